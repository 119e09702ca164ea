// Channel-split convolution kernels of the CIFAR-10 CNN for gfx950 (MI355X): each image is processed
// by S workgroups, workgroup h owning the output channels [h*64/S, (h+1)*64/S).
//
// Replaces TF's Conv2D / BiasAdd / Relu / MaxPool and Conv2DBackpropInput of
// /root/reference/cifar10cnn.py:106-123 at small per-GPU batches.
//
// Why: the per-image kernels (cnn_conv.hip) launch one 8-wave workgroup per image and hold ~130 KB of
// LDS, i.e. one workgroup per CU: at the reference's batch of 128 half the 256 CUs idle, and at 256
// every CU runs one long dependent chain (stage -> MFMA -> pool) with nothing beside it.  Here every
// workgroup keeps <= 72 KB of LDS and <= 128 VGPRs, so B*S workgroups fill the chip and two of them
// share a CU, each one's VALU/LDS phases (staging, pooling) running beside the other's MFMAs.
//   * max-pool is per channel, so a channel slice pools on its own: no exchange between workgroups;
//   * conv1 (K = 75): wave w owns pixel tiles w, w+8, ... and the block's co tiles, weights in
//     registers (the slice of conv1 weights is 10 KB);
//   * conv2 forward / input gradient (K = 1600): the 32-channel weight slice is streamed per kernel
//     row (20 KB) by LDS-DMA, double-buffered; the 8 waves split the K of every kernel row by input-
//     channel half (so both halves consume the same slice at the same time) and own 2-3 pixel tiles
//     x both co tiles; the K halves meet once through LDS at the end (fixed order: deterministic);
//   * the S parts of image b are blocks (b & 7) + 8 h + 8 S (b >> 3): one XCD per image under
//     round-robin placement, so an image's input crosses HBM -> L2 once (placement is speed only).
#include "split_common.h"

namespace dmlc {

// TF-SAME 3x3/2 max pool (pool_emit of conv_common.h) over an LDS image [H*H][CH*8] -> global
// out[q][64] / am[q][64] at channels c0 + 8c, for a workgroup of T threads.
template <int H, int CH, int T>
DEV void pool_emit_c(const bf16* img, bf16* out, uint8_t* am, int c0, int tid) {
  constexpr int HO = H / 2;
  for (int task = tid; task < HO * HO * CH; task += T) {
    const int q = task / CH, c = task - q * CH;
    const int py = q / HO, px = q - py * HO;
    // branch-free (see pool_emit): all 9 taps loaded back to back
    uint4 v[9];
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      const int y = min(2 * py + d / 3, H - 1), x = min(2 * px + d % 3, H - 1);
      v[d] = *reinterpret_cast<const uint4*>(img + swzc<CH>(y * H + x, c));
    }
    uint4 o;
    uint32_t alo, ahi, bmax = 0;
    pool_window(v, o, alo, ahi, bmax);
    st_maybe_nt<kNtX>(reinterpret_cast<uint4*>(out + q * 64 + c0 + c * 8), o);
    st_maybe_nt<kNtX>(reinterpret_cast<uint2*>(am + q * 64 + c0 + c * 8), make_uint2(alo, ahi));
  }
}

// ---------------------------------------------------------------------------------------------
// conv1 (+ uint8 gather / center crop, bias, ReLU, pool1) of NCO output channels of one image.
template <int NCO>
__global__ __launch_bounds__(SP_NT, 4) void k_conv1_fwd_split(DmlcConv1FwdArgs a) {
  constexpr int S = 64 / NCO, CT = NCO / 16, CH = NCO / 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xin = reinterpret_cast<bf16*>(smem);                 // [28][24][16] row windows
  bf16* img = xin + C1_XIN;                                  // [576][NCO] (swzc)
  int b, h;
  split_index<S>(blockIdx.x, b, h);
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), g = lane >> 4, li = lane & 15;
  const int co0 = NCO * h;
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 0);

  const int row = batch_index(a.src, a.B, b);
  uint8_t* raw = reinterpret_cast<uint8_t*>(img) + 16;       // free until the epilogue (16 B of halo slack)
  stage_conv1_raw(raw, a.data + (size_t)row * 3072, (a.xraw && h == 0) ? a.xraw + (size_t)b * 3072 : nullptr, tid);
  // this slice's weights [co0 + 16 ct + li][k = 32 kh + 8 g ..] and biases, in flight with the image
  const bf16* W = reinterpret_cast<const bf16*>(a.w) + (co0 + li) * C1_K + 8 * g;
  bf16x8 wa[CT][3];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int s = 0; s < 3; ++s) wa[ct][s] = glb_b128(W + ct * 16 * C1_K + 32 * s);
  float b4[CT][4];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int i = 0; i < 4; ++i) b4[ct][i] = a.bias[co0 + 16 * ct + 4 * g + i];
  __syncthreads();
  stage_conv1_input(xin, raw, a.cy, a.cx, tid);
  __syncthreads();
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 1);

  // pixel tiles w, w+8, ... (< 36): 5 for waves 0-3, 4 for waves 4-7 (waves w, w+4 share a SIMD)
  auto load_tile = [&](int t, bf16x8 (&bx)[3]) { conv1_frag_tile(xin, t * 16 + li, g, bx); };
  bf16x8 BX[2][3];
  load_tile(w, BX[0]);
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int t = w + 8 * i;
    if (t >= 36) break;                                      // wave-uniform
    const int cur = i & 1;
    wait_lds();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 8 < 36) load_tile(t + 8, BX[cur ^ 1]);
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[ct] = zero4();
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[ct] = mfma16(wa[ct][s], BX[cur][s], acc[ct]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) store_relu_c<CH>(img, t * 16 + li, 16 * ct + 4 * g, acc[ct], b4[ct]);
  }
  __syncthreads();
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 2);
  pool_emit_c<24, CH, SP_NT>(img, reinterpret_cast<bf16*>(a.out) + (size_t)b * 9216, a.am + (size_t)b * 9216, co0, tid);
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 3);
}

// conv2 + bias + ReLU + pool2 of 32 output channels of one image (S = 2 workgroups per image)
__global__ __launch_bounds__(SP_NT, 4) void k_conv2_fwd_split(DmlcConv2FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xin = reinterpret_cast<bf16*>(smem + SP_XIN);
  bf16* ws = reinterpret_cast<bf16*>(smem + SP_WS0);
  bf16* img = xin;                                       // [144][32] conv output, after the core
  int b, h;
  split_index<2>(blockIdx.x, b, h);
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), g = lane >> 4, li = lane & 15;
  DMLC_STAMP(DMLC_TK_CONV2_FWD, 0);
  const bf16* in = reinterpret_cast<const bf16*>(a.in) + (size_t)b * 9216;
  uint4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int s = tid + i * SP_NT, pix = s >> 3, c = s & 7;
    const int iy = (pix >> 4) - 2, ix = (pix & 15) - 2;
    v[i] = load_sel(reinterpret_cast<const uint4*>(in + (iy * 12 + ix) * 64 + c * 8), reinterpret_cast<const uint4*>(in),
                    iy >= 0 && iy < 12 && ix >= 0 && ix < 12);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int s = tid + i * SP_NT;
    *reinterpret_cast<uint4*>(xin + swzpad(s >> 3, s & 7)) = v[i];
  }
  float b4[2][4];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) b4[c][i] = a.bias[32 * h + 16 * c + 4 * g + i];
  split_tiles(reinterpret_cast<const bf16*>(a.w) + (size_t)32 * h * 1600, xin, ws, w, g, li, lane, DMLC_TK_CONV2_FWD,
              [&](int c, int t, const f32x4& acc) { store_relu_c<4>(img, 16 * t + li, 16 * c + 4 * g, acc, b4[c]); });
  __syncthreads();
  DMLC_STAMP(DMLC_TK_CONV2_FWD, 2);
  pool_emit_c<12, 4, SP_NT>(img, reinterpret_cast<bf16*>(a.out) + (size_t)b * 2304, a.am + (size_t)b * 2304, 32 * h, tid);
  DMLC_STAMP(DMLC_TK_CONV2_FWD, 3);
}

__global__ __launch_bounds__(SP_NT, 4) void k_conv2_dgrad_split(DmlcConv2DgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int b, h;
  split_index<2>(blockIdx.x, b, h);
  conv2_dgrad_split_image<false>(a, b, h, smem);
}

}  // namespace dmlc

using namespace dmlc;

extern "C" {

hipError_t dmlc_conv1_fwd_split(const DmlcConv1FwdArgs* a, int nsplit, hipStream_t s) {
  if (a->B % 8 || a->amax) return hipErrorInvalidValue;
  if (nsplit == 2) {
    const size_t lds = (C1_XIN + 576 * 32) * 2;
    hipLaunchKernelGGL(k_conv1_fwd_split<32>, dim3(a->B * 2), dim3(SP_NT), lds, s, *a);
  } else if (nsplit == 4) {
    const size_t lds = (C1_XIN + 576 * 16) * 2;
    hipLaunchKernelGGL(k_conv1_fwd_split<16>, dim3(a->B * 4), dim3(SP_NT), lds, s, *a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t dmlc_conv2_fwd_split(const DmlcConv2FwdArgs* a, hipStream_t s) {
  if (a->B % 8) return hipErrorInvalidValue;
  DMLC_LDS_OPTIN(&k_conv2_fwd_split, SP_LDS);
  hipLaunchKernelGGL(k_conv2_fwd_split, dim3(a->B * 2), dim3(SP_NT), SP_LDS, s, *a);
  return hipGetLastError();
}

hipError_t dmlc_conv2_dgrad_split(const DmlcConv2DgradArgs* a, hipStream_t s) {
  if (a->B % 8 || !a->dp1) return hipErrorInvalidValue;
  DMLC_LDS_OPTIN(&k_conv2_dgrad_split, SP_LDS);
  hipLaunchKernelGGL(k_conv2_dgrad_split, dim3(a->B * 2), dim3(SP_NT), SP_LDS, s, *a);
  return hipGetLastError();
}

}  // extern "C"
