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
// out[q][64] / am[q][64] at channels c0 + 8c, for a workgroup of T threads.  pad_lds (conv12 split):
// the pooled values also go into the zero-padded conv2 input image (swzpad, its channels c0 ..) and
// the global stores are sc1 (write-through: the partner workgroup reads them in the same launch).
template <int H, int CH, int T>
DEV void pool_emit_c(const bf16* img, bf16* out, uint8_t* am, int c0, int tid, bf16* pad_lds = nullptr) {
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
    if (pad_lds) {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), buf_rsrc(out), (uint32_t)(q * 64 + c0 + c * 8) * 2, 0, kSC1);
      st_out8(am, (uint32_t)(q * 64 + c0 + c * 8), make_uint2(alo, ahi));
      *reinterpret_cast<uint4*>(pad_lds + swzpad((py + 2) * (HO + 4) + px + 2, (c0 >> 3) + c)) = o;
    } else {
      st_out16(out, (uint32_t)(q * 64 + c0 + c * 8) * 2, o);           // write-through (common.h)
      st_out8(am, (uint32_t)(q * 64 + c0 + c * 8), make_uint2(alo, ahi));
    }
  }
}

// ---------------------------------------------------------------------------------------------
// conv1 (+ uint8 gather / center crop, bias, ReLU, pool1) of NCO output channels of one image.
// (body shared with the fused conv12 split kernel below: xin [28][24][16] row windows, img
// [576][NCO] (swzc); pad_lds: see pool_emit_c)
template <int NCO>
DEV void conv1_split_body(const DmlcConv1FwdArgs& a, int b, int h, bf16* xin, bf16* img, bf16* pad_lds = nullptr) {
  constexpr int CT = NCO / 16, CH = NCO / 8;
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
  pool_emit_c<24, CH, SP_NT>(img, reinterpret_cast<bf16*>(a.out) + (size_t)b * 9216, a.am + (size_t)b * 9216, co0, tid,
                             pad_lds);
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 3);
}
template <int NCO>
__global__ __launch_bounds__(SP_NT, 4) void k_conv1_fwd_split(DmlcConv1FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int b, h;
  split_index<64 / NCO>(blockIdx.x, b, h);
  bf16* xin = reinterpret_cast<bf16*>(smem);
  conv1_split_body<NCO>(a, b, h, xin, xin + C1_XIN);
}

// conv2 (padded input complete in xin) + bias + ReLU + pool2 of output channels 32h .. 32h+31 of image b
DEV void conv2_split_rest(const DmlcConv2FwdArgs& a, int b, int h, bf16* xin, bf16* ws) {
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), g = lane >> 4, li = lane & 15;
  bf16* img = xin;                                       // [144][32] conv output, after the core
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

// conv2 + bias + ReLU + pool2 of 32 output channels of one image (S = 2 workgroups per image)
__global__ __launch_bounds__(SP_NT, 4) void k_conv2_fwd_split(DmlcConv2FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xin = reinterpret_cast<bf16*>(smem + SP_XIN);
  bf16* ws = reinterpret_cast<bf16*>(smem + SP_WS0);
  int b, h;
  split_index<2>(blockIdx.x, b, h);
  const int tid = threadIdx.x;
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
  conv2_split_rest(a, b, h, xin, ws);
}

// conv1 -> pool1 -> conv2 -> pool2 of image b in ONE launch, two workgroups per image (B <= 128): half
// h computes conv1 / pool1 channels 32h.. straight into its padded conv2 input, stores them write-
// through (sc1) for the backward AND for its partner, raises its flag, waits for the partner's flag,
// reads the partner's 32 channels (sc1) and runs conv2 / pool2 of output channels 32h..  -- the p1
// round trip and the launch boundary between conv1_fwd_split and conv2_fwd_split go away.
// flags[32 * (2b + h)]: zero between launches (the reader resets the flag it consumed).  Both halves
// of an image must be co-resident: grid 2B <= the CU count (one workgroup per CU at this LDS size,
// host-checked); the spin is bounded (the sticky error word) like every other hand-off.
// LDS: [0, 32 KB) the padded conv2 input; then conv1's row windows + output [576][32] (58 KB), which
// conv2's weight slices (40 KB, after pool1) overwrite.
constexpr size_t C12S_X1 = (size_t)C2_XIN * 2, C12S_LDS = C12S_X1 + (size_t)(C1_XIN + 576 * 32) * 2;
static_assert(C12S_LDS <= 160 * 1024 && SP_LDS <= C12S_LDS, "conv12 split LDS map");
__global__ __launch_bounds__(SP_NT, 1) void k_conv12_fwd_split(DmlcConv1FwdArgs a1, DmlcConv2FwdArgs a2,
                                                                unsigned* flags, unsigned* err) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xin2 = reinterpret_cast<bf16*>(smem);
  bf16* xin1 = reinterpret_cast<bf16*>(smem + C12S_X1);
  int b, h;
  split_index<2>(blockIdx.x, b, h);
  const int tid = threadIdx.x;
  for (int s = tid; s < 2048; s += SP_NT) {             // halo of the padded conv2 input
    const int pix = s >> 3, c = s & 7, r = pix >> 4, col = pix & 15;
    if (r < 2 || r >= 14 || col < 2 || col >= 14) *reinterpret_cast<bf16x8*>(xin2 + swzpad(pix, c)) = bf16x8{};
  }
  conv1_split_body<32>(a1, b, h, xin1, xin1 + C1_XIN, xin2);
  wait_vm_all();                                         // this thread's sc1 p1 stores are acknowledged
  __syncthreads();
  unsigned* mine = flags + 32 * (2 * b + h);
  unsigned* theirs = flags + 32 * (2 * b + (h ^ 1));
  if (tid == 0) {
    __hip_atomic_store(mine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool seen = true;
    for (unsigned it = 0; __hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u; ++it) {
      if (it >= DMLC_SPIN_LIMIT) {
        __hip_atomic_fetch_or(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        seen = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    // re-armed for the next launch -- only after a successful wait: a timed-out waiter must not clear
    // a flag its late partner has not raised yet (the engine re-zeroes every flag after an error)
    if (seen) __hip_atomic_store(theirs, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  // the partner's 32 channels: 144 pixels x 4 chunks of 16 B
  const rsrc_t p1 = buf_rsrc(reinterpret_cast<const bf16*>(a1.out) + (size_t)b * 9216);
  const int c0 = 4 * (h ^ 1);
  for (int s = tid; s < 144 * 4; s += SP_NT) {
    const int q = s >> 2, c = c0 + (s & 3), py = q / 12, px = q - py * 12;
    const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(p1, (uint32_t)(q * 64 + c * 8) * 2, 0, kSC1));
    *reinterpret_cast<uint4*>(xin2 + swzpad((py + 2) * 16 + px + 2, c)) = v;
  }
  __syncthreads();
  conv2_split_rest(a2, b, h, xin2, reinterpret_cast<bf16*>(smem + C12S_X1));
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

hipError_t dmlc_conv12_fwd_split(const DmlcConv1FwdArgs* a1, const DmlcConv2FwdArgs* a2, unsigned* flags,
                                 unsigned* err, hipStream_t s) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return hipErrorInvalidValue;
  }
  // both workgroups of an image co-resident: one per CU at this LDS size
  if (a1->B != a2->B || a1->B % 8 || a1->amax || 2 * a1->B > cus || !flags || !err) return hipErrorInvalidValue;
  DMLC_LDS_OPTIN(&k_conv12_fwd_split, C12S_LDS);
  hipLaunchKernelGGL(k_conv12_fwd_split, dim3(a1->B * 2), dim3(SP_NT), C12S_LDS, s, *a1, *a2, flags, err);
  return hipGetLastError();
}

hipError_t dmlc_conv2_dgrad_split(const DmlcConv2DgradArgs* a, hipStream_t s) {
  if (a->B % 8 || !a->dp1) return hipErrorInvalidValue;
  DMLC_LDS_OPTIN(&k_conv2_dgrad_split, SP_LDS);
  hipLaunchKernelGGL(k_conv2_dgrad_split, dim3(a->B * 2), dim3(SP_NT), SP_LDS, s, *a);
  return hipGetLastError();
}

}  // extern "C"
