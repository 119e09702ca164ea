// Convolution kernels of the CIFAR-10 CNN for gfx950 (MI355X), one image per 512-thread workgroup.
//
// Replaces TF's Conv2D / BiasAdd / Relu / MaxPool (+ their gradients) used by
// /root/reference/cifar10cnn.py:106-123.
//
// Design (MI355X-first, not a cuDNN translation):
//   * implicit GEMM on MFMA 16x16x32 bf16 with the GEMM formulated TRANSPOSED (C[channel][pixel]):
//     the weight fragment comes from global/L2 (shared by every workgroup), the pixel fragment is read
//     straight out of an LDS image of the zero-padded input — no im2col buffer ever exists;
//     each lane then owns 4 consecutive channels of one pixel, i.e. an 8-byte NHWC store;
//   * bias + ReLU + TF-SAME 3x3/2 max-pool are fused into the epilogue: the whole conv output of an
//     image stays in LDS, the pool emits the pooled bf16 tensor plus a 1-byte argmax per output
//     (255 encodes "pooled <= 0", i.e. the ReLU mask), so the backward never re-reads activations;
//   * conv1 gathers its uint8 input directly from the device-resident dataset (index list + center
//     crop), so the input pipeline (N1-N3) costs no extra launch;
//   * conv1's K=75 (5x5x3) is laid out as k = kh*16 + kw*3 + ci (K 80, padded to 96 = 3 k-steps):
//     the LDS input holds 5-tap row windows (conv_common.h stage_conv1_input), so every fragment is
//     16 contiguous bytes of it (r4 padded K to 160: kw to 8, ci to 4 -- 40 % of those MFMAs were zeros);
//   * backward: pool/ReLU backward is a *gather* (each input pixel sums the <=4 windows whose argmax
//     points at it: deterministic, no atomics) fused into the staging of the dgrad/wgrad operands;
//     weight gradients read both operands from NHWC LDS images with ds_read_b64_tr_b16 (hardware
//     transpose) so no transposed copies are materialised; they are split-K over image groups with
//     fp32 partial slabs reduced deterministically by the SGD kernel.
#include "conv2_core.h"

namespace dmlc {


// conv1 implicit GEMM of one wave: co tiles 2cp, 2cp+1 (weights wa in registers) x pixel tiles
// 9pq .. 9pq+8.  Software-pipelined: the 3 B fragments of pixel tile t+1 are read from LDS while tile
// t's 6 MFMAs run (wait_lds retires tile t's reads first; see common.h).
// the wave's weight fragments: rows co0 + li (+16 for h = 1) of the [64][96] shadow
DEV void conv1_wfrags(const void* w, int co0, int g, int li, bf16x8 (&wa)[2][3]) {
  const bf16* W = reinterpret_cast<const bf16*>(w) + (co0 + li) * C1_K + 8 * g;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int s = 0; s < 3; ++s) wa[h][s] = glb_b128(W + h * 16 * C1_K + 32 * s);
}
DEV void conv1_mfma(const bf16* xin, const bf16x8 (&wa)[2][3], f32x4 (&acc)[2][9], int pq, int g, int li) {
  auto load_tile = [&](int t, bf16x8 (&bx)[3]) { conv1_frag_tile(xin, (pq * 9 + t) * 16 + li, g, bx); };
#pragma unroll
  for (int t = 0; t < 9; ++t) { acc[0][t] = zero4(); acc[1][t] = zero4(); }
  bf16x8 BX[2][3];
  load_tile(0, BX[0]);
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int cur = t & 1;
    wait_lds();
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < 9) load_tile(t + 1, BX[cur ^ 1]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      acc[0][t] = mfma16(wa[0][s], BX[cur][s], acc[0][t]);
      acc[1][t] = mfma16(wa[1][s], BX[cur][s], acc[1][t]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NT, 1) void k_conv1_fwd(DmlcConv1FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xin = reinterpret_cast<bf16*>(smem);
  bf16* cout = xin + C1_XIN;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int g = lane >> 4, li = lane & 15, cp = w & 1, pq = w >> 1;
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 0);

  const int img = batch_index(a.src, a.B, b);
  uint8_t* raw = reinterpret_cast<uint8_t*>(cout) + 16;     // the conv output region is free until the epilogue
  stage_conv1_raw(raw, a.data + (size_t)img * 3072, a.xraw ? a.xraw + (size_t)b * 3072 : nullptr, tid);
  __syncthreads();
  stage_conv1_input(xin, raw, a.cy, a.cx, tid);

  // A operand: weights [64 co][96 k]; this wave owns co tiles 2cp, 2cp+1 (32 channels) and the
  // pixel tiles 9pq .. 9pq+8 (of 36): every B fragment read from LDS feeds two MFMAs.
  bf16x8 wa[2][3];
  conv1_wfrags(a.w, 32 * cp, g, li, wa);
  float b4[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i) b4[h][i] = a.bias[32 * cp + 16 * h + 4 * g + i];
  __syncthreads();
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 1);

  f32x4 acc[2][9];
  conv1_mfma(xin, wa, acc, pq, g, li);
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      store_relu_tile(cout, (pq * 9 + t) * 16 + li, 32 * cp + 16 * h + 4 * g, acc[h][t], b4[h]);
  __syncthreads();
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 2);
  uint32_t vmax = 0;
  pool_emit<24>(cout, reinterpret_cast<bf16*>(a.out) + (size_t)b * 9216, a.am + (size_t)b * 9216, tid, &vmax);
  if (a.amax) {                                // fp8 path: this image's max of the pooled activations
    // one plain store per image (amax[b]); the fp8 conv2 forward reduces the B maxima itself.  (One
    // same-address atomic per wave serialised at the L2: 8192 of them cost 70 us at B=1024.)
    float* red = reinterpret_cast<float*>(smem + (C1_XIN + C1_OUT) * 2);
    uint32_t m = vmax;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    if ((tid & 63) == 0) red[w] = __uint_as_float(m << 16);   // bf16 bits -> fp32 (pooled >= 0)
    __syncthreads();
    if (tid == 0) {
      float v = red[0];
#pragma unroll
      for (int i = 1; i < NT / 64; ++i) v = fmaxf(v, red[i]);
      a.amax[b] = v;
    }
  }
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 3);
}


__global__ __launch_bounds__(NT, 1) void k_conv2_fwd(DmlcConv2FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xin = reinterpret_cast<bf16*>(smem);
  bf16* cout = xin + C2_XIN;
  bf16* ws = cout + C2_OUT;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int g = lane >> 4, li = lane & 15;
  const bf16* in = reinterpret_cast<const bf16*>(a.in) + (size_t)b * 9216;
  DMLC_STAMP(DMLC_TK_CONV2_FWD, 0);

  uint4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int s = tid + i * NT, pix = s >> 3, c = s & 7;
    const int iy = (pix >> 4) - 2, ix = (pix & 15) - 2;
    v[i] = load_sel(reinterpret_cast<const uint4*>(in + (iy * 12 + ix) * 64 + c * 8), reinterpret_cast<const uint4*>(in),
                    iy >= 0 && iy < 12 && ix >= 0 && ix < 12);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int s = tid + i * NT;
    *reinterpret_cast<uint4*>(xin + swzpad(s >> 3, s & 7)) = v[i];
  }
  ws_dma(reinterpret_cast<const bf16*>(a.w), 0, ws, w, lane);   // kernel row 0, landed by the core's barrier
  float b4[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) b4[c][i] = a.bias[16 * c + 4 * g + i];
  DMLC_STAMP(DMLC_TK_CONV2_FWD, 1);

  conv2_tiles(reinterpret_cast<const bf16*>(a.w), xin, ws, w, g, li, tid, ws, [&](int ct, int t, const f32x4& acc) {
    store_relu_tile(cout, 16 * t + li, 16 * ct + 4 * g, acc, b4[ct]);
  });
  __syncthreads();
  DMLC_STAMP(DMLC_TK_CONV2_FWD, 2);
  pool_emit<12>(cout, reinterpret_cast<bf16*>(a.out) + (size_t)b * 2304, a.am + (size_t)b * 2304, tid);
  DMLC_STAMP(DMLC_TK_CONV2_FWD, 3);
}

__global__ __launch_bounds__(NT, 1) void k_conv2_dgrad(DmlcConv2DgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv2_dgrad_image<false>(a, blockIdx.x, smem);
}

// ---------------------------------------------------------------------------------------------
// conv1 -> pool1 -> conv2 -> pool2 of one image in ONE launch (bf16 path): the images are
// independent, so the pool1 output goes straight into conv2's zero-padded LDS input instead of
// round-tripping through global memory and a second launch (p1 / am1 are still written for the
// backward).  LDS: [0, 80 KB) conv1 output (72 KB), then conv2's two weight-slice buffers;
// [80, 112 KB) conv2's padded input; [112, 130 KB) conv2's output; [130, 151 KB) conv1's input.
// Kernel row 0 of the conv2 weights is loaded into registers at entry and stored into the first
// slice buffer after pool1: its L2 latency hides behind conv1 instead of opening the conv2 core
// (~1 us of the core's first row, r3 phase stamps).
constexpr size_t C12_WS = 0, C12_XIN2 = 81920, C12_OUT2 = C12_XIN2 + C2_XIN * 2;
constexpr size_t C12_XIN1 = C12_OUT2 + C2_OUT * 2, C12_LDS = C12_XIN1 + C1_XIN * 2;
static_assert(C1_OUT * 2 <= C12_XIN2 && WS_BYTES <= C12_XIN2 && C12_LDS <= 160 * 1024, "conv12 LDS map");

__global__ __launch_bounds__(NT, 1) void k_conv12_fwd(DmlcConv1FwdArgs a1, DmlcConv2FwdArgs a2) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xin = reinterpret_cast<bf16*>(smem + C12_XIN1);
  bf16* cout = reinterpret_cast<bf16*>(smem);
  bf16* xin2 = reinterpret_cast<bf16*>(smem + C12_XIN2);
  bf16* cout2 = reinterpret_cast<bf16*>(smem + C12_OUT2);
  bf16* ws = reinterpret_cast<bf16*>(smem + C12_WS);
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int g = lane >> 4, li = lane & 15, cp = w & 1, pq = w >> 1;
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 0);

  // conv1 weights / biases first: in flight together with the index -> image chain
  bf16x8 wa[2][3];
  conv1_wfrags(a1.w, 32 * cp, g, li, wa);
  float b4[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i) b4[h][i] = a1.bias[32 * cp + 16 * h + 4 * g + i];
  uint8_t* raw = reinterpret_cast<uint8_t*>(cout) + 16;     // the conv1 output region is free until its epilogue
  if (a1.xraw_in) {                            // prefetched by the previous step: one load, no index hop
    stage_conv1_raw(raw, a1.xraw + (size_t)b * 3072, nullptr, tid);
  } else {
    const int img = batch_index(a1.src, a1.B, b);
    stage_conv1_raw(raw, a1.data + (size_t)img * 3072, a1.xraw ? a1.xraw + (size_t)b * 3072 : nullptr, tid);
  }
  lds_barrier();   // (the xraw copy's global stores need not drain)
  stage_conv1_input(xin, raw, a1.cy, a1.cx, tid);
  // conv2's padded input: zero halo (rows/cols 0,1,14,15); the interior comes from pool1
  for (int s = tid; s < 2048; s += NT) {
    const int pix = s >> 3, c = s & 7, r = pix >> 4, col = pix & 15;
    if (r < 2 || r >= 14 || col < 2 || col >= 14) *reinterpret_cast<bf16x8*>(xin2 + swzpad(pix, c)) = bf16x8{};
  }
  // conv2 kernel row 0 into registers, in flight during conv1 + pool1 (issued after every load that
  // conv1 waits for, so those waits count past it); stored to LDS once pool1 has freed the conv1 region
  const Slice5 s0v = ws_fetch(reinterpret_cast<const bf16*>(a2.w), 0, w, lane);
  lds_barrier();
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 1);

  {
    f32x4 acc[2][9];
    conv1_mfma(xin, wa, acc, pq, g, li);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        store_relu_tile(cout, (pq * 9 + t) * 16 + li, 32 * cp + 16 * h + 4 * g, acc[h][t], b4[h]);
  }
  lds_barrier();
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 2);
  pool_emit<24>(cout, reinterpret_cast<bf16*>(a1.out) + (size_t)b * 9216, a1.am + (size_t)b * 9216, tid, nullptr, xin2);
  float c2b[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) c2b[c][i] = a2.bias[16 * c + 4 * g + i];
  lds_barrier();                                       // conv2 input complete; conv1 region free
  ws_put(ws, w, lane, s0v);                            // published by the core's first barrier
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 3);

  conv2_tiles(reinterpret_cast<const bf16*>(a2.w), xin2, ws, w, g, li, tid, ws, [&](int ct, int t, const f32x4& acc) {
    store_relu_tile(cout2, 16 * t + li, 16 * ct + 4 * g, acc, c2b[ct]);
  }, DMLC_TK_CONV1_FWD);
  __syncthreads();
  pool_emit<12>(cout2, reinterpret_cast<bf16*>(a2.out) + (size_t)b * 2304, a2.am + (size_t)b * 2304, tid);
  DMLC_STAMP(DMLC_TK_CONV1_FWD, 4);
}

}  // namespace dmlc

using namespace dmlc;


extern "C" {

hipError_t dmlc_conv1_fwd(const DmlcConv1FwdArgs* a, hipStream_t s) {
  const size_t lds = (C1_XIN + C1_OUT) * 2 + 64;        // + the fp8 path's 8 wave maxima
  DMLC_LDS_OPTIN(&k_conv1_fwd, lds);
  hipLaunchKernelGGL(k_conv1_fwd, dim3(a->B), dim3(NT), lds, s, *a);
  return hipGetLastError();
}

hipError_t dmlc_conv2_fwd(const DmlcConv2FwdArgs* a, hipStream_t s) {
  const size_t lds = (C2_XIN + C2_OUT) * 2 + WS_BYTES;
  DMLC_LDS_OPTIN(&k_conv2_fwd, lds);
  hipLaunchKernelGGL(k_conv2_fwd, dim3(a->B), dim3(NT), lds, s, *a);
  return hipGetLastError();
}

hipError_t dmlc_conv12_fwd(const DmlcConv1FwdArgs* a1, const DmlcConv2FwdArgs* a2, hipStream_t s) {
  DMLC_LDS_OPTIN(&k_conv12_fwd, C12_LDS);
  if (a1->B != a2->B || a1->amax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_conv12_fwd, dim3(a1->B), dim3(NT), C12_LDS, s, *a1, *a2);
  return hipGetLastError();
}

hipError_t dmlc_conv2_dgrad(const DmlcConv2DgradArgs* a, hipStream_t s) {
  DMLC_LDS_OPTIN(&k_conv2_dgrad, DG_LDS);
  hipLaunchKernelGGL(k_conv2_dgrad, dim3(a->B), dim3(NT), DG_LDS, s, *a);
  return hipGetLastError();
}

}  // extern "C"
