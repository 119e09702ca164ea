// fp8 (OCP e4m3fn) conv2 forward for the large-batch configuration (BASELINE.json config 5,
// SURVEY.md §2.C "fp8 large-batch").  Same decomposition as the bf16 k_conv2_fwd (one image per
// 512-thread block, weight slices staged through LDS once per block, 2 c_out tiles x 2-3 pixel tiles
// per wave) with both MFMA operands in fp8: __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8 takes
// 8 x fp8 per lane, so every A/B fragment is one ds_read_b64 -- half the LDS and L2 bytes of bf16.
// (On gfx950 the non-scaled fp8 MFMA issues at the bf16 rate; the win is operand traffic, which is
// what bounds this kernel.)  Scaling is per tensor and delayed (graph-capturable, no host sync):
//   activations: sx = 448 / amax(p1), amax accumulated by conv1_fwd's pool epilogue this step;
//   weights:     w2f8 = sat(W2 * sw) written by the SGD kernel together with sw (cnn_sgd.hip).
// Backward stays bf16 (dgrad/wgrad read the bf16 p1 and the bf16 W2 shadows).
#include "conv_common.h"

namespace dmlc {

typedef long fp8x8;                           // 8 packed e4m3 values (MFMA operand)

constexpr int X8_BYTES = 256 * 64;            // [16x16 padded pixels][64 ch] fp8, 8-B chunks swizzled
constexpr int W8_LD = 336;                    // slice row stride (bytes): b64 reads of 16 rows conflict-free
constexpr int W8_SLICE = 64 * W8_LD;
constexpr size_t FP8_LDS = X8_BYTES + 2 * W8_SLICE + 144 * 64 * 2;

DEV int x8_off(int px, int chunk) { return px * 64 + ((chunk ^ (px & 7)) << 3); }

DEV f32x4 mfma_fp8(fp8x8 a, fp8x8 b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a, b, c, 0, 0, 0);
}

DEV void w8_load(uint4 (&v)[3], const uint8_t* __restrict__ W, int kh, int tid) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {                // 64 rows x 20 chunks of 16 B = 1280 chunks
    const int c = min(tid + i * NT, 1279), row = c / 20, k16 = c - row * 20;
    v[i] = *reinterpret_cast<const uint4*>(W + row * 1600 + kh * 320 + k16 * 16);
  }
}
DEV void w8_store(const uint4 (&v)[3], uint8_t* ws, int tid) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int c = tid + i * NT;
    if (c < 1280) {
      const int row = c / 20, k16 = c - row * 20;
      *reinterpret_cast<uint4*>(ws + row * W8_LD + k16 * 16) = v[i];
    }
  }
}

template <int NPX>
DEV void conv2_core_fp8(const uint8_t* __restrict__ W, const uint8_t* x8, uint8_t* ws, f32x4 (&acc)[2][NPX], int pg,
                        int cp, int g, int li, int tid) {
  int pb[NPX];
#pragma unroll
  for (int t = 0; t < NPX; ++t) {
    const int px = 16 * (pg + 4 * t) + li;
    const int y = px / 12;
    pb[t] = y * 16 + (px - y * 12);
  }
#pragma unroll
  for (int t = 0; t < NPX; ++t) { acc[0][t] = zero4(); acc[1][t] = zero4(); }
  uint4 pf[3];
  w8_load(pf, W, 0, tid);
  w8_store(pf, ws, tid);
  __syncthreads();
#pragma unroll
  for (int kh = 0; kh < 5; ++kh) {
    w8_load(pf, W, kh < 4 ? kh + 1 : 4, tid);
    const uint8_t* wsb = ws + (kh & 1) * W8_SLICE + (32 * cp + li) * W8_LD + 8 * g;
#pragma unroll
    for (int kw = 0; kw < 5; ++kw) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const fp8x8 a0 = *reinterpret_cast<const fp8x8*>(wsb + kw * 64 + s * 32);
        const fp8x8 a1 = *reinterpret_cast<const fp8x8*>(wsb + 16 * W8_LD + kw * 64 + s * 32);
#pragma unroll
        for (int t = 0; t < NPX; ++t) {
          const fp8x8 bx = *reinterpret_cast<const fp8x8*>(x8 + x8_off(pb[t] + kh * 16 + kw, 4 * s + g));
          acc[0][t] = mfma_fp8(a0, bx, acc[0][t]);
          acc[1][t] = mfma_fp8(a1, bx, acc[1][t]);
        }
      }
    }
    w8_store(pf, ws + ((kh + 1) & 1) * W8_SLICE, tid);
    __syncthreads();
  }
}

__global__ __launch_bounds__(NT, 1) void k_conv2_fwd_fp8(DmlcConv2FwdFp8Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint8_t* x8 = reinterpret_cast<uint8_t*>(smem);
  uint8_t* ws = x8 + X8_BYTES;
  bf16* cout = reinterpret_cast<bf16*>(ws + 2 * W8_SLICE);
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int g = lane >> 4, li = lane & 15, cp = w & 1, pg = w >> 1;
  const int slot = a.counter ? (int)(*a.counter & 1) : 0;
  const float sx = 448.f / fmaxf(a.amax_x[slot], 1e-20f), sw = a.scale_w[slot];
  const float inv = 1.f / (sx * sw);
  const bf16* in = reinterpret_cast<const bf16*>(a.in) + (size_t)b * 9216;

  // stage: bf16 -> scaled fp8, zero halo (16x16 padded image, pixel (iy,ix) at (iy+2, ix+2))
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
    const uint32_t wv[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
    const uint32_t lo = pk_fp8x4(bf16_lo(wv[0]) * sx, bf16_hi(wv[0]) * sx, bf16_lo(wv[1]) * sx, bf16_hi(wv[1]) * sx);
    const uint32_t hi = pk_fp8x4(bf16_lo(wv[2]) * sx, bf16_hi(wv[2]) * sx, bf16_lo(wv[3]) * sx, bf16_hi(wv[3]) * sx);
    *reinterpret_cast<uint2*>(x8 + x8_off(s >> 3, s & 7)) = make_uint2(lo, hi);
  }
  float b4[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i) b4[h][i] = a.bias[32 * cp + 16 * h + 4 * g + i];
  __syncthreads();

  auto epi = [&](int ct, int t, f32x4 acc) {
    acc[0] *= inv; acc[1] *= inv; acc[2] *= inv; acc[3] *= inv;
    store_relu_tile(cout, 16 * t + li, 16 * ct + 4 * g, acc, b4[ct & 1]);
  };
  if (pg == 0) {
    f32x4 acc[2][3];
    conv2_core_fp8<3>(a.w8, x8, ws, acc, pg, cp, g, li, tid);
#pragma unroll
    for (int t = 0; t < 3; ++t) { epi(2 * cp, pg + 4 * t, acc[0][t]); epi(2 * cp + 1, pg + 4 * t, acc[1][t]); }
  } else {
    f32x4 acc[2][2];
    conv2_core_fp8<2>(a.w8, x8, ws, acc, pg, cp, g, li, tid);
#pragma unroll
    for (int t = 0; t < 2; ++t) { epi(2 * cp, pg + 4 * t, acc[0][t]); epi(2 * cp + 1, pg + 4 * t, acc[1][t]); }
  }
  __syncthreads();
  pool_emit<12>(cout, reinterpret_cast<bf16*>(a.out) + (size_t)b * 2304, a.am + (size_t)b * 2304, tid);
}

// quantise -> dequantise through the hardware converter (numerics test of the fp8 format: OCP e4m3fn)
__global__ void k_fp8_roundtrip(const float* x, float* y, int n, float scale) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t w = pk_fp8x4(x[i] * scale, 0.f, 0.f, 0.f);
  y[i] = __builtin_amdgcn_cvt_f32_fp8((int)w, 0) / scale;
}

}  // namespace dmlc

using namespace dmlc;

namespace {
bool g_fp8 = false;
}

extern "C" {

hipError_t dmlc_conv2_fwd_fp8(const DmlcConv2FwdFp8Args* a, hipStream_t s) {
  if (!g_fp8) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_conv2_fwd_fp8),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)FP8_LDS);
    g_fp8 = true;
  }
  hipLaunchKernelGGL(k_conv2_fwd_fp8, dim3(a->B), dim3(NT), FP8_LDS, s, *a);
  return hipGetLastError();
}

hipError_t dmlc_fp8_roundtrip(const float* x, float* y, int n, float scale, hipStream_t s) {
  hipLaunchKernelGGL(k_fp8_roundtrip, dim3((n + 255) / 256), dim3(256), 0, s, x, y, n, scale);
  return hipGetLastError();
}

}  // extern "C"
