// fp8 (OCP e4m3fn) conv2 forward for the large-batch configuration (BASELINE.json config 5,
// SURVEY.md §2.C "fp8 large-batch") on gfx950's double-rate MFMA, v_mfma_scale_f32_16x16x128_f8f6f4
// (block scales left at 2^0: the tensors carry their own per-tensor scales, below).
//   * K = (tap, ci) runs in chunks of 128 = two 5x5 taps x 64 channels (25 taps + one zero tap = 13
//     chunks); a lane's 32 fp8 of a fragment are 32 consecutive channels of one tap, for the weight
//     row (A, c_out) and the input pixel (B) alike -- the same k order on both sides is all the MFMA
//     needs.
//   * Weight-stationary: a block stages all of W2 (100 KB fp8) ONCE and then runs images b, b + grid,
//     ... (grid = min(B, 256)): at per-GPU batch 1024 a CU reads the weights once for 4 images, not 4
//     times.  The next image's input is prefetched into registers during the current one's MFMAs.
//   * Pixel tiles are 4x4 blocks of the 12x12 output (9 tiles), so with the fp8 input rows (64 B per
//     padded pixel) XOR-swizzled by padded-row parity every B fragment read is conflict-free; weight
//     rows (1792 B) XOR their 16-B units by (row & 1 | ((row >> 1) & 3) << 2): A reads conflict-free.
// Scaling is per tensor and delayed (graph-capturable, no host sync):
//   activations: sx = 448 / amax(p1) of THIS batch: conv1_fwd's pool epilogue stores one maximum per
//                image, every block here reduces the B of them (4 KB at B=1024) behind its weight loads;
//   weights:     w2f8 = sat(W2 * sw) written by the SGD kernel together with sw (cnn_sgd.hip).
// conv2 input gradient (k_conv2_dgrad_fp8): the same weight-stationary core on the flipped, ci-major
// weights (w2d8, quantised by the SGD kernel with the same scale as w2f8) and the pool2/ReLU-backward
// gradient dY2 quantised per IMAGE with sy = 448 / amax(dY2 of that image), reduced in-block from the
// values the block just produced, rounded down to a power of two (r6); the quantised dY2 and its
// scale are also stored (dy8out, sy_img) for the fp8 conv2 weight gradient (cnn_wgrad.hip w2_fp8_main),
// as the forward stores its quantised input and sx (x8out, sx_out).
#include "conv_common.h"

namespace dmlc {

typedef int fp8x32 __attribute__((ext_vector_type(8)));   // 32 packed e4m3 values (MFMA operand)

constexpr int X8_BYTES = 256 * 64;            // [16x16 padded pixels][64 ch] fp8
constexpr int W8_LD = 1792;                   // weight row stride (bytes): 26 taps x 64 used
constexpr int W8_BYTES = 64 * W8_LD;
constexpr size_t FP8_RED = X8_BYTES + W8_BYTES + 144 * 64 * 2;   // 8 wave maxima
constexpr size_t FP8_LDS = FP8_RED + 64;
static_assert(FP8_LDS <= 160 * 1024, "fp8 conv2 LDS");

DEV int x8_addr(int P, int u) { return P * 64 + ((u ^ ((P >> 4) & 1)) << 4); }
DEV int w8_addr(int row, int U) { return row * W8_LD + ((U ^ ((row & 1) | (((row >> 1) & 3) << 2))) << 4); }

DEV f32x4 mfma_fp8(const fp8x32& a, const fp8x32& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}
DEV fp8x32 lds_fp8x32(const uint8_t* lo, const uint8_t* hi) {
  const uint4 a = *reinterpret_cast<const uint4*>(lo), b = *reinterpret_cast<const uint4*>(hi);
  const fp8x32 r = {(int)a.x, (int)a.y, (int)a.z, (int)a.w, (int)b.x, (int)b.y, (int)b.z, (int)b.w};
  return r;
}

// All of an fp8 [64 rows][1600] weight matrix -> LDS: 64 rows x 104 units of 16 B (units 100..103 =
// the zero tap), 13 per thread in two rounds of up to 7 loads in flight.
DEV void stage_w8(const uint8_t* __restrict__ src, uint8_t* w8, int tid) {
#pragma unroll 1
  for (int i0 = 0; i0 < 13; i0 += 7) {
    uint4 wv[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const int e = min(tid + (i0 + i) * NT, 6655), row = e / 104, U = e - row * 104;
      wv[i] = load_sel(reinterpret_cast<const uint4*>(src + row * 1600 + U * 16), reinterpret_cast<const uint4*>(src),
                       U < 100);
    }
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const int e = tid + (i0 + i) * NT, row = e / 104, U = e - row * 104;
      if (e < 6656) *reinterpret_cast<uint4*>(w8 + w8_addr(row, U)) = U < 100 ? wv[i] : make_uint4(0u, 0u, 0u, 0u);
    }
  }
}

// MFMAs of one image: wave (cp, pg) owns c_out tiles 2cp, 2cp+1 x pixel tiles pg, pg+4, pg+8 (< 9).
// Addresses: a padded pixel P = pb + 16 kh + kw never carries into the row bits (x + kw <= 15), so
// its row parity is par(pb) ^ (kh & 1); the two 16-B halves of a lane's 32 B differ in address bit 4
// only (the swizzle XORs 16-B units, u is even), so the second is the first ^ 16.
template <int NPX>
DEV void conv2_core_fp8(const uint8_t* x8, const uint8_t* w8, f32x4 (&acc)[2][NPX], int pg, int cp, int g, int li) {
  const int u = 2 * (g & 1), gh = g >> 1;
  int xb[NPX];                                 // pixel byte base with the unit XOR of tap (0, 0)
#pragma unroll
  for (int t = 0; t < NPX; ++t) {
    const int T = pg + 4 * t, ty = T / 3, tx = T - ty * 3;
    const int pb = (4 * ty + (li >> 2)) * 16 + 4 * tx + (li & 3);   // padded pixel of tap (0, 0)
    xb[t] = pb * 64 + 16 * (u ^ ((pb >> 4) & 1));
    acc[0][t] = zero4();
    acc[1][t] = zero4();
  }
  const int row0 = 32 * cp + li;
  const int hr = (row0 & 1) | (((row0 >> 1) & 3) << 2);          // = h(row0 + 16)
  const uint8_t* wr = w8 + row0 * W8_LD;
#pragma unroll 1
  for (int c = 0; c < 13; ++c) {
    const int tap = 2 * c + gh;                                  // 25 = the zero tap
    const int aoff = ((tap * 4 + u) ^ hr) << 4;
    const fp8x32 a0 = lds_fp8x32(wr + aoff, wr + (aoff ^ 16));
    const fp8x32 a1 = lds_fp8x32(wr + 16 * W8_LD + aoff, wr + 16 * W8_LD + (aoff ^ 16));
    const int tc = tap < 25 ? tap : 24, kh = (tc * 13) >> 6, kw = tc - kh * 5;   // tc / 5 for tc < 64
    const int xoff = (kh * 16 + kw) * 64, flip = (kh & 1) << 4;
    fp8x32 bx[NPX];                            // every read of the chunk in flight before its MFMAs
#pragma unroll
    for (int t = 0; t < NPX; ++t) {
      const int ad = (xb[t] ^ flip) + xoff;
      bx[t] = lds_fp8x32(x8 + ad, x8 + (ad ^ 16));
    }
#pragma unroll
    for (int t = 0; t < NPX; ++t) {
      acc[0][t] = mfma_fp8(a0, bx[t], acc[0][t]);
      acc[1][t] = mfma_fp8(a1, bx[t], acc[1][t]);
    }
  }
}

__global__ __launch_bounds__(NT, 1) void k_conv2_fwd_fp8(DmlcConv2FwdFp8Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint8_t* x8 = reinterpret_cast<uint8_t*>(smem);
  uint8_t* w8 = x8 + X8_BYTES;
  bf16* cout = reinterpret_cast<bf16*>(w8 + W8_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int g = lane >> 4, li = lane & 15, cp = w & 1, pg = w >> 1;
  const int slot = a.counter ? (int)(*a.counter & 1) : 0;
  const float sw = a.scale_w[slot];
  float mx = 0.f;                              // the batch's activation amax from the per-image maxima
  for (int i = tid; i < a.B; i += NT) mx = fmaxf(mx, a.amax_x[i]);

  stage_w8(a.w8, w8, tid);                     // weights -> LDS once
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  float* red = reinterpret_cast<float*>(smem + FP8_RED);
  if (lane == 0) red[w] = mx;
  __syncthreads();
  mx = red[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) mx = fmaxf(mx, red[i]);
  const float sx = 448.f / fmaxf(mx, 1e-20f);
  const float inv = 1.f / (sx * sw);
  if (a.sx_out && blockIdx.x == 0 && tid == 0) a.sx_out[0] = sx;   // (every block computes the same sx)
  float b4[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i) b4[h][i] = a.bias[32 * cp + 16 * h + 4 * g + i];

  // the input of image b: 2048 chunks of 8 channels over the padded 16x16 grid (halo -> 0), 4 per thread
  uint4 v[4];
  auto load = [&](int b) {
    const bf16* in = reinterpret_cast<const bf16*>(a.in) + (size_t)b * 9216;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s = tid + i * NT, pix = s >> 3, c = s & 7;
      const int iy = (pix >> 4) - 2, ix = (pix & 15) - 2;
      v[i] = load_sel(reinterpret_cast<const uint4*>(in + (iy * 12 + ix) * 64 + c * 8), reinterpret_cast<const uint4*>(in),
                      iy >= 0 && iy < 12 && ix >= 0 && ix < 12);
    }
  };
  const int G = gridDim.x;
  load(blockIdx.x);
  for (int b = blockIdx.x; b < a.B; b += G) {
    __syncthreads();                           // the previous image's MFMA / pool reads are done
#pragma unroll
    for (int i = 0; i < 4; ++i) {              // bf16 -> scaled fp8, 8 channels = half a 16-B unit
      const int s = tid + i * NT;
      const uint32_t wv[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
      const uint32_t lo = pk_fp8x4(bf16_lo(wv[0]) * sx, bf16_hi(wv[0]) * sx, bf16_lo(wv[1]) * sx, bf16_hi(wv[1]) * sx);
      const uint32_t hi = pk_fp8x4(bf16_lo(wv[2]) * sx, bf16_hi(wv[2]) * sx, bf16_lo(wv[3]) * sx, bf16_hi(wv[3]) * sx);
      *reinterpret_cast<uint2*>(x8 + x8_addr(s >> 3, (s & 7) >> 1) + (s & 1) * 8) = make_uint2(lo, hi);
      // the fp8 weight gradient's X: the same bytes, unpadded [b][144][64] (interior pixels)
      const int pix = s >> 3, iy = (pix >> 4) - 2, ix = (pix & 15) - 2;
      if (a.x8out && iy >= 0 && iy < 12 && ix >= 0 && ix < 12)
        *reinterpret_cast<uint2*>(a.x8out + ((size_t)b * 144 + iy * 12 + ix) * 64 + (s & 7) * 8) = make_uint2(lo, hi);
    }
    if (b + G < a.B) load(b + G);              // next image's input in flight under this one
    __syncthreads();
    auto epi = [&](int ct, int T, f32x4 acc) {
      acc[0] *= inv; acc[1] *= inv; acc[2] *= inv; acc[3] *= inv;
      const int ty = T / 3, tx = T - ty * 3;
      store_relu_tile(cout, (4 * ty + (li >> 2)) * 12 + 4 * tx + (li & 3), 16 * ct + 4 * g, acc, b4[ct & 1]);
    };
    if (pg == 0) {
      f32x4 acc[2][3];
      conv2_core_fp8<3>(x8, w8, acc, pg, cp, g, li);
#pragma unroll
      for (int t = 0; t < 3; ++t) { epi(2 * cp, pg + 4 * t, acc[0][t]); epi(2 * cp + 1, pg + 4 * t, acc[1][t]); }
    } else {
      f32x4 acc[2][2];
      conv2_core_fp8<2>(x8, w8, acc, pg, cp, g, li);
#pragma unroll
      for (int t = 0; t < 2; ++t) { epi(2 * cp, pg + 4 * t, acc[0][t]); epi(2 * cp + 1, pg + 4 * t, acc[1][t]); }
    }
    __syncthreads();
    pool_emit<12>(cout, reinterpret_cast<bf16*>(a.out) + (size_t)b * 2304, a.am + (size_t)b * 2304, tid);
  }
}

// conv2 input gradient on fp8: per image, pool2/ReLU backward (2x2 ownership, 288 tasks = one per
// thread) -> dY2 (bf16 to global, for the weight gradient) and, in registers, its block amax -> e4m3
// with sy = 448 / amax into the padded swizzled input grid -> the fp8 core against w2d8 -> dp1 =
// acc / (sy * sw) in bf16.  The next image's dp2 / argmax are prefetched into registers under the
// current image's MFMAs.  LDS: x8 16 KB | w8 112 KB | dp2 4.5 KB | argmax 2.25 KB | 8 wave maxima.
constexpr size_t DG8_DP2 = X8_BYTES + W8_BYTES, DG8_AM2 = DG8_DP2 + 2304 * 2, DG8_RED = DG8_AM2 + 2304;
constexpr size_t DG8_LDS = DG8_RED + 64;
static_assert(DG8_LDS <= 160 * 1024, "fp8 conv2 dgrad LDS");

__global__ __launch_bounds__(NT, 1) void k_conv2_dgrad_fp8(DmlcConv2DgradFp8Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint8_t* x8 = reinterpret_cast<uint8_t*>(smem);
  uint8_t* w8 = x8 + X8_BYTES;
  bf16* dp2 = reinterpret_cast<bf16*>(smem + DG8_DP2);
  uint8_t* am2 = reinterpret_cast<uint8_t*>(smem + DG8_AM2);
  float* red = reinterpret_cast<float*>(smem + DG8_RED);
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int g = lane >> 4, li = lane & 15, cp = w & 1, pg = w >> 1;
  const float sw = a.scale_w[0];
  const int G = gridDim.x;

  Prefetch16<288, NT> pd;
  Prefetch16<144, NT> pa;
  pd.load(reinterpret_cast<const bf16*>(a.dp2) + (size_t)blockIdx.x * 2304, tid);
  pa.load(a.am2 + (size_t)blockIdx.x * 2304, tid);
  stage_w8(a.w8, w8, tid);
  for (int s = tid; s < 1024; s += NT) {        // halo of the padded 16x16 grid: zero once
    const int P = s >> 2, r = P >> 4, col = P & 15;
    if (r < 2 || r >= 14 || col < 2 || col >= 14) *reinterpret_cast<uint4*>(x8 + x8_addr(P, s & 3)) = make_uint4(0u, 0u, 0u, 0u);
  }
  for (int b = blockIdx.x; b < a.B; b += G) {
    __syncthreads();                             // the previous image's core / pool reads are done
    pd.store(dp2, tid);
    pa.store(am2, tid);
    if (b + G < a.B) {                           // next image's operands in flight under this one
      pd.load(reinterpret_cast<const bf16*>(a.dp2) + (size_t)(b + G) * 2304, tid);
      pa.load(a.am2 + (size_t)(b + G) * 2304, tid);
    }
    __syncthreads();
    float o[4][8];
    float m = 0.f;
    const int win = tid >> 3, c = tid & 7, py = win / 6, px = win - py * 6;
    if (tid < 288) {
      pool_bwd_2x2<6>(dp2, am2, py, px, c, o);
      bf16* dy2 = reinterpret_cast<bf16*>(a.dy2) + (size_t)b * 9216;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int y = 2 * py + (k >> 1), x = 2 * px + (k & 1);
        *reinterpret_cast<bf16x8*>(dy2 + (y * 12 + x) * 64 + c * 8) = to_bf16x8(o[k]);
#pragma unroll
        for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(o[k][j]));
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    if (lane == 0) red[w] = m;
    __syncthreads();
    float amax = red[0];
#pragma unroll
    for (int i = 1; i < NT / 64; ++i) amax = fmaxf(amax, red[i]);
    // a power of two (round 6): the fp8 weight gradient applies it as the MFMA's E8M0 block scale --
    // kept within 2^+-126 (finite, representable): a saturated softmax leaves images whose largest dY2
    // is denormal (448 / amax overflows); their e4m3 values then flush to zero
    const float sy = amax > 0.f ? exp2f(fminf(fmaxf(floorf(log2f(448.f / amax)), -126.f), 126.f)) : 1.f;
    if (tid == 0 && a.sy_img) a.sy_img[b] = sy;
    if (tid < 288) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int P = (2 * py + (k >> 1) + 2) * 16 + 2 * px + (k & 1) + 2;
        const uint32_t lo = pk_fp8x4(o[k][0] * sy, o[k][1] * sy, o[k][2] * sy, o[k][3] * sy);
        const uint32_t hi = pk_fp8x4(o[k][4] * sy, o[k][5] * sy, o[k][6] * sy, o[k][7] * sy);
        *reinterpret_cast<uint2*>(x8 + x8_addr(P, c >> 1) + (c & 1) * 8) = make_uint2(lo, hi);
        if (a.dy8out) {                      // the fp8 weight gradient's dY: the same bytes, [b][144][64]
          const int y = 2 * py + (k >> 1), x = 2 * px + (k & 1);
          *reinterpret_cast<uint2*>(a.dy8out + ((size_t)b * 144 + y * 12 + x) * 64 + c * 8) = make_uint2(lo, hi);
        }
      }
    }
    __syncthreads();
    const float inv = 1.f / (sy * sw);
    bf16* dp1 = reinterpret_cast<bf16*>(a.dp1) + (size_t)b * 9216;
    auto epi = [&](int ct, int T, f32x4 acc) {
      const int ty = T / 3, tx = T - ty * 3;
      const int p = (4 * ty + (li >> 2)) * 12 + 4 * tx + (li & 3);
      *reinterpret_cast<bf16x4*>(dp1 + p * 64 + 16 * ct + 4 * g) = pack4(acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv);
    };
    if (pg == 0) {
      f32x4 acc[2][3];
      conv2_core_fp8<3>(x8, w8, acc, pg, cp, g, li);
#pragma unroll
      for (int t = 0; t < 3; ++t) { epi(2 * cp, pg + 4 * t, acc[0][t]); epi(2 * cp + 1, pg + 4 * t, acc[1][t]); }
    } else {
      f32x4 acc[2][2];
      conv2_core_fp8<2>(x8, w8, acc, pg, cp, g, li);
#pragma unroll
      for (int t = 0; t < 2; ++t) { epi(2 * cp, pg + 4 * t, acc[0][t]); epi(2 * cp + 1, pg + 4 * t, acc[1][t]); }
    }
  }
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

extern "C" {

hipError_t dmlc_conv2_fwd_fp8(const DmlcConv2FwdFp8Args* a, hipStream_t s) {
  DMLC_LDS_OPTIN(&k_conv2_fwd_fp8, FP8_LDS);
  hipLaunchKernelGGL(k_conv2_fwd_fp8, dim3(a->B < 256 ? a->B : 256), dim3(NT), FP8_LDS, s, *a);
  return hipGetLastError();
}

hipError_t dmlc_conv2_dgrad_fp8(const DmlcConv2DgradFp8Args* a, hipStream_t s) {
  DMLC_LDS_OPTIN(&k_conv2_dgrad_fp8, DG8_LDS);
  hipLaunchKernelGGL(k_conv2_dgrad_fp8, dim3(a->B < 256 ? a->B : 256), dim3(NT), DG8_LDS, s, *a);
  return hipGetLastError();
}

hipError_t dmlc_fp8_roundtrip(const float* x, float* y, int n, float scale, hipStream_t s) {
  hipLaunchKernelGGL(k_fp8_roundtrip, dim3((n + 255) / 256), dim3(256), 0, s, x, y, n, scale);
  return hipGetLastError();
}

}  // extern "C"
