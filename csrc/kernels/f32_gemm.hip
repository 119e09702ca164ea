// fp32 kernels of the fp32-accurate training mode (--dtype fp32 on the GPU): the reference CNN keeps
// every variable and every op in tf.float32 (/root/reference/cifar10cnn.py:97-145, :150-164), and
// this mode reproduces that precision on hand-written CDNA4 code instead of falling back to the
// framework's eager PyTorch ops.
//
//  * k_gemm_f32: C = op(A) op(B) on the fp32 matrix cores (v_mfma_f32_16x16x4_f32 -- true fp32
//    products and fp32 accumulation, no bf16/tf32 operand rounding).  64x64 output tile per
//    256-thread workgroup, 4 waves each owning 32x32 (2x2 MFMA tiles); K in steps of 16 staged
//    through LDS (k-major, row pitch 80 floats so a fragment read -- 4 k-rows x 16 consecutive
//    m/n -- lands in 64 distinct banks), next step register-prefetched under the MFMAs.  Both
//    operand orientations are template parameters, so forward (X W), data gradient (dY W^T) and
//    weight gradient (X^T dY) are the same kernel without transposes in memory.
//  * deterministic split-K: slices write partial products, a second kernel sums them in slice
//    order (+ bias, ReLU) -- the long-K weight gradients (K = B*H*W) get enough workgroups without
//    atomics, so results are bitwise reproducible.
//  * implicit-GEMM convolutions (template CONV = the layer geometry): the A operand is the im2col
//    matrix of an NHWC activation, gathered straight from it by the tile loader -- forward (cols W),
//    weight gradient (cols^T dY, with an optional ones column whose output row is the bias
//    gradient) and data gradient (im2col(dY) against the flipped, transposed weight) never
//    materialise a column matrix;
//  * explicit im2col / col2im (gather form, fixed tap order) for other geometries, and a two-pass
//    column sum for the fc bias gradients.
#include <algorithm>

#include "common.h"
#include "api_f32.h"

namespace dmlc {

constexpr int FT = 256, FBM = 64, FBN = 64, FBK = 64, FLD = 80, FNE = FBK * 64 / FT;   // FNE: elements per thread per operand

DEV f32x4 mfma_f32(float a, float b, const f32x4& c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

// Implicit im2col geometry: x NHWC [B][HW][HW][CH], KSxKS taps, stride 1, zero padding KS/2;
// column (kh*KS + kw)*CH + ci, plus (ones) a constant-1 column at index KS*KS*CH.
template <int CONV> struct ConvGeom;
template <> struct ConvGeom<1> { static constexpr int CH = 3, HW = 24, KS = 5; };    // conv1 input
template <> struct ConvGeom<2> { static constexpr int CH = 64, HW = 12, KS = 5; };   // conv2 input / dY

// Tile-loader state of the implicit im2col operand.  The loop-invariant half of every gathered
// element is computed once per thread: with !TA the thread's 4 tile rows are fixed pixels
// (b, y, x -> base offset), with TA its tile column is a fixed (tap, channel) -- so a k-step costs
// one constant division (channel -> tap, or pixel -> y, x) and a bounds test per element.
template <bool TA, int CONV>
struct ConvA {
  using Gm = ConvGeom<CONV>;
  static constexpr int CH = Gm::CH, HW = Gm::HW, KS = Gm::KS, PAD = KS / 2, KC = KS * KS * CH;
  int y[4], x[4], base[4];      // !TA: per tile row
  int dy, dx, off;              // TA: the column's tap offsets
  bool ones, colok;
  MDEV void init(int M, int m0, int t) {
    if constexpr (!TA) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int gm = min(m0 + (t >> 4) + 16 * i, M - 1);
        const int b = gm / (HW * HW), pp = gm - b * (HW * HW);
        y[i] = pp / HW;
        x[i] = pp - y[i] * HW;
        base[i] = gm * CH;
      }
    } else {
      const int col = m0 + (t & 63);
      colok = col < M;
      ones = col == KC;
      const int c = min(col, KC - 1), tap = c / CH, ci = c - tap * CH, kh = tap / KS, kw = tap - kh * KS;
      dy = kh - PAD;
      dx = kw - PAD;
      off = (dy * HW + dx) * CH + ci;
    }
  }
  // element i of the thread's share of a k-step: op(A)(gm, gk); ok = inside the problem
  MDEV float fetch(const float* X, int i, int gm, int gk, bool ok) const {
    if constexpr (!TA) {                       // gk = im2col column of the fixed pixel row i
      const int tap = gk / CH, ci = gk - tap * CH, kh = tap / KS, kw = tap - kh * KS;
      const int iy = y[i] + kh - PAD, ix = x[i] + kw - PAD;
      const bool in = ok && iy >= 0 && iy < HW && ix >= 0 && ix < HW;
      const float v = X[in ? base[i] + ((kh - PAD) * HW + (kw - PAD)) * CH + ci : 0];
      return in ? v : 0.f;
    } else {                                   // gk = pixel of the fixed column (tap, channel)
      (void)gm;
      const int pp = gk % (HW * HW), yy = pp / HW, xx = pp - yy * HW;
      const int iy = yy + dy, ix = xx + dx;
      const bool in = ok && !ones && iy >= 0 && iy < HW && ix >= 0 && ix < HW;
      const float v = X[in ? (int64_t)gk * CH + off : 0];
      return ones ? (ok ? 1.f : 0.f) : (in ? v : 0.f);
    }
  }
};

struct F32GemmArgs {
  const float* A;
  const float* B;
  const float* bias;
  float* C;
  float* ws;
  int M, N, K, lda, ldb, splits, kc;
  bool relu;
};

// One K-step of operands in registers: thread t owns FNE elements of the 64 x FBK A tile and FNE of
// the FBK x 64 B tile, mapped so that consecutive threads read consecutive addresses of the stored
// matrix (a k-contiguous operand: 16 k x 4 rows per thread-quad pattern; an m/n-contiguous one:
// 64 consecutive m/n).  64 k per step: 256 MFMAs per workgroup between two global round trips.
template <bool T>   // T: the 64-wide index is contiguous in memory
DEV void tile_idx(int t, int i, int& mn, int& k) {
  if (T) { mn = t & 63; k = (t >> 6) + 4 * i; }
  else { mn = (t >> 4) + 16 * (i & 3); k = (t & 15) + 16 * (i >> 2); }
}

template <bool TA, bool TB, int CONV>
struct F32Tile {
  float a[FNE], b[FNE];
  ConvA<TA, CONV == 0 ? 1 : CONV> cv;
  MDEV void load(const F32GemmArgs& p, int m0, int n0, int k0, int kend, int t) {
#pragma unroll
    for (int i = 0; i < FNE; ++i) {
      int m, k;
      tile_idx<TA>(t, i, m, k);
      const int gm = m0 + m, gk = k0 + k;
      const bool ok = gm < p.M && gk < kend;
      if constexpr (CONV != 0) {                // op(A) = im2col(x) (pixel, column) or its transpose
        a[i] = cv.fetch(p.A, i & 3, gm, gk, ok);
      } else {
        const int64_t off = TA ? (int64_t)gk * p.lda + gm : (int64_t)gm * p.lda + gk;
        const float v = p.A[ok ? off : 0];
        a[i] = ok ? v : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < FNE; ++i) {
      int n, k;
      tile_idx<!TB>(t, i, n, k);
      const int gn = n0 + n, gk = k0 + k;
      const bool ok = gn < p.N && gk < kend;
      const int64_t off = TB ? (int64_t)gn * p.ldb + gk : (int64_t)gk * p.ldb + gn;
      const float v = p.B[ok ? off : 0];
      b[i] = ok ? v : 0.f;
    }
  }
  MDEV void store(float* As, float* Bs, int t) const {
#pragma unroll
    for (int i = 0; i < FNE; ++i) {
      int m, k;
      tile_idx<TA>(t, i, m, k);
      As[k * FLD + m] = a[i];
    }
#pragma unroll
    for (int i = 0; i < FNE; ++i) {
      int n, k;
      tile_idx<!TB>(t, i, n, k);
      Bs[k * FLD + n] = b[i];
    }
  }
};

template <bool TA, bool TB, int CONV>
__global__ __launch_bounds__(FT) void k_gemm_f32(F32GemmArgs p) {
  __shared__ float As[FBK * FLD], Bs[FBK * FLD];
  const int t = threadIdx.x, lane = t & 63, w = wave_id();
  const int m0 = blockIdx.x * FBM, n0 = blockIdx.y * FBN, z = blockIdx.z;
  const int kbeg = z * p.kc, kend = min(p.K, kbeg + p.kc);
  const int wm = (w & 1) * 32, wn = (w >> 1) * 32, r = lane & 15, q = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero4();
  F32Tile<TA, TB, CONV> tile;
  if constexpr (CONV != 0) tile.cv.init(p.M, m0, t);
  tile.load(p, m0, n0, kbeg, kend, t);
  for (int k0 = kbeg; k0 < kend; k0 += FBK) {
    tile.store(As, Bs, t);
    __syncthreads();
    if (k0 + FBK < kend) tile.load(p, m0, n0, k0 + FBK, kend, t);   // next step under the MFMAs
#pragma unroll
    for (int kk = 0; kk < FBK / 4; ++kk) {
      const float* ar = As + (4 * kk + q) * FLD + wm + r;
      const float* br = Bs + (4 * kk + q) * FLD + wn + r;
      const float a0 = ar[0], a1 = ar[16], b0 = br[0], b1 = br[16];
      acc[0][0] = mfma_f32(a0, b0, acc[0][0]);
      acc[0][1] = mfma_f32(a0, b1, acc[0][1]);
      acc[1][0] = mfma_f32(a1, b0, acc[1][0]);
      acc[1][1] = mfma_f32(a1, b1, acc[1][1]);
    }
    __syncthreads();
  }
  const bool epi = p.splits == 1;
  float* out = epi ? p.C : p.ws + (int64_t)z * p.M * p.N;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn + 16 * j + r;
    if (col >= p.N) continue;
    const float bv = (epi && p.bias) ? p.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm + 16 * i + 4 * q + e;
        if (row >= p.M) continue;
        float v = acc[i][j][e] + bv;
        if (epi && p.relu) v = fmaxf(v, 0.f);
        out[(int64_t)row * p.N + col] = v;
      }
  }
}

// out[e] = sum_z ws[z][e] (slice order) + bias[e % N], optional ReLU
__global__ __launch_bounds__(FT) void k_f32_reduce(const float* ws, float* out, const float* bias, int64_t mn, int N,
                                                   int S, bool relu) {
  const int64_t stride = (int64_t)gridDim.x * FT;
  for (int64_t e = (int64_t)blockIdx.x * FT + threadIdx.x; e < mn; e += stride) {
    float s = ws[e];
#pragma unroll 8
    for (int z = 1; z < S; ++z) s += ws[(int64_t)z * mn + e];   // loads independent: 8 in flight
    if (bias) s += bias[e % N];
    if (relu) s = fmaxf(s, 0.f);
    out[e] = s;
  }
}

__global__ __launch_bounds__(FT) void k_f32_im2col(const float* x, float* cols, int B, int H, int W, int C, int KH,
                                                   int KW, int pad) {
  const int64_t KC = (int64_t)KH * KW * C, total = (int64_t)B * H * W * KC;
  const int64_t stride = (int64_t)gridDim.x * FT;
  for (int64_t e = (int64_t)blockIdx.x * FT + threadIdx.x; e < total; e += stride) {
    const int64_t row = e / KC;
    const int col = (int)(e - row * KC), tap = col / C, c = col - tap * C, kh = tap / KW, kw = tap - kh * KW;
    const int b = (int)(row / (H * W)), pix = (int)(row - (int64_t)b * H * W), y = pix / W, xx = pix - y * W;
    const int iy = y + kh - pad, ix = xx + kw - pad;
    const bool ok = iy >= 0 && iy < H && ix >= 0 && ix < W;
    const float v = x[ok ? (((int64_t)b * H + iy) * W + ix) * C + c : 0];
    cols[e] = ok ? v : 0.f;
  }
}

__global__ __launch_bounds__(FT) void k_f32_col2im(const float* dcols, float* dx, int B, int H, int W, int C, int KH,
                                                   int KW, int pad) {
  const int64_t KC = (int64_t)KH * KW * C, total = (int64_t)B * H * W * C;
  const int64_t stride = (int64_t)gridDim.x * FT;
  for (int64_t e = (int64_t)blockIdx.x * FT + threadIdx.x; e < total; e += stride) {
    const int64_t pix = e / C;
    const int c = (int)(e - pix * C);
    const int b = (int)(pix / (H * W)), pp = (int)(pix - (int64_t)b * H * W), y = pp / W, xx = pp - y * W;
    float s = 0.f;
    for (int kh = 0; kh < KH; ++kh) {
      const int oy = y - kh + pad;
      if (oy < 0 || oy >= H) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int ox = xx - kw + pad;
        if (ox < 0 || ox >= W) continue;
        s += dcols[(((int64_t)b * H + oy) * W + ox) * KC + (kh * KW + kw) * C + c];
      }
    }
    dx[e] = s;
  }
}

// partial column sums: workgroup (column block, row slice), 4 row phases reduced through LDS
__global__ __launch_bounds__(FT) void k_f32_colsum_part(const float* x, float* ws, int M, int N, int rc) {
  __shared__ float red[4][64];
  const int t = threadIdx.x, col = blockIdx.x * 64 + (t & 63), g = t >> 6, s = blockIdx.y;
  const int r0 = s * rc, r1 = min(M, r0 + rc);
  float acc = 0.f;
  if (col < N)
    for (int r = r0 + g; r < r1; r += 4) acc += x[(int64_t)r * N + col];
  red[g][t & 63] = acc;
  __syncthreads();
  if (g == 0 && col < N) ws[(int64_t)s * N + col] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
}

int grid_for(int64_t n) { return (int)std::min<int64_t>((n + FT - 1) / FT, 8192); }

}  // namespace dmlc

using namespace dmlc;

extern "C" {

hipError_t dmlc_f32_gemm(const float* A, const float* B, const float* bias, float* C, float* ws, int M, int N,
                         int K, int lda, int ldb, bool ta, bool tb, bool relu, int splits, int kc, int conv,
                         hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || splits < 1 || kc % FBK || (int64_t)splits * kc < K || (splits > 1 && !ws))
    return hipErrorInvalidValue;
  if (conv < 0 || conv > 2 || (conv && tb)) return hipErrorInvalidValue;
  F32GemmArgs p{A, B, bias, C, ws, M, N, K, lda, ldb, splits, kc, relu};
  const dim3 grid((M + FBM - 1) / FBM, (N + FBN - 1) / FBN, splits);
  if (conv == 1) {
    if (ta) hipLaunchKernelGGL((k_gemm_f32<true, false, 1>), grid, dim3(FT), 0, s, p);
    else hipLaunchKernelGGL((k_gemm_f32<false, false, 1>), grid, dim3(FT), 0, s, p);
  } else if (conv == 2) {
    if (ta) hipLaunchKernelGGL((k_gemm_f32<true, false, 2>), grid, dim3(FT), 0, s, p);
    else hipLaunchKernelGGL((k_gemm_f32<false, false, 2>), grid, dim3(FT), 0, s, p);
  } else if (ta && tb) hipLaunchKernelGGL((k_gemm_f32<true, true, 0>), grid, dim3(FT), 0, s, p);
  else if (ta) hipLaunchKernelGGL((k_gemm_f32<true, false, 0>), grid, dim3(FT), 0, s, p);
  else if (tb) hipLaunchKernelGGL((k_gemm_f32<false, true, 0>), grid, dim3(FT), 0, s, p);
  else hipLaunchKernelGGL((k_gemm_f32<false, false, 0>), grid, dim3(FT), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || splits == 1) return e;
  const int64_t mn = (int64_t)M * N;
  hipLaunchKernelGGL(k_f32_reduce, dim3(grid_for(mn)), dim3(FT), 0, s, ws, C, bias, mn, N, splits, relu);
  return hipGetLastError();
}

hipError_t dmlc_f32_im2col(const float* x, float* cols, int B, int H, int W, int C, int KH, int KW, int pad,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_f32_im2col, dim3(grid_for((int64_t)B * H * W * KH * KW * C)), dim3(FT), 0, s, x, cols, B, H,
                     W, C, KH, KW, pad);
  return hipGetLastError();
}

hipError_t dmlc_f32_col2im(const float* dcols, float* dx, int B, int H, int W, int C, int KH, int KW, int pad,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_f32_col2im, dim3(grid_for((int64_t)B * H * W * C)), dim3(FT), 0, s, dcols, dx, B, H, W, C,
                     KH, KW, pad);
  return hipGetLastError();
}

hipError_t dmlc_f32_colsum(const float* x, float* out, float* ws, int M, int N, int splits, hipStream_t s) {
  if (M <= 0 || N <= 0 || splits < 1) return hipErrorInvalidValue;
  const int rc = (M + splits - 1) / splits;
  hipLaunchKernelGGL(k_f32_colsum_part, dim3((N + 63) / 64, splits), dim3(FT), 0, s, x, ws, M, N, rc);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_f32_reduce, dim3(grid_for(N)), dim3(FT), 0, s, ws, out, nullptr, (int64_t)N, N, splits,
                     false);
  return hipGetLastError();
}

}  // extern "C"
