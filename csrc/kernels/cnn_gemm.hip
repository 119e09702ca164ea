// Grouped bf16 GEMM for the fully-connected layers (/root/reference/cifar10cnn.py:130-145; TF MatMul
// and its gradients, SURVEY.md §2.B N10, §2.C linear_fwd / linear_bwd_dx / linear_bwd_dw).
//
// Up to 8 independent problems share ONE launch (blockIdx ranges), so e.g. the fc1 input-gradient,
// the three weight gradients and the three bias gradients of the backward are a single kernel
// instead of seven.  Each problem picks its operand layouts:
//   * k-major operands are staged as [rows][32 k] and read with ds_read_b128;
//   * m/n-major operands (the weight-gradient case, where the reduction runs over the batch) are
//     staged untransposed as [32 k][rows] and read with the gfx950 hardware transpose
//     ds_read_b64_tr_b16 — no transposed copy of any activation is ever written.
// 64x64 tiles, 4 waves in 2x2, each wave 2x2 MFMA 16x16x32 tiles, register-staged double buffer,
// optional split-K into fp32 partial slabs (reduced by the consumer kernel's prologue).
#include "common.h"
#include "api.h"

namespace dmlc {

constexpr int KC_LD = 40;   // k-major tile row stride (bf16): 80 B rows, 16-B aligned
constexpr int MC_LD = 72;   // m-major tile row stride (bf16): 144 B rows, 16-B aligned
constexpr int TILE_ELEMS = 64 * KC_LD > 32 * MC_LD ? 64 * KC_LD : 32 * MC_LD;

struct Stage {
  bf16x8 v;
  int dst;
};

// Load one 16-byte piece of a 64-row x 32-k operand tile into registers.
DEV Stage load_piece(const bf16* __restrict__ X, int ld, int kmajor, int R, int K, int r0, int k0, int tid) {
  Stage st;
  if (kmajor) {
    const int row = tid >> 2, kc = tid & 3;
    const int gr = r0 + row, gk = k0 + 8 * kc;
    st.v = (gr < R && gk < K) ? glb_b128(X + (size_t)gr * ld + gk) : bf16x8{};
    st.dst = row * KC_LD + 8 * kc;
  } else {
    const int kk = tid >> 3, rc = tid & 7;
    const int gk = k0 + kk, gr = r0 + 8 * rc;
    st.v = (gk < K && gr < R) ? glb_b128(X + (size_t)gk * ld + gr) : bf16x8{};
    st.dst = kk * MC_LD + 8 * rc;
  }
  return st;
}

DEV bf16x8 frag(const bf16* sm, int kmajor, int rr0, int g, int li) {
  if (kmajor) return lds_b128(sm + (rr0 + li) * KC_LD + 8 * g);
  const int q = li >> 2, p = li & 3;
  return tr_frag(sm + (8 * g + q) * MC_LD + rr0 + 4 * p, sm + (8 * g + 4 + q) * MC_LD + rr0 + 4 * p);
}

DEV void colsum_block(const DmlcGemmProblem& P, int local, float* red) {
  // C[m] = sum_k A(m,k) with A m-major ([K rows][M cols], lda)
  const int tid = threadIdx.x;
  const int col = local * 64 + (tid & 63);
  const bf16* A = reinterpret_cast<const bf16*>(P.A);
  float s = 0.f;
  if (col < P.M)
    for (int k = tid >> 6; k < P.K; k += 4) s += (float)A[(size_t)k * P.lda + col];
  red[tid] = s;
  __syncthreads();
  if (tid < 64 && col < P.M && col < P.nvalid)
    reinterpret_cast<float*>(P.C)[col] = red[tid] + red[tid + 64] + red[tid + 128] + red[tid + 192];
}

__global__ __launch_bounds__(256) void k_gemm_grouped(DmlcGemmGroup G) {
  __shared__ __attribute__((aligned(16))) bf16 sA[2][TILE_ELEMS];
  __shared__ __attribute__((aligned(16))) bf16 sB[2][TILE_ELEMS];
  const int blk = blockIdx.x;
  int pi = 0;
  while (pi + 1 < G.nprob && blk >= G.p[pi + 1].block_start) ++pi;
  const DmlcGemmProblem P = G.p[pi];
  const int local = blk - P.block_start;
  if (P.c_mode == 3) { colsum_block(P, local, reinterpret_cast<float*>(&sA[0][0])); return; }

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int per_split = P.tiles_m * P.tiles_n;
  const int split = local / per_split, t = local - split * per_split;
  const int m0 = (t / P.tiles_n) * 64, n0 = (t % P.tiles_n) * 64;
  const int ksteps = (P.K + 31) >> 5;
  const int per = (ksteps + P.ksplit - 1) / P.ksplit;
  const int ks0 = split * per, ks1 = min(ksteps, ks0 + per);
  const bf16* A = reinterpret_cast<const bf16*>(P.A);
  const bf16* B = reinterpret_cast<const bf16*>(P.B);
  const int wm = w >> 1, wn = w & 1;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) { acc[i][0] = zero4(); acc[i][1] = zero4(); }

  if (ks0 < ks1) {
    Stage pa = load_piece(A, P.lda, P.a_kmajor, P.M, P.K, m0, ks0 * 32, tid);
    Stage pb = load_piece(B, P.ldb, P.b_kmajor, P.N, P.K, n0, ks0 * 32, tid);
    *reinterpret_cast<bf16x8*>(&sA[0][pa.dst]) = pa.v;
    *reinterpret_cast<bf16x8*>(&sB[0][pb.dst]) = pb.v;
    __syncthreads();
    int buf = 0;
    for (int ks = ks0; ks < ks1; ++ks) {
      const bool more = ks + 1 < ks1;
      if (more) {
        pa = load_piece(A, P.lda, P.a_kmajor, P.M, P.K, m0, (ks + 1) * 32, tid);
        pb = load_piece(B, P.ldb, P.b_kmajor, P.N, P.K, n0, (ks + 1) * 32, tid);
      }
      const bf16x8 a0 = frag(sA[buf], P.a_kmajor, 32 * wm, g, li);
      const bf16x8 a1 = frag(sA[buf], P.a_kmajor, 32 * wm + 16, g, li);
      const bf16x8 b0 = frag(sB[buf], P.b_kmajor, 32 * wn, g, li);
      const bf16x8 b1 = frag(sB[buf], P.b_kmajor, 32 * wn + 16, g, li);
      acc[0][0] = mfma16(a0, b0, acc[0][0]);
      acc[0][1] = mfma16(a0, b1, acc[0][1]);
      acc[1][0] = mfma16(a1, b0, acc[1][0]);
      acc[1][1] = mfma16(a1, b1, acc[1][1]);
      if (more) {
        *reinterpret_cast<bf16x8*>(&sA[buf ^ 1][pa.dst]) = pa.v;
        *reinterpret_cast<bf16x8*>(&sB[buf ^ 1][pb.dst]) = pb.v;
      }
      __syncthreads();
      buf ^= 1;
    }
  }

  // epilogue: acc[i][j] holds C[m0+32wm+16i+4g+r][n0+32wn+16j+li]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 32 * wn + 16 * j + li;
      if (n >= P.nvalid) continue;
      const float bn = P.bias ? P.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 32 * wm + 16 * i + 4 * g + r;
        if (m >= P.M) continue;
        float v = acc[i][j][r];
        if (P.c_mode == 2) {
          reinterpret_cast<float*>(P.C)[(size_t)split * P.M * P.ldc + (size_t)m * P.ldc + n] = v;
          continue;
        }
        v += bn;
        if (P.relu) v = fmaxf(v, 0.f);
        if (P.c_mode == 0) reinterpret_cast<float*>(P.C)[(size_t)m * P.ldc + n] = v;
        else reinterpret_cast<bf16*>(P.C)[(size_t)m * P.ldc + n] = (bf16)v;
      }
    }
}

}  // namespace dmlc

using namespace dmlc;

extern "C" hipError_t dmlc_gemm_grouped(DmlcGemmGroup* G, hipStream_t s) {
  int blocks = 0;
  for (int i = 0; i < G->nprob; ++i) {
    DmlcGemmProblem& P = G->p[i];
    P.tiles_m = (P.M + 63) / 64;
    P.tiles_n = P.c_mode == 3 ? 1 : (P.N + 63) / 64;
    if (P.ksplit < 1) P.ksplit = 1;
    if (P.c_mode == 3) P.ksplit = 1;
    P.block_start = blocks;
    blocks += P.tiles_m * P.tiles_n * P.ksplit;
  }
  G->nblocks = blocks;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gemm_grouped, dim3(blocks), dim3(256), 0, s, *G);
  return hipGetLastError();
}
