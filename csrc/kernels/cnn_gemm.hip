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
// 64x64 tiles, 4 waves in 2x2, each wave 2x2 MFMA 16x16x32 tiles; K is staged in 128-deep chunks
// (4 k-steps, 8 x 16-B loads per thread in flight) with the next chunk's loads issued before the
// current chunk's MFMAs (register-staged double buffer); optional split-K into fp32 partial slabs
// (reduced by the consumer kernel's prologue).
#include "common.h"
#include "api.h"

namespace dmlc {

constexpr int KC = 128;                     // K chunk staged per phase (4 MFMA k-steps)
// LDS images, modelled with the gfx950 lane groups (MI355X_MICROARCH.md §LDS; tools/lds_banks.py):
//  * k-major [64 rows][128 k]: 288-B rows (a row is 8 banks further on), so the 16 lanes of every
//    ds_read_b128 group land on 64 distinct banks (272-B rows: 2-way, 8 cycles instead of 4);
//  * m-major [128 k rows][64 cols]: unpadded 128-B rows with the 16-B chunk index XORed by row bits 1
//    and 3 (mswz): the 8 rows {q, 8+q} a ds_read_b64_tr_b16 half-wave touches then cover all 64
//    banks exactly once (any plain row pad: 2-way, 4 cycles instead of 2); the 16-B stores of a row
//    stay one contiguous permuted row (conflict-free).
constexpr int KC_LD = KC + 16;              // k-major tile row stride (bf16)
constexpr int MC_LD = 64;                   // m-major tile row stride (bf16), swizzled by mswz
constexpr int TILE_ELEMS = 64 * KC_LD > KC * MC_LD ? 64 * KC_LD : KC * MC_LD;
constexpr int PIECES = 64 * KC / 8 / 256;   // 16-byte pieces per thread per operand per chunk (4)
constexpr size_t GEMM_LDS = (size_t)2 * 2 * TILE_ELEMS * 2;

// One operand's share of a 64-row x KC-deep chunk, held in registers between the global load and the
// LDS store (so the next chunk's loads are in flight while the current chunk is multiplied).
// element offset of (row, col) in the swizzled m-major image (col: multiple of 4)
DEV int mswz(int row, int col) {
  const int f = 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
  return row * MC_LD + (((col >> 3) ^ f) << 3) + (col & 7);
}

struct Chunk {
  uint4 v[PIECES];
  MDEV void load(const bf16* __restrict__ X, int ld, int kmajor, int R, int K, int r0, int k0, int tid) {
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const int c = tid + i * 256;
      int gr, gk;
      if (kmajor) { gr = r0 + (c >> 4); gk = k0 + 8 * (c & 15); }
      else { gk = k0 + (c >> 3); gr = r0 + 8 * (c & 7); }
      v[i] = load_sel(reinterpret_cast<const uint4*>(kmajor ? X + (size_t)gr * ld + gk : X + (size_t)gk * ld + gr),
                      reinterpret_cast<const uint4*>(X), gr < R && gk < K);
    }
  }
  MDEV void store(bf16* sm, int kmajor, int tid) const {
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const int c = tid + i * 256;
      const int off = kmajor ? (c >> 4) * KC_LD + 8 * (c & 15) : mswz(c >> 3, 8 * (c & 7));
      *reinterpret_cast<uint4*>(sm + off) = v[i];
    }
  }
};

DEV bf16x8 frag(const bf16* sm, int kmajor, int rr0, int kk, int g, int li) {
  if (kmajor) return lds_b128(sm + (rr0 + li) * KC_LD + kk * 32 + 8 * g);
  const int q = li >> 2, p = li & 3;
  return tr_frag(sm + mswz(kk * 32 + 8 * g + q, rr0 + 4 * p), sm + mswz(kk * 32 + 8 * g + 4 + q, rr0 + 4 * p));
}

DEV void colsum_block(const DmlcGemmProblem& P, int local, float* red) {
  // C[m] = sum_k A(m,k) with A m-major ([K rows][M cols], lda)
  const int tid = threadIdx.x;
  const int col = local * 64 + (tid & 63);
  const bf16* A = reinterpret_cast<const bf16*>(P.A);
  float s = 0.f;
  if (col < P.M) {
#pragma unroll 8
    for (int k = tid >> 6; k < P.K; k += 4) s += (float)A[(size_t)k * P.lda + col];
  }
  red[tid] = s;
  __syncthreads();
  if (tid < 64 && col < P.M && col < P.nvalid)
    reinterpret_cast<float*>(P.C)[col] = red[tid] + red[tid + 64] + red[tid + 128] + red[tid + 192];
}

__global__ __launch_bounds__(256) void k_gemm_grouped(DmlcGemmGroup G) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* sA = reinterpret_cast<bf16*>(smem);             // [2][TILE_ELEMS]
  bf16* sB = sA + 2 * TILE_ELEMS;                        // [2][TILE_ELEMS]
  const int blk = blockIdx.x;
  // problem lookup: every block_start compared at once (independent scalar loads, one latency; a
  // search loop paid one dependent kernarg load per problem before the last problem's blocks began)
  int pi = 0;
#pragma unroll
  for (int i = 1; i < DMLC_MAX_GEMM; ++i) pi += (i < G.nprob && blk >= G.p[i].block_start) ? 1 : 0;
  const DmlcGemmProblem P = G.p[pi];
  const int local = blk - P.block_start;
  DMLC_STAMP(DMLC_TK_GEMM, 0);
  if (P.c_mode == 3) { colsum_block(P, local, reinterpret_cast<float*>(smem)); return; }

  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int g = lane >> 4, li = lane & 15;
  const int per_split = P.tiles_m * P.tiles_n;
  // XCD-aware order (G.xcd_map): the problem's blocks are padded to 8 * per_x; block local runs on
  // XCD local % 8 (round-robin dispatch, block_start % 8 == 0) and takes tile (local % 8) * per_x +
  // local / 8, so each XCD owns a contiguous run of tiles -- split-major, then along the LARGER
  // operand (n-major when B = N x K outweighs A = M x K) -- and reads that operand's tiles into its
  // own L2 once instead of every XCD pulling all of it through the fabric.  Placement is a speed
  // matter only: any block->XCD assignment computes the same tiles.
  int lin = local;
  if (G.xcd_map) {
    const int nb = per_split * P.ksplit, per_x = (nb + 7) >> 3;
    lin = (local & 7) * per_x + (local >> 3);
    if (lin >= nb) return;                     // padding block
  }
  const int split = lin / per_split, t = lin - split * per_split;
  const bool nmaj = G.xcd_map && P.N > P.M;
  const int m0 = (nmaj ? t % P.tiles_m : t / P.tiles_n) * 64, n0 = (nmaj ? t / P.tiles_m : t % P.tiles_n) * 64;
  const int ksteps = (P.K + 31) >> 5;
  const int per = (ksteps + P.ksplit - 1) / P.ksplit;
  const int kbeg = split * per * 32, kend = min(P.K, (split * per + per) * 32);
  // step parity (double-buffered bf16 weight shadows, fused SGD epilogue): one scalar load
  const int64_t st = ((P.b_par != 0 || P.c_mode == 4) && G.step) ? *G.step : 0;
  const bf16* A = reinterpret_cast<const bf16*>(P.A);
  const bf16* B = reinterpret_cast<const bf16*>(P.B) + ((st & 1) ? P.b_par : 0);
  const int wm = w >> 1, wn = w & 1;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) { acc[i][0] = zero4(); acc[i][1] = zero4(); }

  // fused SGD (c_mode 4): this tile's fp32 master weights are loaded NOW, under the mainloop, not
  // after it (the epilogue's one dependent memory round trip was ~1 us of every dW1 block)
  float4 wv[4];
  int ok[4];
  if (P.c_mode == 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + u * 256, rr = e >> 4, cc = (e & 15) * 4;
      const int m = m0 + rr, n = n0 + cc;
      ok[u] = m < P.M && n < P.nvalid;
      wv[u] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(P.C) + (ok[u] ? (size_t)m * P.ldc + n : 0));
    }
  }

  // Two chunks of operand loads in flight (64 KB per block): the loads of chunk i+2 are issued as
  // soon as chunk i's registers are in LDS.  With one chunk in flight every 128-deep chunk paid a
  // whole memory latency under load (~1.6-2 us per chunk, in-kernel stamps); a K slice of up to two
  // chunks (fc1 forward, dW1) now pays one.  Unrolled by two so the register sets stay static.
  auto mma = [&](const bf16* a_s, const bf16* b_s, int nk) {
    for (int kk = 0; kk < nk; ++kk) {
      const bf16x8 a0 = frag(a_s, P.a_kmajor, 32 * wm, kk, g, li);
      const bf16x8 a1 = frag(a_s, P.a_kmajor, 32 * wm + 16, kk, g, li);
      const bf16x8 b0 = frag(b_s, P.b_kmajor, 32 * wn, kk, g, li);
      const bf16x8 b1 = frag(b_s, P.b_kmajor, 32 * wn + 16, kk, g, li);
      acc[0][0] = mfma16(a0, b0, acc[0][0]);
      acc[0][1] = mfma16(a0, b1, acc[0][1]);
      acc[1][0] = mfma16(a1, b0, acc[1][0]);
      acc[1][1] = mfma16(a1, b1, acc[1][1]);
    }
  };
  if (kbeg < kend) {
    Chunk ca0, cb0, ca1, cb1;
    ca0.load(A, P.lda, P.a_kmajor, P.M, kend, m0, kbeg, tid);
    cb0.load(B, P.ldb, P.b_kmajor, P.N, kend, n0, kbeg, tid);
    if (kbeg + KC < kend) {
      ca1.load(A, P.lda, P.a_kmajor, P.M, kend, m0, kbeg + KC, tid);
      cb1.load(B, P.ldb, P.b_kmajor, P.N, kend, n0, kbeg + KC, tid);
    }
    // buffer b was last read by the MFMAs two chunks ago, which every wave finished before the
    // barrier of the chunk in between
    for (int k0 = kbeg; k0 < kend; k0 += 2 * KC) {
      ca0.store(sA, P.a_kmajor, tid);
      cb0.store(sB, P.b_kmajor, tid);
      if (k0 + 2 * KC < kend) {
        ca0.load(A, P.lda, P.a_kmajor, P.M, kend, m0, k0 + 2 * KC, tid);
        cb0.load(B, P.ldb, P.b_kmajor, P.N, kend, n0, k0 + 2 * KC, tid);
      }
      __syncthreads();
      mma(sA, sB, min(KC, kend - k0 + 31) >> 5);
      if (k0 + KC >= kend) break;
      ca1.store(sA + TILE_ELEMS, P.a_kmajor, tid);
      cb1.store(sB + TILE_ELEMS, P.b_kmajor, tid);
      if (k0 + 3 * KC < kend) {
        ca1.load(A, P.lda, P.a_kmajor, P.M, kend, m0, k0 + 3 * KC, tid);
        cb1.load(B, P.ldb, P.b_kmajor, P.N, kend, n0, k0 + 3 * KC, tid);
      }
      __syncthreads();
      mma(sA + TILE_ELEMS, sB + TILE_ELEMS, min(KC, kend - k0 - KC + 31) >> 5);
    }
  }
  DMLC_STAMP(DMLC_TK_GEMM, 1);

  // epilogue: acc[i][j] holds C[m0+32wm+16i+4g+r][n0+32wn+16j+li] -- 4 rows of ONE column per lane,
  // i.e. 4-byte stores scattered over rows.  The tile goes through LDS instead ([64][68] fp32 over
  // the A buffers, free once every wave is past the last chunk) and leaves as 16-B row vectors.
  float* ct = reinterpret_cast<float*>(smem);
  constexpr int CT_LD = 68;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) ct[(32 * wm + 16 * i + 4 * g + r) * CT_LD + 32 * wn + 16 * j + li] = acc[i][j][r];
  __syncthreads();
  const bool vec = (P.ldc & 3) == 0;
  if (P.c_mode == 4) {
    // fused SGD (single GPU): acc is the complete weight gradient of this tile (K = the whole batch,
    // no split); master update + the next step's bf16 shadow, both 16-B row vectors (ldc % 4 == 0,
    // nvalid == N, checked by the binding)
    const float f = lr_sched(G.lr0, G.decay, G.decay_steps, G.staircase, G.warmup, st) * G.grad_scale;
    bf16* S = reinterpret_cast<bf16*>(P.S) + (((st + 1) & 1) ? P.s_par : 0);
    void* cbase = const_cast<void*>(uni(P.C));   // buffer descriptors live in SGPRs
    void* sbase = const_cast<void*>(uni(S));
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (!ok[u]) continue;
      const int e = tid + u * 256, rr = e >> 4, cc = (e & 15) * 4;
      const size_t q = (size_t)(m0 + rr) * P.ldc + n0 + cc;
      const float4 g = *reinterpret_cast<const float4*>(ct + rr * CT_LD + cc);
      float4 v = wv[u];
      v.x -= f * g.x; v.y -= f * g.y; v.z -= f * g.z; v.w -= f * g.w;
      // write-through: no dirty master / shadow lines for the kernel-boundary write-back (as the fc
      // chain's epilogue, fc_common.h)
      st_out16(cbase, (uint32_t)(q * 4), __builtin_bit_cast(uint4, make_float4(v.x, v.y, v.z, v.w)));
      st_out8(sbase, (uint32_t)(q * 2), __builtin_bit_cast(uint2, pack4(v.x, v.y, v.z, v.w)));
    }
    DMLC_STAMP(DMLC_TK_GEMM, 2);
    return;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = tid + u * 256, rr = e >> 4, cc = (e & 15) * 4;
    const int m = m0 + rr, n = n0 + cc;
    if (m >= P.M || n >= P.nvalid) continue;
    float4 v = *reinterpret_cast<const float4*>(ct + rr * CT_LD + cc);
    float vv[4] = {v.x, v.y, v.z, v.w};
    if (P.c_mode != 2) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        vv[k] += (P.bias && n + k < P.nvalid) ? P.bias[n + k] : 0.f;
        if (P.relu) vv[k] = fmaxf(vv[k], 0.f);
      }
    }
    const size_t base = (P.c_mode == 2 ? (size_t)split * P.M * P.ldc : 0) + (size_t)m * P.ldc + n;
    if (vec && n + 4 <= P.nvalid) {
      if (P.c_mode == 1) *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(P.C) + base) = pack4(vv[0], vv[1], vv[2], vv[3]);
      else {
        const f32x4 o = {vv[0], vv[1], vv[2], vv[3]};
        st_maybe_nt<kNtGemm>(reinterpret_cast<f32x4*>(reinterpret_cast<float*>(P.C) + base), o);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (n + k >= P.nvalid) break;
        if (P.c_mode == 1) reinterpret_cast<bf16*>(P.C)[base + k] = (bf16)vv[k];
        else reinterpret_cast<float*>(P.C)[base + k] = vv[k];
      }
    }
  }
  DMLC_STAMP(DMLC_TK_GEMM, 2);
}

}  // namespace dmlc

using namespace dmlc;

extern "C" hipError_t dmlc_gemm_grouped(DmlcGemmGroup* G, hipStream_t s) {
#ifndef DMLC_GEMM_FIFO
  // Longest blocks first: workgroups are dispatched in blockIdx order, so the problems are laid out
  // by descending k-steps per block (stable).  In the B > 256 backward the K = batch weight-gradient
  // tiles (dW1: 216 blocks of 32 k-steps at B = 1024) otherwise start behind the 576 short dp2 tiles
  // and end the launch alone.  The kernel locates a problem by its block range only.
  {
    auto work = [](const DmlcGemmProblem& P) {     // k-steps per block
      const int ks = (P.K + 31) / 32, sp = P.ksplit > 1 ? P.ksplit : 1;
      return P.c_mode == 3 ? 0 : (ks + sp - 1) / sp;
    };
    for (int i = 1; i < G->nprob; ++i)
      for (int j = i; j > 0 && work(G->p[j]) > work(G->p[j - 1]); --j) {
        const DmlcGemmProblem t = G->p[j];
        G->p[j] = G->p[j - 1];
        G->p[j - 1] = t;
      }
  }
#endif
  int blocks = 0;
  for (int i = 0; i < G->nprob; ++i) {
    DmlcGemmProblem& P = G->p[i];
    P.tiles_m = (P.M + 63) / 64;
    P.tiles_n = P.c_mode == 3 ? 1 : (P.N + 63) / 64;
    if (P.ksplit < 1) P.ksplit = 1;
    if (P.c_mode == 3) P.ksplit = 1;
    P.block_start = blocks;
    const int nb = P.tiles_m * P.tiles_n * P.ksplit;
    blocks += G->xcd_map ? (nb + 7) / 8 * 8 : nb;
  }
  G->nblocks = blocks;
  if (blocks == 0) return hipSuccess;
  DMLC_LDS_OPTIN(&k_gemm_grouped, GEMM_LDS);
  hipLaunchKernelGGL(k_gemm_grouped, dim3(blocks), dim3(256), GEMM_LDS, s, *G);
  return hipGetLastError();
}
