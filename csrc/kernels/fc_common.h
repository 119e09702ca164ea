// Building blocks of the fully-connected chain shared by the persistent fc-chain launch
// (cnn_fc.hip) and the weight-gradient launch (cnn_wgrad.hip, apply mode: the fc weight gradients
// and their SGD run in the conv1 blocks' idle time there).  See cnn_fc.hip for the design.
#pragma once
#include "common.h"
#include "api.h"

namespace dmlc {

DEV const bf16* P2(const DmlcFcArgs& a) { return reinterpret_cast<const bf16*>(a.p2); }
DEV bf16* W1S(const DmlcFcArgs& a) { return reinterpret_cast<bf16*>(a.w1); }
DEV bf16* DP2(const DmlcFcArgs& a) { return reinterpret_cast<bf16*>(a.dp2); }

constexpr int FT = 512;                        // 8 waves
constexpr int FC_BLOCKS = 256;
constexpr int FC_S = 8;                        // fc1 forward K split (288 = 9 k-steps each)
constexpr int FC_KS = 2304 / FC_S;
constexpr int FC_RB = 4;                       // head rows per block

// ---- LDS images ---------------------------------------------------------------------------------
// k-major [rows][stride] bf16 with stride = 16 (mod 128) elements: a row is 8 banks further on, so
// the 16 lanes of every ds_read_b128 lane group hit 64 distinct banks (as cnn_gemm.hip's KC_LD)
constexpr int KST_A = 400;                     // K <= 384 (fc1 forward slice 288, dp2 384)
// m-major [k rows][64 cols] bf16, unpadded 128-B rows, 16-B chunk index XORed by row bits 1 and 3
// (cnn_gemm.hip mswz: conflict-free ds_read_b64_tr_b16 and conflict-free 16-B stores)
DEV int mz(int row, int col) {
  const int f = 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
  return row * 64 + (((col >> 3) ^ f) << 3) + (col & 7);
}
DEV bf16x8 kfrag(const bf16* img, int stride, int r0, int kk, int g, int li) {
  return lds_b128(img + (r0 + li) * stride + kk * 32 + 8 * g);
}
DEV bf16x8 mfrag(const bf16* img, int c0, int kk, int g, int li) {
  const int q = li >> 2, p = li & 3;
  return tr_frag(img + mz(kk * 32 + 8 * g + q, c0 + 4 * p), img + mz(kk * 32 + 8 * g + 4 + q, c0 + 4 * p));
}

// GEMM task LDS: dp2 = dh1 rows [64][400] + W1 rows [128][400]; dW1 = p2 columns 2 x [256][64] +
// dh1 columns [256][64]; fc1 forward = p2 rows [64][400] + W1 slice [288][64]
constexpr int L_DP2_A = 0, L_DP2_B = 64 * KST_A * 2;
constexpr int L_DP2_END = L_DP2_B + 128 * KST_A * 2;
constexpr int L_W1_A = 0, L_W1_B = 2 * 256 * 64 * 2;
constexpr int L_FWD_A = 0, L_FWD_B = 64 * KST_A * 2;
constexpr int L_RED = L_W1_B + 256 * 64 * 2;   // [8][64] fp32 bias-gradient partials (dW tasks)
// ---- sync words (DmlcFcArgs::sync, uints, each counter on its own 128-B line) --------------------
// (common.h Seam: each seam's arrivals are spread over several words, polled side by side)
// a.sync + 32 * 9: launch epoch E; a.sync + 32 * 10 .. + 32 * 19: the two-level end-of-launch ticket
// (common.h last_arrival)
DEV unsigned* epochW(const DmlcFcArgs& a) { return a.sync + 32 * 9; }
// fc1 forward task (m, nt, s) -> word (m, nt): FC_S arrivals each; the head blocks of row tile m wait
// for the tile's 6 words
constexpr int SY_A = 28, SY_B = SY_A + 24, SY_D = SY_B + 16, SY_END = SY_D + 2 * 4 * 18;
static_assert(SY_END == 212, "engine/fused.py fc_sync and the binding size the sync words");
DEV unsigned* cntA(const DmlcFcArgs& a, int m, int nt) { return a.sync + 32 * (SY_A + 6 * m + nt); }
DEV Seam seamA(const DmlcFcArgs& a, int m) { return Seam{cntA(a, m, 0), 6, (unsigned)FC_S}; }
// head block hb (row tile m = hb >> 4) -> word (m, hb & 3): a quarter of the tile's head blocks each
DEV unsigned* cntB(const DmlcFcArgs& a, int m, int q) { return a.sync + 32 * (SY_B + 4 * m + q); }
DEV unsigned head_quarter(const DmlcFcArgs& a, int m) { return (unsigned)(min(64, a.B - 64 * m) / FC_RB / 4); }
DEV Seam seamB(const DmlcFcArgs& a, int m) { return Seam{cntB(a, m, 0), 4, head_quarter(a, m)}; }
// dp2 task (m, j) -> one flag word of set E & 1 (the launch's last arrival re-arms the OTHER set and
// bumps E, so it can arrive before the dgrad's waits are done); the dgrad of an image in row tile m
// waits for the tile's 18 words
constexpr unsigned DP2_COL_TILES = 2304 / 128;
DEV unsigned* cntD(const DmlcFcArgs& a, unsigned set, int m, int j) {
  return a.sync + 32 * (SY_D + 72 * (set & 1) + 18 * m + j);
}
DEV Seam seamD(const DmlcFcArgs& a, unsigned set, int m) { return Seam{cntD(a, set, m, 0), (int)DP2_COL_TILES, 1u}; }

DEV unsigned ld_relaxed(unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// one lane: spin until *p >= target (bounded; on give-up the sticky error word is set)
DEV void wait_ge(unsigned* p, unsigned target, unsigned* err) {
  for (unsigned it = 0; ld_relaxed(p) < target; ++it) {
    if (it >= DMLC_SPIN_LIMIT) {
      __hip_atomic_fetch_or(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
// every storing wave drains its write-through stores, the workgroup meets, one lane signals
DEV void publish(unsigned* c) {
  wait_vm_all();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// wave 0 waits, then the workgroup meets (every later load of the handed-off bytes is sc1)
DEV void consume(const Seam& s, unsigned* err) {
  if (threadIdx.x < 64) seam_wait(s, threadIdx.x, err, 2u);
  __syncthreads();
}

DEV uint4 ld16(rsrc_t r, uint32_t off) {      // sc1 16-B load (hand-off bytes)
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSC1));
}
DEV void st16(rsrc_t r, uint32_t off, const uint4& v) {   // sc1 16-B store (hand-off bytes)
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, kSC1);
}

// ---- one MFMA k-step accumulate of a 32x32 wave tile --------------------------------------------
struct Acc {
  f32x4 c[2][2];
  MDEV void zero() {
#pragma unroll
    for (int i = 0; i < 2; ++i) { c[i][0] = zero4(); c[i][1] = zero4(); }
  }
  MDEV void mma(const bf16x8& a0, const bf16x8& a1, const bf16x8& b0, const bf16x8& b1) {
    c[0][0] = mfma16(a0, b0, c[0][0]);
    c[0][1] = mfma16(a0, b1, c[0][1]);
    c[1][0] = mfma16(a1, b0, c[1][0]);
    c[1][1] = mfma16(a1, b1, c[1][1]);
  }
  // into an fp32 LDS tile [rows][ld]: acc[i][j][r] = C[r0 + 16i + 4g + r][c0 + 16j + li]
  MDEV void to_lds(float* t, int ld, int r0, int c0, int g, int li) const {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) t[(r0 + 16 * i + 4 * g + r) * ld + c0 + 16 * j + li] = c[i][j][r];
  }
  MDEV void add_lds(float* t, int ld, int r0, int c0, int g, int li) const {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) t[(r0 + 16 * i + 4 * g + r) * ld + c0 + 16 * j + li] += c[i][j][r];
  }
};
constexpr int CT_LD = 68;                     // fp32 staging rows (64 + 4): conflict-free 4-B writes

// =================================================================================================
// Phase C tasks.  Types (in task order): dp2 (64 rows x 128 k1 of dp2 = dh1 W1^T, K = 384),
// dW1 (128 k1 x 64 n of p2^T dh1, K = B; fused SGD or gradient), dW2 (128 x 64 of h1^T dh2),
// dW3 (128 x 16 of h2^T dl); the first M tile of each dW also sums its dh1 / dh2 / dl columns into
// db1 / db2 / db3.
// =================================================================================================
struct CTask { int kind, i, j; };   // kind 0 dp2, 1 dW1, 2 dW2, 3 dW3
DEV CTask ctask_(const DmlcFcArgs& a, int t);
// (wave-uniform fields: held in SGPRs, so the task branches are uniform and no kernel argument has
// to live in divergent-code VGPRs -- without this hipcc copied the argument block to scratch)
DEV CTask ctask(const DmlcFcArgs& a, int t) {
  const CTask T = ctask_(a, t);
  return {__builtin_amdgcn_readfirstlane(T.kind), __builtin_amdgcn_readfirstlane(T.i), __builtin_amdgcn_readfirstlane(T.j)};
}
DEV CTask ctask_(const DmlcFcArgs& a, int t) {
  const int ndp2 = a.mtiles * 18;
  if (t < ndp2) return {0, t / 18, t % 18};
  if (!a.dw_tasks) return {-1, 0, 0};          // the weight-gradient launch runs the dW tiles
  t -= ndp2;
  if (t < 108) return {1, t / 6, t % 6};
  t -= 108;
  if (t < 9) return {2, t / 3, t % 3};
  t -= 9;
  if (t < 2) return {3, t, 0};
  return {-1, 0, 0};
}
// (the bias gradients ride along: the i == 0 tiles of dW1 / dW2 / dW3 hold dh1 / dh2 / dl columns in
// LDS and sum them -- three column-sum tasks of their own were each a chain of dependent row loads)
constexpr int FC_DW_TASKS = 108 + 9 + 2;      // dW1, dW2, dW3 tiles
DEV int ctask_count(const DmlcFcArgs& a) { return a.mtiles * 18 + (a.dw_tasks ? FC_DW_TASKS : 0); }
// dW task d (0 <= d < FC_DW_TASKS) as a C task (what the weight-gradient launch runs)
DEV CTask dw_ctask(int d) {
  const CTask T = d < 108 ? CTask{1, d / 6, d % 6} : d < 117 ? CTask{2, (d - 108) / 3, (d - 108) % 3}
                                                             : CTask{3, d - 117, 0};
  return {__builtin_amdgcn_readfirstlane(T.kind), __builtin_amdgcn_readfirstlane(T.i), __builtin_amdgcn_readfirstlane(T.j)};
}

// what a dp2 / dW1 task stages before its seam: 12 x 16 B (W1 rows, or p2 columns) + 4 float4 of
// the fp32 master (dW1 with the fused SGD); always the same number of loads (static vmcnt counts)
struct PreRegs { uint4 v[12]; float4 m[4]; };
// branch-free: every block issues the same 16 loads whatever its task (others read valid dummy
// addresses and discard), so the forward task's waits count them statically
DEV void pre_issue(const DmlcFcArgs& a, const CTask& T, int parity, PreRegs& R, int tid) {
  const bf16* W1 = W1S(a) + (parity ? 884736 : 0);
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int c = tid + i * FT;
    const int rw0 = c / 48, kc0 = c - rw0 * 48;          // dp2: W1 rows [128 j .. +128][384]
    const int rw1 = c >> 4, cc1 = c & 15;                // dW1: p2 columns [B rows][128 i .. +128]
    const bool ok1 = T.kind == 1 && rw1 < a.B;
    const bf16* p = T.kind == 0 ? W1 + (size_t)(128 * T.j + rw0) * 384 + 8 * kc0
                                : ok1 ? P2(a) + (size_t)rw1 * 2304 + 128 * T.i + 8 * cc1 : P2(a);
    R.v[i] = load_sel(reinterpret_cast<const uint4*>(p), reinterpret_cast<const uint4*>(P2(a)), T.kind == 0 || ok1);
  }
  // master tile [128][64] fp32: dW1 with a fused SGD (gw1 = the fc1 master), dW2 with every fc
  // parameter fused (mw2, [384][192])
  const bool fc2m = T.kind == 2 && a.fuse_sgd == 2;
  const float* mb = fc2m ? (const float*)uni(a.mw2) : (const float*)uni(a.gw1);
  const int mld = fc2m ? 192 : 384;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = tid + u * FT, rr = e >> 4, cc = (e & 15) * 4;
    const bool ok = (T.kind == 1 && a.fuse_sgd != 0) || fc2m;
    R.m[u] = load_sel(reinterpret_cast<const float4*>(mb + (size_t)(128 * T.i + rr) * mld + 64 * T.j + cc),
                      reinterpret_cast<const float4*>(mb), ok);
  }
}
DEV void pre_store(const DmlcFcArgs& a, const CTask& T, const PreRegs& R, char* smem, int tid) {
  if (T.kind == 0) {
    bf16* sb = reinterpret_cast<bf16*>(smem + L_DP2_B);
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const int c = tid + i * FT, rw = c / 48, kc = c - rw * 48;
      *reinterpret_cast<uint4*>(sb + rw * KST_A + 8 * kc) = R.v[i];
    }
  } else if (T.kind == 1) {
    bf16* sa = reinterpret_cast<bf16*>(smem + L_W1_A);
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const int c = tid + i * FT, rw = c >> 4, cc = c & 15;
      if (rw < 256) *reinterpret_cast<uint4*>(sa + (cc >> 3) * 256 * 64 + mz(rw, 8 * (cc & 7))) = R.v[i];
    }
  }
}

// m-major hand-off operand [K = B rows][64 cols c0 ..] of a bf16 [B][ld] matrix (sc1 loads; columns
// >= ncol and rows >= B read as zero) into the image at `img`
// (all of a thread's loads in flight at once: Kpad <= 256 rows x 8 chunks = at most 4 per thread)
DEV void stage_m_sc1(const void* base, int ld, int c0, int ncol, int B, bf16* img, int Kpad, int tid) {
  const rsrc_t r = buf_rsrc(base);
  uint4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + i * FT, rw = c >> 3, col = c0 + 8 * (c & 7);
    const bool ok = rw < B && col < ncol;
    v[i] = ld16(r, ok ? (uint32_t)(rw * ld + col) * 2 : 0u);
    if (!ok) v[i] = make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + i * FT, rw = c >> 3;
    if (rw < Kpad) *reinterpret_cast<uint4*>(img + mz(rw, 8 * (c & 7))) = v[i];
  }
}

// 128 (M) x 64 (N) x K=Kpad product of two m-major images: A = na 64-col images (cols 64 x img),
// B one 64-col image; waves: wm = w >> 1 (32-row quarter), wn = w & 1
DEV void mma_128x64(const bf16* sa, const bf16* sb, int ksteps, Acc& acc, int w, int g, int li) {
  const int wm = w >> 1, wn = w & 1;
  const bf16* ia = sa + (wm >> 1) * 256 * 64;
  const int ca = 32 * (wm & 1);
  for (int kk = 0; kk < ksteps; ++kk)
    acc.mma(mfrag(ia, ca, kk, g, li), mfrag(ia, ca + 16, kk, g, li), mfrag(sb, 32 * wn, kk, g, li),
            mfrag(sb, 32 * wn + 16, kk, g, li));
}


DEV void dp2_task(const DmlcFcArgs& a, const CTask& T, char* smem, int tid, unsigned epoch) {
  bf16* sa = reinterpret_cast<bf16*>(smem + L_DP2_A);
  bf16* sb = reinterpret_cast<bf16*>(smem + L_DP2_B);
  const int mt = T.i, n0 = 128 * T.j;
  const int rows = min(64, a.B - 64 * mt);
  consume(seamB(a, mt), a.err);
  DMLC_STAMP(DMLC_TK_GEMM, 3);
  {
    const rsrc_t r = buf_rsrc(a.dh1);
    uint4 v[6];                                // dh1 rows [64][384]: 6 x 16 B per thread, all in flight
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int c = tid + i * FT, rw = c / 48, kc = c - rw * 48;
      const bool ok = rw < rows;
      v[i] = ld16(r, ok ? (uint32_t)((64 * mt + rw) * 384 + 8 * kc) * 2 : 0u);
      if (!ok) v[i] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int c = tid + i * FT, rw = c / 48, kc = c - rw * 48;
      *reinterpret_cast<uint4*>(sa + rw * KST_A + 8 * kc) = v[i];
    }
  }
  __syncthreads();
  const int w = wave_id(), lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int wm = w & 1, wn = w >> 1;
  Acc acc;
  acc.zero();
  bf16x8 F[2][4];                              // software-pipelined as mma_128x64
  auto frags = [&](int kk, bf16x8 (&f)[4]) __attribute__((always_inline)) {
    f[0] = kfrag(sa, KST_A, 32 * wm, kk, g, li);
    f[1] = kfrag(sa, KST_A, 32 * wm + 16, kk, g, li);
    f[2] = kfrag(sb, KST_A, 32 * wn, kk, g, li);
    f[3] = kfrag(sb, KST_A, 32 * wn + 16, kk, g, li);
  };
  frags(0, F[0]);
#pragma unroll
  for (int kk = 0; kk < 12; ++kk) {
    const int cur = kk & 1;
    wait_lds();
    __builtin_amdgcn_sched_barrier(0);
    if (kk + 1 < 12) frags(kk + 1, F[cur ^ 1]);
    __builtin_amdgcn_sched_barrier(0);
    acc.mma(F[cur][0], F[cur][1], F[cur][2], F[cur][3]);
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  DMLC_STAMP(DMLC_TK_GEMM, 4);
  float* ct = reinterpret_cast<float*>(smem);  // [64][132]
  constexpr int LD = 132;
  acc.to_lds(ct, LD, 32 * wm, 32 * wn, g, li);
  __syncthreads();
  // sc1 stores + the row tile's counter: the launch's conv2 dgrad (one image per workgroup) reads
  // these rows as soon as all 18 column tiles of its row tile are published
  const rsrc_t rd = buf_rsrc(a.dp2);
#pragma unroll
  for (int u = 0; u < 2; ++u) {                // 64 x 128 bf16 = 1024 x 16-B pieces
    const int e = tid + u * FT, rr = e >> 4, cc = (e & 15) * 8;
    if (rr < rows) {
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(ct + rr * LD + cc);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(ct + rr * LD + cc + 4);
      const uint2 lo = __builtin_bit_cast(uint2, pack4(v0[0], v0[1], v0[2], v0[3]));
      const uint2 hi = __builtin_bit_cast(uint2, pack4(v1[0], v1[1], v1[2], v1[3]));
      st16(rd, (uint32_t)((64 * mt + rr) * 2304 + n0 + cc) * 2, make_uint4(lo.x, lo.y, hi.x, hi.y));
    }
  }
  publish(cntD(a, epoch, mt, T.j));
}

// dW1 / dW2 / dW3: 128 x 64 tile of A^T B over the batch (A, B: bf16 [B][lda], [B][ldb])
// One 16-B chunk per thread of a 64-row tile of an m-major hand-off operand: rows 64 m + (tid >> 3),
// columns c0 + 8 (tid & 7) of a bf16 [B][ld] matrix (sc1; rows >= B / columns >= ncol read as zero)
// (SC1 = false: the operand comes from an earlier launch -- plain loads, which may hit this XCD's L2;
// the tasks sharing a column slice then fetch it from memory once per XCD, not once each)
template <bool SC1 = true>
DEV uint4 ld_mtile(const void* base, int ld, int c0, int ncol, int B, int m, int tid) {
  const int rw = 64 * m + (tid >> 3), col = c0 + 8 * (tid & 7);
  const bool ok = rw < B && col < ncol;
  const uint32_t off = ok ? (uint32_t)(rw * ld + col) * 2 : 0u;
  const uint4 v = SC1 ? ld16(buf_rsrc(base), off)
                      : __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(buf_rsrc(base), off, 0, 0));
  return ok ? v : make_uint4(0, 0, 0, 0);
}
DEV void st_mtile(bf16* img, int m, const uint4& v, int tid) {
  *reinterpret_cast<uint4*>(img + mz(64 * m + (tid >> 3), 8 * (tid & 7))) = v;
}

// HANDOFF (the fc-chain launch): the dh1 / h1 / h2 / dh2 / dl rows come from the head blocks of the
// same launch -- wait for each 64-row tile's counter, sc1 loads.  Otherwise (the weight-gradient
// launch) they were written by an earlier launch: no waits.
struct NoOp { __device__ void operator()() const {} };
// after_issue (no hand-off only): runs once every operand load is in flight (the wgrad launch's
// conv1 blocks drain their slab stores and arrive at their barrier there, under the loads)
template <bool HANDOFF, class F = NoOp>
DEV void dw_task(const DmlcFcArgs& a, const CTask& T, const PreRegs& R, int64_t step, char* smem, int tid,
                 F&& after_issue = F{}) {
  bf16* sa = reinterpret_cast<bf16*>(smem + L_W1_A);
  bf16* sb = reinterpret_cast<bf16*>(smem + L_W1_B);
  const int Kpad = (a.B + 31) & ~31;
  const int m0 = 128 * T.i, n0 = 64 * T.j;
  // dW1 = p2^T dh1 (A staged before the seam), dW2 = h1^T dh2, dW3 = h2^T dl (10 columns)
  const int M = T.kind == 1 ? 2304 : T.kind == 2 ? 384 : 192;
  const int N = T.kind == 1 ? 384 : T.kind == 2 ? 192 : 10;
  const int ldc = N;
  // The K (= batch) range is the head blocks' rows: lanes 0..15 of wave 0 poll the 4 x 4 head words
  // side by side (one memory round trip per poll round for all of them), then every tile's loads go
  // out at once.  (r4 waited for each tile's counter in turn, issuing that tile's loads in between --
  // the head blocks finish together, so that bought no overlap and cost a round trip per tile.)  The
  // barrier is an s_barrier (lds_barrier), not __syncthreads: that would drain the prefetched loads
  // already in flight.
  // (the operand of each kind, selected branch-free: the same three loads per tile for every kind)
  // (every candidate made opaque BEFORE the select: a select between two argument fields becomes a
  // load through a selected address into the argument block, and hipcc then copies the whole block
  // to scratch)
  const void* pa = T.kind == 2 ? uni(a.h1) : uni(a.h2);
  const void* pb = T.kind == 1 ? uni(a.dh1) : T.kind == 2 ? uni(a.dh2) : uni(a.dl);
  const int lda = __builtin_amdgcn_readfirstlane(T.kind == 2 ? 384 : 192);
  const int ldb = __builtin_amdgcn_readfirstlane(T.kind == 1 ? 384 : T.kind == 2 ? 192 : 16);
  const int cb = T.kind == 3 ? 0 : n0;
  const bool need_a = T.kind != 1;
  // (written out per tile: as a loop over the tiles it stayed rolled and its register arrays went
  // to scratch)
  struct T3 { uint4 a0, a1, b; };
  if (HANDOFF) {
    if (tid < 64)                              // lane 4m + q: word (m, q) of row tile m < mtiles
      seam_wait(Seam{cntB(a, 0, 0), 4 * a.mtiles, 0u}, tid, a.err, 2u, (int)head_quarter(a, min(tid >> 2, 3)));
    lds_barrier();
  }
  auto tile = [&](int m) __attribute__((always_inline)) {
    const bool on = m < a.mtiles;
    const int Bm = on ? a.B : 0;            // a tile past the batch reads nothing (zeros)
    T3 r;
    r.b = ld_mtile<HANDOFF>(pb, ldb, cb, ldb, Bm, m, tid);
    r.a0 = ld_mtile<HANDOFF>(pa, lda, m0, need_a ? lda : 0, Bm, m, tid);
    r.a1 = ld_mtile<HANDOFF>(pa, lda, m0 + 64, need_a ? lda : 0, Bm, m, tid);
    return r;
  };
  auto put = [&](int m, const T3& r) __attribute__((always_inline)) {
    if (64 * m + (tid >> 3) < Kpad) {
      st_mtile(sb, m, r.b, tid);
      if (need_a) {
        st_mtile(sa, m, r.a0, tid);
        st_mtile(sa + 256 * 64, m, r.a1, tid);
      }
    }
  };
  const T3 t0 = tile(0), t1 = tile(1), t2 = tile(2), t3 = tile(3);
  if (HANDOFF) DMLC_STAMP(DMLC_TK_GEMM, 3);
  // no hand-off (inputs from earlier launches): the caller issued R and returned at once, so the
  // prefetch and the tile loads are in flight together -- one memory round trip, not two
  if (!HANDOFF) {
    after_issue();
    __syncthreads();                           // the previous role's LDS reads are done
    pre_store(a, T, R, smem, tid);
    DMLC_STAMP(DMLC_TK_GEMM, 5);
  }
  put(0, t0); put(1, t1); put(2, t2); put(3, t3);
  __syncthreads();
  const int w = wave_id(), lane = tid & 63, g = lane >> 4, li = lane & 15;
  // bias gradient of the B columns (first M tile only): 8 row groups x 64 columns, fixed order
  float* red = reinterpret_cast<float*>(smem + L_RED);
  const bool bias = T.i == 0;
  if (bias) {
    const int col = tid & 63, rg = tid >> 6;
    // 8 rows per round in flight (a rolled loop waited one LDS latency per row: ~1.3 us at B=256 on
    // the three tasks that carry a bias); rows past Kpad read row 0 and add 0
    float sum = 0.f;
    for (int r0 = rg; r0 < Kpad; r0 += 64) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int rw = r0 + 8 * u;
        v[u] = rw < Kpad ? (float)sb[mz(rw < Kpad ? rw : 0, col)] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) sum += v[u];
    }
    red[rg * 64 + col] = sum;
  }
  Acc acc;
  acc.zero();
  mma_128x64(sa, sb, Kpad >> 5, acc, w, g, li);
  __syncthreads();
  if (HANDOFF) DMLC_STAMP(DMLC_TK_GEMM, 4);
  else DMLC_STAMP(DMLC_TK_GEMM, 6);
  // fused SGD modes: the SGD kernel's update expression (w -= (lr * grad_scale) * g), so the weights
  // are bit-identical to the gradient + SGD-launch path
  const float f = lr_sched(a.lr0, a.decay, a.decay_steps, a.staircase, a.warmup, step) * a.grad_scale;
  const bool all_fused = a.fuse_sgd == 2;
  if (bias && tid < 64 && n0 + tid < N) {
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) sum += red[k * 64 + tid];
    if (all_fused) {
      float* mb = (float*)(T.kind == 1 ? uni(a.mb1) : T.kind == 2 ? uni(a.mb2) : uni(a.mb3));
      float v = mb[n0 + tid];
      v -= f * sum;
      mb[n0 + tid] = v;
    } else if (a.grad_bf16) {
      ((bf16*)(T.kind == 1 ? uni(a.gb1) : T.kind == 2 ? uni(a.gb2) : uni(a.gb3)))[n0 + tid] = (bf16)sum;
    } else {
      ((float*)(T.kind == 1 ? uni(a.gb1) : T.kind == 2 ? uni(a.gb2) : uni(a.gb3)))[n0 + tid] = sum;
    }
  }
  float* ct = reinterpret_cast<float*>(smem);  // [128][68]
  acc.to_lds(ct, CT_LD, 32 * (w >> 1), 32 * (w & 1), g, li);
  __syncthreads();
  if (T.kind == 1 && a.fuse_sgd) {
    // fused SGD (single GPU): the complete dW1 tile; master update + the NEXT step's bf16 shadow
    // (the expression of cnn_gemm.hip's c_mode 4 and the SGD kernel: bit-identical weights)
    bf16* S = W1S(a) + ((step & 1) ? 0 : 884736);    // the shadow the NEXT step reads
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + u * FT, rr = e >> 4, cc = (e & 15) * 4;
      const size_t q = (size_t)(m0 + rr) * 384 + n0 + cc;
      const float4 gv = *reinterpret_cast<const float4*>(ct + rr * CT_LD + cc);
      float4 v = R.m[u];
      v.x -= f * gv.x; v.y -= f * gv.y; v.z -= f * gv.z; v.w -= f * gv.w;
      // write-through (sc1): 3.5 MB of master + 1.8 MB of shadow per step would otherwise sit dirty
      // in the L2s for the kernel boundary's write-back (common.h st_out16); 77.7-78.4 vs 79.0-79.3
      // us/step at B=256 with nt stores (profiles/r5_fc1_epilogue_wt_ab.txt)
      st_out16(a.gw1, (uint32_t)(q * 4), __builtin_bit_cast(uint4, make_float4(v.x, v.y, v.z, v.w)));
      st_out8(S, (uint32_t)(q * 2), __builtin_bit_cast(uint2, pack4(v.x, v.y, v.z, v.w)));
    }
    return;
  }
  if (T.kind == 2 && all_fused) {
    // fc2 weights [384 k][192 n]: master, the same-layout shadow fc2n and (through an LDS transpose)
    // fc2t [192 n][384 k] -- as the SGD kernel's fc2 role writes them
    constexpr int TL = 136;                    // bf16 row stride of the [64 n][128 k] transpose tile
    bf16* tl = reinterpret_cast<bf16*>(smem + 40960);
    float* mw = (float*)uni(a.mw2);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + u * FT, rr = e >> 4, cc = (e & 15) * 4;
      const size_t q = (size_t)(m0 + rr) * 192 + n0 + cc;
      const float4 gv = *reinterpret_cast<const float4*>(ct + rr * CT_LD + cc);
      float4 v = R.m[u];
      v.x -= f * gv.x; v.y -= f * gv.y; v.z -= f * gv.z; v.w -= f * gv.w;
      *reinterpret_cast<float4*>(mw + q) = v;
      *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.fc2n) + q) = pack4(v.x, v.y, v.z, v.w);
      tl[(cc + 0) * TL + rr] = (bf16)v.x; tl[(cc + 1) * TL + rr] = (bf16)v.y;
      tl[(cc + 2) * TL + rr] = (bf16)v.z; tl[(cc + 3) * TL + rr] = (bf16)v.w;
    }
    lds_barrier();
#pragma unroll
    for (int u = 0; u < 2; ++u) {              // 64 n rows x 16 pieces of 8 k
      const int e = tid + u * FT, nn = e >> 4, k8 = e & 15;
      *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(a.fc2t) + (size_t)(n0 + nn) * 384 + m0 + 8 * k8) =
          *reinterpret_cast<const bf16x8*>(tl + nn * TL + 8 * k8);
    }
    return;
  }
  if (T.kind == 3 && all_fused) {
    // fc3 weights [192 k][10 n]: master, fc3t [16 n][192 k] and fc3d [192 k][32 n] (as the SGD
    // kernel's fc tail role)
    float* mw = (float*)uni(a.mw3);
    for (int e = tid; e < 128 * 10; e += FT) {
      const int rr = e / 10, n = e - rr * 10, m = m0 + rr;
      if (m >= 192) continue;
      float v = mw[m * 10 + n];
      v -= f * ct[rr * CT_LD + n];
      mw[m * 10 + n] = v;
      reinterpret_cast<bf16*>(a.fc3t)[n * 192 + m] = (bf16)v;
      reinterpret_cast<bf16*>(a.fc3d)[m * 32 + n] = (bf16)v;
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = tid + u * FT, rr = e >> 4, cc = (e & 15) * 4;
    const int m = m0 + rr, n = n0 + cc;
    if (m >= M || n >= N) continue;
    const float4 v = *reinterpret_cast<const float4*>(ct + rr * CT_LD + cc);
    if (a.grad_bf16) {                         // the bf16 flat gradient (RCCL bf16 wire)
      bf16* Cb = (bf16*)(T.kind == 1 ? uni(a.gw1) : T.kind == 2 ? uni(a.gw2) : uni(a.gw3));
      const float vv[4] = {v.x, v.y, v.z, v.w};
      if (ldc % 4 == 0 && n + 4 <= N) {
        *reinterpret_cast<bf16x4*>(Cb + (size_t)m * ldc + n) = pack4(v.x, v.y, v.z, v.w);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) if (n + k < N) Cb[(size_t)m * ldc + n + k] = (bf16)vv[k];
      }
      continue;
    }
    float* C = (float*)(T.kind == 1 ? uni(a.gw1) : T.kind == 2 ? uni(a.gw2) : uni(a.gw3));
    if (ldc % 4 == 0 && n + 4 <= N) {
      *reinterpret_cast<float4*>(C + (size_t)m * ldc + n) = v;
    } else {
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) if (n + k < N) C[(size_t)m * ldc + n + k] = vv[k];
    }
  }
}

DEV void c_task(const DmlcFcArgs& a, const CTask& T, const PreRegs& R, int64_t step, char* smem, int tid,
                unsigned epoch) {
  if (T.kind == 0) dp2_task(a, T, smem, tid, epoch);
  else dw_task<true>(a, T, R, step, smem, tid);
}

}  // namespace dmlc
