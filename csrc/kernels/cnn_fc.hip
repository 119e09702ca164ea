// The whole fully-connected part of a training step in ONE persistent launch (B <= 256):
//   fc1 forward (split-K) -> MLP head (fc1 reduce/bias/ReLU, fc2, fc3, ReLU logits, softmax xent,
//   accuracy, dlogits -> dh2 -> dh1) -> fc backward (dp2 = dh1 W1^T for the conv backward, dW1 with
//   the fused fc1 SGD epilogue, dW2, dW3, db1..3).
// Replaces /root/reference/cifar10cnn.py:126-176 and their autodiff through :163 (TF MatMul,
// BiasAdd, Relu, SparseSoftmaxCrossEntropyWithLogits + gradients).
//
// Why one launch: the three launches it replaces (grouped fc1 GEMM, head, grouped backward GEMM)
// were each a latency chain of ~6-8 us for < 1.5 GFLOP (tools/gemm_probe.py: a one-tile GEMM costs
// 4 us per graph-replayed launch), so every seam paid a launch boundary, a grid ramp and a cold
// operand fetch.  Here every block knows its whole schedule up front and loads what does not depend
// on the seam BEFORE waiting at it:
//   * head blocks (the first H = B/4 blocks, 4 batch rows each) stage all of fc2's weights (144 KB)
//     into LDS while the fc1 forward runs, then wait for their 64-row tile of fc1 partials;
//   * GEMM blocks (the rest) run one fc1-forward task (64 x 64 tile of one K slice), then stage the
//     operands of their backward task that are already known -- 128 fc1 weight rows (dp2 tasks) or
//     128 columns of the pooled conv2 output + the fp32 master tile (dW1 tasks) -- and only then
//     wait for the head's dh1 rows.
// Hand-offs (MI355X_MICROARCH.md, Valid forms, first table row): producers store the handed-off
// bytes write-through (sc1 buffer stores), every storing wave drains (vmcnt(0)), the workgroup
// barriers, ONE lane adds to a counter (agent-scope atomic); the consumer's one lane polls that
// counter with relaxed atomic loads, the workgroup barriers, and EVERY load of handed-off bytes is an
// sc1 buffer load.  Counters: one per 64-row tile for the fc1 partials (cntA) and for the head
// outputs (cntB) plus a total; the last block to finish re-arms them (zero) for the next launch.
// Every spin is bounded and sets the sticky error word (the engine's wgrad barrier error word) --
// all 256 blocks must be co-resident (one per CU: ~150 KB of LDS each; host-checked).
#include "common.h"
#include "api.h"

namespace dmlc {

// typed views of the DmlcFcArgs pointers
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

// head LDS (cnn_head.hip layouts): fc2 weights [192 n][384 k] swizzled, activations of RB rows + a
// zero row
constexpr int W2_LD = 384, H1_LD = 392, H2_LD = 200, DL_LD = 40;
DEV int w2swz(int row, int col) {
  return row * W2_LD + (((col >> 3) ^ (2 * (row & 3) + 8 * ((row >> 3) & 1))) << 3) + (col & 7);
}
struct HL {
  static constexpr int W2 = 0;
  static constexpr int H1 = W2 + 192 * W2_LD * 2;
  static constexpr int H2 = H1 + (FC_RB + 1) * H1_LD * 2;
  static constexpr int DH2 = H2 + (FC_RB + 1) * H2_LD * 2;
  static constexpr int DL = DH2 + (FC_RB + 1) * H2_LD * 2;
  static constexpr int LG = DL + (FC_RB + 1) * DL_LD * 2;
  static constexpr int BYTES = LG + 16 * 17 * 4;
};
// GEMM task LDS: dp2 = dh1 rows [64][400] + W1 rows [128][400]; dW1 = p2 columns 2 x [256][64] +
// dh1 columns [256][64]; fc1 forward = p2 rows [64][400] + W1 slice [288][64]
constexpr int L_DP2_A = 0, L_DP2_B = 64 * KST_A * 2;
constexpr int L_DP2_END = L_DP2_B + 128 * KST_A * 2;
constexpr int L_W1_A = 0, L_W1_B = 2 * 256 * 64 * 2;
constexpr int L_FWD_A = 0, L_FWD_B = 64 * KST_A * 2;
constexpr int L_RED = L_W1_B + 256 * 64 * 2;   // [8][64] fp32 bias-gradient partials (dW tasks)
constexpr int FC_LDS = L_DP2_END > HL::BYTES ? L_DP2_END : HL::BYTES;
static_assert(FC_LDS <= 160 * 1024, "fc chain LDS exceeds a CU");
static_assert(L_FWD_B + FC_KS * 64 * 2 <= FC_LDS && L_RED + 8 * 64 * 4 <= FC_LDS, "task images");

// ---- sync words (DmlcFcArgs::sync, uints, each counter on its own 128-B line) --------------------
DEV unsigned* cntA(const DmlcFcArgs& a, int m) { return a.sync + 32 * m; }          // m < 4
DEV unsigned* cntB(const DmlcFcArgs& a, int m) { return a.sync + 32 * (4 + m); }    // m < 4
DEV unsigned* cntBall(const DmlcFcArgs& a) { return a.sync + 32 * 8; }
// a.sync + 32 * 10 .. + 32 * 19: the two-level end-of-launch ticket (common.h last_arrival)

DEV unsigned ld_relaxed(unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// one lane: spin until *p >= target (bounded; on give-up the sticky error word is set)
DEV void wait_ge(unsigned* p, unsigned target, unsigned* err) {
  for (unsigned it = 0; ld_relaxed(p) < target; ++it) {
    if (it > (1u << 20)) {
      __hip_atomic_fetch_or(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
// every storing wave drains its write-through stores, the workgroup meets, one lane signals
DEV void publish(unsigned* c1, unsigned* c2) {
  wait_vm_all();
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(c1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (c2) __hip_atomic_fetch_add(c2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// one lane waits, then the workgroup meets (every later load of the handed-off bytes is sc1)
DEV void consume(unsigned* c, unsigned target, unsigned* err) {
  if (threadIdx.x == 0) wait_ge(c, target, err);
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
// Phase A: fc1 forward task t = (mt, nt, s): h1part[s][64 mt .. +64][64 nt .. +64] =
//   p2[rows][288 s .. +288] x W1[288 s .. +288][cols].  Waves 0-3 take k-steps 0..4, waves 4-7
//   k-steps 5..8 of the slice (2 x 2 waves x 32 x 32 each), summed in LDS; write-through stores.
// =================================================================================================
struct FwdRegs { uint4 a[5], b[5]; };
// always the same 10 loads (task-less blocks read valid dummy addresses): the waits that follow
// count them statically
DEV void fwd_issue(const DmlcFcArgs& a, int t, bool has, int parity, FwdRegs& R, int tid) {
  const int s = t % FC_S, nt = (t / FC_S) % 6, mt = t / (6 * FC_S);
  const bf16* W1 = W1S(a) + (parity ? 884736 : 0);
  const int k0 = s * FC_KS;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int c = tid + i * FT;               // A: 64 rows x 36 chunks; B: 288 k rows x 8 chunks
    const int ra = c / 36, ka = c - ra * 36;
    const int rowa = 64 * mt + ra;
    const bool oka = has && c < 64 * 36 && rowa < a.B;
    R.a[i] = load_sel(reinterpret_cast<const uint4*>(P2(a) + (size_t)rowa * 2304 + k0 + 8 * ka),
                      reinterpret_cast<const uint4*>(P2(a)), oka);
    const int kb = c >> 3, cb = c & 7;
    const bool okb = has && c < FC_KS * 8;
    R.b[i] = load_sel(reinterpret_cast<const uint4*>(W1 + (size_t)(k0 + kb) * 384 + 64 * nt + 8 * cb),
                      reinterpret_cast<const uint4*>(W1), okb);
  }
}
DEV void fwd_task(const DmlcFcArgs& a, int t, const FwdRegs& R, char* smem, int tid) {
  bf16* sa = reinterpret_cast<bf16*>(smem + L_FWD_A);
  bf16* sb = reinterpret_cast<bf16*>(smem + L_FWD_B);
  const int s = t % FC_S, nt = (t / FC_S) % 6, mt = t / (6 * FC_S);
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int c = tid + i * FT;
    if (c < 64 * 36) {
      const int ra = c / 36, ka = c - ra * 36;
      *reinterpret_cast<uint4*>(sa + ra * KST_A + 8 * ka) = R.a[i];
    }
    if (c < FC_KS * 8) *reinterpret_cast<uint4*>(sb + mz(c >> 3, 8 * (c & 7))) = R.b[i];
  }
  __syncthreads();
  const int w = wave_id(), lane = tid & 63, g = lane >> 4, li = lane & 15;
  const int h = w >> 2, wm = (w >> 1) & 1, wn = w & 1;
  Acc acc;
  acc.zero();
  const int kb = h ? 5 : 0, ke = h ? 9 : 5;
  for (int kk = kb; kk < ke; ++kk)
    acc.mma(kfrag(sa, KST_A, 32 * wm, kk, g, li), kfrag(sa, KST_A, 32 * wm + 16, kk, g, li),
            mfrag(sb, 32 * wn, kk, g, li), mfrag(sb, 32 * wn + 16, kk, g, li));
  __syncthreads();                             // operand images are dead: reuse the LDS
  float* ct = reinterpret_cast<float*>(smem);
  if (h == 1) acc.to_lds(ct, CT_LD, 32 * wm, 32 * wn, g, li);
  __syncthreads();
  if (h == 0) acc.add_lds(ct, CT_LD, 32 * wm, 32 * wn, g, li);   // fixed order: (k-steps 5..8) + (0..4)
  __syncthreads();
  const rsrc_t out = buf_rsrc(a.h1part);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = tid + u * FT, rr = e >> 4, cc = (e & 15) * 4;
    const int row = 64 * mt + rr;
    if (row < a.B) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(ct + rr * CT_LD + cc);
      st_sc1(out, (uint32_t)(((size_t)s * a.B + row) * 384 + 64 * nt + cc) * 4, v);
    }
  }
  publish(cntA(a, mt), nullptr);
}

// =================================================================================================
// Phase B: MLP head of rows r0 .. r0+3 (cnn_head.hip's math at 8 waves)
// =================================================================================================
DEV bf16x4 relu_mask4(const f32x4& acc, const bf16x4& h) {
  return pack4((float)h[0] > 0.f ? acc[0] : 0.f, (float)h[1] > 0.f ? acc[1] : 0.f,
               (float)h[2] > 0.f ? acc[2] : 0.f, (float)h[3] > 0.f ? acc[3] : 0.f);
}

DEV void head_task(const DmlcFcArgs& a, int hb, char* smem, int tid) {
  bf16* w2s = reinterpret_cast<bf16*>(smem + HL::W2);
  bf16* h1s = reinterpret_cast<bf16*>(smem + HL::H1);
  bf16* h2s = reinterpret_cast<bf16*>(smem + HL::H2);
  bf16* dh2s = reinterpret_cast<bf16*>(smem + HL::DH2);
  bf16* dls = reinterpret_cast<bf16*>(smem + HL::DL);
  const int lane = tid & 63, w = wave_id(), g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  constexpr int RB = FC_RB;
  const int r0 = hb * RB, mt = r0 >> 6;
  const bool rv = li < RB;
  const int rr = rv ? li : RB;
  DMLC_STAMP(DMLC_TK_HEAD, 0);
  DMLC_STAMP(DMLC_TK_CONV2_FWD, 0);

  // --- everything the seam does not gate, issued first: fc2 weights (18 x 16 B per thread), the
  //     small operands, the labels
  int label = 0;
  if (w == 7 && lane < RB) label = a.labels[batch_index(a.src, a.B, r0 + lane)];
  {
    constexpr int WCH = 192 * 48 / FT;
    uint4 wv[WCH];
#pragma unroll
    for (int i = 0; i < WCH; ++i) wv[i] = *(reinterpret_cast<const uint4*>(a.w2t) + tid + i * FT);
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int c = tid + i * FT, n2 = c / 48, k8 = c - n2 * 48;
      *reinterpret_cast<uint4*>(w2s + w2swz(n2, k8 * 8)) = wv[i];
    }
  }
  // fc2 output tiles: waves 0-3 tiles w and w + 8, waves 4-7 tile w
  float4 b2v[2];
  bf16x8 w3d[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int nt = w + 8 * j;
    const bool ok = nt < 12;
    b2v[j] = ok ? *reinterpret_cast<const float4*>(a.b2 + 16 * nt + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
    w3d[j] = ok ? glb_b128(reinterpret_cast<const bf16*>(a.w3d) + (16 * nt + li) * 32 + 8 * g) : bf16x8{};
  }
  bf16x8 w3f[6];
  float b3v[4] = {0.f, 0.f, 0.f, 0.f};
  if (w == 7) {
    const bf16* W = reinterpret_cast<const bf16*>(a.w3t) + li * 192 + 8 * g;
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) w3f[ks] = glb_b128(W + ks * 32);
#pragma unroll
    for (int i = 0; i < 4; ++i) b3v[i] = load_sel(a.b3 + 4 * g + i, a.b3, 4 * g + i < 10);
  }
  const bool act = tid < RB * 96;
  const int ec = act ? tid : 0, r = ec / 96, n = (ec - r * 96) * 4;
  const float4 b1v = *reinterpret_cast<const float4*>(a.b1 + n);
  // zero rows (row RB of every activation tile)
  if (tid < 96) *reinterpret_cast<bf16x4*>(h1s + RB * H1_LD + tid * 4) = pack4(0.f, 0.f, 0.f, 0.f);
  else if (tid < 144) *reinterpret_cast<bf16x4*>(h2s + RB * H2_LD + (tid - 96) * 4) = pack4(0.f, 0.f, 0.f, 0.f);
  else if (tid < 192) *reinterpret_cast<bf16x4*>(dh2s + RB * H2_LD + (tid - 144) * 4) = pack4(0.f, 0.f, 0.f, 0.f);
  else if (tid < 200) *reinterpret_cast<bf16x4*>(dls + RB * DL_LD + (tid - 192) * 4) = pack4(0.f, 0.f, 0.f, 0.f);
  else if (tid < 200 + 2 * RB)                 // dlogit columns 16..31 of the real rows (K pad)
    *reinterpret_cast<uint4*>(dls + ((tid - 200) >> 1) * DL_LD + 16 + 8 * ((tid - 200) & 1)) = make_uint4(0, 0, 0, 0);

  // --- seam 1: every fc1 forward task of this 64-row tile
  DMLC_STAMP(DMLC_TK_HEAD, 1);
  consume(cntA(a, mt), 6 * FC_S, a.err);
  DMLC_STAMP(DMLC_TK_HEAD, 2);
  {
    const rsrc_t part = buf_rsrc(a.h1part);
    float4 v[FC_S];
#pragma unroll
    for (int s = 0; s < FC_S; ++s)
      v[s] = ld_sc1(part, (uint32_t)(((size_t)s * a.B + r0 + r) * 384 + n) * 4);
    float4 acc = b1v;
#pragma unroll
    for (int s = 0; s < FC_S; ++s) { acc.x += v[s].x; acc.y += v[s].y; acc.z += v[s].z; acc.w += v[s].w; }
    if (act)
      *reinterpret_cast<bf16x4*>(h1s + r * H1_LD + n) =
          pack4(fmaxf(acc.x, 0.f), fmaxf(acc.y, 0.f), fmaxf(acc.z, 0.f), fmaxf(acc.w, 0.f));
  }
  lds_barrier();
  DMLC_STAMP(DMLC_TK_HEAD, 3);

  // (b) h2 = relu(h1 W2 + b2): C[n][r] = sum_k W2t[n][k] h1[r][k]
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int nt = w + 8 * j;
    if (nt >= 12) break;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 12; ++ks)
      acc = mfma16(lds_b128(w2s + w2swz(16 * nt + li, 8 * g + 32 * ks)), lds_b128(h1s + rr * H1_LD + ks * 32 + 8 * g), acc);
    const float4 bb = b2v[j];
    const bf16x4 o = pack4(fmaxf(acc[0] + bb.x, 0.f), fmaxf(acc[1] + bb.y, 0.f), fmaxf(acc[2] + bb.z, 0.f),
                           fmaxf(acc[3] + bb.w, 0.f));
    if (rv) *reinterpret_cast<bf16x4*>(h2s + li * H2_LD + 16 * nt + 4 * g) = o;
  }
  lds_barrier();

  DMLC_STAMP(DMLC_TK_CONV2_FWD, 1);            // (head-internal phase stamps: the conv2_fwd row)
  // (c)+(d) wave 7, in registers: logits = [relu](h2 W3 + b3) as one 16x16 tile (K = 192), lane
  //   (g, li) holding classes 4g..4g+3 of row li; the row max / argmax / exp-sum meet across the
  //   four lane groups by two xor shuffles -- softmax cross-entropy, accuracy and dlogits without an
  //   LDS round trip or a barrier in between (fixed shuffle order: deterministic)
  if (w == 7) {
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) acc = mfma16(w3f[ks], lds_b128(h2s + rr * H2_LD + ks * 32 + 8 * g), acc);
    float v[4];
    float m = -INFINITY;
    int am = 16;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = acc[i] + b3v[i];
      if (a.relu_logits) v[i] = fmaxf(v[i], 0.f);
      if (4 * g + i < 10 && v[i] > m) { m = v[i]; am = 4 * g + i; }   // first maximum within the lane
    }
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {       // larger value wins, ties go to the smaller class
      const float m2 = __shfl_xor(m, o);
      const int a2 = __shfl_xor(am, o);
      if (m2 > m || (m2 == m && a2 < am)) { m = m2; am = a2; }
    }
    float se = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) se += 4 * g + i < 10 ? __expf(v[i] - m) : 0.f;
    se += __shfl_xor(se, 16);
    se += __shfl_xor(se, 32);
    const float lse = m + __logf(se);
    const int lab = __shfl(label, li);          // wave 7 lane r < RB loaded row r's label
    const bool rowok = li < RB;
    const float vr = rowok && r0 + li < a.nvalid ? 1.f : 0.f;
    float loss = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) if (4 * g + i == lab) loss = vr * (lse - v[i]);
    const float corr = g == 0 ? vr * (am == lab ? 1.f : 0.f) : 0.f;
    if (rowok) {
      bf16x4 d4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 4 * g + i;
        float d = 0.f;
        if (c < 10) {
          d = (__expf(v[i] - lse) - (c == lab ? 1.f : 0.f)) * a.inv_batch * vr;
          if (a.relu_logits && !(v[i] > 0.f)) d = 0.f;
        }
        d4[i] = (bf16)d;
      }
      *reinterpret_cast<bf16x4*>(dls + li * DL_LD + 4 * g) = d4;
    }
    const float ls = wave_sum(rowok ? loss : 0.f), cs = wave_sum(corr);
    if (lane == 0) {
      a.loss_part[hb] = ls;
      a.correct_part[hb] = (int)(cs + 0.5f);
    }
  }
  lds_barrier();

  DMLC_STAMP(DMLC_TK_CONV2_FWD, 2);
  // (e) dh2 = (dl W3^T) * (h2 > 0), K = 32 (one MFMA)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int nt = w + 8 * j;
    if (nt >= 12) break;
    const f32x4 acc = mfma16(w3d[j], lds_b128(dls + rr * DL_LD + 8 * g), zero4());
    const int nn = 16 * nt + 4 * g;
    const bf16x4 o = relu_mask4(acc, *reinterpret_cast<const bf16x4*>(h2s + rr * H2_LD + nn));
    if (rv) *reinterpret_cast<bf16x4*>(dh2s + li * H2_LD + nn) = o;
  }
  lds_barrier();

  DMLC_STAMP(DMLC_TK_CONV2_FWD, 3);
  // (f) dh1 = (dh2 W2^T) * (h1 > 0): 24 k tiles, 3 per wave, K = 192 (transposed fc2 fragments);
  //     the rows go through LDS over the dead W2 image to the write-through stores below
  f32x4 dacc[3];
  bf16x4 hm[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int k0 = 16 * (w + 8 * j);
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) {
      const bf16x8 af = tr_frag(w2s + w2swz(32 * ks + 8 * g + q, k0 + 4 * p), w2s + w2swz(32 * ks + 8 * g + 4 + q, k0 + 4 * p));
      acc = mfma16(af, lds_b128(dh2s + rr * H2_LD + ks * 32 + 8 * g), acc);
    }
    dacc[j] = acc;
    hm[j] = *reinterpret_cast<const bf16x4*>(h1s + rr * H1_LD + k0 + 4 * g);
  }
  __syncthreads();                             // every fc2 fragment read: the W2 image is dead
  bf16* d1 = reinterpret_cast<bf16*>(smem + HL::W2);   // dh1 rows [RB][384] over the W2 image
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int k0 = 16 * (w + 8 * j);
    if (rv) *reinterpret_cast<bf16x4*>(d1 + li * 384 + k0 + 4 * g) = relu_mask4(dacc[j], hm[j]);
  }
  lds_barrier();
  DMLC_STAMP(DMLC_TK_HEAD, 4);

  // (g) hand-off rows, write-through: h1, h2, dh2, dl, dh1 (16-B pieces; per row 48 + 24 + 24 + 2 + 48)
  const rsrc_t rh1 = buf_rsrc(a.h1), rh2 = buf_rsrc(a.h2), rdh2 = buf_rsrc(a.dh2), rdl = buf_rsrc(a.dl),
               rdh1 = buf_rsrc(a.dh1);
  for (int c = tid; c < RB * 146; c += FT) {
    const int rw = c / 146, qq = c - rw * 146, b = r0 + rw;
    if (qq < 48) st16(rh1, (uint32_t)(b * 384 + 8 * qq) * 2, *reinterpret_cast<const uint4*>(h1s + rw * H1_LD + 8 * qq));
    else if (qq < 72) st16(rh2, (uint32_t)(b * 192 + 8 * (qq - 48)) * 2, *reinterpret_cast<const uint4*>(h2s + rw * H2_LD + 8 * (qq - 48)));
    else if (qq < 96) st16(rdh2, (uint32_t)(b * 192 + 8 * (qq - 72)) * 2, *reinterpret_cast<const uint4*>(dh2s + rw * H2_LD + 8 * (qq - 72)));
    else if (qq < 98) st16(rdl, (uint32_t)(b * 16 + 8 * (qq - 96)) * 2, *reinterpret_cast<const uint4*>(dls + rw * DL_LD + 8 * (qq - 96)));
    else st16(rdh1, (uint32_t)(b * 384 + 8 * (qq - 98)) * 2, *reinterpret_cast<const uint4*>(d1 + rw * 384 + 8 * (qq - 98)));
  }
  publish(cntB(a, mt), cntBall(a));
  DMLC_STAMP(DMLC_TK_HEAD, 5);
}

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
DEV int ctask_count(const DmlcFcArgs& a) { return a.mtiles * 18 + 108 + 9 + 2; }

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
#pragma unroll
  for (int u = 0; u < 4; ++u) {                // master tile [128][64] fp32 of dW1 (fused SGD)
    const int e = tid + u * FT, rr = e >> 4, cc = (e & 15) * 4;
    const bool ok = T.kind == 1 && a.fuse_sgd;
    R.m[u] = load_sel(reinterpret_cast<const float4*>(a.gw1 + (size_t)(128 * T.i + rr) * 384 + 64 * T.j + cc),
                      reinterpret_cast<const float4*>(a.gw1), ok);
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

DEV void dp2_task(const DmlcFcArgs& a, const CTask& T, char* smem, int tid) {
  bf16* sa = reinterpret_cast<bf16*>(smem + L_DP2_A);
  bf16* sb = reinterpret_cast<bf16*>(smem + L_DP2_B);
  const int mt = T.i, n0 = 128 * T.j;
  const int rows = min(64, a.B - 64 * mt);
  consume(cntB(a, mt), (unsigned)(rows / FC_RB), a.err);
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
#pragma unroll 4
  for (int kk = 0; kk < 12; ++kk)
    acc.mma(kfrag(sa, KST_A, 32 * wm, kk, g, li), kfrag(sa, KST_A, 32 * wm + 16, kk, g, li),
            kfrag(sb, KST_A, 32 * wn, kk, g, li), kfrag(sb, KST_A, 32 * wn + 16, kk, g, li));
  __syncthreads();
  DMLC_STAMP(DMLC_TK_GEMM, 4);
  float* ct = reinterpret_cast<float*>(smem);  // [64][132]
  constexpr int LD = 132;
  acc.to_lds(ct, LD, 32 * wm, 32 * wn, g, li);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {                // 64 x 128 bf16 = 2048 x 8-B pieces
    const int e = tid + u * FT, rr = e >> 5, cc = (e & 31) * 4;
    if (rr < rows) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(ct + rr * LD + cc);
      st_maybe_nt<kNtGemm>(reinterpret_cast<bf16x4*>(DP2(a) + (size_t)(64 * mt + rr) * 2304 + n0 + cc),
                           pack4(v[0], v[1], v[2], v[3]));
    }
  }
}

// dW1 / dW2 / dW3: 128 x 64 tile of A^T B over the batch (A, B: bf16 [B][lda], [B][ldb])
// One 16-B chunk per thread of a 64-row tile of an m-major hand-off operand: rows 64 m + (tid >> 3),
// columns c0 + 8 (tid & 7) of a bf16 [B][ld] matrix (sc1; rows >= B / columns >= ncol read as zero)
// a pointer the compiler cannot prove wave-uniform, made so (buffer descriptors live in SGPRs; a
// VGPR descriptor makes hipcc wrap every buffer op in a waterfall loop -- guide T20)
DEV const void* uni(const void* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<const void*>(((uint64_t)hi << 32) | lo);
}
DEV uint4 ld_mtile(const void* base, int ld, int c0, int ncol, int B, int m, int tid) {
  const int rw = 64 * m + (tid >> 3), col = c0 + 8 * (tid & 7);
  const bool ok = rw < B && col < ncol;
  const uint4 v = ld16(buf_rsrc(base), ok ? (uint32_t)(rw * ld + col) * 2 : 0u);
  return ok ? v : make_uint4(0, 0, 0, 0);
}
DEV void st_mtile(bf16* img, int m, const uint4& v, int tid) {
  *reinterpret_cast<uint4*>(img + mz(64 * m + (tid >> 3), 8 * (tid & 7))) = v;
}

DEV void dw_task(const DmlcFcArgs& a, const CTask& T, const PreRegs& R, int64_t step, char* smem, int tid) {
  bf16* sa = reinterpret_cast<bf16*>(smem + L_W1_A);
  bf16* sb = reinterpret_cast<bf16*>(smem + L_W1_B);
  const int Kpad = (a.B + 31) & ~31;
  const int m0 = 128 * T.i, n0 = 64 * T.j;
  // dW1 = p2^T dh1 (A staged before the seam), dW2 = h1^T dh2, dW3 = h2^T dl (10 columns)
  const int M = T.kind == 1 ? 2304 : T.kind == 2 ? 384 : 192;
  const int N = T.kind == 1 ? 384 : T.kind == 2 ? 192 : 10;
  const int ldc = N;
  // The K (= batch) range arrives one 64-row tile at a time: wait for that tile's head blocks only
  // (its own counter: the polls spread over mtiles words instead of all hitting the total) and
  // issue its operand loads before waiting for the next tile.  The barrier between is an s_barrier
  // (lds_barrier), not __syncthreads: that would drain the loads already in flight.
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
  // (written out per tile: with the spin inside, a loop over the tiles stayed rolled and its register
  // arrays went to scratch)
  struct T3 { uint4 a0, a1, b; };
  auto tile = [&](int m) __attribute__((always_inline)) {
    const bool on = m < a.mtiles;
    if (on && tid == 0) wait_ge(cntB(a, m), (unsigned)(min(64, a.B - 64 * m) / FC_RB), a.err);
    lds_barrier();
    const int Bm = on ? a.B : 0;            // a tile past the batch reads nothing (zeros)
    T3 r;
    r.b = ld_mtile(pb, ldb, cb, ldb, Bm, m, tid);
    r.a0 = ld_mtile(pa, lda, m0, need_a ? lda : 0, Bm, m, tid);
    r.a1 = ld_mtile(pa, lda, m0 + 64, need_a ? lda : 0, Bm, m, tid);
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
  DMLC_STAMP(DMLC_TK_GEMM, 3);
  put(0, t0); put(1, t1); put(2, t2); put(3, t3);
  __syncthreads();
  const int w = wave_id(), lane = tid & 63, g = lane >> 4, li = lane & 15;
  // bias gradient of the B columns (first M tile only): 8 row groups x 64 columns, fixed order
  float* red = reinterpret_cast<float*>(smem + L_RED);
  const bool bias = T.i == 0;
  if (bias) {
    const int col = tid & 63, rg = tid >> 6;
    float sum = 0.f;
    for (int rw = rg; rw < Kpad; rw += 8) sum += (float)sb[mz(rw, col)];
    red[rg * 64 + col] = sum;
  }
  Acc acc;
  acc.zero();
  mma_128x64(sa, sb, Kpad >> 5, acc, w, g, li);
  __syncthreads();
  DMLC_STAMP(DMLC_TK_GEMM, 4);
  if (bias && tid < 64 && n0 + tid < N) {
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) sum += red[k * 64 + tid];
    ((float*)(T.kind == 1 ? uni(a.gb1) : T.kind == 2 ? uni(a.gb2) : uni(a.gb3)))[n0 + tid] = sum;
  }
  float* ct = reinterpret_cast<float*>(smem);  // [128][68]
  acc.to_lds(ct, CT_LD, 32 * (w >> 1), 32 * (w & 1), g, li);
  __syncthreads();
  if (T.kind == 1 && a.fuse_sgd) {
    // fused SGD (single GPU): the complete dW1 tile; master update + the NEXT step's bf16 shadow
    // (the expression of cnn_gemm.hip's c_mode 4 and the SGD kernel: bit-identical weights)
    const float f = lr_sched(a.lr0, a.decay, a.decay_steps, a.staircase, a.warmup, step) * a.grad_scale;
    bf16* S = W1S(a) + ((step & 1) ? 0 : 884736);    // the shadow the NEXT step reads
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + u * FT, rr = e >> 4, cc = (e & 15) * 4;
      const size_t q = (size_t)(m0 + rr) * 384 + n0 + cc;
      const float4 gv = *reinterpret_cast<const float4*>(ct + rr * CT_LD + cc);
      float4 v = R.m[u];
      v.x -= f * gv.x; v.y -= f * gv.y; v.z -= f * gv.z; v.w -= f * gv.w;
      const f32x4 vo = {v.x, v.y, v.z, v.w};
      st_maybe_nt<kNtX>(reinterpret_cast<f32x4*>(a.gw1 + q), vo);
      st_maybe_nt<kNtX>(reinterpret_cast<bf16x4*>(S + q), pack4(v.x, v.y, v.z, v.w));
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = tid + u * FT, rr = e >> 4, cc = (e & 15) * 4;
    const int m = m0 + rr, n = n0 + cc;
    if (m >= M || n >= N) continue;
    const float4 v = *reinterpret_cast<const float4*>(ct + rr * CT_LD + cc);
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

DEV void c_task(const DmlcFcArgs& a, const CTask& T, const PreRegs& R, int64_t step, char* smem, int tid) {
  if (T.kind == 0) dp2_task(a, T, smem, tid);
  else dw_task(a, T, R, step, smem, tid);
}

__global__ __launch_bounds__(FT, 1) void k_fc_chain(DmlcFcArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, blk = blockIdx.x;
  const int H = a.B / FC_RB;
  const int64_t step = a.step ? *a.step : 0;   // fc1 shadow parity, LR of the fused SGD
  const int parity = (int)(step & 1);
  if (blk == 0 && tid == 0 && a.step_copy) *a.step_copy = step;
  const int nc = ctask_count(a);
  if (blk < H) {
    // head block: its rows, then (after every head) the C tasks past the GEMM blocks' share
    head_task(a, blk, smem, tid);
    const int G = FC_BLOCKS - H;
    for (int t = G + blk; t < nc; t += H) {
      __syncthreads();
      PreRegs R;
      const CTask T = ctask(a, t);
      pre_issue(a, T, parity, R, tid);
      pre_store(a, T, R, smem, tid);
      c_task(a, T, R, step, smem, tid);
    }
    DMLC_STAMP(DMLC_TK_HEAD, 6);
  } else {
    DMLC_STAMP(DMLC_TK_GEMM, 0);
    const int j = blk - H;
    const int na = a.mtiles * 6 * FC_S;
    const bool has_a = j < na;
    if (has_a) {
      FwdRegs F;
      fwd_issue(a, j, true, parity, F, tid);
      fwd_task(a, j, F, smem, tid);
    }
    DMLC_STAMP(DMLC_TK_GEMM, 1);
    // the backward task's seam-independent operands, issued only once the forward task has
    // published: its loads would otherwise share this CU's fabric rate with the forward's operands
    // (and the publish's vmcnt(0) would wait for them); the head's ~9 us covers their latency
    const CTask T = ctask(a, j);
    if (T.kind >= 0) {
      PreRegs R;
      pre_issue(a, T, parity, R, tid);
      __syncthreads();                         // the forward's LDS staging is dead
      pre_store(a, T, R, smem, tid);
      DMLC_STAMP(DMLC_TK_GEMM, 2);
      c_task(a, T, R, step, smem, tid);
      DMLC_STAMP(DMLC_TK_GEMM, 5);
    }
  }
  // the last block to finish re-arms the counters for the next launch (two-level ticket: one
  // counter taking 256 arrivals in a row serialises them at the memory side)
  __syncthreads();
  if (tid == 0) {
    wait_vm_all();
    if (last_arrival(a.sync + 32 * 10, blk, FC_BLOCKS)) {
      for (int m = 0; m < 4; ++m) {
        __hip_atomic_store(cntA(a, m), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(cntB(a, m), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __hip_atomic_store(cntBall(a), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (blk < H) DMLC_STAMP(DMLC_TK_HEAD, 7);
  else DMLC_STAMP(DMLC_TK_GEMM, 6);
}

}  // namespace dmlc

using namespace dmlc;

extern "C" hipError_t dmlc_fc_chain(const DmlcFcArgs* a, hipStream_t s) {
  if (a->B < 16 || a->B > 256 || a->B % 16 != 0 || a->mtiles != (a->B + 63) / 64 || !a->sync || !a->err)
    return hipErrorInvalidValue;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return hipErrorInvalidValue;
  }
  if (cus < FC_BLOCKS) return hipErrorInvalidValue;   // every block must be co-resident (one per CU)
  DMLC_LDS_OPTIN(&k_fc_chain, FC_LDS);
  hipLaunchKernelGGL(k_fc_chain, dim3(FC_BLOCKS), dim3(FT), FC_LDS, s, *a);
  return hipGetLastError();
}
