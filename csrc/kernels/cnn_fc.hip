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
// sc1 buffer load.  Counters (fc_common.h, each seam spread over several words that the consumer's
// lanes poll side by side): the fc1 partials (cntA), the head outputs (cntB) and the dp2 tiles (cntD);
// the last block to finish re-arms them (zero) for the next launch.
// Every spin is bounded and sets the sticky error word (the engine's wgrad barrier error word) --
// all 256 blocks must be co-resident (one per CU: ~150 KB of LDS each; host-checked).
#include <string.h>

#include "fc_common.h"
#include "conv2_core.h"
#include "split_common.h"

namespace dmlc {

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
constexpr int FC_LDS = L_DP2_END > HL::BYTES ? L_DP2_END : HL::BYTES;
static_assert(FC_LDS <= 160 * 1024, "fc chain LDS exceeds a CU");
constexpr int FC_LDS_ALL = FC_LDS > (int)DG_LDS ? FC_LDS : (int)DG_LDS;   // with the conv2 dgrad
static_assert(FT == NT && FC_LDS_ALL <= 160 * 1024, "the dgrad runs in the chain's workgroups");
static_assert(FT == SP_NT && SP_LDS <= (size_t)FC_LDS_ALL, "... and so does the split dgrad");
static_assert(L_FWD_B + FC_KS * 64 * 2 <= FC_LDS && L_RED + 8 * 64 * 4 <= FC_LDS, "task images");

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
  publish(cntA(a, mt, nt));
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
  consume(seamA(a, mt), a.err);
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
  publish(cntB(a, mt, hb & 3));
  DMLC_STAMP(DMLC_TK_HEAD, 5);
}


// Each block's second phase (backward tasks, ticket, conv2 dgrad) reads its arguments through
// late_kernarg (common.h), so the entry block loads only what the head / forward tasks need; the
// launch epoch's load is in flight through the first phase.
#ifdef DMLC_EAGER_ARGS                         // A/B build: every field loaded in the entry block
#define late_fc() a
#define late_dg() dg
#else
#define late_fc() late_kernarg<DmlcFcArgs>(0)
#define late_dg() late_kernarg<DmlcConv2DgradArgs>(kernarg_second<DmlcFcArgs, DmlcConv2DgradArgs>())
#endif
__global__ __launch_bounds__(FT, 1) void k_fc_chain(DmlcFcArgs a, DmlcConv2DgradArgs dg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, blk = blockIdx.x;
  const int H = a.B / FC_RB;
  const int64_t step = a.step ? *a.step : 0;   // fc1 shadow parity, LR of the fused SGD
  const int parity = (int)(step & 1);
  if (blk == 0 && tid == 0 && a.step_copy) *a.step_copy = step;
  __shared__ unsigned s_epoch;
  unsigned e0 = 0;
  if (tid == 0) e0 = ld_relaxed(epochW(a));   // (in hand before this block can arrive below)
  if (blk < H) {
    // head block: its rows, then (after every head) the C tasks past the GEMM blocks' share
    head_task(a, blk, smem, tid);
    if (tid == 0) s_epoch = e0;
    const DmlcFcArgs& L = late_fc();
    const int G = FC_BLOCKS - H, nc = ctask_count(L);
    for (int t = G + blk; t < nc; t += H) {
      __syncthreads();
      PreRegs R;
      const CTask T = ctask(L, t);
      pre_issue(L, T, parity, R, tid);
      pre_store(L, T, R, smem, tid);
      c_task(L, T, R, step, smem, tid, s_epoch);
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
    if (tid == 0) s_epoch = e0;
    DMLC_STAMP(DMLC_TK_GEMM, 1);
    // the backward task's seam-independent operands, issued only once the forward task has
    // published: its loads would otherwise share this CU's fabric rate with the forward's operands
    // (and the publish's vmcnt(0) would wait for them); the head's ~9 us covers their latency
    const DmlcFcArgs& L = late_fc();
    const CTask T = ctask(L, j);
    if (T.kind >= 0) {
      PreRegs R;
      pre_issue(L, T, parity, R, tid);
      __syncthreads();                         // the forward's LDS staging is dead
      pre_store(L, T, R, smem, tid);
      DMLC_STAMP(DMLC_TK_GEMM, 2);
      c_task(L, T, R, step, smem, tid, s_epoch);
      DMLC_STAMP(DMLC_TK_GEMM, 5);
    }
  }
  // the last block to finish its chain work re-arms the counters for the next launch (two-level
  // ticket: one counter taking 256 arrivals in a row serialises them at the memory side); the
  // dgrad's dp2 counters are the epoch's set, so the ticket need not wait for the dgrad
  __syncthreads();
  const unsigned epoch = s_epoch;
  const DmlcFcArgs& L = late_fc();
  if (tid == 0) {
    wait_vm_all();
    if (last_arrival(L.sync + 32 * 10, blk, FC_BLOCKS)) {
      for (int w = SY_A; w < SY_D; ++w)        // cntA, cntB
        __hip_atomic_store(L.sync + 32 * w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int k = 0; k < 72; ++k)             // the other dp2 set
        __hip_atomic_store(cntD(L, epoch + 1, 0, 0) + 32 * k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(epochW(L), epoch + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // the conv2 input gradient of image blk (dg.B = 0: a separate launch does it): its dp2 row tile
  // comes from this launch's dp2 tasks; everything else it reads was written by earlier launches
  const DmlcConv2DgradArgs& D = late_dg();
  if (D.split) {                               // B <= 128: image b's input-channel half h
    if (blk < 2 * D.B) {
      int b, h;
      split_index<2>(blk, b, h);
      conv2_dgrad_split_image<true>(D, b, h, smem, seamD(L, epoch, b >> 6), L.err);
    }
  } else if (blk < D.B) {
    conv2_dgrad_image<true>(D, blk, smem, seamD(L, epoch, blk >> 6), L.err);
  }
  if (blk < H) DMLC_STAMP(DMLC_TK_HEAD, 7);
  else DMLC_STAMP(DMLC_TK_GEMM, 6);
}

}  // namespace dmlc

using namespace dmlc;

extern "C" hipError_t dmlc_fc_chain(const DmlcFcArgs* a, const DmlcConv2DgradArgs* dg, hipStream_t s) {
  if (a->B < 16 || a->B > 256 || a->B % 16 != 0 || a->mtiles != (a->B + 63) / 64 || !a->sync || !a->err)
    return hipErrorInvalidValue;
  DmlcConv2DgradArgs d;
  memset(&d, 0, sizeof(d));
  if (dg) {
    // one image per workgroup of the 256: the batch rows are the chain's, dp2 its own output
    if (dg->B != a->B || dg->dp2 != a->dp2 || !dg->am2 || !dg->wd || !dg->dp1 || !dg->dy2) return hipErrorInvalidValue;
    if (dg->split && (2 * dg->B > FC_BLOCKS || dg->B % 8)) return hipErrorInvalidValue;
    d = *dg;
  }
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return hipErrorInvalidValue;
  }
  if (cus < FC_BLOCKS) return hipErrorInvalidValue;   // every block must be co-resident (one per CU)
  DMLC_LDS_OPTIN(&k_fc_chain, FC_LDS_ALL);
  hipLaunchKernelGGL(k_fc_chain, dim3(FC_BLOCKS), dim3(FT), d.B ? FC_LDS_ALL : FC_LDS, s, *a, d);
  return hipGetLastError();
}
