// MLP head of the CIFAR-10 CNN, one launch for forward AND backward of the small layers:
//   fc1 split-K reduction + bias + ReLU (prologue), fc2 + ReLU, fc3 (+ ReLU on the logits, D4),
//   sparse softmax cross-entropy + batch accuracy, then dlogits -> dh2 -> dh1 (with ReLU masks).
// Replaces /root/reference/cifar10cnn.py:130-176 (full1..full3, cifar_loss, batch_accuracy) and the
// corresponding autodiff ops (SURVEY.md §2.B N7/N8/N10-N12, §2.C xent10_fwd_bwd + linear_bwd_dx).
//
// Rows-parallel: RB (2 or 4) batch rows per workgroup of 16 waves; everything per row stays in LDS.
// What bounds this launch is the bytes every CU must pull in -- each workgroup needs ALL of fc2's
// 384 x 192 weights, at the ~11-15 B/clk a CU gets from the fabric -- not MFMA work.  So the fc2
// weight matrix is staged ONCE per workgroup into LDS (144 KB of the 160 KB) and read there in both
// orientations: row fragments (ds_read_b128) for h2 = h1 W2 and hardware-transposed fragments
// (ds_read_b64_tr_b16) for dh1 = dh2 W2^T -- half the bytes of fetching fc2 and its transpose.
// Every product is computed TRANSPOSED (C[feature][row]); the MFMA tiles keep 16 row columns and
// lanes of rows >= RB read a zero LDS row (their columns compute zeros and are never stored).
// Small operands (biases, fc3 fragments) are fetched at entry: a load issued inside a phase is an
// exposed memory latency on the serial chain.  Weight *gradients* of fc1/fc2/fc3 need a reduction
// over the whole batch: the grouped GEMM kernel does them.
#include "common.h"
#include "api.h"

namespace dmlc {

constexpr int HT = 1024;     // 16 waves
// fc2 weights in LDS, [192 n][384 k]: unpadded 768-B rows with the 16-B chunk index XORed by
// w2h(row) = 2 (row & 3) + 8 ((row >> 3) & 1).  Modelled with the gfx950 lane groups
// (tools/lds_banks.py): the ds_read_b128 row fragments (16 rows x one chunk per lane group) and the
// ds_read_b64_tr_b16 column fragments (rows {q, 8+q} x two chunks per half-wave) both hit 64
// distinct banks, and the staging stores stay conflict-free; 784-B padded rows were 2-way on both
// reads (8 / 4 LDS cycles instead of 4 / 2).
constexpr int W2_LD = 384;
constexpr int H1_LD = 392;   // 784-B rows: 16-B aligned, rows land on distinct bank slots
constexpr int H2_LD = 200;   // 400-B rows
constexpr int DL_LD = 40;    // 80-B rows (k padded to 32 with zeros)

DEV int w2swz(int row, int col) {
  return row * W2_LD + (((col >> 3) ^ (2 * (row & 3) + 8 * ((row >> 3) & 1))) << 3) + (col & 7);
}

template <int RB>
struct HeadLds {             // byte offsets into the dynamic LDS; RB real rows + one zero row
  static constexpr int W2 = 0;
  static constexpr int H1 = W2 + 192 * W2_LD * 2;
  static constexpr int H2 = H1 + (RB + 1) * H1_LD * 2;
  static constexpr int DH2 = H2 + (RB + 1) * H2_LD * 2;
  static constexpr int DL = DH2 + (RB + 1) * H2_LD * 2;
  static constexpr int LG = DL + (RB + 1) * DL_LD * 2;
  static constexpr int BYTES = LG + 16 * 17 * 4;
  static_assert(BYTES <= 160 * 1024, "head LDS exceeds the 160 KB of a CU");
};

DEV bf16x4 relu_mask4(const f32x4& acc, const bf16x4& h) {
  return pack4((float)h[0] > 0.f ? acc[0] : 0.f, (float)h[1] > 0.f ? acc[1] : 0.f,
               (float)h[2] > 0.f ? acc[2] : 0.f, (float)h[3] > 0.f ? acc[3] : 0.f);
}

template <int RB>
__global__ __launch_bounds__(HT, 1) void k_head(DmlcHeadArgs a) {
  if (a.step_copy && blockIdx.x == 0 && threadIdx.x == 0) *a.step_copy = *a.step;
  using L = HeadLds<RB>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* w2s = reinterpret_cast<bf16*>(smem + L::W2);
  bf16* h1s = reinterpret_cast<bf16*>(smem + L::H1);
  bf16* h2s = reinterpret_cast<bf16*>(smem + L::H2);
  bf16* dh2s = reinterpret_cast<bf16*>(smem + L::DH2);
  bf16* dls = reinterpret_cast<bf16*>(smem + L::DL);
  float (*lg)[17] = reinterpret_cast<float (*)[17]>(smem + L::LG);
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int r0 = blockIdx.x * RB;
  const bool rv = li < RB;                      // this lane's row column is a real batch row
  const int rr = rv ? li : RB;                  // LDS row it reads (RB = the zero row)
  DMLC_STAMP(DMLC_TK_HEAD, 0);

  // the loss wave's labels (counter -> index -> label chain) are fetched at entry
  int label = 0;
  if (w == 12 && lane < RB) label = a.labels[batch_index(a.src, a.B, r0 + lane)];

  // fc2 weights (a.w2t = [192 n][384 k]) -> LDS: 9216 chunks of 16 B, 9 per thread, all in flight
  constexpr int WCH = 192 * 48 / HT;
  uint4 wv[WCH];
#pragma unroll
  for (int i = 0; i < WCH; ++i) {
    const int c = tid + i * HT;
    wv[i] = *(reinterpret_cast<const uint4*>(a.w2t) + c);
  }
  // small operands of the later phases
  const float4 b2v = w < 12 ? *reinterpret_cast<const float4*>(a.b2 + 16 * w + 4 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
  bf16x8 w3f[6], w3d;
  float b3v[4] = {0.f, 0.f, 0.f, 0.f};
  if (w < 12 && a.train) w3d = glb_b128(reinterpret_cast<const bf16*>(a.w3d) + (16 * w + li) * 32 + 8 * g);
  if (w == 12) {
    const bf16* W = reinterpret_cast<const bf16*>(a.w3t) + li * 192 + 8 * g;
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) w3f[ks] = glb_b128(W + ks * 32);
#pragma unroll
    for (int i = 0; i < 4; ++i) b3v[i] = load_sel(a.b3 + 4 * g + i, a.b3, 4 * g + i < 10);
  }

  // (a) h1 = relu(sum_s part[s] + b1): RB x 96 float4, one per thread (threads < RB * 96)
  {
    const bool act = tid < RB * 96;
    const int ec = act ? tid : 0;                             // branch-free: clamp, discard later
    const int r = ec / 96, n = (ec - r * 96) * 4;
    float4 acc = *reinterpret_cast<const float4*>(a.b1 + n);
    const float* hp = a.h1part + (size_t)(r0 + r) * 384 + n;
    const size_t sstride = (size_t)a.B * 384;
    // up to 9 split-K partials (every fc1_split the engine picks) loaded at once, branch-free
    // (clamped to partial 0, zeroed after): one memory latency, not one per group of four
    constexpr int SP = 9;
    float4 v[SP];
#pragma unroll
    for (int k = 0; k < SP; ++k) v[k] = *reinterpret_cast<const float4*>(hp + (k < a.nsplit ? k : 0) * sstride);
#pragma unroll
    for (int k = 0; k < SP; ++k)
      if (k < a.nsplit) { acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w; }
    for (int sp = SP; sp < a.nsplit; ++sp) {
      const float4 v = *reinterpret_cast<const float4*>(hp + sp * sstride);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    // zero rows (row RB of every activation tile)
    if (tid < 96) *reinterpret_cast<bf16x4*>(h1s + RB * H1_LD + tid * 4) = pack4(0.f, 0.f, 0.f, 0.f);
    else if (tid < 144) *reinterpret_cast<bf16x4*>(h2s + RB * H2_LD + (tid - 96) * 4) = pack4(0.f, 0.f, 0.f, 0.f);
    else if (tid < 192) *reinterpret_cast<bf16x4*>(dh2s + RB * H2_LD + (tid - 144) * 4) = pack4(0.f, 0.f, 0.f, 0.f);
    else if (tid < 200) *reinterpret_cast<bf16x4*>(dls + RB * DL_LD + (tid - 192) * 4) = pack4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      const int c = tid + i * HT, n2 = c / 48, k8 = c - n2 * 48;
      *reinterpret_cast<uint4*>(w2s + w2swz(n2, k8 * 8)) = wv[i];
    }
    if (act) {
      const bf16x4 o = pack4(fmaxf(acc.x, 0.f), fmaxf(acc.y, 0.f), fmaxf(acc.z, 0.f), fmaxf(acc.w, 0.f));
      *reinterpret_cast<bf16x4*>(h1s + r * H1_LD + n) = o;
    }
  }
  lds_barrier();
  DMLC_STAMP(DMLC_TK_HEAD, 1);

  // (b) h2 = relu(h1 W2 + b2): C[n][r] = sum_k W2t[n][k] h1[r][k], waves 0..11 = n tiles
  if (w < 12) {
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 12; ++ks)
      acc = mfma16(lds_b128(w2s + w2swz(16 * w + li, 8 * g + 32 * ks)), lds_b128(h1s + rr * H1_LD + ks * 32 + 8 * g), acc);
    const int n = 16 * w + 4 * g;
    const bf16x4 o = pack4(fmaxf(acc[0] + b2v.x, 0.f), fmaxf(acc[1] + b2v.y, 0.f),
                           fmaxf(acc[2] + b2v.z, 0.f), fmaxf(acc[3] + b2v.w, 0.f));
    if (rv) *reinterpret_cast<bf16x4*>(h2s + li * H2_LD + n) = o;
  }
  lds_barrier();
  DMLC_STAMP(DMLC_TK_HEAD, 2);

  // (c) logits = [relu](h2 W3 + b3): wave 12, one 16x16 tile, K = 192
  if (w == 12) {
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) acc = mfma16(w3f[ks], lds_b128(h2s + rr * H2_LD + ks * 32 + 8 * g), acc);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = 4 * g + i;
      if (n < 10) {
        float v = acc[i] + b3v[i];
        if (a.relu_logits) v = fmaxf(v, 0.f);
        lg[li][n] = v;
      }
    }
  }
  lds_barrier();

  // (d) softmax cross-entropy, accuracy, dlogits (wave 12, lanes 0..RB-1 = rows)
  float loss_w = 0.f, corr_w = 0.f;
  if (w == 12) {
    float loss = 0.f, corr = 0.f;
    if (lane < RB) {
      const int b = r0 + lane;
      const float vr = b < a.nvalid ? 1.f : 0.f;     // padding rows (any-B tail): weight 0
      float m = lg[lane][0];
      int am = 0;
#pragma unroll
      for (int j = 1; j < 10; ++j) if (lg[lane][j] > m) { m = lg[lane][j]; am = j; }
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < 10; ++j) se += __expf(lg[lane][j] - m);
      const float lse = m + __logf(se);
      loss = vr * (lse - lg[lane][label]);
      corr = vr * (am == label ? 1.f : 0.f);
      if (a.logits_out) {
#pragma unroll
        for (int j = 0; j < 10; ++j) a.logits_out[b * 10 + j] = lg[lane][j];
      }
      if (a.train) {
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          float d = 0.f;
          if (j < 10) {
            d = (__expf(lg[lane][j] - lse) - (j == label ? 1.f : 0.f)) * a.inv_batch * vr;
            if (a.relu_logits && !(lg[lane][j] > 0.f)) d = 0.f;
          }
          dls[lane * DL_LD + j] = (bf16)d;
        }
      }
    }
    loss = wave_sum(loss);
    corr = wave_sum(corr);
    if (lane == 0 && !a.train) {                   // eval: nothing follows
      a.loss_part[blockIdx.x] = loss;
      a.correct_part[blockIdx.x] = (int)(corr + 0.5f);
    }
    loss_w = loss;
    corr_w = corr;
  }
  if (!a.train) return;
  lds_barrier();
  DMLC_STAMP(DMLC_TK_HEAD, 3);

  // (e) dh2 = (dl W3^T) * (h2 > 0): C[n][r] = sum_k W3d[n][k] dl[r][k], K = 32 (one step), waves 0..11
  if (w < 12) {
    const f32x4 acc = mfma16(w3d, lds_b128(dls + rr * DL_LD + 8 * g), zero4());
    const int n = 16 * w + 4 * g;
    const bf16x4 o = relu_mask4(acc, *reinterpret_cast<const bf16x4*>(h2s + rr * H2_LD + n));
    if (rv) *reinterpret_cast<bf16x4*>(dh2s + li * H2_LD + n) = o;
  }
  lds_barrier();
  DMLC_STAMP(DMLC_TK_HEAD, 4);

  // (f) dh1 = (dh2 W2^T) * (h1 > 0): C[k][r] = sum_n W2[k][n] dh2[r][n], k tiles w and w+16 (w < 8),
  // K = 192.  The A fragment (lane li: k = k0 + li, n = 32 ks + 8 g + j) is a column of the [n][k]
  // LDS image: two ds_read_b64_tr_b16 per fragment (wave-uniform control flow: EXEC all ones).
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j == 1 && w >= 8) break;
    const int k0 = 16 * (w + 16 * j);
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) {
      const bf16x8 af = tr_frag(w2s + w2swz(32 * ks + 8 * g + q, k0 + 4 * p), w2s + w2swz(32 * ks + 8 * g + 4 + q, k0 + 4 * p));
      acc = mfma16(af, lds_b128(dh2s + rr * H2_LD + ks * 32 + 8 * g), acc);
    }
    const int n = k0 + 4 * g;
    const bf16x4 o = relu_mask4(acc, *reinterpret_cast<const bf16x4*>(h1s + rr * H1_LD + n));
    if (rv) *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.dh1) + (size_t)(r0 + li) * 384 + n) = o;
  }
  // (g) the intermediates the fc weight-gradient GEMMs read (h1, h2, dl, dh2) and the loss partials
  // leave last, from LDS: vmcnt counts stores too, so a global store issued ahead of a load the wave
  // later waits for holds that wait until the store is acknowledged.
  if (w == 12 && lane == 0) {
    a.loss_part[blockIdx.x] = loss_w;
    a.correct_part[blockIdx.x] = (int)(corr_w + 0.5f);
  }
  for (int c = tid; c < RB * 98; c += HT) {       // per row: 48 + 24 + 24 + 2 chunks of 16 B
    const int r = c / 98, qq = c - r * 98;
    const bf16* src;
    bf16* dst;
    if (qq < 48) { src = h1s + r * H1_LD + 8 * qq; dst = reinterpret_cast<bf16*>(a.h1) + (size_t)(r0 + r) * 384 + 8 * qq; }
    else if (qq < 72) {
      src = h2s + r * H2_LD + 8 * (qq - 48); dst = reinterpret_cast<bf16*>(a.h2) + (size_t)(r0 + r) * 192 + 8 * (qq - 48);
    } else if (qq < 96) {
      src = dh2s + r * H2_LD + 8 * (qq - 72); dst = reinterpret_cast<bf16*>(a.dh2) + (size_t)(r0 + r) * 192 + 8 * (qq - 72);
    } else {
      src = dls + r * DL_LD + 8 * (qq - 96); dst = reinterpret_cast<bf16*>(a.dl) + (size_t)(r0 + r) * 16 + 8 * (qq - 96);
    }
    *reinterpret_cast<bf16x8*>(dst) = lds_b128(src);
  }
  DMLC_STAMP(DMLC_TK_HEAD, 5);
}

template <int RB>
hipError_t launch_head(const DmlcHeadArgs* a, hipStream_t s) {
  DMLC_LDS_OPTIN(&k_head<RB>, HeadLds<RB>::BYTES);
  hipLaunchKernelGGL(k_head<RB>, dim3(a->B / RB), dim3(HT), HeadLds<RB>::BYTES, s, *a);
  return hipGetLastError();
}

}  // namespace dmlc

using namespace dmlc;

extern "C" hipError_t dmlc_head(const DmlcHeadArgs* a, hipStream_t s) {
  switch (a->rows) {
    case 2: return launch_head<2>(a, s);
    case 4: return launch_head<4>(a, s);
    default: return hipErrorInvalidValue;
  }
}
