// Fused ResNet-20 training kernels for gfx950 (BASELINE.json config 4; SURVEY.md §2.C "Extra kernels
// not in the reference": conv3x3 fwd/dgrad/wgrad with stride 1/2, train-mode batch-norm, residual add,
// global average pool).  Model: models/resnet.py (the eager oracle).
//
// Design (MI355X-first):
//   * every 3x3 conv is an implicit GEMM on MFMA 16x16x32 bf16 over an LDS image of ONE zero-padded
//     input (one image per 256-thread block for fwd/dgrad), no im2col buffer; the K order is
//     (tap, channel) so each 8-wide B fragment is one 16-byte LDS read (CIN padded to 8 for the stem);
//   * train-mode BatchNorm never gets its own kernel: a layer's forward kernel writes z and adds
//     per-block channel sums / sums of squares into fp64 accumulators; the NEXT conv applies
//     scale/shift + ReLU (+ the option-A residual) while staging its input (and materialises a for
//     the backward); the backward mirrors it: each dgrad's epilogue produces g_y of the layer below
//     plus its two BN reductions (sum g_y, sum g_y*xhat), and the consumer rebuilds
//     g_z = gamma*rstd*(g_y - R1/N - xhat*R2/N) in its prologue;
//   * the statistics are exact fixed-point sums: every block splits each fp32 channel partial into an
//     integer part and a 48-bit fraction and adds both with 64-bit integer atomics into one of NSLOT
//     copies (slot = blockIdx & 7, i.e. one per XCD under round-robin dispatch) so 256 blocks do not
//     serialise on 64 addresses; integer addition is associative, so the totals -- and everything
//     downstream -- are bitwise reproducible (graph replay == eager launches) at the cost of fp64
//     atomics (r6: the ticketed per-slot-group flush this replaces cost 54 us per step); consumers fold
//     the slots once per block (64 threads) into LDS coefficient tables;
//   * stride-2 dgrad is a stride-1 correlation over a zero-inserted LDS image (pad 2/0);
//   * weight gradients: split-K over image groups x m-chunks, several images staged per barrier, both
//     operands read with ds_read_b64_tr_b16 from NHWC LDS images (per-lane row addresses absorb stride
//     and taps);
//   * the SGD kernel reduces the slabs in fixed order (per-layer split factor so every thread issues
//     <= 8 loads), updates BN running statistics, refreshes both bf16 weight shadows and bumps the
//     device step counter (graph-capturable).
#include "conv_common.h"
#include "api_resnet.h"

namespace dmlc {
namespace rn {

constexpr int RT = 256;
// streaming (nt) stores for the activations / gradients / slabs the next launches read (common.h:
// fewer dirty L2 lines to write back at every one of the ~58 kernel boundaries): 0.695 -> 0.682 ms
constexpr bool kNtRn = kNtDefault;
#ifdef DMLC_RN_SLAB_PLAIN   // A/B build, slabs stored plain: 640.4-641.5 vs 611.7-611.9 us (r6s3_rn_slab_plain_ab.txt)
constexpr bool kNtSlab = false;
#else
constexpr bool kNtSlab = kNtRn;
#endif
// activation stores (z, a, g_y -> the next launch): write-through (common.h st_out16 / st_out8) unless
// -DDMLC_RN_NT (the r3 streaming form); the fp32 slabs stay streaming (their 4-B write-through
// stores are one fabric write each: 375 vs 401 k images/s, r5 same-box A/B)
#ifdef DMLC_RN_NT
DEV void st_rn16(void* base, uint32_t off, const uint4& v) {
  st_maybe_nt<kNtRn>(reinterpret_cast<uint4*>(reinterpret_cast<char*>(base) + off), v);
}
DEV void st_rn8(void* base, uint32_t off, const bf16x4& v) {
  st_maybe_nt<kNtRn>(reinterpret_cast<bf16x4*>(reinterpret_cast<char*>(base) + off), v);
}
#else
DEV void st_rn16(void* base, uint32_t off, const uint4& v) { st_out16(base, off, v); }
DEV void st_rn8(void* base, uint32_t off, const bf16x4& v) { st_out8(base, off, __builtin_bit_cast(uint2, v)); }
#endif
constexpr int NSLOT = DMLC_RN_NSLOT;          // statistics copies per layer: [NSLOT][hi 128 | lo 128] int64
constexpr double BN_EPS = 1e-3;

__host__ __device__ constexpr int round32(int x) { return (x + 31) / 32 * 32; }

// Fixed-point BN statistics.  A slot holds, per statistic e (0..63 sum / R1, 64..127 sum of squares /
// R2), an int64 integer part at [e] and a uint64 fraction in units of 2^-48 at [128 + e].  One add
// splits x = floor(x) + f exactly (|x| < 2^50, so x - floor(x) and f * 2^48 are exact in fp64) and
// rounds f * 2^48 to an integer (error <= 2^-49 per add, far below the fp32 partial's own rounding).
// A non-finite or absurd partial adds the poison 2^56 to the integer part; legitimate slot totals stay
// below 2^55 in magnitude (<= 32 adds of < 2^50 each at B = 256), so the decoder turns any slot at or
// beyond 2^55 into NaN -- a diverged step still shows up as NaN downstream.
constexpr double FX_ONE = 281474976710656.0;             // 2^48
constexpr double FX_LIM = 1125899906842624.0;            // 2^50
constexpr long long FX_POISON = 1LL << 56;
constexpr long long FX_BAD = 1LL << 55;

DEV void fx_add(long long* slot, int e, float v) {
  const double x = (double)v;
  long long hi;
  unsigned long long lo;
  if (__builtin_fabs(x) < FX_LIM) {
    const double f = __builtin_floor(x);
    hi = (long long)f;
    lo = (unsigned long long)__builtin_rint((x - f) * FX_ONE);   // in [0, 2^48]
  } else {
    hi = FX_POISON;
    lo = 0;
  }
  atomicAdd(reinterpret_cast<unsigned long long*>(slot + e), (unsigned long long)hi);
  atomicAdd(reinterpret_cast<unsigned long long*>(slot + 128 + e), lo);
}

// total of statistic e over the NSLOT copies of one layer's slotted accumulator (all loads first)
DEV double fx_total(const long long* st, int e) {
  long long h[NSLOT];
  unsigned long long l[NSLOT];
#pragma unroll
  for (int k = 0; k < NSLOT; ++k) {
    h[k] = st[k * 256 + e];
    l[k] = (unsigned long long)st[k * 256 + 128 + e];
  }
  long long hs = 0;
  unsigned long long ls = 0;
  bool bad = false;
#pragma unroll
  for (int k = 0; k < NSLOT; ++k) {
    hs += h[k];
    ls += l[k];
    bad |= h[k] >= FX_BAD || h[k] <= -FX_BAD;
  }
  return bad ? __builtin_nan("") : (double)hs + (double)ls * (1.0 / FX_ONE);
}

// channel c of a slotted accumulator: (sum, sum of squares) or (R1, R2)
DEV void slot_sums(const long long* st, int c, double& s1, double& s2) {
  s1 = fx_total(st, c);
  s2 = fx_total(st, 64 + c);
}

// (no FMA contraction in the coefficient math: the backend's -ffp-contract=fast choices depend on
// the surrounding kernel, and every kernel that rebuilds these coefficients must get the same bits)
DEV void bn_mean_rstd(const long long* stat, int c, float inv_n, float& mean, float& rstd) {
#pragma clang fp contract(off)
  double s1, s2;
  slot_sums(stat, c, s1, s2);
  const double m = s1 * (double)inv_n;
  double var = s2 * (double)inv_n - m * m;
  var = var > 0.0 ? var : 0.0;
  mean = (float)m;
  rstd = (float)(1.0 / sqrt(var + BN_EPS));
}

// BN backward: g_z = A*g_y + Bc*z + Cc  with  A = gamma*rstd, Bc = -gamma*rstd^2*R2/N, Cc = -A*R1/N - Bc*mean
DEV void bnb_coeffs(const long long* stat, const long long* red, const float* gamma, int c, float inv_n, float& A,
                    float& Bc, float& Cc) {
#pragma clang fp contract(off)
  float mean, rstd;
  bn_mean_rstd(stat, c, inv_n, mean, rstd);
  double r1, r2;
  slot_sums(red, c, r1, r2);
  A = gamma[c] * rstd;
  Bc = -A * rstd * (float)(r2 * (double)inv_n);
  Cc = -A * (float)(r1 * (double)inv_n) - Bc * mean;
}

// g_z = A*g_y + Bc*z + Cc with the rounding pinned (two explicit FMAs): the dgrad, the wgrad and the
// per-image backward each rebuild g_z from the same bf16 inputs and must agree bit for bit
DEV float bnb_apply(float A, float Bc, float Cc, float gy, float z) {
  return __builtin_fmaf(A, gy, __builtin_fmaf(Bc, z, Cc));
}

DEV uint32_t pack2(float a, float b) {
  const bf16x4 v = pack4(a, b, 0.f, 0.f);
  return __builtin_bit_cast(uint2, v).x;
}

// block-level channel reduction of per-lane partials (lanes with equal li share a channel group), then
// one fixed-point add per statistic into this block's slot
template <int CT, int C>
DEV void reduce_flush(float (&s1)[4], float (&s2)[4], float* red, long long* dst, int w, int g, int li,
                      int tid) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) { s1[r] += __shfl_xor(s1[r], o); s2[r] += __shfl_xor(s2[r], o); }
  const int ct = w % CT;
  if (li == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[(w * 2 + 0) * 64 + 16 * ct + 4 * g + r] = s1[r];
      red[(w * 2 + 1) * 64 + 16 * ct + 4 * g + r] = s2[r];
    }
  }
  __syncthreads();
  float t1 = 0.f, t2 = 0.f;
  if (tid < C) {
#pragma unroll
    for (int ww = 0; ww < 4; ++ww)
      if (ww % CT == tid / 16) { t1 += red[(ww * 2) * 64 + tid]; t2 += red[(ww * 2 + 1) * 64 + tid]; }
  }
  if (tid < C) {
    long long* d = dst + (blockIdx.x & (NSLOT - 1)) * 256;
    fx_add(d, tid, t1);
    fx_add(d, 64 + tid, t2);
  }
}

// uint8 NHWC pixel (3 channels) -> 8 bf16 lanes (ci 3..7 zero)
DEV uint4 px_u8_to_bf16x8(uint32_t v) {
  return make_uint4(pack2((float)(v & 0xff), (float)((v >> 8) & 0xff)), pack2((float)((v >> 16) & 0xff), 0.f), 0u, 0u);
}
DEV uint32_t load_px_u8(const uint8_t* img, int cy, int cx, int iy, int ix, bool ok) {
  const uint8_t* s = img + (ok ? ((cy + iy) * 32 + cx + ix) * 3 : 0);
  const uint32_t v = (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16);
  return ok ? v : 0u;
}

// ================================ forward ======================================================
template <int CIN, int COUT, int HIN, int S>
struct Fwd {
  static constexpr int CINP = CIN < 8 ? 8 : CIN;
  static constexpr int HOUT = HIN / S;
  static constexpr int PADB = S == 1 ? 1 : 0;
  static constexpr int HP = HIN + (S == 1 ? 2 : 1);
  static constexpr int KP = round32(9 * CINP), KS = KP / 32;
  static constexpr int CT = COUT / 16, WPC = 4 / CT, NPXT = HOUT * HOUT / 16, NPT = NPXT / WPC;
  static constexpr int NCH = HP * HP * CINP / 8;               // 16-B chunks of the padded image
  static constexpr int IT = (NCH + RT - 1) / RT;
  static constexpr size_t XB = (size_t)HP * HP * CINP * 2;
  static constexpr size_t LDS = XB + 4 * 2 * 64 * 4 + 2 * 64 * 4;
};

template <int CIN, int COUT, int HIN, int S>
__global__ __launch_bounds__(RT) void k_rn_fwd(DmlcRnFwdArgs a) {
  using F = Fwd<CIN, COUT, HIN, S>;
  constexpr int CINP = F::CINP, HP = F::HP, HOUT = F::HOUT, KP = F::KP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xs = reinterpret_cast<bf16*>(smem);
  float* red = reinterpret_cast<float*>(smem + F::XB);          // [4][2][64]
  float* cf = red + 4 * 2 * 64;                                  // [2][64] BN scale / shift of layer l-1
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = wave_id(), g = lane >> 4, li = lane & 15;
  // timing build only (tools/rn_ktiming.py): phases of the stage-1 16->16 forward, kernel id 0
  constexpr bool TS = CIN == 16 && COUT == 16 && S == 1;
  if (TS) DMLC_STAMP(0, 0);
  // weight fragments first (independent of everything): their latency overlaps the prologue's
  const int ct = w % F::CT, pt0 = w / F::CT;
  const bf16* W = reinterpret_cast<const bf16*>(a.w) + (16 * ct + li) * KP + 8 * g;
  bf16x8 wa[F::KS];
#pragma unroll
  for (int ks = 0; ks < F::KS; ++ks) wa[ks] = glb_b128(W + 32 * ks);

  // ---- prologue: padded input image (stem: dataset gather; else BN-apply of layer l-1) ----
  if constexpr (CIN == 3) {
    const uint8_t* img = a.data + (size_t)batch_index(a.src, a.B, b) * 3072;
    uint32_t px3[F::IT];
#pragma unroll
    for (int i = 0; i < F::IT; ++i) {
      const int e = min(tid + i * RT, F::NCH - 1);
      const int iy = e / HP - F::PADB, ix = e % HP - F::PADB;
      px3[i] = load_px_u8(img, a.cy, a.cx, iy, ix, iy >= 0 && iy < HIN && ix >= 0 && ix < HIN);
    }
#pragma unroll
    for (int i = 0; i < F::IT; ++i) {
      const int e = tid + i * RT;
      if (e < F::NCH) reinterpret_cast<uint4*>(xs)[e] = px_u8_to_bf16x8(px3[i]);
    }
  } else {
    constexpr int C8 = CIN / 8;
    const int c8 = tid % C8;                  // fixed channel chunk of this thread (RT % C8 == 0)
    const uint4* zp = reinterpret_cast<const uint4*>(a.z_prev) + (size_t)b * HIN * HIN * C8;
    const uint4* ss = reinterpret_cast<const uint4*>(a.sc_src);
    uint4 zv[F::IT], sv[F::IT];
#pragma unroll
    for (int i = 0; i < F::IT; ++i) {
      const int e = min(tid + i * RT, F::NCH - 1);
      const int pp = e / C8, iy = pp / HP - F::PADB, ix = pp % HP - F::PADB;
      const bool ok = iy >= 0 && iy < HIN && ix >= 0 && ix < HIN;
      const int pin = ok ? iy * HIN + ix : 0;
      zv[i] = zp[pin * C8 + c8];
      sv[i] = make_uint4(0, 0, 0, 0);
      if (a.sc_mode == 1) sv[i] = ss[((size_t)b * HIN * HIN + pin) * C8 + c8];
      else if (a.sc_mode == 2) {               // option A: x[2y][2x][c] for c < CIN/2, zero above
        const bool lowc = c8 < C8 / 2;
        const size_t q = ((size_t)b * 4 * HIN * HIN + (ok ? (2 * iy) * (2 * HIN) + 2 * ix : 0)) * (C8 / 2) + (lowc ? c8 : 0);
        const uint4 v = ss[q];
        sv[i] = lowc ? v : make_uint4(0, 0, 0, 0);
      }
    }
    // BN_{l-1} coefficients, once per block: the statistics reads go out behind the image loads
    // (computed first, they added a dependent memory round trip to the prologue)
    if (tid < CIN) {
      float mean, rstd;
      bn_mean_rstd(a.stat_prev, tid, a.inv_n_prev, mean, rstd);
      const float sc = a.gamma_prev[tid] * rstd;
      cf[tid] = sc;
      cf[64 + tid] = a.beta_prev[tid] - mean * sc;
    }
    lds_barrier();
    float sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = cf[c8 * 8 + j]; sh[j] = cf[64 + c8 * 8 + j]; }
    uint4* ao = reinterpret_cast<uint4*>(a.a_out) + (size_t)b * HIN * HIN * C8;
#pragma unroll
    for (int i = 0; i < F::IT; ++i) {
      const int e = tid + i * RT;
      if (e < F::NCH) {
        const int pp = e / C8, iy = pp / HP - F::PADB, ix = pp % HP - F::PADB;
        const bool ok = iy >= 0 && iy < HIN && ix >= 0 && ix < HIN;
        const uint32_t zw[4] = {zv[i].x, zv[i].y, zv[i].z, zv[i].w};
        const uint32_t sw[4] = {sv[i].x, sv[i].y, sv[i].z, sv[i].w};
        uint32_t ow[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float y0 = fmaxf(bf16_lo(zw[k]) * sc[2 * k] + sh[2 * k] + bf16_lo(sw[k]), 0.f);
          const float y1 = fmaxf(bf16_hi(zw[k]) * sc[2 * k + 1] + sh[2 * k + 1] + bf16_hi(sw[k]), 0.f);
          ow[k] = ok ? pack2(y0, y1) : 0u;
        }
        const uint4 o = make_uint4(ow[0], ow[1], ow[2], ow[3]);
        reinterpret_cast<uint4*>(xs)[e] = o;
        if (ok) st_rn16(ao, (uint32_t)((iy * HIN + ix) * C8 + c8) * 16, o);
      }
    }
  }
  if (TS) DMLC_STAMP(0, 1);                       // 1: input image staged (BN-apply done)
  __syncthreads();
  if (TS) DMLC_STAMP(0, 2);                       // 2: weights in registers, barrier passed

  // ---- implicit GEMM: C[co][px] = sum_k W[co][k] X[px][k] ----
  f32x4 acc[F::NPT];
#pragma unroll
  for (int i = 0; i < F::NPT; ++i) acc[i] = zero4();
#pragma unroll
  for (int i = 0; i < F::NPT; ++i) {
    const int px = 16 * (pt0 + F::WPC * i) + li;
    const int oy = px / HOUT, ox = px - (px / HOUT) * HOUT;
    const int base = (oy * S) * HP + ox * S;
#pragma unroll
    for (int ks = 0; ks < F::KS; ++ks) {
      const int k0 = 32 * ks + 8 * g;
      const int tap = min(k0 / CINP, 8), ci0 = k0 % CINP;
      const int kh = tap / 3, kw = tap - 3 * (tap / 3);
      const bf16x8 bx = lds_b128(xs + (base + kh * HP + kw) * CINP + ci0);
      acc[i] = mfma16(wa[ks], bx, acc[i]);
    }
  }
  if (TS) DMLC_STAMP(0, 3);                       // 3: MFMAs issued
  // ---- epilogue: z (bf16) + BN partial sums ----
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  bf16* zo = reinterpret_cast<bf16*>(a.z) + (size_t)b * HOUT * HOUT * COUT;
#pragma unroll
  for (int i = 0; i < F::NPT; ++i) {
    const int px = 16 * (pt0 + F::WPC * i) + li;
    st_rn8(zo, (uint32_t)(px * COUT + 16 * ct + 4 * g) * 2, pack4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]));
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[r] += acc[i][r]; s2[r] += acc[i][r] * acc[i][r]; }
  }
  if (TS) DMLC_STAMP(0, 4);                       // 4: z stored, partial sums ready
  if (b >= a.nvalid) {                            // batch padding: not part of the BN statistics
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[r] = 0.f; s2[r] = 0.f; }
  }
  reduce_flush<F::CT, COUT>(s1, s2, red, a.stat, w, g, li, tid);
  if (TS) DMLC_STAMP(0, 5);                       // 5: statistics flushed (end)
}

// ================================ dgrad ========================================================
template <int CIN, int COUT, int HIN, int S>
struct Dg {
  static constexpr int HOUT = HIN / S;
  static constexpr int HPD = HIN + 2;
  static constexpr int KPD = round32(9 * COUT), KS = KPD / 32;
  static constexpr int CT = CIN / 16, WPC = 4 / CT, NPXT = HIN * HIN / 16, NPT = NPXT / WPC;
  static constexpr int NCH = HPD * HPD * COUT / 8;
  static constexpr int IT = (NCH + RT - 1) / RT;
  static constexpr size_t GB = (size_t)HPD * HPD * COUT * 2;
  static constexpr size_t LDS = GB + 4 * 2 * 64 * 4 + 5 * 64 * 4;
};

template <int CIN, int COUT, int HIN, int S>
DEV void rn_dgrad_body(const DmlcRnDgradArgs& a) {   // workgroup blockIdx.x = image (grid starts with these)
  using D = Dg<CIN, COUT, HIN, S>;
  constexpr int HOUT = D::HOUT, HPD = D::HPD, KPD = D::KPD, C8 = COUT / 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* gs = reinterpret_cast<bf16*>(smem);
  float* red = reinterpret_cast<float*>(smem + D::GB);           // [4][2][64]
  float* cf = red + 4 * 2 * 64;                                   // [5][64]: A, Bc, Cc (layer l); mean, rstd (l-1)
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = wave_id(), g = lane >> 4, li = lane & 15;
  constexpr bool TS = CIN == 16 && COUT == 16 && S == 1;   // timing build: stage-1 dgrad, kernel id 1
  if (TS) DMLC_STAMP(1, 0);

  if (tid < COUT) {
    float A, Bc, Cc;
    bnb_coeffs(a.stat, a.red, a.gamma, tid, a.inv_n, A, Bc, Cc);
    cf[tid] = A; cf[64 + tid] = Bc; cf[128 + tid] = Cc;
  } else if (tid >= 128 && tid < 128 + CIN) {
    float mean, rstd;
    bn_mean_rstd(a.stat_prev, tid - 128, a.inv_n_prev, mean, rstd);
    cf[192 + tid - 128] = mean; cf[256 + tid - 128] = rstd;
  }
  // ---- prologue: g_z of layer l on the (zero-inserted for S = 2) padded grid ----
  {
    const int c8 = tid % C8;
    const uint4* gyp = reinterpret_cast<const uint4*>(a.gy) + (size_t)b * HOUT * HOUT * C8;
    const uint4* zp = reinterpret_cast<const uint4*>(a.z) + (size_t)b * HOUT * HOUT * C8;
    uint4 gv[D::IT], zv[D::IT];
    bool okv[D::IT];
#pragma unroll
    for (int i = 0; i < D::IT; ++i) {
      const int e = min(tid + i * RT, D::NCH - 1);
      const int pp = e / C8, py = pp / HPD, px = pp % HPD;
      int oy, ox;
      bool ok;
      if (S == 1) { oy = py - 1; ox = px - 1; ok = oy >= 0 && oy < HOUT && ox >= 0 && ox < HOUT; }
      else {
        oy = (py - 2) >> 1; ox = (px - 2) >> 1;
        ok = py >= 2 && px >= 2 && !((py - 2) & 1) && !((px - 2) & 1) && oy < HOUT && ox < HOUT;
      }
      const int q = (ok ? oy * HOUT + ox : 0) * C8 + c8;
      gv[i] = gyp[q];
      zv[i] = zp[q];
      okv[i] = ok && (tid + i * RT) < D::NCH && b < a.nvalid;   // padding image: g_z = 0
    }
    lds_barrier();
    float A[8], Bc[8], Cc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { A[j] = cf[c8 * 8 + j]; Bc[j] = cf[64 + c8 * 8 + j]; Cc[j] = cf[128 + c8 * 8 + j]; }
#pragma unroll
    for (int i = 0; i < D::IT; ++i) {
      const int e = tid + i * RT;
      if (e < D::NCH) {
        const uint32_t gw[4] = {gv[i].x, gv[i].y, gv[i].z, gv[i].w}, zw[4] = {zv[i].x, zv[i].y, zv[i].z, zv[i].w};
        uint32_t ow[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float v0 = bnb_apply(A[2 * k], Bc[2 * k], Cc[2 * k], bf16_lo(gw[k]), bf16_lo(zw[k]));
          const float v1 = bnb_apply(A[2 * k + 1], Bc[2 * k + 1], Cc[2 * k + 1], bf16_hi(gw[k]), bf16_hi(zw[k]));
          ow[k] = okv[i] ? pack2(v0, v1) : 0u;
        }
        reinterpret_cast<uint4*>(gs)[e] = make_uint4(ow[0], ow[1], ow[2], ow[3]);
      }
    }
  }
  const int ct = w % D::CT, pt0 = w / D::CT;
  const bf16* Wd = reinterpret_cast<const bf16*>(a.wd) + (16 * ct + li) * KPD + 8 * g;
  bf16x8 wa[D::KS];
#pragma unroll
  for (int ks = 0; ks < D::KS; ++ks) wa[ks] = glb_b128(Wd + 32 * ks);
  __syncthreads();
  if (TS) DMLC_STAMP(1, 1);                       // 1: g_z staged, weights in registers

  // Epilogue operands of layer l-1 (activation for the ReLU mask, z for x-hat, the shortcut's g_y),
  // 4 pixel tiles per chunk, software-pipelined: chunk 0 is issued here, under the MFMAs, and chunk
  // c+1 before chunk c's stores.  (Loaded inside the store loop, every tile paid a full memory
  // latency -- the stores may alias the loads -- 11 of the kernel's 22 us at 16 tiles per wave.)
  struct EpiIn { uint2 a, z, s; };
  constexpr int EC = D::NPT < 4 ? D::NPT : 4;
  const int c0 = 16 * ct + 4 * g;
  const bf16* ap = reinterpret_cast<const bf16*>(a.a_prev) + (size_t)b * HIN * HIN * CIN;
  const bf16* zpp = reinterpret_cast<const bf16*>(a.z_prev) + (size_t)b * HIN * HIN * CIN;
  auto epi_load = [&](int i, EpiIn& e) {
    const int px = 16 * (pt0 + D::WPC * i) + li;
    const int iy = px / HIN, ix = px - (px / HIN) * HIN;
    e.a = *reinterpret_cast<const uint2*>(ap + px * CIN + c0);
    e.z = *reinterpret_cast<const uint2*>(zpp + px * CIN + c0);
    e.s = make_uint2(0u, 0u);
    if (a.sc_mode == 1) {
      e.s = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16*>(a.gy_sc) + ((size_t)b * HIN * HIN + px) * CIN + c0);
    } else if (a.sc_mode == 2) {
      const bool even = !(iy & 1) && !(ix & 1);
      const int HB = HIN / 2;
      const size_t q = ((size_t)b * HB * HB + (even ? (iy / 2) * HB + ix / 2 : 0)) * (2 * CIN) + c0;
      const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16*>(a.gy_sc) + q);
      e.s = even ? v : make_uint2(0u, 0u);
    }
  };
  EpiIn cur[EC];
#pragma unroll
  for (int j = 0; j < EC; ++j) epi_load(j, cur[j]);

  // ---- C[ci][px_in] = sum_{tap', co} Wd[ci][tap'*COUT + co] G[(iy+kh')*HPD + ix + kw'][co] ----
  f32x4 acc[D::NPT];
#pragma unroll
  for (int i = 0; i < D::NPT; ++i) acc[i] = zero4();
#pragma unroll
  for (int i = 0; i < D::NPT; ++i) {
    const int px = 16 * (pt0 + D::WPC * i) + li;
    const int iy = px / HIN, ix = px - (px / HIN) * HIN;
    const int base = iy * HPD + ix;
#pragma unroll
    for (int ks = 0; ks < D::KS; ++ks) {
      const int k0 = 32 * ks + 8 * g;
      const int tap = min(k0 / COUT, 8), co0 = k0 % COUT;
      const int kh = tap / 3, kw = tap - 3 * (tap / 3);
      const bf16x8 bx = lds_b128(gs + (base + kh * HPD + kw) * COUT + co0);
      acc[i] = mfma16(wa[ks], bx, acc[i]);
    }
  }

  if (TS) DMLC_STAMP(1, 2);                       // 2: MFMAs issued
  // ---- epilogue: g_a_{l-1} (+ shortcut) -> g_y_{l-1} + its BN reductions ----
  float mean[4], rstd[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { mean[r] = cf[192 + c0 + r]; rstd[r] = cf[256 + c0 + r]; }
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  bf16* gyo = reinterpret_cast<bf16*>(a.gy_prev) + (size_t)b * HIN * HIN * CIN;
#pragma unroll
  for (int c = 0; c < D::NPT; c += EC) {
    EpiIn nxt[EC];
    if (c + EC < D::NPT) {
#pragma unroll
      for (int j = 0; j < EC; ++j) epi_load(c + EC + j, nxt[j]);
    }
#pragma unroll
    for (int j = 0; j < EC; ++j) {
      const int i = c + j;
      const int px = 16 * (pt0 + D::WPC * i) + li;
      const uint2 av = cur[j].a, zv = cur[j].z, sv = cur[j].s;
      const float sc4[4] = {bf16_lo(sv.x), bf16_hi(sv.x), bf16_lo(sv.y), bf16_hi(sv.y)};
      const float av4[4] = {bf16_lo(av.x), bf16_hi(av.x), bf16_lo(av.y), bf16_hi(av.y)};
      const float zv4[4] = {bf16_lo(zv.x), bf16_hi(zv.x), bf16_lo(zv.y), bf16_hi(zv.y)};
      float gy[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gy[r] = av4[r] > 0.f ? acc[i][r] + sc4[r] : 0.f;
        s1[r] += gy[r];
        s2[r] = __builtin_fmaf(gy[r] * (zv4[r] - mean[r]), rstd[r], s2[r]);   // pinned (bitwise across kernels)
      }
      st_rn8(gyo, (uint32_t)(px * CIN + c0) * 2, pack4(gy[0], gy[1], gy[2], gy[3]));
    }
    if (c + EC < D::NPT) {
#pragma unroll
      for (int j = 0; j < EC; ++j) cur[j] = nxt[j];
    }
  }
  if (TS) DMLC_STAMP(1, 3);                       // 3: g_y stored, partial sums ready
  reduce_flush<D::CT, CIN>(s1, s2, red, a.red_prev, w, g, li, tid);
  if (TS) DMLC_STAMP(1, 4);                       // 4: reductions flushed (end)
}

// ================================ wgrad ========================================================
// Block (grp, mc): images [grp*B/G, (grp+1)*B/G), slab rows of m-tiles [mc*MCH, (mc+1)*MCH); NB images are
// staged per barrier (LDS budget ~120 KB) so their global loads are all in flight together.
template <int CIN, int COUT, int HIN, int S>
struct Wg {
  static constexpr int CINP = CIN < 8 ? 8 : CIN;
  static constexpr int HOUT = HIN / S;
  static constexpr int PADB = S == 1 ? 1 : 0;
  static constexpr int HP = HIN + (S == 1 ? 2 : 1);
  static constexpr int KP = round32(9 * CINP);
  static constexpr int MT = KP / 16;
  static constexpr int MC = MT <= 12 ? 1 : (MT <= 24 ? 2 : 3);           // m-chunks (grid.y)
  static constexpr int MCH = (MT + MC - 1) / MC;
  static constexpr int MJ = (MCH + 3) / 4;                               // m-tiles per wave
  static constexpr int NT = COUT / 16;
  static constexpr int NPIX = HOUT * HOUT, KSTEPS = NPIX / 32;
  static constexpr int GLD = COUT + 8;                                   // g_z LDS row stride (bf16)
  static constexpr int XE = HP * HP * CINP, GE = NPIX * GLD;            // bf16 elements per image
  static constexpr int XCH = XE / 8, GCH = NPIX * COUT / 8;             // 16-B chunks per image
  static constexpr int PER_IMG = (XE + GE) * 2;
  static constexpr int NB = (120 * 1024 / PER_IMG) < 1 ? 1 : ((120 * 1024 / PER_IMG) > 4 ? 4 : 120 * 1024 / PER_IMG);
  static constexpr int XIT = (NB * XCH + RT - 1) / RT, GIT = (NB * GCH + RT - 1) / RT;
  static constexpr size_t LDS = (size_t)NB * PER_IMG + 3 * 64 * 4;
};

template <int CIN, int COUT, int HIN, int S>
DEV void rn_wgrad_body(const DmlcRnWgradArgs& a, const int grp, const int mc) {
  using G = Wg<CIN, COUT, HIN, S>;
  constexpr int CINP = G::CINP, HP = G::HP, HOUT = G::HOUT, KP = G::KP, NT = G::NT, GLD = G::GLD, NB = G::NB;
  constexpr int C8 = COUT / 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xs = reinterpret_cast<bf16*>(smem);                       // [NB][XE]
  bf16* gz = xs + NB * G::XE;                                     // [NB][GE]
  float* cf = reinterpret_cast<float*>(gz + NB * G::GE);          // [3][64]
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int b0 = grp * a.B / a.G, b1 = (grp + 1) * a.B / a.G;
  constexpr bool TS = CIN == 16 && COUT == 16 && S == 1;   // timing build: stage-1 wgrad, kernel id 2
  if (TS) DMLC_STAMP(2, 0);

  if (tid < COUT) {
    float A, Bc, Cc;
    bnb_coeffs(a.stat, a.red, a.gamma, tid, a.inv_n, A, Bc, Cc);
    cf[tid] = A; cf[64 + tid] = Bc; cf[128 + tid] = Cc;
  }
  const int c8 = tid % C8;                                        // RT % (C8) == 0 and GCH % C8 == 0

  f32x4 acc[G::MJ][NT];
#pragma unroll
  for (int j = 0; j < G::MJ; ++j)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[j][n] = zero4();

  // stem: the dataset rows of the block's images, once per image (thread i -> image b0 + i), published
  // by the first loop barrier.  Evaluated per staged element, the generated-order index (a keyed
  // Feistel, ~150 instructions) ran XIT times per thread per image batch.
  [[maybe_unused]] int* srow = nullptr;
  if constexpr (CIN == 3) {
    __shared__ int srow_s[RT];
    srow = srow_s;
    if (b1 - b0 <= RT && tid < b1 - b0) srow_s[tid] = batch_index(a.src, a.B, b0 + tid);
  }
  for (int bb = b0; bb < b1; bb += NB) {
    const int nb = min(NB, b1 - bb);
    __syncthreads();
    // ---- x images (padded) ----
    if constexpr (CIN == 3) {
      uint32_t px3[G::XIT];
#pragma unroll
      for (int i = 0; i < G::XIT; ++i) {
        const int e = min(tid + i * RT, NB * G::XCH - 1);
        const int im = min(e / G::XCH, nb - 1), e1 = e - (e / G::XCH) * G::XCH;
        const int row = b1 - b0 <= RT ? srow[bb - b0 + im] : batch_index(a.src, a.B, bb + im);
        const uint8_t* img = a.data + (size_t)row * 3072;
        const int iy = e1 / HP - G::PADB, ix = e1 % HP - G::PADB;
        px3[i] = load_px_u8(img, a.cy, a.cx, iy, ix, iy >= 0 && iy < HIN && ix >= 0 && ix < HIN);
      }
#pragma unroll
      for (int i = 0; i < G::XIT; ++i) {
        const int e = tid + i * RT;
        if (e < NB * G::XCH) reinterpret_cast<uint4*>(xs)[e] = px_u8_to_bf16x8(px3[i]);
      }
    } else {
      constexpr int X8 = CIN / 8;
      uint4 xv[G::XIT];
#pragma unroll
      for (int i = 0; i < G::XIT; ++i) {
        const int e = min(tid + i * RT, NB * G::XCH - 1);
        const int im = min(e / G::XCH, nb - 1), e1 = e - (e / G::XCH) * G::XCH;
        const uint4* xp = reinterpret_cast<const uint4*>(a.x) + (size_t)(bb + im) * HIN * HIN * X8;
        const int pp = e1 / X8, iy = pp / HP - G::PADB, ix = pp % HP - G::PADB;
        const bool ok = iy >= 0 && iy < HIN && ix >= 0 && ix < HIN;
        xv[i] = load_sel(xp + (ok ? (iy * HIN + ix) * X8 + e1 % X8 : 0), xp, ok);
      }
#pragma unroll
      for (int i = 0; i < G::XIT; ++i) {
        const int e = tid + i * RT;
        if (e < NB * G::XCH) reinterpret_cast<uint4*>(xs)[e] = xv[i];
      }
    }
    // ---- g_z images [NB][NPIX][GLD] ----
    {
      uint4 gv[G::GIT], zv[G::GIT];
#pragma unroll
      for (int i = 0; i < G::GIT; ++i) {
        const int e = min(tid + i * RT, NB * G::GCH - 1);
        const int im = min(e / G::GCH, nb - 1), e1 = e - (e / G::GCH) * G::GCH;
        const size_t off = (size_t)(bb + im) * G::GCH + e1;
        gv[i] = reinterpret_cast<const uint4*>(a.gy)[off];
        zv[i] = reinterpret_cast<const uint4*>(a.z)[off];
      }
      float A[8], Bc[8], Cc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { A[j] = cf[c8 * 8 + j]; Bc[j] = cf[64 + c8 * 8 + j]; Cc[j] = cf[128 + c8 * 8 + j]; }
#pragma unroll
      for (int i = 0; i < G::GIT; ++i) {
        const int e = tid + i * RT;
        if (e < NB * G::GCH) {
          const int im = e / G::GCH, e1 = e - im * G::GCH;
          const uint32_t gw[4] = {gv[i].x, gv[i].y, gv[i].z, gv[i].w}, zw[4] = {zv[i].x, zv[i].y, zv[i].z, zv[i].w};
          const bool real = bb + im < a.nvalid;          // batch padding: g_z = 0
          uint32_t ow[4];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            ow[k] = real ? pack2(bnb_apply(A[2 * k], Bc[2 * k], Cc[2 * k], bf16_lo(gw[k]), bf16_lo(zw[k])),
                                 bnb_apply(A[2 * k + 1], Bc[2 * k + 1], Cc[2 * k + 1], bf16_hi(gw[k]), bf16_hi(zw[k])))
                         : 0u;
          *reinterpret_cast<uint4*>(gz + im * G::GE + (e1 / C8) * GLD + (e1 % C8) * 8) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
        }
      }
    }
    __syncthreads();
    if (TS && bb == b0) DMLC_STAMP(2, 1);         // 1: first staging step in LDS
    // ---- MFMA over the staged images' pixels ----
    // Software-pipelined: the next k-step's fragments (ds_read_b64_tr_b16) are read under this
    // k-step's MFMAs -- with the reads in line, every k-step waited one LDS latency (the phase took
    // 7 us for one 32x32x16 image, tools/rn_ktiming.py).  The wave's m-tiles are loop-invariant.
    int moff[G::MJ], mci[G::MJ];
    bool mok[G::MJ];
#pragma unroll
    for (int j = 0; j < G::MJ; ++j) {
      const int m = mc * G::MCH + w + 4 * j;
      mok[j] = w + 4 * j < G::MCH && m < G::MT;          // wave-uniform
      int tap, ci0;
      if (CINP >= 16) { tap = (16 * m) / CINP; ci0 = (16 * m) % CINP + 4 * p; }
      else { tap = 2 * m + (p >> 1); ci0 = 4 * (p & 1); }
      tap = min(tap, 8);
      const int kh = tap / 3, kw = tap - 3 * (tap / 3);
      moff[j] = kh * HP + kw;
      mci[j] = ci0;
    }
    for (int im = 0; im < nb; ++im) {
      const bf16* xi = xs + im * G::XE;
      const bf16* gi = gz + im * G::GE;
      auto frags = [&](int s, bf16x8 (&bf)[NT], bf16x8 (&af)[G::MJ]) {
        const int rA = 32 * s + 8 * g + q, rB = rA + 4;
#pragma unroll
        for (int n = 0; n < NT; ++n) bf[n] = tr_frag(gi + rA * GLD + 16 * n + 4 * p, gi + rB * GLD + 16 * n + 4 * p);
        const int oyA = rA / HOUT, oxA = rA - oyA * HOUT, oyB = rB / HOUT, oxB = rB - oyB * HOUT;
        const int pA = (oyA * S) * HP + oxA * S, pB = (oyB * S) * HP + oxB * S;
#pragma unroll
        for (int j = 0; j < G::MJ; ++j)
          if (mok[j]) af[j] = tr_frag(xi + (pA + moff[j]) * CINP + mci[j], xi + (pB + moff[j]) * CINP + mci[j]);
      };
      bf16x8 bf[NT], af[G::MJ];
      frags(0, bf, af);
      for (int s = 0; s < G::KSTEPS; ++s) {
        bf16x8 bn[NT], an[G::MJ];
        wait_lds();                                  // step s's fragments have landed
        __builtin_amdgcn_sched_barrier(0);
        if (s + 1 < G::KSTEPS) frags(s + 1, bn, an);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < G::MJ; ++j)
          if (mok[j]) {
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[j][n] = mfma16(af[j], bf[n], acc[j][n]);
          }
#pragma unroll
        for (int n = 0; n < NT; ++n) bf[n] = bn[n];
#pragma unroll
        for (int j = 0; j < G::MJ; ++j) af[j] = an[j];
      }
    }
  }
  if (TS) DMLC_STAMP(2, 2);                       // 2: all MFMAs issued
  // slab rows k = 16m + 4g + i, cols co = 16n + li
  float* out = a.part + (size_t)grp * KP * COUT;
#pragma unroll
  for (int j = 0; j < G::MJ; ++j) {
    const int m = mc * G::MCH + w + 4 * j;
    if (w + 4 * j < G::MCH && m < G::MT) {
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) st_maybe_nt<kNtSlab>(out + (16 * m + 4 * g + i) * COUT + 16 * n + li, acc[j][n][i]);
    }
  }
  if (TS) DMLC_STAMP(2, 3);                       // 3: slab written (end)
}

template <int CIN, int COUT, int HIN, int S>
__global__ __launch_bounds__(RT) void k_rn_dgrad(DmlcRnDgradArgs a) { rn_dgrad_body<CIN, COUT, HIN, S>(a); }

template <int CIN, int COUT, int HIN, int S>
__global__ __launch_bounds__(RT) void k_rn_wgrad(DmlcRnWgradArgs a) {
  rn_wgrad_body<CIN, COUT, HIN, S>(a, blockIdx.x, blockIdx.y);
}

// Layer l's input gradient AND weight gradient in ONE launch (both only read what layer l+1's dgrad
// produced): workgroups [0, B) run the dgrad body (one image each, the same blockIdx as its own
// launch, so the BN-reduction slots are unchanged), the rest the wgrad body (group, m-chunk).  One
// launch per layer instead of two, with no stream fork/join in the step graph.
template <int CIN, int COUT, int HIN, int S>
__global__ __launch_bounds__(RT, 2) void k_rn_bwd(DmlcRnDgradArgs d, DmlcRnWgradArgs w) {
  if ((int)blockIdx.x < d.B) {
    rn_dgrad_body<CIN, COUT, HIN, S>(d);
  } else {
    const int t = (int)blockIdx.x - d.B;
    rn_wgrad_body<CIN, COUT, HIN, S>(w, t % w.G, t / w.G);
  }
}

// ============================ per-image backward (stride 1, one slab per image) ====================
// Layer l's input gradient AND its weight gradient from ONE workgroup per image: the g_z image the
// dgrad stages (padded, [HPD][HPD][COUT]) is also the weight gradient's B operand, and the layer
// input a_{l-1} is staged once into LDS (padded) for both the dgrad epilogue's ReLU mask and the
// weight gradient's A operand -- the separate wgrad blocks re-read g_y, z and a_{l-1} from memory
// (96 KB per 32x32x16 image).  Needs one split-K group per image (w.G == B, the 16-channel layers'
// choice at B <= 256): the slab of image b is part[b].  Same per-image sums in the same k-step
// order as the grouped wgrad body: the step is bitwise the merged launch's.
template <int CIN, int COUT, int HIN>
struct BwdImg {
  using D = Dg<CIN, COUT, HIN, 1>;
  static constexpr int HP = HIN + 2, CINP = CIN;
  static constexpr int XCH = HP * HP * CIN / 8, XIT = (XCH + RT - 1) / RT;
  static constexpr size_t XB = (size_t)HP * HP * CIN * 2;
  static constexpr int KP = round32(9 * CIN), MT = KP / 16, MJ = (MT + 3) / 4, NT = COUT / 16;
  static constexpr int NPIX = HIN * HIN, KSTEPS = NPIX / 32;
  static constexpr size_t LDS = D::GB + XB + 4 * 2 * 64 * 4 + 5 * 64 * 4;
  static_assert(CIN == COUT && CIN % 16 == 0 && NPIX % 32 == 0, "per-image backward: square stride-1 layers");
};

template <int CIN, int COUT, int HIN>
__global__ __launch_bounds__(RT, 2) void k_rn_bwd_img(DmlcRnDgradArgs a, DmlcRnWgradArgs wa_) {
  using D = Dg<CIN, COUT, HIN, 1>;
  using I = BwdImg<CIN, COUT, HIN>;
  constexpr int HPD = D::HPD, KPD = D::KPD, C8 = COUT / 8, HP = I::HP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* gs = reinterpret_cast<bf16*>(smem);
  bf16* xs = reinterpret_cast<bf16*>(smem + D::GB);
  float* red = reinterpret_cast<float*>(smem + D::GB + I::XB);   // [4][2][64]
  float* cf = red + 4 * 2 * 64;                                  // [5][64]
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = wave_id(), g = lane >> 4, li = lane & 15;
  const int q = li >> 2, p = li & 3;

  if (tid < COUT) {
    float A, Bc, Cc;
    bnb_coeffs(a.stat, a.red, a.gamma, tid, a.inv_n, A, Bc, Cc);
    cf[tid] = A; cf[64 + tid] = Bc; cf[128 + tid] = Cc;
  } else if (tid >= 128 && tid < 128 + CIN) {
    float mean, rstd;
    bn_mean_rstd(a.stat_prev, tid - 128, a.inv_n_prev, mean, rstd);
    cf[192 + tid - 128] = mean; cf[256 + tid - 128] = rstd;
  }
  // ---- prologue: g_z of layer l on the padded grid (as rn_dgrad_body, stride 1) ----
  {
    const int c8 = tid % C8;
    const uint4* gyp = reinterpret_cast<const uint4*>(a.gy) + (size_t)b * HIN * HIN * C8;
    const uint4* zp = reinterpret_cast<const uint4*>(a.z) + (size_t)b * HIN * HIN * C8;
    uint4 gv[D::IT], zv[D::IT];
    bool okv[D::IT];
#pragma unroll
    for (int i = 0; i < D::IT; ++i) {
      const int e = min(tid + i * RT, D::NCH - 1);
      const int pp = e / C8, py = pp / HPD, px = pp % HPD;
      const int oy = py - 1, ox = px - 1;
      const bool ok = oy >= 0 && oy < HIN && ox >= 0 && ox < HIN;
      const int qq = (ok ? oy * HIN + ox : 0) * C8 + c8;
      gv[i] = gyp[qq];
      zv[i] = zp[qq];
      okv[i] = ok && (tid + i * RT) < D::NCH && b < a.nvalid;   // padding image: g_z = 0
    }
    lds_barrier();
    float A[8], Bc[8], Cc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { A[j] = cf[c8 * 8 + j]; Bc[j] = cf[64 + c8 * 8 + j]; Cc[j] = cf[128 + c8 * 8 + j]; }
#pragma unroll
    for (int i = 0; i < D::IT; ++i) {
      const int e = tid + i * RT;
      if (e < D::NCH) {
        const uint32_t gw[4] = {gv[i].x, gv[i].y, gv[i].z, gv[i].w}, zw[4] = {zv[i].x, zv[i].y, zv[i].z, zv[i].w};
        uint32_t ow[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float v0 = bnb_apply(A[2 * k], Bc[2 * k], Cc[2 * k], bf16_lo(gw[k]), bf16_lo(zw[k]));
          const float v1 = bnb_apply(A[2 * k + 1], Bc[2 * k + 1], Cc[2 * k + 1], bf16_hi(gw[k]), bf16_hi(zw[k]));
          ow[k] = okv[i] ? pack2(v0, v1) : 0u;
        }
        reinterpret_cast<uint4*>(gs)[e] = make_uint4(ow[0], ow[1], ow[2], ow[3]);
      }
    }
  }
  // the layer input a_{l-1} (padded, halo 0): its loads fly during the dgrad MFMAs
  uint4 xv[I::XIT];
  {
    constexpr int X8 = CIN / 8;
    const uint4* xp = reinterpret_cast<const uint4*>(a.a_prev) + (size_t)b * HIN * HIN * X8;
#pragma unroll
    for (int i = 0; i < I::XIT; ++i) {
      const int e = min(tid + i * RT, I::XCH - 1);
      const int pp = e / X8, iy = pp / HP - 1, ix = pp % HP - 1;
      const bool ok = iy >= 0 && iy < HIN && ix >= 0 && ix < HIN;
      xv[i] = load_sel(xp + (ok ? (iy * HIN + ix) * X8 + e % X8 : 0), xp, ok);
    }
  }
  const int ct = w % D::CT, pt0 = w / D::CT;
  const bf16* Wd = reinterpret_cast<const bf16*>(a.wd) + (16 * ct + li) * KPD + 8 * g;
  bf16x8 wdf[D::KS];
#pragma unroll
  for (int ks = 0; ks < D::KS; ++ks) wdf[ks] = glb_b128(Wd + 32 * ks);
  __syncthreads();

  // ---- dgrad MFMAs (as rn_dgrad_body) ----
  f32x4 acc[D::NPT];
#pragma unroll
  for (int i = 0; i < D::NPT; ++i) acc[i] = zero4();
#pragma unroll
  for (int i = 0; i < D::NPT; ++i) {
    const int px = 16 * (pt0 + D::WPC * i) + li;
    const int iy = px / HIN, ix = px - (px / HIN) * HIN;
    const int base = iy * HPD + ix;
#pragma unroll
    for (int ks = 0; ks < D::KS; ++ks) {
      const int k0 = 32 * ks + 8 * g;
      const int tap = min(k0 / COUT, 8), co0 = k0 % COUT;
      const int kh = tap / 3, kw = tap - 3 * (tap / 3);
      const bf16x8 bx = lds_b128(gs + (base + kh * HPD + kw) * COUT + co0);
      acc[i] = mfma16(wdf[ks], bx, acc[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < I::XIT; ++i) {
    const int e = tid + i * RT;
    if (e < I::XCH) reinterpret_cast<uint4*>(xs)[e] = xv[i];
  }
  __syncthreads();                                // xs complete (the epilogue's mask reads it)

  // ---- dgrad epilogue: g_a_{l-1} (+ shortcut) -> g_y_{l-1} + its BN reductions ----
  struct EpiIn { uint2 z, s; };
  constexpr int EC = D::NPT < 4 ? D::NPT : 4;
  const int c0 = 16 * ct + 4 * g;
  const bf16* zpp = reinterpret_cast<const bf16*>(a.z_prev) + (size_t)b * HIN * HIN * CIN;
  auto epi_load = [&](int i, EpiIn& e) {
    const int px = 16 * (pt0 + D::WPC * i) + li;
    const int iy = px / HIN, ix = px - (px / HIN) * HIN;
    e.z = *reinterpret_cast<const uint2*>(zpp + px * CIN + c0);
    e.s = make_uint2(0u, 0u);
    if (a.sc_mode == 1) {
      e.s = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16*>(a.gy_sc) + ((size_t)b * HIN * HIN + px) * CIN + c0);
    } else if (a.sc_mode == 2) {
      const bool even = !(iy & 1) && !(ix & 1);
      const int HB = HIN / 2;
      const size_t qq = ((size_t)b * HB * HB + (even ? (iy / 2) * HB + ix / 2 : 0)) * (2 * CIN) + c0;
      const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16*>(a.gy_sc) + qq);
      e.s = even ? v : make_uint2(0u, 0u);
    }
  };
  EpiIn cur[EC];
#pragma unroll
  for (int j = 0; j < EC; ++j) epi_load(j, cur[j]);
  float mean[4], rstd[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { mean[r] = cf[192 + c0 + r]; rstd[r] = cf[256 + c0 + r]; }
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  bf16* gyo = reinterpret_cast<bf16*>(a.gy_prev) + (size_t)b * HIN * HIN * CIN;
#pragma unroll
  for (int c = 0; c < D::NPT; c += EC) {
    EpiIn nxt[EC];
    if (c + EC < D::NPT) {
#pragma unroll
      for (int j = 0; j < EC; ++j) epi_load(c + EC + j, nxt[j]);
    }
#pragma unroll
    for (int j = 0; j < EC; ++j) {
      const int i = c + j;
      const int px = 16 * (pt0 + D::WPC * i) + li;
      const int iy = px / HIN, ix = px - (px / HIN) * HIN;
      const uint2 av = *reinterpret_cast<const uint2*>(xs + ((iy + 1) * HP + ix + 1) * CIN + c0);
      const uint2 zv = cur[j].z, sv = cur[j].s;
      const float sc4[4] = {bf16_lo(sv.x), bf16_hi(sv.x), bf16_lo(sv.y), bf16_hi(sv.y)};
      const float av4[4] = {bf16_lo(av.x), bf16_hi(av.x), bf16_lo(av.y), bf16_hi(av.y)};
      const float zv4[4] = {bf16_lo(zv.x), bf16_hi(zv.x), bf16_lo(zv.y), bf16_hi(zv.y)};
      float gy[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gy[r] = av4[r] > 0.f ? acc[i][r] + sc4[r] : 0.f;
        s1[r] += gy[r];
        s2[r] = __builtin_fmaf(gy[r] * (zv4[r] - mean[r]), rstd[r], s2[r]);   // pinned (bitwise across kernels)
      }
      st_rn8(gyo, (uint32_t)(px * CIN + c0) * 2, pack4(gy[0], gy[1], gy[2], gy[3]));
    }
    if (c + EC < D::NPT) {
#pragma unroll
      for (int j = 0; j < EC; ++j) cur[j] = nxt[j];
    }
  }
  reduce_flush<D::CT, CIN>(s1, s2, red, a.red_prev, w, g, li, tid);

  // ---- weight gradient of this image: C[k = (tap, ci)][co] = sum_px X[px + tap][ci] g_z[px][co] ----
  // m-tile m: k = 16m .. 16m+15 = tap (16m) / CIN, channels (16m) % CIN .. +15 (taps past 8: K padding)
  int moff[I::MJ], mci[I::MJ];
  bool mok[I::MJ];
#pragma unroll
  for (int j = 0; j < I::MJ; ++j) {
    const int m = w + 4 * j;
    mok[j] = m < I::MT;                             // wave-uniform
    const int tap = min((16 * m) / CIN, 8);
    moff[j] = (tap / 3) * HP + tap % 3;
    mci[j] = (16 * m) % CIN + 4 * p;
  }
  auto prow = [&](int r) { return ((r / HIN) + 1) * HPD + (r % HIN) + 1; };   // padded g_z row of pixel r
  auto frags = [&](int s_, bf16x8 (&bf)[I::NT], bf16x8 (&af)[I::MJ]) {
    const int rA = 32 * s_ + 8 * g + q, rB = rA + 4;
#pragma unroll
    for (int n = 0; n < I::NT; ++n)
      bf[n] = tr_frag(gs + prow(rA) * COUT + 16 * n + 4 * p, gs + prow(rB) * COUT + 16 * n + 4 * p);
    const int pA = (rA / HIN) * HP + rA % HIN, pB = (rB / HIN) * HP + rB % HIN;
#pragma unroll
    for (int j = 0; j < I::MJ; ++j)
      if (mok[j]) af[j] = tr_frag(xs + (pA + moff[j]) * CIN + mci[j], xs + (pB + moff[j]) * CIN + mci[j]);
  };
  f32x4 wacc[I::MJ][I::NT];
#pragma unroll
  for (int j = 0; j < I::MJ; ++j)
#pragma unroll
    for (int n = 0; n < I::NT; ++n) wacc[j][n] = zero4();
  bf16x8 bfr[I::NT], afr[I::MJ];
  frags(0, bfr, afr);
  for (int s_ = 0; s_ < I::KSTEPS; ++s_) {
    bf16x8 bn[I::NT], an[I::MJ];
    wait_lds();
    __builtin_amdgcn_sched_barrier(0);
    if (s_ + 1 < I::KSTEPS) frags(s_ + 1, bn, an);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < I::MJ; ++j)
      if (mok[j]) {
#pragma unroll
        for (int n = 0; n < I::NT; ++n) wacc[j][n] = mfma16(afr[j], bfr[n], wacc[j][n]);
      }
#pragma unroll
    for (int n = 0; n < I::NT; ++n) bfr[n] = bn[n];
#pragma unroll
    for (int j = 0; j < I::MJ; ++j) afr[j] = an[j];
  }
  float* out = wa_.part + (size_t)b * I::KP * COUT;
#pragma unroll
  for (int j = 0; j < I::MJ; ++j) {
    const int m = w + 4 * j;
    if (mok[j]) {
#pragma unroll
      for (int n = 0; n < I::NT; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) st_maybe_nt<kNtSlab>(out + (16 * m + 4 * g + i) * COUT + 16 * n + li, wacc[j][n][i]);
    }
  }
}

// ================================ head =========================================================
// per image: a18 = relu(bn(z18) + x_in) -> mean pool -> fc 64x10 -> softmax-xent -> backward to g_y18
__global__ __launch_bounds__(RT) void k_rn_head(DmlcRnHeadArgs a) {
  if (a.step_copy && blockIdx.x == 0 && threadIdx.x == 0) *a.step_copy = *a.step;
  __shared__ float pool_part[4][64];
  __shared__ float pooled[64], dlog[16], gpool[64], cf[2][64];
  __shared__ float redl[2][4][64];
  __shared__ float fcw_s[650];                  // fc weight [64][10] + bias [10]
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int c = lane;                           // thread -> channel c, pixels w, w+4, ... (16 each)
  // every small operand of the later phases is loaded at entry, beside the activations: the fc
  // weights / bias into LDS, gamma / beta into registers (each was one more exposed memory latency
  // on the serial chain pool -> logits -> dlogits -> pooled gradient)
  float fv[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int e = tid + i * RT;                 // clamped addresses: every load in bounds
    const float wv = a.fcw[e < 640 ? e : 0], bv = a.fcb[e >= 640 && e < 650 ? e - 640 : 0];
    fv[i] = e < 640 ? wv : (e < 650 ? bv : 0.f);
  }
  const float gam = a.gamma[c], bet = a.beta[c];
  if (tid < 64) {
    float mean, rstd;
    bn_mean_rstd(a.stat, tid, a.inv_n, mean, rstd);
    cf[0][tid] = mean; cf[1][tid] = rstd;
  }
  const bf16* zp = reinterpret_cast<const bf16*>(a.z) + (size_t)b * 4096;
  const bf16* sp = reinterpret_cast<const bf16*>(a.sc) + (size_t)b * 4096;
  float zv[16], sv[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int px = w + 4 * k;
    zv[k] = (float)zp[px * 64 + c];
    sv[k] = (float)sp[px * 64 + c];
  }
  int label = 0;
  if (tid == 0) label = a.labels[batch_index(a.src, a.B, b)];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int e = tid + i * RT;
    if (e < 650) fcw_s[e] = fv[i];
  }
  __syncthreads();
  const float mean = cf[0][c], rstd = cf[1][c];
  const float sc = gam * rstd, sh = bet - mean * sc;
  float av[16];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    av[k] = fmaxf(zv[k] * sc + sh + sv[k], 0.f);
    s += av[k];
  }
  pool_part[w][c] = s;
  __syncthreads();
  if (tid < 64) pooled[tid] = (pool_part[0][tid] + pool_part[1][tid] + pool_part[2][tid] + pool_part[3][tid]) * (1.f / 64.f);
  __syncthreads();
  if (tid < 64) {                               // wave 0: logits / softmax / dlogits
    float lg = 0.f;
    if (lane < 10) {
      lg = fcw_s[640 + lane];
      for (int k = 0; k < 64; ++k) lg += pooled[k] * fcw_s[k * 10 + lane];
    }
    const float lgm = lane < 10 ? lg : -INFINITY;
    float m = lgm;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    float e = lane < 10 ? __expf(lg - m) : 0.f;
    float se = e;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o);
    const int lab = __shfl(label, 0);
    int am = lane < 10 && lg == m ? lane : 64;  // first maximum (accuracy)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) am = min(am, __shfl_xor(am, o));
    const float lse = m + __logf(se);
    const float lgl = __shfl(lg, lab);
    const bool real = b < a.nvalid;             // batch padding: no loss, accuracy or gradient
    if (lane == 0) { a.loss_img[b] = real ? lse - lgl : 0.f; a.correct_img[b] = real && am == lab ? 1 : 0; }
    if (lane < 10) {
      if (a.logits_out) a.logits_out[b * 10 + lane] = lg;
      dlog[lane] = real ? (e / se - (lane == lab ? 1.f : 0.f)) * a.inv_batch : 0.f;
    }
  }
  __syncthreads();
  if (tid < 64) {
    float gp = 0.f;
#pragma unroll
    for (int n = 0; n < 10; ++n) gp += fcw_s[tid * 10 + n] * dlog[n];
    gpool[tid] = gp * (1.f / 64.f);
    float* fp = a.fc_part + (size_t)b * 656;
#pragma unroll
    for (int n = 0; n < 10; ++n) fp[tid * 10 + n] = pooled[tid] * dlog[n];
    if (tid < 10) fp[640 + tid] = dlog[tid];
  }
  __syncthreads();
  const float gpc = gpool[c];
  bf16* gyo = reinterpret_cast<bf16*>(a.gy) + (size_t)b * 4096;
  float r1 = 0.f, r2 = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int px = w + 4 * k;
    const float gy = av[k] > 0.f ? gpc : 0.f;
    gyo[px * 64 + c] = (bf16)gy;
    r1 += gy;
    r2 += gy * (zv[k] - mean) * rstd;
  }
  redl[0][w][c] = r1;
  redl[1][w][c] = r2;
  __syncthreads();
  const float t1 = tid < 64 ? redl[0][0][tid] + redl[0][1][tid] + redl[0][2][tid] + redl[0][3][tid] : 0.f;
  const float t2 = tid < 64 ? redl[1][0][tid] + redl[1][1][tid] + redl[1][2][tid] + redl[1][3][tid] : 0.f;
  if (tid < 64) {
    long long* d = a.red + (b & (NSLOT - 1)) * 256;
    fx_add(d, tid, t1);
    fx_add(d, 64 + tid, t2);
  }
}

// ================================ SGD ==========================================================
DEV float4 add4r(float4 x, float4 y) { return make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w); }

// thread (sp = tid / O, idx = tid % O) sums slabs q = sp, sp+S, ...; the block folds the S splits
// in fixed order -> threads tid < O return the total of output idx (deterministic)
DEV float4 split_reduce(const float* p, size_t stride, int n, int S, float4* lds) {
  const int O = RT / S, sp = threadIdx.x / O, idx = threadIdx.x - sp * O;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  int q = sp;
  for (; q + 7 * S < n; q += 8 * S) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(p + (size_t)(q + u * S) * stride);
#pragma unroll
    for (int u = 0; u < 8; ++u) s = add4r(s, v[u]);
  }
  for (; q < n; q += S) s = add4r(s, *reinterpret_cast<const float4*>(p + (size_t)q * stride));
  lds[threadIdx.x] = s;
  __syncthreads();
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (threadIdx.x < O)
    for (int k = 0; k < S; ++k) t = add4r(t, lds[k * O + idx]);
  return t;
}

// modes: 0 reduce slabs + apply (1 GPU); 1 reduce slabs into `grad` (DP, before the all-reduce);
//        2 apply grad_scale * `grad` (DP, after it); 3 refresh the bf16 shadows from the master only
// blocks: [conv layer 0..18 | fc | BN layer 0..18]
__global__ __launch_bounds__(RT) void k_rn_sgd(DmlcRnSgdArgs a) {
  __shared__ float4 lds[RT];
  __shared__ float lred[2][4];
  const int64_t step = *a.step_rd;
  const float lr0 = a.staircase ? a.lr0 * powf(a.decay, floorf((float)step / a.decay_steps)) : a.lr0;
  const float lr = a.warmup > 0.f && (float)step < a.warmup ? lr0 * ((float)step + 1.f) / a.warmup : lr0;
  const int mode = a.mode;
  const bool reduce = mode <= 1, apply = mode == 0 || mode == 2;
  const int blk = blockIdx.x, tid = threadIdx.x;
  constexpr int NL = DMLC_RN_LAYERS;
  // (the BN blocks dispatched first instead of last measured no better: 612.0-612.9 vs 608.4-611.3
  // us/step, profiles/r6s3_rn_sgd_bn_first_ab.txt -- they are not the launch's tail)
  // block role: every range start compared at once (21 independent kernarg loads, one latency; the
  // search loop paid one dependent scalar load per range -- ~20 in a row for the BN blocks)
  int l = 0;
#pragma unroll
  for (int i = 1; i <= NL + 1; ++i) l += blk >= a.blk_start[i] ? 1 : 0;
  if (l < NL) {                                  // conv layer l
    const int S = a.split[l], O = RT / S;
    const int cin = a.cin[l], cout = a.cout[l], cinp = cin < 8 ? 8 : cin;
    const int kp = (9 * cinp + 31) / 32 * 32, kpd = (9 * cout + 31) / 32 * 32;
    const int n4 = 9 * cin * cout / 4, co4n = cout / 4;
    const int o4 = (blk - a.blk_start[l]) * O + tid % O;
    const bool valid = o4 < n4;
    const int oc = valid ? o4 : 0;
    const int row = oc / co4n, co = (oc - row * co4n) * 4;          // HWIO row = tap*cin + ci
    const int tap = row / cin, ci = row - tap * cin, k = tap * cinp + ci;
    const size_t off = (size_t)a.conv_off[l] + (size_t)row * cout + co;
    float4 gsum = make_float4(0.f, 0.f, 0.f, 0.f);
    if (reduce) gsum = split_reduce(a.part[l] + (size_t)k * cout + co, (size_t)kp * cout, a.G[l], S, lds);
    if (tid < O && valid) {
      if (mode == 1) {
        *reinterpret_cast<float4*>(a.grad + off) = gsum;
      } else {
        if (mode == 2) {
          const float4 gv = *reinterpret_cast<const float4*>(a.grad + off);
          gsum = make_float4(gv.x * a.grad_scale, gv.y * a.grad_scale, gv.z * a.grad_scale, gv.w * a.grad_scale);
        }
        float* m = a.master + off;
        float4 wv = *reinterpret_cast<float4*>(m);
        if (apply) {
          wv.x -= lr * gsum.x; wv.y -= lr * gsum.y; wv.z -= lr * gsum.z; wv.w -= lr * gsum.w;
          *reinterpret_cast<float4*>(m) = wv;
        }
        bf16* wf = reinterpret_cast<bf16*>(a.wf[l]);
        wf[(co + 0) * kp + k] = (bf16)wv.x; wf[(co + 1) * kp + k] = (bf16)wv.y;
        wf[(co + 2) * kp + k] = (bf16)wv.z; wf[(co + 3) * kp + k] = (bf16)wv.w;
        if (a.wd[l])
          *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.wd[l]) + (size_t)ci * kpd + (8 - tap) * cout + co) =
              pack4(wv.x, wv.y, wv.z, wv.w);
      }
    }
  } else if (l == NL) {                          // fc: 164 float4 of [640 dW | 10 db | pad], split over images
    const int S = a.split[NL], O = RT / S;
    const int o4 = (blk - a.blk_start[l]) * O + tid % O;
    const bool valid = o4 < 164;
    float4 gsum = make_float4(0.f, 0.f, 0.f, 0.f);
    if (reduce) gsum = split_reduce(a.fc_part + 4 * (valid ? o4 : 0), 656, a.B, S, lds);
    if (tid < O && valid && mode != 3) {
      const float gv[4] = {gsum.x, gsum.y, gsum.z, gsum.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = 4 * o4 + j;
        if (e < 650) {
          const size_t off = e < 640 ? (size_t)a.fcw_off + e : (size_t)a.fcb_off + e - 640;
          if (mode == 1) a.grad[off] = gv[j];
          else a.master[off] -= lr * (mode == 2 ? a.grad[off] * a.grad_scale : gv[j]);
        }
      }
    }
  } else if (mode != 3 && a.tail) {               // BN layer L: gamma/beta + running statistics
    const int L = blk - a.blk_start[NL + 1];
    const int c = tid;
    // every load of this block first (gradient and statistics slots, master gamma / beta, running
    // statistics, layer 0: the per-image loss / accuracy), then the arithmetic and the stores: the
    // chain of dependent round trips made these 19 blocks the launch's tail
    const bool act = c < a.cout[L];
    const int cc = act ? c : 0;
    const size_t og = (size_t)a.gamma_off[L] + cc, ob = (size_t)a.beta_off[L] + cc;
    const long long* rp = a.red + (size_t)L * NSLOT * 256;
    const long long* sp = a.stat + (size_t)L * NSLOT * 256;
    // (fx_total issues its 16 loads before any arithmetic; the four totals are independent)
    const double r1 = fx_total(rp, cc), r2 = fx_total(rp, 64 + cc);
    const double s1 = fx_total(sp, cc), s2 = fx_total(sp, 64 + cc);
    float* mm = a.state + a.mm_off[L] + cc;
    float* mv = a.state + a.mv_off[L] + cc;
    // (a.grad exists only in the data-parallel modes 1/2; the running statistics are only updated
    // by the applying modes)
    float mg = 0.f, mb = 0.f, gg = 0.f, gb = 0.f, mmv = 0.f, mvv = 0.f;
    if (mode != 1) { mg = a.master[og]; mb = a.master[ob]; mmv = *mm; mvv = *mv; }
    if (mode == 2) { gg = a.grad[og]; gb = a.grad[ob]; }
    float lsv = 0.f, csv = 0.f;
    if (L == 0 && apply)
      for (int q = tid; q < a.B; q += RT) { lsv += a.loss_img[q]; csv += (float)a.correct_img[q]; }
    if (act) {
      if (mode == 1) {
        a.grad[og] = (float)r2;
        a.grad[ob] = (float)r1;
      } else {
        a.master[og] = mg - lr * (mode == 2 ? gg * a.grad_scale : (float)r2);
        a.master[ob] = mb - lr * (mode == 2 ? gb * a.grad_scale : (float)r1);
        const double inv = (double)a.inv_n[L];
        const double mean = s1 * inv;
        double var = s2 * inv - mean * mean;
        var = var > 0.0 ? var : 0.0;
        const double nn = 1.0 / inv;
        const float m = a.bn_momentum;
        *mm = (1.f - m) * mmv + m * (float)mean;
        *mv = (1.f - m) * mvv + m * (float)(var * nn / (nn - 1.0));
      }
    }
    if (L == 0 && apply) {                       // batch loss / accuracy -> stats ring (fields 1, 2)
      float ls = lsv, cs = csv;
      ls = wave_sum(ls);
      cs = wave_sum(cs);
      if ((tid & 63) == 0) { lred[0][tid >> 6] = ls; lred[1][tid >> 6] = cs; }
      __syncthreads();
      if (tid == 0) {
        float* st = a.stats + (size_t)(step % a.stats_len) * 4;
        st[1] = (lred[0][0] + lred[0][1] + lred[0][2] + lred[0][3]) / (float)a.nvalid;
        st[2] = (lred[1][0] + lred[1][1] + lred[1][2] + lred[1][3]) / (float)a.nvalid;
        if (a.step_rd != a.step) {               // no block reads *a.step: publish + bump here
          st[0] = (float)(step + 1);
          st[3] = lr;
          *a.step = step + 1;
        }
      }
    }
  }
  if (!apply || !a.tail || a.step_rd != a.step) return;   // partial launch / ticketless: nothing more
  __syncthreads();
  if (tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (last_arrival(a.ticket, blockIdx.x, gridDim.x)) {   // last block: publish the step
      float* st = a.stats + (size_t)(step % a.stats_len) * 4;
      st[0] = (float)(step + 1);
      st[3] = lr;
      *a.step = step + 1;
    }
  }
}

}  // namespace rn
}  // namespace dmlc

using namespace dmlc;
using namespace dmlc::rn;

namespace {


// the ResNet-20 layer shapes (CIN, COUT, HIN, S)
#define DMLC_RN_SHAPES(X) \
  X(3, 16, 32, 1)         \
  X(16, 16, 32, 1)        \
  X(16, 32, 32, 2)        \
  X(32, 32, 16, 1)        \
  X(32, 64, 16, 2)        \
  X(64, 64, 8, 1)

template <int CI, int CO, int H, int ST>
hipError_t launch_fwd(const DmlcRnFwdArgs& a, hipStream_t s) {
  using F = Fwd<CI, CO, H, ST>;
  DMLC_LDS_OPTIN((&k_rn_fwd<CI, CO, H, ST>), F::LDS);
  hipLaunchKernelGGL((k_rn_fwd<CI, CO, H, ST>), dim3(a.B), dim3(RT), F::LDS, s, a);
  return hipGetLastError();
}

template <int CI, int CO, int H, int ST>
hipError_t launch_dgrad(const DmlcRnDgradArgs& a, hipStream_t s) {
  if constexpr (CI < 16) {
    return hipErrorInvalidValue;             // the stem has no input gradient
  } else {
    using D = Dg<CI, CO, H, ST>;
    DMLC_LDS_OPTIN((&k_rn_dgrad<CI, CO, H, ST>), D::LDS);
    hipLaunchKernelGGL((k_rn_dgrad<CI, CO, H, ST>), dim3(a.B), dim3(RT), D::LDS, s, a);
    return hipGetLastError();
  }
}

template <int CI, int CO, int H, int ST>
hipError_t launch_bwd(const DmlcRnDgradArgs& d, const DmlcRnWgradArgs& w, hipStream_t s) {
  if constexpr (CI < 16) {
    return hipErrorInvalidValue;             // the stem has no input gradient
  } else {
    using D = Dg<CI, CO, H, ST>;
    using G = Wg<CI, CO, H, ST>;
    constexpr size_t lds = D::LDS > G::LDS ? D::LDS : G::LDS;
    DMLC_LDS_OPTIN((&k_rn_bwd<CI, CO, H, ST>), lds);
    hipLaunchKernelGGL((k_rn_bwd<CI, CO, H, ST>), dim3(d.B + w.G * G::MC), dim3(RT), lds, s, d, w);
    return hipGetLastError();
  }
}

template <int C, int H>
hipError_t launch_bwd_img(const DmlcRnDgradArgs& d, const DmlcRnWgradArgs& w, hipStream_t s) {
  using I = BwdImg<C, C, H>;
  if (w.G != d.B) return hipErrorInvalidValue;   // one slab per image
  DMLC_LDS_OPTIN((&k_rn_bwd_img<C, C, H>), I::LDS);
  hipLaunchKernelGGL((k_rn_bwd_img<C, C, H>), dim3(d.B), dim3(RT), I::LDS, s, d, w);
  return hipGetLastError();
}

template <int CI, int CO, int H, int ST>
hipError_t launch_wgrad(const DmlcRnWgradArgs& a, hipStream_t s) {
  using G = Wg<CI, CO, H, ST>;
  DMLC_LDS_OPTIN((&k_rn_wgrad<CI, CO, H, ST>), G::LDS);
  hipLaunchKernelGGL((k_rn_wgrad<CI, CO, H, ST>), dim3(a.G, G::MC), dim3(RT), G::LDS, s, a);
  return hipGetLastError();
}

}  // namespace

extern "C" {

hipError_t dmlc_rn_fwd(const DmlcRnLayerGeom* g, const DmlcRnFwdArgs* a, hipStream_t s) {
#define X(CI, CO, H, ST) \
  if (g->cin == CI && g->cout == CO && g->hin == H && g->stride == ST) return launch_fwd<CI, CO, H, ST>(*a, s);
  DMLC_RN_SHAPES(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t dmlc_rn_dgrad(const DmlcRnLayerGeom* g, const DmlcRnDgradArgs* a, hipStream_t s) {
#define X(CI, CO, H, ST) \
  if (CI >= 16 && g->cin == CI && g->cout == CO && g->hin == H && g->stride == ST) return launch_dgrad<CI, CO, H, ST>(*a, s);
  DMLC_RN_SHAPES(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t dmlc_rn_wgrad(const DmlcRnLayerGeom* g, const DmlcRnWgradArgs* a, hipStream_t s) {
#define X(CI, CO, H, ST) \
  if (g->cin == CI && g->cout == CO && g->hin == H && g->stride == ST) return launch_wgrad<CI, CO, H, ST>(*a, s);
  DMLC_RN_SHAPES(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t dmlc_rn_bwd(const DmlcRnLayerGeom* g, const DmlcRnDgradArgs* d, const DmlcRnWgradArgs* w, hipStream_t s) {
  if (d->B != w->B) return hipErrorInvalidValue;
  if (g->per_image) {                              // one workgroup per image: dgrad + wgrad
    if (g->cin == 16 && g->cout == 16 && g->hin == 32 && g->stride == 1) return launch_bwd_img<16, 32>(*d, *w, s);
    if (g->cin == 32 && g->cout == 32 && g->hin == 16 && g->stride == 1) return launch_bwd_img<32, 16>(*d, *w, s);
    return hipErrorInvalidValue;
  }
#define X(CI, CO, H, ST) \
  if (CI >= 16 && g->cin == CI && g->cout == CO && g->hin == H && g->stride == ST) return launch_bwd<CI, CO, H, ST>(*d, *w, s);
  DMLC_RN_SHAPES(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t dmlc_rn_head(const DmlcRnHeadArgs* a, hipStream_t s) {
  hipLaunchKernelGGL(k_rn_head, dim3(a->B), dim3(RT), 0, s, *a);
  return hipGetLastError();
}

static int split_for(int n) {                 // slabs per thread <= 8
  int S = 4;
  while (S < 64 && S * 8 < n) S <<= 1;
  return S;
}

hipError_t dmlc_rn_sgd(DmlcRnSgdArgs* a, hipStream_t s) {
  if (a->layer_lo < 0 || a->layer_hi > DMLC_RN_LAYERS || a->layer_lo > a->layer_hi) return hipErrorInvalidValue;
  if (!a->tail && (a->mode == 1 || a->mode == 2 || a->mode == 3)) return hipErrorInvalidValue;   // partial: mode 0
  int blocks = 0;
  for (int l = 0; l < DMLC_RN_LAYERS; ++l) {      // layers outside the range get no blocks
    a->split[l] = split_for(a->G[l]);
    a->blk_start[l] = blocks;
    const int O = RT / a->split[l];
    if (l >= a->layer_lo && l < a->layer_hi) blocks += (9 * a->cin[l] * a->cout[l] / 4 + O - 1) / O;
  }
  a->split[DMLC_RN_LAYERS] = split_for(a->B);
  a->blk_start[DMLC_RN_LAYERS] = blocks;                     // fc
  if (a->tail) blocks += (164 + RT / a->split[DMLC_RN_LAYERS] - 1) / (RT / a->split[DMLC_RN_LAYERS]);
  a->blk_start[DMLC_RN_LAYERS + 1] = blocks;                 // BN, one block per layer
  if (a->tail) blocks += DMLC_RN_LAYERS;
  a->blk_start[DMLC_RN_LAYERS + 2] = blocks;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rn_sgd, dim3(blocks), dim3(RT), 0, s, *a);
  return hipGetLastError();
}

}  // extern "C"
