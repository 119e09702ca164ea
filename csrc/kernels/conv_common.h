// Device helpers shared by the convolution kernels (cnn_conv.hip, cnn_wgrad.hip).
#pragma once
#include "common.h"
#include "api.h"

namespace dmlc {

constexpr int NT = 512;   // per-image conv kernels: 8 waves, 2 per SIMD hide each other's latency

// Copy N 16-byte chunks global -> LDS with every load of the thread issued before any store, so
// the block pays one memory latency instead of one per iteration.
template <int N>
DEV void stage16(void* dst, const void* src, int tid) {
  constexpr int IT = (N + 255) / 256;
  uint4 v[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int c = tid + i * 256;
    v[i] = load_sel(reinterpret_cast<const uint4*>(src) + c, reinterpret_cast<const uint4*>(src), c < N);
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int c = tid + i * 256;
    if (c < N) reinterpret_cast<uint4*>(dst)[c] = v[i];
  }
}

// Register prefetch of N 16-byte chunks (thread's share), split in two halves so a kernel can issue
// the loads of the NEXT item before computing the current one.
template <int N, int T = 256>
struct Prefetch16 {
  static constexpr int IT = (N + T - 1) / T;
  uint4 v[IT];
  MDEV void load(const void* src, int tid) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int c = tid + i * T;
      v[i] = load_sel(reinterpret_cast<const uint4*>(src) + c, reinterpret_cast<const uint4*>(src), c < N);
    }
  }
  MDEV void store(void* dst, int tid) const {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int c = tid + i * T;
      if (c < N) reinterpret_cast<uint4*>(dst)[c] = v[i];
    }
  }
};

// Register prefetch of N 16-byte chunks with NO predicate on any load or store: in the last round
// the surplus threads re-load (and later re-store) a chunk another thread owns -- identical bytes to
// the same LDS address.  Every load is then consumed by an unconditional store on every path.  With
// a predicated store (Prefetch16), hipcc's waitcnt pass sees a path on which the previous prefetch is
// still in flight when its registers are reloaded, and waits for it in the MIDDLE of issuing the
// next prefetch -- one exposed memory latency per item again (seen in the wgrad loop's .s).
template <int N, int T>
struct PrefetchAll {
  static constexpr int IT = (N + T - 1) / T;
  static constexpr int TAIL = N - (IT - 1) * T;
  uint4 v[IT];
  MDEV void load(const void* src, int tid) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int c = i < IT - 1 ? tid + i * T : (IT - 1) * T + (TAIL == T ? tid : tid % TAIL);
      v[i] = reinterpret_cast<const uint4*>(src)[c];
    }
  }
  MDEV void store(void* dst, int tid) const {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int c = i < IT - 1 ? tid + i * T : (IT - 1) * T + (TAIL == T ? tid : tid % TAIL);
      reinterpret_cast<uint4*>(dst)[c] = v[i];
    }
  }
};

DEV bf16x8 to_bf16x8(const float (&v)[8]) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
  return o;
}

// conv1 input as 5-tap row windows: the 24x24 crop of the uint8 NHWC image at (cy,cx) with a zero
// halo of 2, stored as [28 padded rows r][24 output columns x][16] bf16 where element j = kw*3 + ci
// (j < 15; j = 15 is zero) is input pixel (r - 2, x + kw - 2), channel ci.  An MFMA B fragment (8
// consecutive k of the K = 80 layout k = kh*16 + kw*3 + ci) is then ONE 16-B read at row y + kh,
// half (k >> 3) & 1 -- K padded to 96 (3 k-steps) instead of 160 (5; kw padded to 8 and ci to 4).
constexpr int C1_XIN = 28 * 24 * 16;       // 10752 bf16
constexpr int C1_K = 96;                   // conv1 weight shadow row: [64 co][96], k = kh*16 + kw*3 + ci
constexpr int C1_OUT = 576 * 64;           // 36864 bf16

// The whole 3 KB uint8 image in ONE 16-byte load per thread (threads 0..191) into LDS (`raw`), and
// optionally out to xraw (the weight-gradient kernel then reads it without the index -> dataset
// chain); then expanded from LDS.  Call stage_conv1_raw, barrier, stage_conv1_input.
DEV void stage_conv1_raw(uint8_t* raw, const uint8_t* src, uint8_t* xraw, int tid) {
  if (tid < 192) {
    const uint4 v = reinterpret_cast<const uint4*>(src)[tid];
    reinterpret_cast<uint4*>(raw)[tid] = v;
    if (xraw) reinterpret_cast<uint4*>(xraw)[tid] = v;
  }
}

// (elements j of a window are consecutive bytes of the raw NHWC row: pixel x + kw - 2, channel ci
// sits at byte (x - 2) * 3 + j of the crop row, so a half window is the 8 raw bytes at `off`, read
// as two aligned 8-B words and funnel-shifted -- 8 byte reads per half measured ~0.9 us slower.
// raw needs 8 readable bytes before it (the left halo reads them and masks them out) and after.
DEV void stage_conv1_input(bf16* xin, const uint8_t* raw, int cy, int cx, int tid) {
  const int h = tid & 1;                       // NT is even: every task of a thread has the same half
  for (int t = tid; t < 28 * 24 * 2; t += NT) {
    const int px = t >> 1, r = px / 24, x = px - r * 24, iy = r - 2;
    const bool rok = iy >= 0 && iy < 24;
    const int off = rok ? ((cy + iy) * 32 + cx + x - 2) * 3 + 8 * h : 8;
    const int a0 = off & ~7, sh = (off & 7) * 8;
    const uint64_t lo = *reinterpret_cast<const uint64_t*>(raw + a0);
    const uint64_t hi = *reinterpret_cast<const uint64_t*>(raw + a0 + 8);
    const uint64_t v = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
    float f[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int j = 8 * h + e, ix = x + j / 3 - 2;
      f[e] = rok && j < 15 && ix >= 0 && ix < 24 ? (float)((uint32_t)(v >> (8 * e)) & 0xffu) : 0.f;
    }
    *reinterpret_cast<bf16x8*>(xin + px * 16 + 8 * h) = to_bf16x8(f);
  }
}

// conv1 B fragments of pixel px (lane li of its tile): k-step s, lane group g holds k = 32s + 8g ..
// +7 = kernel row 2s + (g >> 1), window half g & 1; the pad rows k >= 80 (s = 2, g >= 2) re-read
// row 4 against zero weights.
DEV void conv1_frag_tile(const bf16* xin, int px, int g, bf16x8 (&bx)[3]) {
  const int y = px / 24, x = px - y * 24;
  const bf16* base = xin + (y * 24 + x) * 16 + 8 * (g & 1);
#pragma unroll
  for (int s = 0; s < 3; ++s) bx[s] = lds_b128(base + min(2 * s + (g >> 1), 4) * 24 * 16);
}

// conv2 input / output LDS images: padded [16*16][64] (swzpad) and [144][64] bf16
constexpr int C2_XIN = 256 * 64;
constexpr int C2_OUT = 144 * 64;

DEV float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
DEV float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// TF-SAME 3x3/2 max-pool backward, "2x2 ownership" form.  Pooled window (py,px) owns the conv
// output pixels (2py+dy, 2px+dx), dy,dx in {0,1}; with windows overlapping by one row/column, those
// pixels receive gradient only from (py,px), its left (py,px-1), upper (py-1,px) and upper-left
// neighbour, at fixed in-window positions d = 3*dy + dx:
//   o[3] (2py+1,2px+1) : W d4
//   o[2] (2py+1,2px)   : W d3 + L d5
//   o[1] (2py,  2px+1) : W d1 + U d7
//   o[0] (2py,  2px)   : W d0 + L d2 + U d6 + UL d8
// (the argmax byte 255 = "pooled <= 0" never matches, giving the ReLU mask for free).  No loops, no
// atomics, fixed summation order -> deterministic.  dp/am: LDS [HO*HO][64]; chunk c = channels 8c..8c+7.
template <int HO>
DEV void pool_bwd_2x2(const bf16* dp, const uint8_t* am, int py, int px, int c, float (&o)[4][8]) {
  const int base = (py * HO + px) * 64 + c * 8;
  const uint2 aw = *reinterpret_cast<const uint2*>(am + base);
  const uint4 vw = *reinterpret_cast<const uint4*>(dp + base);
  // neighbours outside the grid read the window itself (valid address) and get argmax 255 (no match)
  const int ol = px > 0 ? 64 : 0, ou = py > 0 ? HO * 64 : 0;
  uint2 al = *reinterpret_cast<const uint2*>(am + base - ol);
  uint2 au = *reinterpret_cast<const uint2*>(am + base - ou);
  uint2 aul = *reinterpret_cast<const uint2*>(am + base - ol - ou);
  const uint4 vl = *reinterpret_cast<const uint4*>(dp + base - ol);
  const uint4 vu = *reinterpret_cast<const uint4*>(dp + base - ou);
  const uint4 vul = *reinterpret_cast<const uint4*>(dp + base - ol - ou);
  const uint2 none = make_uint2(0xffffffffu, 0xffffffffu);
  if (!ol) al = none;
  if (!ou) au = none;
  if (!ol || !ou) aul = none;
  const uint32_t vwa[4] = {vw.x, vw.y, vw.z, vw.w}, vla[4] = {vl.x, vl.y, vl.z, vl.w};
  const uint32_t vua[4] = {vu.x, vu.y, vu.z, vu.w}, vula[4] = {vul.x, vul.y, vul.z, vul.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int sh = (j & 3) * 8;
    const uint32_t bw = ((j < 4 ? aw.x : aw.y) >> sh) & 0xff, bl = ((j < 4 ? al.x : al.y) >> sh) & 0xff;
    const uint32_t bu = ((j < 4 ? au.x : au.y) >> sh) & 0xff, bul = ((j < 4 ? aul.x : aul.y) >> sh) & 0xff;
    const float fw = (j & 1) ? bf16_hi(vwa[j >> 1]) : bf16_lo(vwa[j >> 1]);
    const float fl = (j & 1) ? bf16_hi(vla[j >> 1]) : bf16_lo(vla[j >> 1]);
    const float fu = (j & 1) ? bf16_hi(vua[j >> 1]) : bf16_lo(vua[j >> 1]);
    const float ful = (j & 1) ? bf16_hi(vula[j >> 1]) : bf16_lo(vula[j >> 1]);
    o[3][j] = bw == 4 ? fw : 0.f;
    o[2][j] = (bw == 3 ? fw : 0.f) + (bl == 5 ? fl : 0.f);
    o[1][j] = (bw == 1 ? fw : 0.f) + (bu == 7 ? fu : 0.f);
    o[0][j] = ((bw == 0 ? fw : 0.f) + (bl == 2 ? fl : 0.f)) + ((bu == 6 ? fu : 0.f) + (bul == 8 ? ful : 0.f));
  }
}

// Reduce per-thread channel sums (thread's chunk = tid & 7) over the workgroup: red[waves][64] partials.
DEV void block_chunk_sum(float (&v)[8], float* red /*[waves][64]*/, int tid) {
  const int lane = tid & 63, w = wave_id();
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float s = v[j];
    s += __shfl_xor(s, 8);
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    v[j] = s;
  }
  if (lane < 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[w * 64 + lane * 8 + j] = v[j];
  }
}

// Epilogue helper: acc (C[4g+i][px]) + bias -> ReLU -> bf16 -> LDS [px][64] swizzled.
DEV void store_relu_tile(bf16* cout, int px, int co_base, const f32x4& acc, const float* b4) {
  const bf16x4 v = pack4(fmaxf(acc[0] + b4[0], 0.f), fmaxf(acc[1] + b4[1], 0.f),
                         fmaxf(acc[2] + b4[2], 0.f), fmaxf(acc[3] + b4[3], 0.f));
  const int chunk = co_base >> 3, half = (co_base >> 2) & 1;
  *reinterpret_cast<bf16x4*>(cout + swz128(px, chunk) + half * 4) = v;
}

// The 3x3 window max + first argmax of 8 channels from the window's 9 taps (16-B chunks of 8 bf16).
// Each candidate is a signed 32-bit key (bits << 16 | 15 - d): post-ReLU values order like their
// bit patterns, a -0.0 (sign bit set) ranks below the initial key 0, and one integer max per
// element and tap keeps value AND first argmax (ties -> smallest d).  A tap in the bottom / right
// TF-SAME padding is read clamped to the last row / column, i.e. it repeats tap d-3 / d-1 (and
// d-4) with a smaller tag, so it can never win and needs no mask.  (r4 masked the sign bit and the
// padding taps: ~4 VALU per element and tap; this is 1.5.)  Output bits / argmax bytes (255 =
// "pooled <= 0", the ReLU mask for the backward).
DEV void pool_window(const uint4 (&v)[9], uint4& o, uint32_t& alo, uint32_t& ahi, uint32_t& bmax) {
  int key[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) key[j] = 0;
#pragma unroll
  for (int d = 0; d < 9; ++d) {
    const uint32_t tag = 15 - d;
    const uint32_t wv[4] = {v[d].x, v[d].y, v[d].z, v[d].w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      key[2 * i] = max(key[2 * i], (int)((wv[i] << 16) | tag));
      key[2 * i + 1] = max(key[2 * i + 1], (int)((wv[i] & 0xffff0000u) | tag));
    }
  }
  uint32_t* ow = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
  for (int i = 0; i < 4; ++i) ow[i] = ((uint32_t)key[2 * i] >> 16) | ((uint32_t)key[2 * i + 1] & 0xffff0000u);
  alo = 0;
  ahi = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t hv = (uint32_t)key[j] >> 16;
    bmax = max(bmax, hv);
    const uint32_t arg = hv ? 15 - (key[j] & 15) : 255;
    if (j < 4) alo |= arg << (8 * j);
    else ahi |= arg << (8 * (j - 4));
  }
}

// TF-SAME 3x3/2 max-pool over an LDS image [H*W][64] (swizzled) -> global out [HO*WO][64] bf16 +
// argmax bytes.  Padding is bottom/right only (in = 2*out), padded cells never win.
// The window max / argmax: pool_window.
// pad_lds (optional): also writes the pooled image into an LDS [(HO+4) x (HO+4)][64] swizzled image
// at offset (2, 2) -- the zero-padded input of the next 5x5 conv (fused conv1 -> conv2 forward).
template <int H>
DEV void pool_emit(const bf16* cout, bf16* out, uint8_t* am, int tid, uint32_t* vmax = nullptr,
                   bf16* pad_lds = nullptr) {
  // (r5: 4-channel tasks -- 2304 half tasks, 4.5 per thread instead of 2.25 -- measured 0.5 us slower)
  constexpr int HO = H / 2;
  uint32_t bmax = 0;                           // max pooled bf16 bits of this thread (fp8 scaling)
  for (int task = tid; task < HO * HO * 8; task += NT) {
    const int q = task >> 3, c = task & 7;
    const int py = q / HO, px = q - py * HO;
    // Branch-free: all 9 taps are loaded (a tap in the bottom / right TF-SAME padding reads the last
    // row / column instead: see pool_window), so the 9 LDS reads issue back to back and the task
    // pays one LDS latency.  (With `if (tap valid) load` -- a divergent condition -- hipcc put each
    // load in its own EXEC-masked block with its own lgkmcnt(0).)
    uint4 v[9];
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      const int y = min(2 * py + d / 3, H - 1), x = min(2 * px + d % 3, H - 1);
      v[d] = *reinterpret_cast<const uint4*>(cout + swz128(y * H + x, c));
    }
    uint4 o;
    uint32_t alo, ahi;
    pool_window(v, o, alo, ahi, bmax);
    st_out16(out, (uint32_t)(q * 64 + c * 8) * 2, o);
    st_out8(am, (uint32_t)(q * 64 + c * 8), make_uint2(alo, ahi));
    if (pad_lds) *reinterpret_cast<uint4*>(pad_lds + swzpad((py + 2) * (HO + 4) + px + 2, c)) = o;
  }
  if (vmax) *vmax = bmax;
}

}  // namespace dmlc
