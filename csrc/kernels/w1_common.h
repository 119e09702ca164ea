// conv1 weight gradient of ONE image, as device building blocks shared by the stand-alone conv1
// wgrad kernel (cnn_wgrad.hip, image groups) and the fused conv2-dgrad + conv1-wgrad kernel
// (cnn_conv.hip, one image per workgroup; TF Conv2DBackpropFilter + BiasAddGrad of conv1,
// /root/reference/cifar10cnn.py:107 via the autodiff of :163).
//
//   dW1[k''][co] = sum_px X[px][k''] dY1[px][co],  k'' = kh*16 + kw*3 + ci  (k'' % 16 == 15 unused)
//  * dY1 (the conv1 output gradient) is produced in LDS by the TF-SAME pool1 backward, scattered
//    from the pool1 gradient + argmax bytes in 4 deterministic phases (w1_pool_bwd);
//  * the bias gradient comes out of the same MFMAs (a ones plane in the unused K'' row 15);
//  * X is kept as 15 channel-planar, column-shifted copies of the padded 28x24 crop (plane kw*3+ci =
//    Xpad[ci][y][x+kw]) so a K'' tile of 16 is one kernel row (15 taps + 1 zero plane) and every B
//    fragment is ONE aligned ds_read_b128 of 8 consecutive pixels;
//  * 8 waves split the 18 pixel k-steps (ks = w >> 1) and the co tile pairs (ch = w & 1); each wave owns
//    20 MFMA accumulators, reduced across the 4 k-step groups in fixed order by w1_flush.
#pragma once
#include "conv_common.h"

namespace dmlc {

// dY1 LDS row stride (bf16): 128 B, one dword bank per channel pair whatever the pixel -- the
// scatter's random-row writes are conflict-free; the MFMA's tr reads of it are 4-way.  (Swizzling
// the 16-column tiles by row bits 1 and 3 makes those reads conflict-free and the scatter ~3-way:
// measured 1 us slower per launch.  Staging by LDS-DMA instead of registers: 0.5 us slower.)
constexpr int W1_DY_LD = 64;
constexpr int W1_PL = 28 * 24 + 8;            // shifted-plane stride (bf16): 1360 B, b128 reads conflict-free
constexpr int W1_DYT = 576 * W1_DY_LD;        // bf16 elements
constexpr int W1_XS = 16 * W1_PL;
constexpr int W1T = 512;                      // 8 waves (2 per SIMD) for the VALU-heavy gather phases
constexpr int W1_FL_BYTES = 4 * 10 * 64 * 16; // cross-wave reduction buffer (f32x4 per lane per tile, 2 rounds)

// plane 15 (the unused K'' row of every kernel-row tile) holds ONES: row 15 of each kernel-row
// tile of the MFMA product is then sum_px dY1[px][co], the conv1 bias gradient, for free
DEV void w1_ones_plane15(bf16* xs, int tid) {
  bf16x8 one;
#pragma unroll
  for (int j = 0; j < 8; ++j) one[j] = (bf16)1.0f;
  for (int e = tid; e < W1_PL / 8; e += W1T) *reinterpret_cast<bf16x8*>(xs + 15 * W1_PL + e * 8) = one;
}

// (a) shifted channel planes straight from the uint8 image in LDS: task (yy, x8, kw) -> planes
//     kw*3+{0,1,2}, 8 pixels: plane[kw*3+ci][yy][x] = crop[ci][yy-2][x+kw-2] (0 outside the crop)
DEV void w1_planes(bf16* xs, const uint8_t* img, int cy, int cx, int tid) {
  for (int task = tid; task < 28 * 3 * 5; task += W1T) {
    const int kw = task % 5, r = task / 5, x8 = r % 3, yy = r / 3, iy = yy - 2;
    const bool rok = iy >= 0 && iy < 24;
    const uint8_t* srow = img + ((cy + (rok ? iy : 0)) * 32 + cx) * 3;
    bf16x8 o0, o1, o2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ix = x8 * 8 + kw + j - 2;
      const bool ok = rok && ix >= 0 && ix < 24;
      const uint8_t* px = srow + (ok ? ix : 0) * 3;
      const float f0 = px[0], f1 = px[1], f2 = px[2];
      o0[j] = (bf16)(ok ? f0 : 0.f); o1[j] = (bf16)(ok ? f1 : 0.f); o2[j] = (bf16)(ok ? f2 : 0.f);
    }
    bf16* dst = xs + (kw * 3) * W1_PL + yy * 24 + x8 * 8;
    *reinterpret_cast<bf16x8*>(dst) = o0;
    *reinterpret_cast<bf16x8*>(dst + W1_PL) = o1;
    *reinterpret_cast<bf16x8*>(dst + 2 * W1_PL) = o2;
  }
}

// (b) pool1 / ReLU backward -> dY1 (bf16, LDS) as a SCATTER: every pool1 window adds its gradient
//     to its argmax pixel (read-modify-write into a zeroed tile) instead of every pixel gathering from
//     the up-to-4 windows that may have picked it (~10 VALU per output element).  One instruction
//     covers the 64 channels of one window (lanes 0-31: even channels, 32-63: odd), so with 128-B
//     dY1 rows its 32-lane groups hit 32 distinct banks whatever pixels the argmaxes pick (a lane per
//     window instead measured 55 % of the LDS cycles in bank conflicts).  Windows whose (py, px)
//     parities agree never overlap: the 4 parity classes run as 4 barrier-separated phases (36
//     windows each, window l -> wave l % 8), so no two adds of one phase hit the same element and an
//     element that receives several gradients receives them in the fixed phase order --
//     deterministic.  The first add into an element is exact (0 + bf16), the second is one rounding,
//     like the rounding of an fp32 sum.  (LDS bf16 atomics instead: 2x slower.)
DEV int w1_class_window(int ph, int l) {      // pool1 window (py * 12 + px) of class ph, index l < 36
  const int r = l / 6;
  return (2 * r + (ph >> 1)) * 12 + 2 * (l - r * 6) + (ph & 1);
}

DEV void w1_zero_dy(bf16* dyt, int tid) {
  for (int e = tid; e < W1_DYT / 8; e += W1T) *reinterpret_cast<bf16x8*>(dyt + e * 8) = bf16x8{};
}

// dps: pool1 gradient [144][64] bf16, ams: argmax bytes [144][64] (255 = no gradient), both in LDS.
// Call after w1_zero_dy + a barrier; ends with a barrier (dY1 complete).
DEV void w1_pool_bwd(bf16* dyt, const bf16* dps, const uint8_t* ams, int w, int lane) {
  // (d / 3) * 24 + d % 3 for the in-window position d = 3 dy + dx, 6 bits per entry; code 255 reads
  // bits 58.. (shift taken mod 64): offset 0, and adds 0 to the window's own corner element
  constexpr uint64_t kOff = 0ull | 1ull << 6 | 2ull << 12 | 24ull << 18 | 25ull << 24 | 26ull << 30 | 48ull << 36 |
                            49ull << 42 | 50ull << 48;
  const int ch = 2 * (lane & 31) + (lane >> 5);
#pragma unroll
  for (int ph = 0; ph < 4; ++ph) {
    // straight-line reads for all 5 items (the 5th exists for waves 0-3 only; the others read
    // window 35 again and write nothing), so their LDS latencies overlap
    int addr[5];
    float add[5], old[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {            // windows w, w + 8, ... (< 36) of this class
      const int l = min(w + 8 * k, 35);
      const int win = w1_class_window(ph, l), py = win / 12, px = win - py * 12;
      const uint32_t code = ams[win * 64 + ch];
      const float f = (float)dps[win * 64 + ch];
      addr[k] = ((py * 48 + 2 * px) + (int)((kOff >> ((6 * code) & 63u)) & 63u)) * W1_DY_LD + ch;
      add[k] = code < 9 ? f : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) old[k] = (float)dyt[addr[k]];
#pragma unroll
    for (int k = 0; k < 4; ++k) dyt[addr[k]] = (bf16)(old[k] + add[k]);
    if (w < 4) dyt[addr[4]] = (bf16)(old[4] + add[4]);
    lds_barrier();
  }
}

// (c) MFMA over one image: this wave's k-steps s = ks, ks+4, ... of the 18 (32 pixels each), co
//     tiles 2ch, 2ch+1, kernel rows t = 0..4 (16 K'' each).  Software-pipelined: the next k-step's
//     7 fragments are read under this k-step's 10 MFMAs (two waves per SIMD do not hide an LDS
//     latency per k-step).
DEV void w1_mfma(const bf16* dyt, const bf16* xs, f32x4 (&acc)[2][5], int ks, int ch, int g, int li) {
  const int q = li >> 2, p = li & 3;
  auto frags = [&](int s, bf16x8 (&af)[2], bf16x8 (&bx)[5]) {
    const int rA = 32 * s + 8 * g + q, rB = rA + 4;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ct = 2 * ch + h;
      af[h] = tr_frag(dyt + rA * W1_DY_LD + 16 * ct + 4 * p, dyt + rB * W1_DY_LD + 16 * ct + 4 * p);
    }
    const bf16* xp = xs + li * W1_PL + 32 * s + 8 * g;   // pixel row y, column x0: y * 24 + x0 = 32 s + 8 g
#pragma unroll
    for (int t = 0; t < 5; ++t) bx[t] = lds_b128(xp + t * 24);
  };
  bf16x8 af[2], bx[5];
  frags(ks, af, bx);
  for (int s = ks; s < 18; s += 4) {
    bf16x8 an[2], bn[5];
    wait_lds();                                // this k-step's fragments have landed
    __builtin_amdgcn_sched_barrier(0);
    if (s + 4 < 18) frags(s + 4, an, bn);      // uniform per wave
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h) acc[h][t] = mfma16(af[h], bx[t], acc[h][t]);
#pragma unroll
    for (int h = 0; h < 2; ++h) af[h] = an[h];
#pragma unroll
    for (int t = 0; t < 5; ++t) bx[t] = bn[t];
  }
}

// Cross-wave reduction (fixed order) through `fl` (W1_FL_BYTES of LDS no longer read by anyone), one
// co-tile half per round, then the fp32 slab out[80 k''][64 co] and the bias-grad row outb[64]
// (= row 15, the ones plane).  Call after a barrier that retired every wave's MFMA reads of the region.
// coh: agent-coherent stores (st_sc1) -- the slab is reduced by other blocks of the SAME launch.
DEV void w1_flush(char* fl_mem, const f32x4 (&acc)[2][5], float* out, float* outb, int ks, int ch, int lane,
                  int tid, bool coh = false) {
  f32x4* fl = reinterpret_cast<f32x4*>(fl_mem);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h) lds_barrier();                      // round 0's reads are done
#pragma unroll
    for (int t = 0; t < 5; ++t) fl[(ks * 10 + ch * 5 + t) * 64 + lane] = acc[h][t];
    lds_barrier();
    for (int e = tid; e < 10 * 64; e += W1T) {
      const f32x4 s = ((fl[e] + fl[640 + e]) + (fl[1280 + e] + fl[1920 + e]));
      const int tile = e >> 6, ln = e & 63, cp = tile / 5, t = tile - cp * 5;
      const int co = 16 * (2 * cp + h) + 4 * (ln >> 4), kk = 16 * t + (ln & 15);
      if (coh) {
        st_sc1(buf_rsrc(out), (uint32_t)(kk * 64 + co) * 4, s);
        if (kk == 15) st_sc1(buf_rsrc(outb), (uint32_t)co * 4, s);
      } else {
        st_maybe_nt<kNtW1>(reinterpret_cast<f32x4*>(out + kk * 64 + co), s);
        if (kk == 15) *reinterpret_cast<f32x4*>(outb + co) = s;
      }
    }
  }
}

}  // namespace dmlc
