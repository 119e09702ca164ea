// conv1 weight gradient of ONE image, as device building blocks shared by the stand-alone conv1
// wgrad kernel (cnn_wgrad.hip, image groups) and the fused conv2-dgrad + conv1-wgrad kernel
// (cnn_conv.hip, one image per workgroup; TF Conv2DBackpropFilter + BiasAddGrad of conv1,
// /root/reference/cifar10cnn.py:107 via the autodiff of :163).
//
//   dW1[k''][co] = sum_px X[px][k''] dY1[px][co],  k'' = kh*16 + kw*3 + ci  (k'' % 16 == 15 unused)
//  * dY1 (the conv1 output gradient) is produced in LDS by the TF-SAME pool1 backward in "2x2
//    ownership" form from the pool1 gradient + argmax bytes (conv_common.h pool_bwd_2x2);
//  * X is kept as 15 channel-planar, column-shifted copies of the padded 28x24 crop (plane kw*3+ci =
//    Xpad[ci][y][x+kw]) so a K'' tile of 16 is one kernel row (15 taps + 1 zero plane) and every B
//    fragment is ONE aligned ds_read_b128 of 8 consecutive pixels;
//  * 8 waves split the 18 pixel k-steps (ks = w >> 1) and the co tile pairs (ch = w & 1); each wave owns
//    20 MFMA accumulators, reduced across the 4 k-step groups in fixed order by w1_flush.
#pragma once
#include "conv_common.h"

namespace dmlc {

constexpr int W1_DY_LD = 72;                  // dY1 LDS row stride (bf16): 144 B, tr reads conflict-free
constexpr int W1_PL = 28 * 24 + 8;            // shifted-plane stride (bf16): 1360 B, b128 reads conflict-free
constexpr int W1_DYT = 576 * W1_DY_LD;        // bf16 elements
constexpr int W1_XS = 16 * W1_PL;
constexpr int W1T = 512;                      // 8 waves (2 per SIMD) for the VALU-heavy gather phases
constexpr int W1_FL_BYTES = 4 * 20 * 64 * 16; // cross-wave reduction buffer (f32x4 per lane per tile)

// plane 15 (the zero K'' row of every kernel-row tile)
DEV void w1_zero_plane15(bf16* xs, int tid) {
  for (int e = tid; e < W1_PL / 8; e += W1T) *reinterpret_cast<bf16x8*>(xs + 15 * W1_PL + e * 8) = bf16x8{};
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

// (b) pool1 / ReLU backward -> dY1 (bf16, LDS) + bias-grad sums (fp32).  dps: pool1 gradient, LDS
//     [144][64] bf16 unswizzled; ams: argmax bytes [144][64].
DEV void w1_pool_bwd(bf16* dyt, const bf16* dps, const uint8_t* ams, float (&bsum)[8], int tid) {
  for (int task = tid; task < 144 * 8; task += W1T) {
    const int win = task >> 3, c = task & 7, py = win / 12, px = win - py * 12;
    float o[4][8];
    pool_bwd_2x2<12>(dps, ams, py, px, c, o);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int y = 2 * py + (k >> 1), x = 2 * px + (k & 1);
      *reinterpret_cast<bf16x8*>(dyt + (y * 24 + x) * W1_DY_LD + c * 8) = to_bf16x8(o[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) bsum[j] += o[k][j];
    }
  }
}

// (c) MFMA over one image: this wave's k-steps s = ks, ks+4, ... of the 18 (32 pixels each), co
//     tiles 2ch, 2ch+1, kernel rows t = 0..4 (16 K'' each)
DEV void w1_mfma(const bf16* dyt, const bf16* xs, f32x4 (&acc)[2][5], int ks, int ch, int g, int li) {
  const int q = li >> 2, p = li & 3;
  for (int s = ks; s < 18; s += 4) {
    const int rA = 32 * s + 8 * g + q, rB = rA + 4;
    bf16x8 af[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ct = 2 * ch + h;
      af[h] = tr_frag(dyt + rA * W1_DY_LD + 16 * ct + 4 * p, dyt + rB * W1_DY_LD + 16 * ct + 4 * p);
    }
    const int r0 = 32 * s + 8 * g, y = r0 / 24, x0 = r0 - y * 24;
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const bf16x8 bx = lds_b128(xs + li * W1_PL + (y + t) * 24 + x0);
#pragma unroll
      for (int h = 0; h < 2; ++h) acc[h][t] = mfma16(af[h], bx, acc[h][t]);
    }
  }
}

// Cross-wave reduction (fixed order) through `fl` (W1_FL_BYTES of LDS no longer read by anyone),
// then the fp32 slab out[80 k''][64 co] and the bias-grad row outb[64].  Call after a barrier that
// retired every wave's MFMA reads of the region; red: LDS [8][64] floats.
DEV void w1_flush(char* fl_mem, float* red, const f32x4 (&acc)[2][5], float (&bsum)[8], float* out, float* outb,
                  int ks, int ch, int lane, int tid) {
  f32x4* fl = reinterpret_cast<f32x4*>(fl_mem);
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int t = 0; t < 5; ++t) fl[(ks * 20 + (2 * ch + h) * 5 + t) * 64 + lane] = acc[h][t];
  block_chunk_sum(bsum, red, tid);
  __syncthreads();
  for (int e = tid; e < 20 * 64; e += W1T) {
    const f32x4 s = ((fl[e] + fl[1280 + e]) + (fl[2560 + e] + fl[3840 + e]));
    const int tile = e >> 6, ln = e & 63, ct = tile / 5, t = tile - ct * 5;
    const int co = 16 * ct + 4 * (ln >> 4), kk = 16 * t + (ln & 15);
    *reinterpret_cast<f32x4*>(out + kk * 64 + co) = s;
  }
  if (tid < 64) {
    float sb = 0.f;
#pragma unroll
    for (int k = 0; k < W1T / 64; ++k) sb += red[k * 64 + tid];
    outb[tid] = sb;
  }
}

}  // namespace dmlc
