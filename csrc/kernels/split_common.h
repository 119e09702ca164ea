// Channel-split building blocks (cnn_split.hip's design notes): block -> (image, part) placement, the
// [pixel][channels] LDS swizzle, the 32-row conv2-shaped core with its K halves, and the conv2 input
// gradient of one image's 32-channel half -- shared by the split launches (cnn_split.hip) and the fc
// chain launch, which runs the split dgrad at B <= 128 (cnn_fc.hip).
#pragma once
#include "w1_common.h"

namespace dmlc {

template <int S>
DEV void split_index(int blk, int& b, int& h) {
  h = (blk >> 3) % S;
  b = (blk & 7) + 8 * (blk / (8 * S));
}

// [pixel][CH x 16-B chunks] LDS images (CH = channels / 8): chunk c of pixel p at slot c ^ key(p), the
// key stepping once per bank row of pixels so that 16 consecutive pixels (an MFMA epilogue store) and
// the stride-2 pixels of the pool windows spread over the bank slots.
template <int CH>
DEV int swzc(int px, int c) {
  if constexpr (CH == 8) return px * 64 + ((c ^ (px & 7)) << 3);
  else if constexpr (CH == 4) return px * 32 + ((c ^ ((px >> 1) & 3)) << 3);
  else return px * 16 + ((c ^ ((px >> 2) & 1)) << 3);
}

// acc (C[co 4g+i][px]) + bias -> ReLU -> bf16 -> LDS [px][CH*8] (swzc)
template <int CH>
DEV void store_relu_c(bf16* img, int px, int co, const f32x4& acc, const float* b4) {
  const bf16x4 v = pack4(fmaxf(acc[0] + b4[0], 0.f), fmaxf(acc[1] + b4[1], 0.f),
                         fmaxf(acc[2] + b4[2], 0.f), fmaxf(acc[3] + b4[3], 0.f));
  *reinterpret_cast<bf16x4*>(img + swzc<CH>(px, co >> 3) + ((co >> 2) & 1) * 4) = v;
}

constexpr int SP_NT = 512;

// ---------------------------------------------------------------------------------------------
// conv2-shaped implicit GEMM over 32 output rows (c_out for the forward, c_in for the input gradient):
//   C[r][px] = sum_{kh,kw,ci} Wg[r][(kh*5+kw)*64 + ci] * Xpad[(y+kh)*16 + x+kw][ci]
// Xpad: LDS [16*16][64] bf16 (swzpad).  Wave w: K half kk = w >> 2 (input channels 32kk..32kk+31 of
// every tap), pixel group pg (tiles pg, pg+4, and 8 for pg 0), both 16-row tiles.  pg is rotated by
// the wave's SIMD partner (w, w+4) so the 3-tile group is not paired with itself: 5/4/4/5 tiles per SIMD.
constexpr int SP_WS = 32 * 320;                         // one kernel-row slice of 32 rows (bf16, 20 KB)
constexpr size_t SP_XIN = 0, SP_WS0 = (size_t)C2_XIN * 2, SP_LDS = SP_WS0 + 2 * (size_t)SP_WS * 2;
static_assert(SP_LDS <= 80 * 1024, "two split workgroups per CU");

// slice kh of Wg[32 rows][1600] -> LDS (physical chunk P = row*40 + (lc ^ (row & 7))), 20 x 1 KB DMAs
DEV void ws_dma32(const bf16* Wg, int kh, bf16* buf, int w, int lane) {
  for (int j = w; j < 20; j += SP_NT / 64) {
    const int P = j * 64 + lane, row = P / 40, pc = P - row * 40, lc = pc ^ (row & 7);
    __builtin_amdgcn_global_load_lds(Wg + row * 1600 + kh * 320 + lc * 8, (LDS_AS void*)(buf + j * 512), 16, 0, 0);
  }
}

template <int NPX>
DEV void split_core(const bf16* Wg, const bf16* xin, bf16* ws, f32x4 (&acc)[2][NPX], int pg, int kk, int g,
                    int li, int w, int lane, int tk) {
  int xo[NPX][8];
#pragma unroll
  for (int t = 0; t < NPX; ++t) {
    const int px = 16 * (pg + 4 * t) + li;
    const int y = px / 12, x = px - y * 12;
    const int pb = y * 16 + x, key0 = (x + 4 * y) & 7;
#pragma unroll
    for (int d = 0; d < 8; ++d) xo[t][d] = pb * 64 + (((4 * kk + g) ^ ((key0 + d) & 7)) << 3);
  }
  const int ao = li * 320 + (((4 * kk + g) ^ (li & 7)) << 3);
#pragma unroll
  for (int t = 0; t < NPX; ++t) { acc[0][t] = zero4(); acc[1][t] = zero4(); }
  auto load_chunk = [&](int kh, int kw, bf16x8& a0, bf16x8& a1, bf16x8 (&bx)[NPX]) {
    const bf16* wr = ws + (kh & 1) * SP_WS + kw * 64 + ao;
    a0 = lds_b128(wr);
    a1 = lds_b128(wr + 16 * 320);
#pragma unroll
    for (int t = 0; t < NPX; ++t) bx[t] = lds_b128(xin + xo[t][(kw + 4 * kh) & 7] + (kh * 16 + kw) * 64);
  };
  ws_dma32(Wg, 0, ws, w, lane);
  __syncthreads();                                       // slice 0 landed (vmcnt(0)), Xpad complete
  DMLC_STAMP(tk, 1);
#pragma unroll
  for (int kh = 0; kh < 5; ++kh) {
    if (kh < 4) ws_dma32(Wg, kh + 1, ws + ((kh + 1) & 1) * SP_WS, w, lane);
    bf16x8 A0[2], A1[2], BX[2][NPX];
    load_chunk(kh, 0, A0[0], A1[0], BX[0]);
#pragma unroll
    for (int kw = 0; kw < 5; ++kw) {
      const int cur = kw & 1;
      wait_lds();
      __builtin_amdgcn_sched_barrier(0);
      if (kw + 1 < 5) load_chunk(kh, kw + 1, A0[cur ^ 1], A1[cur ^ 1], BX[cur ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < NPX; ++t) {
        acc[0][t] = mfma16(A0[cur], BX[cur][t], acc[0][t]);
        acc[1][t] = mfma16(A1[cur], BX[cur][t], acc[1][t]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (kh < 4) __syncthreads();                         // next slice landed; this one fully read
  }
}

// Runs the core, adds the two K halves in fixed order (kk = 1 publishes through the slice buffer the
// last kernel row did not use) and calls fn(row_tile, px_tile, acc) on the kk = 0 waves.
template <class F>
DEV void split_tiles(const bf16* Wg, const bf16* xin, bf16* ws, int w, int g, int li, int lane, int tk, F&& fn) {
  const int kk = w >> 2, pg = (w + (w >> 2)) & 3;
  f32x4* red = reinterpret_cast<f32x4*>(ws + SP_WS);    // slice buffer 1: free after kernel row 3
  auto finish = [&](auto& acc, auto npx) {
    constexpr int NPX = decltype(npx)::value;
    if (kk == 1) {
#pragma unroll
      for (int t = 0; t < NPX; ++t)
#pragma unroll
        for (int c = 0; c < 2; ++c) red[((pg + 4 * t) * 2 + c) * 64 + lane] = acc[c][t];
    }
    lds_barrier();
    if (kk == 0) {
#pragma unroll
      for (int t = 0; t < NPX; ++t)
#pragma unroll
        for (int c = 0; c < 2; ++c) fn(c, pg + 4 * t, acc[c][t] + red[((pg + 4 * t) * 2 + c) * 64 + lane]);
    }
  };
  if (pg == 0) {
    f32x4 acc[2][3];
    split_core<3>(Wg, xin, ws, acc, pg, kk, g, li, w, lane, tk);
    finish(acc, std::integral_constant<int, 3>{});
  } else {
    f32x4 acc[2][2];
    split_core<2>(Wg, xin, ws, acc, pg, kk, g, li, w, lane, tk);
    finish(acc, std::integral_constant<int, 2>{});
  }
}
static_assert(9 * 2 * 64 * 16 <= SP_WS * 2, "K-half partials fit one slice buffer");

// pool2 / ReLU backward (-> dY2, all 64 channels in LDS; this block stores its 32 to global) + the conv2
// input gradient of 32 input channels of one image (S = 2 workgroups per image)
// IN_LAUNCH (the fc chain, B <= 128: its 2B workgroups run the dgrad of image b, half h once the
// chain's dp2 row tile is published -- as conv2_dgrad_image<true>): dp2 is read with sc1 loads after
// the seam; everything else was written by earlier launches.
template <bool IN_LAUNCH>
DEV void conv2_dgrad_split_image(const DmlcConv2DgradArgs& a, int b, int h, char* smem,
                                 Seam seam = Seam{nullptr, 0, 0u}, unsigned* err = nullptr) {
  bf16* dyp = reinterpret_cast<bf16*>(smem + SP_XIN);
  bf16* ws = reinterpret_cast<bf16*>(smem + SP_WS0);
  bf16* dp2 = ws + SP_WS;                                   // [36][64] in slice buffer 1 (free until
  uint8_t* am2 = reinterpret_cast<uint8_t*>(dp2 + 2304);    //  the slice-1 DMA, after the pool bwd)
  bf16* img = dyp;                                          // [144][32] dp1 slice, after the core
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id(), g = lane >> 4, li = lane & 15;
  DMLC_STAMP(DMLC_TK_DGRAD, 0);
  if (!IN_LAUNCH) stage16<288>(dp2, reinterpret_cast<const bf16*>(a.dp2) + (size_t)b * 2304, tid);
  stage16<144>(am2, a.am2 + (size_t)b * 2304, tid);
  for (int s = tid; s < 2048; s += SP_NT) {                 // halo of the padded 16x16 grad image
    const int pix = s >> 3, c = s & 7, r = pix >> 4, col = pix & 15;
    if (r < 2 || r >= 14 || col < 2 || col >= 14) *reinterpret_cast<bf16x8*>(dyp + swzpad(pix, c)) = bf16x8{};
  }
  if (IN_LAUNCH) {
    if (tid < 64) seam_wait(seam, tid, err, 2u);
    lds_barrier();
    if (tid < 288)
      reinterpret_cast<uint4*>(dp2)[tid] = __builtin_bit_cast(
          uint4, __builtin_amdgcn_raw_buffer_load_b128(buf_rsrc(a.dp2), (uint32_t)(b * 2304 + 8 * tid) * 2, 0, kSC1));
  }
  __syncthreads();
  bf16* dy2 = reinterpret_cast<bf16*>(a.dy2) + (size_t)b * 9216;
  if (tid < 36 * 8) {
    const int task = tid, win = task >> 3, c = task & 7, py = win / 6, px = win - py * 6;
    float o[4][8];
    pool_bwd_2x2<6>(dp2, am2, py, px, c, o);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int y = 2 * py + (k >> 1), x = 2 * px + (k & 1);
      const bf16x8 v = to_bf16x8(o[k]);
      *reinterpret_cast<bf16x8*>(dyp + swzpad((y + 2) * 16 + x + 2, c)) = v;
      if ((c >> 2) == h) st_out16(dy2, (uint32_t)((y * 12 + x) * 64 + c * 8) * 2, __builtin_bit_cast(uint4, v));
    }
  }
  lds_barrier();   // dyp published (dy2's global stores need not drain); dp2 / am2 reads done
  split_tiles(reinterpret_cast<const bf16*>(a.wd) + (size_t)32 * h * 1600, dyp, ws, w, g, li, lane, DMLC_TK_DGRAD,
              [&](int c, int t, const f32x4& acc) {
                const int px = 16 * t + li, cb = 16 * c + 4 * g;
                *reinterpret_cast<bf16x4*>(img + swzc<4>(px, cb >> 3) + ((cb >> 2) & 1) * 4) =
                    pack4(acc[0], acc[1], acc[2], acc[3]);
              });
  __syncthreads();
  DMLC_STAMP(DMLC_TK_DGRAD, 2);
  bf16* dp1 = reinterpret_cast<bf16*>(a.dp1) + (size_t)b * 9216 + 32 * h;
  for (int s = tid; s < 144 * 4; s += SP_NT) {
    const int p = s >> 2, c = s & 3;
    st_out16(dp1, (uint32_t)(p * 64 + c * 8) * 2, __builtin_bit_cast(uint4, lds_b128(img + swzc<4>(p, c))));
  }
  DMLC_STAMP(DMLC_TK_DGRAD, 3);
}

}  // namespace dmlc
