// conv2-shaped implicit-GEMM core (forward, dgrad) and the conv2 input gradient of one image, shared
// by the per-image conv kernels (cnn_conv.hip) and the fc chain launch, which runs the dgrad of its
// block's image once the chain's dp2 row tile is complete (cnn_fc.hip).
#pragma once
#include "w1_common.h"

namespace dmlc {

// ---------------------------------------------------------------------------------------------
// conv2-shaped implicit GEMM core shared by forward and dgrad:
//   C[c_out][px] = sum_{kh,kw,c_in} Wt[c_out][(kh*5+kw)*64 + c_in] * Xpad[(y+kh)*16 + x+kw][c_in]
// Xpad: LDS [16*16][64] bf16 (swizzled), wave w -> c_out tile 16w, 9 pixel tiles of 16.

// conv2-shaped implicit GEMM core, weights staged through LDS.
// The 64 x 1600 weight matrix is consumed one kh slice (64 co x 320 k, 40 KB) at a time.  Each slice
// is copied global -> LDS by LDS-DMA (global_load_lds_dwordx4: 40 wave-instructions of 1 KB, 5 per
// wave, no registers), issued for slice kh+1 into the other buffer before slice kh's MFMAs and
// waited for at the end of the slice -- the copy is hidden behind the MFMAs.  (Register-staged, the
// compiler sank the loads down to their LDS stores -- one exposed L2 latency per slice -- and pinning
// them spilled the staging registers to scratch.)  Every weight byte crosses L2 -> CU once per block.
// Rows are 640 B with the 16-B chunks XOR-swizzled by (row & 7), which keeps the A-fragment reads
// (16 co rows x 4 chunks per ds_read_b128) conflict-free.
// Tile ownership: see conv2_core below (per k-chunk a wave reads 2 A and 2-3 B fragments,
// ds_read_b128, conflict-free, for 4-5 MFMAs).
constexpr int WS_ELEMS = 64 * 320;            // one slice, bf16
constexpr size_t WS_BYTES = 2 * WS_ELEMS * 2;

// slice kh of W[64 co][1600] -> LDS slice buffer (physical chunk P = row*40 + (lc ^ (row & 7)))
DEV void ws_dma(const bf16* Wg, int kh, bf16* buf, int w, int lane) {
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int j = w * 5 + i;                            // wave-uniform: 1 KB of LDS per instruction
    const int P = j * 64 + lane, row = P / 40, pc = P - row * 40, lc = pc ^ (row & 7);
    __builtin_amdgcn_global_load_lds(Wg + row * 1600 + kh * 320 + lc * 8, (LDS_AS void*)(buf + j * 512), 16, 0, 0);
  }
}

// s0: where kernel row 0 of the weights already sits (the caller issued its LDS-DMA at kernel entry,
// so its latency hides behind the staging instead of opening the core), or null: the core copies it
// into ws.  Rows 1..4 alternate between the two ws buffers (row kh in buffer kh & 1).
DEV const bf16* slice_buf(const bf16* s0, const bf16* ws, int kh) { return kh == 0 ? s0 : ws + (kh & 1) * WS_ELEMS; }

// The same copy through registers: the loads can be issued long before the LDS is free (kernel entry)
// and stored once it is.  (An early LDS-DMA instead makes hipcc wait vmcnt(0) before every later LDS
// read it cannot prove disjoint -- e.g. each pool iteration -- and its waits stop counting in order.)
// (named members, passed by value: as an array hipcc kept the five chunks in scratch)
struct Slice5 { uint4 a, b, c, d, e; };
DEV uint4 ws_chunk(const bf16* Wg, int kh, int w, int lane, int i) {
  const int P = (w * 5 + i) * 64 + lane, row = P / 40, pc = P - row * 40, lc = pc ^ (row & 7);
  return *reinterpret_cast<const uint4*>(Wg + row * 1600 + kh * 320 + lc * 8);
}
DEV Slice5 ws_fetch(const bf16* Wg, int kh, int w, int lane) {
  return Slice5{ws_chunk(Wg, kh, w, lane, 0), ws_chunk(Wg, kh, w, lane, 1), ws_chunk(Wg, kh, w, lane, 2),
                ws_chunk(Wg, kh, w, lane, 3), ws_chunk(Wg, kh, w, lane, 4)};
}
DEV void ws_put(bf16* buf, int w, int lane, Slice5 v) {
  uint4* p = reinterpret_cast<uint4*>(buf) + w * 5 * 64 + lane;
  p[0] = v.a; p[64] = v.b; p[128] = v.c; p[192] = v.d; p[256] = v.e;
}

// Tile ownership (r5): wave w = (cp, pg), cp = w & 1, pg = w >> 1, owns c_out tiles 2cp, 2cp+1 of the
// pixel tiles pg and pg+4 (4 tile-units of 50 k-chunks each), and waves 0-3 also pixel tile 8 for
// ONE c_out tile, 2cp + pg (EXTRA: 5 units).  Waves w and w+4 share a SIMD, so every SIMD carries 9
// of the 36 units -- the earlier 2-3 pixel tiles x 2 c_out tiles per wave put 10 on two SIMDs and 8
// on the other two.  Every output tile is still summed by one wave in the same k order, so the
// results are bit-identical to that tiling.
template <bool EXTRA>
DEV void conv2_core(const bf16* Wg, const bf16* xin, bf16* ws, f32x4 (&acc)[2][2], f32x4& accx, int pg, int cp,
                    int xsel, int g, int li, int tid, const bf16* s0, int tk = -1) {
  constexpr int NPX = EXTRA ? 3 : 2;
  const int w = wave_id(), lane = tid & 63, sw = li & 7;
  // Per-lane LDS element offsets, computed once: every fragment read of the loop is then one
  // ds_read_b128 at (offset register + compile-time immediate), no per-chunk address VALU (the swizzle
  // arithmetic had made this loop VALU-issue-bound: ~3 integer ops per MFMA).
  //  * B (input image, swzpad layout): tile t's pixel for tap (kh, kw) is pb[t] + 16 kh + kw and its
  //    XOR key is (key0 + kw + 4 kh) & 7 (no carry out of the 16-wide row: x + kw <= 15), so the
  //    lane's offset is xo[t][d][s] + (16 kh + kw) * 64 with d = (kw + 4 kh) & 7;
  //  * A (weight slice, chunk c ^ (row & 7)): kw * 64 + ao[s].
  int xo[NPX][8][2];
#pragma unroll
  for (int t = 0; t < NPX; ++t) {
    const int px = 16 * (t < 2 ? pg + 4 * t : 8) + li;
    const int y = px / 12, x = px - y * 12;
    const int pb = y * 16 + x, key0 = (x + 4 * y) & 7;
#pragma unroll
    for (int d = 0; d < 8; ++d)
#pragma unroll
      for (int s = 0; s < 2; ++s) xo[t][d][s] = pb * 64 + (((4 * s + g) ^ ((key0 + d) & 7)) << 3);
  }
  int ao[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) ao[s] = (32 * cp + li) * 320 + (((4 * s + g) ^ sw) << 3);
#pragma unroll
  for (int t = 0; t < 2; ++t) { acc[0][t] = zero4(); acc[1][t] = zero4(); }
  accx = zero4();
  if (!s0) ws_dma(Wg, 0, ws, w, lane);
  const bf16* sb0 = s0 ? s0 : ws;
  __syncthreads();                                       // (waits vmcnt(0): the DMA has landed)
  // One k-chunk (kw, s) = 2 A + NPX B fragments.  The fragments of chunk j+1 are read into the other
  // register set BEFORE chunk j's MFMAs issue, so the LDS latency of a chunk hides behind the previous
  // chunk's MFMAs (lgkmcnt waits for the older reads only) instead of one exposed latency per chunk.
  auto load_chunk = [&](int kh, int j, bf16x8& a0, bf16x8& a1, bf16x8 (&bx)[NPX]) {
    const int kw = j >> 1, s = j & 1;
    const bf16* wr = slice_buf(sb0, ws, kh) + kw * 64 + ao[s];
    a0 = lds_b128(wr);
    a1 = lds_b128(wr + 16 * 320);
#pragma unroll
    for (int t = 0; t < NPX; ++t) bx[t] = lds_b128(xin + xo[t][(kw + 4 * kh) & 7][s] + (kh * 16 + kw) * 64);
  };
#pragma unroll
  for (int kh = 0; kh < 5; ++kh) {
    if (kh < 4) ws_dma(Wg, kh + 1, ws + ((kh + 1) & 1) * WS_ELEMS, w, lane);   // buffer freed by the last barrier
    bf16x8 A0[2], A1[2], BX[2][NPX];
    load_chunk(kh, 0, A0[0], A1[0], BX[0]);
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const int cur = j & 1;
      // chunk j's reads (issued one chunk ago) complete; then chunk j+1's reads go out ahead of chunk
      // j's MFMAs (sched barriers keep the scheduler from sinking them back next to their use)
      wait_lds();
      __builtin_amdgcn_sched_barrier(0);
      if (j + 1 < 10) load_chunk(kh, j + 1, A0[cur ^ 1], A1[cur ^ 1], BX[cur ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        acc[0][t] = mfma16(A0[cur], BX[cur][t], acc[0][t]);
        acc[1][t] = mfma16(A1[cur], BX[cur][t], acc[1][t]);
      }
      if constexpr (EXTRA) accx = mfma16(xsel ? A1[cur] : A0[cur], BX[cur][NPX - 1], accx);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (kh < 4) __syncthreads();                         // next slice landed; this one fully read
    if (tk >= 0 && (kh == 0 || kh == 2)) DMLC_STAMP(tk, 5 + kh / 2);
  }
  if (tk >= 0) DMLC_STAMP(tk, 7);
}

// fn(co_tile, px_tile, acc) for every finished 16x16 output tile (called by the wave that owns it).
// (A 4-c_out-tile-per-wave variant with a K split measured 0.8-1.3 % slower per step in r3: the core
// is not bound by its LDS read bandwidth; removed in r5.)
template <class F>
DEV void conv2_tiles(const bf16* Wg, const bf16* xin, bf16* ws, int w, int g, int li, int tid, const bf16* s0,
                     F&& fn, int tk = -1) {
  const int cp = w & 1, pg = w >> 1;
  f32x4 acc[2][2], accx;
  if (w < 4) {
    conv2_core<true>(Wg, xin, ws, acc, accx, pg, cp, pg, g, li, tid, s0, tk);
    fn(2 * cp + pg, 8, accx);
  } else {
    conv2_core<false>(Wg, xin, ws, acc, accx, pg, cp, 0, g, li, tid, s0, tk);
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) { fn(2 * cp, pg + 4 * t, acc[0][t]); fn(2 * cp + 1, pg + 4 * t, acc[1][t]); }
}

// conv2 input gradient of image b: pool2/ReLU backward (gather over the 2x2 ownership windows) into
// the zero-padded LDS image, then the conv2-shaped core with the flipped weights, dY2 and dP1 out.
// LDS: [conv2 input | outputs | dp2 | argmax2 | weight slices], (C2_XIN + C2_OUT) * 2 + 2304 * 3 + WS_BYTES.
// IN_LAUNCH: dp2 is produced by other workgroups of the same launch (the fc chain's dp2 tiles, sc1
// stores + a per-row-tile counter): everything that does not depend on it (argmax, kernel row 0 of
// the weights, the halo) is issued first, then one lane waits for the counter (bounded, sticky error
// word) and dp2 is read with sc1 loads (another XCD's L2 may hold a stale copy of those lines).
constexpr size_t DG_LDS = (C2_XIN + C2_OUT) * 2 + 2304 * 3 + WS_BYTES;

template <bool IN_LAUNCH>
DEV void conv2_dgrad_image(const DmlcConv2DgradArgs& a, int b, char* smem, Seam seam = Seam{nullptr, 0, 0u},
                           unsigned* err = nullptr) {
  bf16* dyp = reinterpret_cast<bf16*>(smem);
  bf16* outs = dyp + C2_XIN;
  bf16* dp2 = outs + C2_OUT;                                    // [36][64] staged pool2 grad
  uint8_t* am2 = reinterpret_cast<uint8_t*>(dp2 + 2304);        // [36][64] staged argmax
  bf16* ws = reinterpret_cast<bf16*>(am2 + 2304);               // weight slices (conv2_core)
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int g = lane >> 4, li = lane & 15;
  DMLC_STAMP(DMLC_TK_DGRAD, 0);
  if (!IN_LAUNCH) stage16<288>(dp2, reinterpret_cast<const bf16*>(a.dp2) + (size_t)b * 2304, tid);
  stage16<144>(am2, a.am2 + (size_t)b * 2304, tid);
  // kernel row 0 of the weights into registers: in flight during the pool backward (see ws_fetch)
  const Slice5 s0v = ws_fetch(reinterpret_cast<const bf16*>(a.wd), 0, w, lane);
  bf16* dy2 = reinterpret_cast<bf16*>(a.dy2) + (size_t)b * 9216;

  // halo of the padded 16x16 grad image
  for (int s = tid; s < 2048; s += NT) {
    const int pix = s >> 3, c = s & 7;
    const int r = pix >> 4, col = pix & 15;
    if (r < 2 || r >= 14 || col < 2 || col >= 14) *reinterpret_cast<bf16x8*>(dyp + swzpad(pix, c)) = bf16x8{};
  }
  if (IN_LAUNCH) {
    if (tid < 64) seam_wait(seam, tid, err, 2u);
    lds_barrier();
    if (tid < 288)
      reinterpret_cast<uint4*>(dp2)[tid] = __builtin_bit_cast(
          uint4, __builtin_amdgcn_raw_buffer_load_b128(buf_rsrc(a.dp2), (uint32_t)(b * 2304 + 8 * tid) * 2, 0, kSC1));
  }
  lds_barrier();   // (not __syncthreads: its vmcnt(0) would wait for the row-0 loads right here)
  DMLC_STAMP(DMLC_TK_DGRAD, 1);
  static_assert(36 * 8 <= NT, "one pool-bwd task per thread");
  const int win = tid >> 3, pc = tid & 7, py = win / 6, px = win - py * 6;
  bf16x8 dv[4];
  if (tid < 36 * 8) {
    float o[4][8];
    pool_bwd_2x2<6>(dp2, am2, py, px, pc, o);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int y = 2 * py + (k >> 1), x = 2 * px + (k & 1);
      dv[k] = to_bf16x8(o[k]);
      *reinterpret_cast<bf16x8*>(dyp + swzpad((y + 2) * 16 + x + 2, pc)) = dv[k];
    }
  }
  // kernel row 0 into its slice buffer BEFORE the dy2 stores go out: the wait for the row-0 loads
  // then cannot include them (a store in one branch of a join makes hipcc wait vmcnt(0))
  ws_put(ws, w, lane, s0v);                        // published by the core's first barrier
  if (tid < 36 * 8) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int y = 2 * py + (k >> 1), x = 2 * px + (k & 1);
      st_out16(dy2, (uint32_t)((y * 12 + x) * 64 + pc * 8) * 2, __builtin_bit_cast(uint4, dv[k]));
    }
  }
  lds_barrier();   // publishes dyp only; the dy2 global stores need not drain here
  DMLC_STAMP(DMLC_TK_DGRAD, 2);

  conv2_tiles(reinterpret_cast<const bf16*>(a.wd), dyp, ws, w, g, li, tid, ws, [&](int ct, int t, const f32x4& acc) {
    const int px = 16 * t + li, cb = 16 * ct + 4 * g;
    const bf16x4 v = pack4(acc[0], acc[1], acc[2], acc[3]);
    *reinterpret_cast<bf16x4*>(outs + swz128(px, cb >> 3) + ((cb >> 2) & 1) * 4) = v;
  });
  __syncthreads();
  DMLC_STAMP(DMLC_TK_DGRAD, 3);
  bf16* dp1 = reinterpret_cast<bf16*>(a.dp1) + (size_t)b * 9216;
  for (int s = tid; s < 1152; s += NT) {
    const int p = s >> 3, c = s & 7;
    st_out16(dp1, (uint32_t)(p * 64 + c * 8) * 2, __builtin_bit_cast(uint4, lds_b128(outs + swz128(p, c))));
  }
  DMLC_STAMP(DMLC_TK_DGRAD, 4);
}

}  // namespace dmlc
