// Weight gradients of the two convolutions (TF Conv2DBackpropFilter + BiasAddGrad of
// /root/reference/cifar10cnn.py:107/:118 via the autodiff of :163; SURVEY.md §2.B N5/N7, §2.C
// conv5x5_wgrad).  Results are fp32 split-K partial slabs, one per image group, reduced in fixed order
// by the SGD kernel.
//
//   conv1  dW1[k''][co] = sum_{b,px} X[b,px][k''] dY1[b,px][co],  k'' = kh*16 + kw*3 + ci
//     one 8-wave block per image group (w1_common.h): dY1 is scattered in LDS from the pool1 gradient
//     and argmax bytes, which every thread loads straight into registers for exactly the (window,
//     chunk) tasks it scatters (no LDS staging); X as 15 column-shifted channel planes.
//   conv2  dW2[(kh,kw,ci)][co] = sum_{b,px} Xpad[b][px+(kh,kw)][ci] dY2[b,px][co]
//     one 8-wave block per (ci quarter, image group): per image it loads the group's dY2 (18 KB) and
//     only ITS 16 input channels of the conv2 input (4.6 KB) -- 23 KB per image per block where a
//     (kh, group) partition moved 37 KB (five kernel-row blocks each re-reading dY2 and 12 input rows):
//     the per-CU load rate, not the MFMA, bounded that layout.  Wave w owns taps 3w..3w+2 x the 4 co
//     tiles (12 accumulators) and waves 0-3 also tap 24 x co tile w: 25 MFMAs per k-step on every SIMD.
// Both: the NEXT image's global data is prefetched into registers while the current image computes.
#include "w1_common.h"
#include "sgd_common.h"
#include "fc_common.h"

namespace dmlc {

// ---------------------------------------------------------------------------------------------
// dY1 | shifted planes | pool1 grad (bf16) | raw uint8 image [32][32][3] | argmax bytes
constexpr size_t W1_LDS = (size_t)(W1_DYT + W1_XS + 9216) * 2 + 3072 + 9216;
static_assert(W1_FL_BYTES <= (W1_DYT + W1_XS) * 2, "flush buffer over dY1 + planes");

DEV void conv1_wgrad_block(const DmlcConv1WgradArgs& a, const int grp, char* smem, bool coh = false) {
  bf16* dyt = reinterpret_cast<bf16*>(smem);
  bf16* xs = dyt + W1_DYT;
  bf16* dps = xs + W1_XS;
  uint8_t* img = reinterpret_cast<uint8_t*>(dps + 9216);
  uint8_t* ams = img + 3072;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int g = lane >> 4, li = lane & 15;
  const int ch = w & 1, ks = w >> 1;                     // MFMA: co tiles 2ch, 2ch+1; k-steps ks mod 4
  // image group grp = images grp, grp + g1, ...: with g1 % 8 == 0 all of them were produced on this
  // block's XCD (blockIdx % 8) by the forward / dgrad blocks of the same index (placement is a
  // speed matter only)
  const int G = a.g1, b0 = grp, last = grp < a.B ? grp + (a.B - 1 - grp) / G * G : grp;
  DMLC_STAMP(DMLC_TK_W1, 0);

  w1_ones_plane15(xs, tid);

  f32x4 acc[2][5];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int t = 0; t < 5; ++t) acc[h][t] = zero4();

  // Every load below is unconditional (image indices clamped to the block's last image, surplus
  // threads duplicating chunks): see PrefetchAll.  The dataset row of image b+1 is read one image
  // ahead of its pixels, so no index -> pixels dependency is exposed inside the loop.
  // Per thread: 1 chunk of the whole uint8 image (3072 B = 192 chunks, 16-B aligned dataset rows),
  // 3 of the pool1 gradient (1152), 2 of the argmax bytes (576).  Named registers, not member
  // arrays: with the arrays in a struct hipcc kept them in scratch.
  const int cI = tid % 192, cD2 = 1024 + (tid & 127), cA1 = 512 + (tid & 63);
  uint4 vI, vD0, vD1, vD2, vA0, vA1;
  auto load = [&](int idx, int bb) {
    const uint4* si = reinterpret_cast<const uint4*>(a.xraw ? a.xraw + (size_t)bb * 3072 : a.data + (size_t)idx * 3072);
    const uint4* sd = reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.dp1) + (size_t)bb * 9216);
    const uint4* sa = reinterpret_cast<const uint4*>(a.am1 + (size_t)bb * 9216);
    vI = si[cI];
    vD0 = sd[tid]; vD1 = sd[tid + 512]; vD2 = sd[cD2];
    vA0 = sa[tid]; vA1 = sa[cA1];
  };
  // with the forward's image copy (xraw) no dataset index is needed at all
  auto row_index = [&](int bb) { return a.xraw ? 0 : batch_index(a.src, a.B, bb); };
  load(row_index(b0 < last ? b0 : last), b0 < last ? b0 : last);
  int nidx = row_index(b0 + G < last ? b0 + G : last);
  for (int b = b0; b < a.B; b += G) {
    lds_barrier();                             // previous image's MFMA reads are done
    reinterpret_cast<uint4*>(img)[cI] = vI;
    reinterpret_cast<uint4*>(dps)[tid] = vD0;
    reinterpret_cast<uint4*>(dps)[tid + 512] = vD1;
    reinterpret_cast<uint4*>(dps)[cD2] = vD2;
    reinterpret_cast<uint4*>(ams)[tid] = vA0;
    reinterpret_cast<uint4*>(ams)[cA1] = vA1;
    w1_zero_dy(dyt, tid);
    load(nidx, b + G < last ? b + G : last);   // prefetch the next image while this one computes
    nidx = row_index(b + 2 * G < last ? b + 2 * G : last);
    lds_barrier();
    if (b == b0) DMLC_STAMP(DMLC_TK_W1, 1);
    if (b == b0 + G) DMLC_STAMP(DMLC_TK_W1, 6);
    w1_planes(xs, img, a.cy, a.cx, tid);
    w1_pool_bwd(dyt, dps, ams, w, lane);       // ends with a barrier: dY1 and the planes complete
    if (b == b0) DMLC_STAMP(DMLC_TK_W1, 2);
    if (b == b0 + G) DMLC_STAMP(DMLC_TK_W1, 7);
    w1_mfma(dyt, xs, acc, ks, ch, g, li);
    if (b == b0) DMLC_STAMP(DMLC_TK_W1, 5);
  }
  __syncthreads();
  DMLC_STAMP(DMLC_TK_W1, 3);
  w1_flush(smem, acc, a.part1 + (size_t)grp * 80 * 64, a.partb1 + grp * 64, ks, ch, lane, tid, coh);
  DMLC_STAMP(DMLC_TK_W1, 4);
}

// ---------------------------------------------------------------------------------------------
constexpr int W2T = 512;
// dY rows: 128 B with the 16-column tiles XOR-swizzled by row bits 1 and 3 -- the tr reads of rows
// {r..r+3, r+8..r+11} land on 8 distinct bank windows (a 144-B row stride left them 2-way)
constexpr int W2_LD = 64;
DEV int w2_dy_col(int row, int col) { return col ^ (16 * (((row >> 1) & 1) | ((row >> 2) & 2))); }
constexpr int W2_DY = 160 * W2_LD;             // 144 pixels + 16 zero rows
constexpr int W2_LDX = 16;                     // conv2 input: 16 channels per padded pixel, 32-B rows
constexpr int W2_XT = 256 * W2_LDX;            // the padded 16x16 image (halo 2)
constexpr int W2_ST = 68;                      // epilogue staging rows (floats): conflict-free writes
constexpr size_t W2_LDS_MAIN = (size_t)(W2_XT + W2_DY) * 2;
constexpr size_t W2_LDS_ST = (size_t)(W2T / 64) * 16 * W2_ST * 4;
constexpr size_t W2_LDS = W2_LDS_MAIN > W2_LDS_ST ? W2_LDS_MAIN : W2_LDS_ST;

// Block blk (base + blk = blockIdx.x) -> (c4, group): input channels 16*c4 .. 16*c4+15 of image group
// `group` = images group, group + g2, ...; fills rows (tap, 16*c4 .. 16*c4+15) of slab `group` (the
// 4 blocks of a group write disjoint quarters).  With g2 % 8 == 0 and base % 8 == 0 the 4 blocks of a
// group sit on one XCD (blockIdx % 8), the one whose dgrad / forward blocks wrote the group's dY2 and
// input (placement is a speed matter only).  (Double-buffering the image operands in LDS, with or
// without reading k-step s+1's fragments under k-step s's MFMAs, measured 0.3-1 us slower.)
DEV void w2_block_pos(const DmlcConv2WgradArgs& a, int blk, int base, int& c4, int& grp) {
  const bool xcd = a.g2 % 8 == 0 && base % 8 == 0;
  c4 = xcd ? (blk >> 3) & 3 : blk & 3;
  grp = xcd ? (blk & 7) + 8 * (blk >> 5) : blk >> 2;
}

// ---------------------------------------------------------------------------------------------
// fp8 conv2 weight gradient (BASELINE config 5; a.x8 set): the same blocks, accumulators and epilogue
// as the bf16 body below, with the MFMA on v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3: twice the
// bf16 rate per clock) over the e4m3 operands the producers already quantised -- X by the fp8 forward
// (per-batch scale sx), dY2 by the fp8 dgrad (a power-of-two scale per image) -- so the staging is a
// plain copy of half the bf16 bytes.
//   * K = output pixels of a UNIT of two images, each laid out as a 12 x 16 grid whose columns 12..15
//     carry dY = 0: a 16-wide K row makes every tap's input rows a LINEAR shift of the output rows
//     (padded pixel = k + 16 kh + kw), and 2 x 192 = 384 = three K chunks of 128;
//   * dY's per-image scale rides on the MFMA's E8M0 block scales: lane l's scale byte covers K rows
//     {0..15, 32..47} + 64 ((l >> 4) & 1) + 16 (l >> 5) of the chunk (tools/probes/mx_scale_probe.hip),
//     so a block never straddles the image boundary at row 192; acc / sx at the end;
//   * the conv2 bias gradient from the same dY bytes: one extra MFMA against an all-ones A per chunk
//     on waves 4-7 of the c4 == 0 blocks (they carry one MFMA less than waves 0-3);
//   * fragments by ds_read_b64_tr_b8 (lane 2q+p addresses row q, bytes 8p..; lane i receives column i
//     of the 8-row x 16-byte block -- tools/probes/fp8_wgrad_probe.hip).  Lane group g's four reads
//     j take the 8-row K segments g + 4j (the MFMA's K order only has to agree between A and B): the
//     two groups of a half-wave then read rows 8 apart, so the 16-B X rows are conflict-free as they
//     stand and the 64-B dY rows need only an XOR of the 16-B co tile with row bits 2 and 3 -- both
//     per-lane constants, as is the image of every read (the boundary at row 192 falls between reads
//     j = 1 and 2 of chunk 1): every fragment address is a lane base + an immediate offset.  LDS is
//     double-buffered per unit, the next unit's 16-B chunks in registers under this unit's MFMAs; one
//     barrier per unit.
typedef int w8x32 __attribute__((ext_vector_type(8)));
typedef int w8x2 __attribute__((ext_vector_type(2)));
constexpr int W8_XROWS = 272;                  // padded 16 x 16 input grid + 16 zero rows (garbage-column reads)
constexpr int W8_XIMG = W8_XROWS * 16;         // bytes per image: [row][16 ci] e4m3
constexpr int W8_YIMG = 192 * 64;              // [12 x 16 output grid][64 co] e4m3
constexpr int W8_XU = 2 * W8_XIMG, W8_BUF = 2 * (W8_XIMG + W8_YIMG);
constexpr size_t W8_LDS = 2 * (size_t)W8_BUF + 64 * 4;   // double buffer + the bias tile
DEV int w8_ychunk(int r, int ct) { return ct ^ (((r >> 2) & 1) | (((r >> 3) & 1) << 1)); }
DEV w8x2 tr8(const uint8_t* p) { return __builtin_amdgcn_ds_read_tr8_b64_v2i32((LDS_AS w8x2*)(p)); }
DEV f32x4 mfma8(const w8x32& a, const w8x32& b, const f32x4& c, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, sb);
}

DEV void w2_fp8_main(const DmlcConv2WgradArgs& a, int c4, int grp, char* smem, f32x4 (&acc)[13], float (&bsum)[8]) {
  uint8_t* lds = reinterpret_cast<uint8_t*>(smem);
  float* btile = reinterpret_cast<float*>(smem + 2 * W8_BUF);
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int g = lane >> 4, q = (lane & 15) >> 1, p = lane & 1, half = (lane >> 4) & 1;
  const int G = a.g2, nimg = grp < a.B ? (a.B - 1 - grp) / G + 1 : 0, nunits = (nimg + 1) >> 1;
  const bool bias = c4 == 0 && w >= 4;         // wave 4 + ct: the bias gradient of co tile ct
  // zero both buffers once: halo / slack X rows and dY columns 12..15 are never written again
  for (int i = tid; i < 2 * W8_BUF / 16; i += W2T) reinterpret_cast<uint4*>(lds)[i] = make_uint4(0u, 0u, 0u, 0u);

  // staging map (16-B chunks): X chunk s < 288 (image s / 144, pixel s % 144: this quarter's 16 ci),
  // thread s = tid; dY chunk s < 1152 (image s / 576, pixel (s % 576) >> 2, co tile s & 3), s = tid +
  // 512 m for m < 3 (the last for tid < 128)
  uint4 vx, vy[3];
  float syv[2];                                // the unit's two dY scales (prefetched with its chunks)
  int ey[2];                                   // ... as E8M0 block scales, 127 - log2 sy
  auto img_of = [&](int u, int i) { return grp + G * (2 * u + i); };
  auto load = [&](int u, uint4& vx, uint4 (&vy)[3], float (&syv)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int b = img_of(u, i);
      syv[i] = load_sel(a.sy_img + b, a.sy_img, b < a.B);
    }
    {
      const int i = tid >= 144, px = tid - 144 * i, b = img_of(u, i);
      vx = load_sel(reinterpret_cast<const uint4*>(a.x8 + ((size_t)b * 144 + px) * 64 + 16 * c4),
                    reinterpret_cast<const uint4*>(a.x8), tid < 288 && b < a.B);
    }
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      const int s = tid + 512 * m, i = s >= 576, k = s - 576 * i, b = img_of(u, i);
      vy[m] = load_sel(reinterpret_cast<const uint4*>(a.y8 + ((size_t)b * 144 + (k >> 2)) * 64 + 16 * (k & 3)),
                       reinterpret_cast<const uint4*>(a.y8), (m < 2 || tid < 128) && b < a.B);
    }
  };
  auto store = [&](int buf, const uint4& vx, const uint4 (&vy)[3]) __attribute__((always_inline)) {
    uint8_t* X8 = lds + buf * W8_BUF;
    uint8_t* Y8 = X8 + W8_XU;
    if (tid < 288) {
      const int i = tid >= 144, px = tid - 144 * i, y = px / 12, x = px - 12 * y;
      *reinterpret_cast<uint4*>(X8 + i * W8_XIMG + ((y + 2) * 16 + x + 2) * 16) = vx;
    }
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      if (m == 2 && tid >= 128) break;
      const int s = tid + 512 * m, i = s >= 576, k = s - 576 * i, px = k >> 2, y = px / 12, x = px - 12 * y;
      const int r = i * 192 + y * 16 + x;
      *reinterpret_cast<uint4*>(Y8 + r * 64 + 16 * w8_ychunk(r, k & 3)) = vy[m];
    }
  };
  auto scales = [&](const float (&syv)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) ey[i] = syv[i] > 0.f ? 127 - (int)log2f(syv[i]) : 127;   // (exact powers of two)
  };
  // fragment bases: dY row (8 g + q) of chunk 0, tile ct (swizzle f = row bits 2, 3: per lane); X row
  // (8 g + q) + the wave's tap offsets (16 kh + kw rows); chunk c, read j, image 1 by immediates
  const int f = ((q >> 2) & 1) | ((g & 1) << 1);
  const int yl = (8 * g + q) * 64 + 8 * p, xl = (8 * g + q) * 16 + 8 * p;
  int xt[4];
#pragma unroll
  for (int t = 0; t < 3; ++t) xt[t] = xl + ((3 * w + t) / 5 * 16 + (3 * w + t) % 5) * 16;
  xt[3] = xl + (4 * 16 + 4) * 16;
  const w8x32 ones = {0x38383838, 0x38383838, 0x38383838, 0x38383838,   // e4m3 1.0
                      0x38383838, 0x38383838, 0x38383838, 0x38383838};
  f32x4 accb = zero4();
  __syncthreads();                             // the zeroing is done before any staging store
  // (loads two units ahead -- a second register set -- spill at this kernel's register budget)
  if (nunits > 0) load(0, vx, vy, syv);
  for (int u = 0; u < nunits; ++u) {
    const int buf = u & 1;
    store(buf, vx, vy);                        // (buffer buf was last read two units ago)
    scales(syv);
    if (u + 1 < nunits) load(u + 1, vx, vy, syv);   // the next unit's operands in flight under the MFMAs
    lds_barrier();
    if (u == 0) DMLC_STAMP(DMLC_TK_W2, 1);
    const uint8_t* Y8 = lds + buf * W8_BUF + W8_XU + yl;
    const uint8_t* X8 = lds + buf * W8_BUF;
    // chunk c's fragments: rows 128 c + 8 g + 32 j + q; image 1 for c == 2 and for j >= 2 of c == 1
    // (one set of fragments: a second set for a read-ahead spills -- the partner wave of the SIMD
    // covers this wave's read latency with its MFMAs)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      w8x32 bf[4], af[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int img = c == 2 || (c == 1 && j >= 2);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const w8x2 v = tr8(Y8 + 16 * (ct ^ f) + c * 8192 + j * 2048);
          bf[ct][2 * j] = v.x; bf[ct][2 * j + 1] = v.y;
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (t == 3 && w >= 4) break;
          const w8x2 v = tr8(X8 + xt[t] + c * 2048 + j * 512 + img * (W8_XIMG - 192 * 16));
          af[t][2 * j] = v.x; af[t][2 * j + 1] = v.y;
        }
      }
      // this lane's dY block scale: its block is image 1 for c == 2, and for the upper half-wave's
      // blocks (reads j >= 2) of c == 1
      const int sb = c == 0 ? ey[0] : c == 2 ? ey[1] : lane >= 32 ? ey[1] : ey[0];
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[4 * t + ct] = mfma8(af[t], bf[ct], acc[4 * t + ct], sb);
      if (w < 4) {
        const w8x32 bw = w == 0 ? bf[0] : w == 1 ? bf[1] : w == 2 ? bf[2] : bf[3];
        acc[12] = mfma8(af[3], bw, acc[12], sb);
      } else if (bias) {
        const w8x32 bw = w == 4 ? bf[0] : w == 5 ? bf[1] : w == 6 ? bf[2] : bf[3];
        accb = mfma8(ones, bw, accb, sb);
      }
    }
    if (u == 0) DMLC_STAMP(DMLC_TK_W2, 4);
  }
  const float inv = 1.f / a.sx[0];
#pragma unroll
  for (int j = 0; j < 13; ++j) acc[j] *= inv;
  // the bias tile (row 0 of the ones product: lanes 0..15) -> bsum of threads 0..7 in the layout
  // block_chunk_sum reduces (thread t < 8, j: channel 8 t + j; every other thread 0)
  __syncthreads();                             // every MFMA read of LDS is done
  if (bias && lane < 16) btile[16 * (w - 4) + lane] = accb[0];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum[j] = c4 == 0 && tid < 8 ? btile[8 * tid + j] : 0.f;
}

// coh: the slabs and bias partials are reduced by other blocks of the same launch (apply mode):
// agent-coherent stores instead of streaming ones
DEV void conv2_wgrad_block(const DmlcConv2WgradArgs& a, const int blk, const int base, char* smem, bool coh = false) {
  bf16* xt = reinterpret_cast<bf16*>(smem);
  bf16* dyt = xt + W2_XT;
  const int tid = threadIdx.x, lane = tid & 63, w = wave_id();
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  int c4, grp;
  w2_block_pos(a, blk, base, c4, grp);
  const int G = a.g2, b0 = grp, last = grp < a.B ? grp + (a.B - 1 - grp) / G * G : grp;
  DMLC_STAMP(DMLC_TK_W2, 0);

  f32x4 acc[13];
#pragma unroll
  for (int j = 0; j < 13; ++j) acc[j] = zero4();
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // conv2 bias grad (c4 == 0 blocks)
  if (a.x8) {
    w2_fp8_main(a, c4, grp, smem, acc, bsum);
  } else {
  // zero the whole padded input once (the interior is overwritten per image) and the 16 pad dY rows
  *reinterpret_cast<bf16x8*>(xt + tid * 8) = bf16x8{};
  if (tid < 128) *reinterpret_cast<bf16x8*>(dyt + (144 + (tid >> 3)) * W2_LD + (tid & 7) * 8) = bf16x8{};

  // prefetch per image: 1 chunk of this quarter's input (288 chunks: pixel k >> 1, half k & 1;
  // threads >= 288 duplicate chunks of lower threads) and 3 of dY (1152 chunks; in the third,
  // threads >= 128 duplicate those of threads 0..127).  No predicate on any load or store.
  const int kx = tid % 288, pxl = kx >> 1, xy = pxl / 12;
  bf16* xdst = xt + ((xy + 2) * 16 + pxl - xy * 12 + 2) * W2_LDX + 8 * (kx & 1);
  const int kd[3] = {tid, tid + 512, 1024 + (tid & 127)};
  uint4 vx, vd[3];
  auto load = [&](int b) {
    const uint4* x = reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.p1) + (size_t)b * 9216);
    const uint4* d = reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.dy2) + (size_t)b * 9216);
    vx = x[pxl * 8 + 2 * c4 + (kx & 1)];
#pragma unroll
    for (int i = 0; i < 3; ++i) vd[i] = d[kd[i]];
  };

  // per-lane pixel rows of the 5 k-steps (tr reads: rows rA = 32s + 8g + q and rB = rA + 4; input
  // rows past pixel 143 are clamped -- their dY rows are zero)
  int xa[5], xb[5];
#pragma unroll
  for (int s = 0; s < 5; ++s) {
    const int cA = min(32 * s + 8 * g + q, 143), cB = min(32 * s + 8 * g + q + 4, 143);
    xa[s] = ((cA / 12) * 16 + cA % 12) * W2_LDX + 4 * p;
    xb[s] = ((cB / 12) * 16 + cB % 12) * W2_LDX + 4 * p;
  }
  int toff[3];                                 // this wave's taps 3w .. 3w+2 (kh * 16 + kw pixels)
#pragma unroll
  for (int j = 0; j < 3; ++j) toff[j] = ((3 * w + j) / 5 * 16 + (3 * w + j) % 5) * W2_LDX;
  constexpr int T24 = (4 * 16 + 4) * W2_LDX;

  load(b0 < last ? b0 : last);
  for (int b = b0; b < a.B; b += G) {
    lds_barrier();                             // previous image's MFMA reads are done
    *reinterpret_cast<uint4*>(xdst) = vx;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int k = kd[i];
      *reinterpret_cast<uint4*>(dyt + (k >> 3) * W2_LD + w2_dy_col(k >> 3, (k & 7) * 8)) = vd[i];
      if (c4 == 0 && (i < 2 || tid < 128)) {   // chunk k & 7 == tid & 7: channels 8c..8c+7
        const uint32_t d4[4] = {vd[i].x, vd[i].y, vd[i].z, vd[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) { bsum[2 * j] += bf16_lo(d4[j]); bsum[2 * j + 1] += bf16_hi(d4[j]); }
      }
    }
    load(b + G < last ? b + G : last);
    lds_barrier();
    if (b == b0) DMLC_STAMP(DMLC_TK_W2, 1);
    // k-step s+1's fragments are read into the other register set BEFORE k-step s's MFMAs issue,
    // so each k-step's LDS latency hides behind the previous one's MFMAs (as conv2_core): MFMA
    // phase 15.5 -> 14.3 us, 77.8-78.2 -> 76.8-77.1 us/step at B=256 (profiles/r5_w2_kpipe_ab.txt)
    bf16x8 BF[2][4], AF[2][4];
    auto frags = [&](int s, bf16x8 (&bf)[4], bf16x8 (&af)[4]) __attribute__((always_inline)) {
      const int rA = 32 * s + 8 * g + q, rB = rA + 4;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        bf[ct] = tr_frag(dyt + rA * W2_LD + w2_dy_col(rA, 16 * ct + 4 * p), dyt + rB * W2_LD + w2_dy_col(rB, 16 * ct + 4 * p));
#pragma unroll
      for (int j = 0; j < 3; ++j) af[j] = tr_frag(xt + xa[s] + toff[j], xt + xb[s] + toff[j]);
      if (w < 4) af[3] = tr_frag(xt + xa[s] + T24, xt + xb[s] + T24);
    };
    frags(0, BF[0], AF[0]);
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      const int cur = s & 1;
      wait_lds();
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < 5) frags(s + 1, BF[cur ^ 1], AF[cur ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[4 * j + ct] = mfma16(AF[cur][j], BF[cur][ct], acc[4 * j + ct]);
      if (w < 4) {                             // tap 24 x co tile w
        const bf16x8 bw = w == 0 ? BF[cur][0] : w == 1 ? BF[cur][1] : w == 2 ? BF[cur][2] : BF[cur][3];
        acc[12] = mfma16(AF[cur][3], bw, acc[12]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (b == b0) DMLC_STAMP(DMLC_TK_W2, 4);
  }
  }
  DMLC_STAMP(DMLC_TK_W2, 2);
  // slab element e of this group (fp32 partial sum over G-th of the batch)
  const size_t slab0 = (size_t)grp * 1600 * 64;
  auto put4 = [&](size_t e, const f32x4& v) {
    if (coh) st_sc1(buf_rsrc(a.part2), (uint32_t)(slab0 + e) * 4, v);
    else st_maybe_nt<kNtDefault>(reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.part2) + slab0 + e), v);
  };
  auto put1 = [&](size_t e, float v) {
    if (coh) st_sc1(buf_rsrc(a.part2), (uint32_t)(slab0 + e) * 4, v);
    else reinterpret_cast<float*>(a.part2)[slab0 + e] = v;
  };
  __syncthreads();                             // every MFMA read of LDS is done: reuse it for staging
  if (c4 == 0) {
    float* red = reinterpret_cast<float*>(smem);
    block_chunk_sum(bsum, red, tid);
    __syncthreads();
    if (tid < 64) {
      float sb = 0.f;
#pragma unroll
      for (int k = 0; k < W2T / 64; ++k) sb += red[k * 64 + tid];
      if (coh) st_sc1(buf_rsrc(a.partb2), (uint32_t)(grp * 64 + tid) * 4, sb);
      else a.partb2[grp * 64 + tid] = sb;
    }
    __syncthreads();
  }
  DMLC_STAMP(DMLC_TK_W2, 5);
  // full taps: each wave stages one 16 ci x 64 co tap slice in LDS and writes it as 4 rows of 256 B
  float* st = reinterpret_cast<float*>(smem) + w * 16 * W2_ST;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int i = 0; i < 4; ++i) st[(4 * g + i) * W2_ST + 16 * ct + li] = acc[4 * j + ct][i];
    lds_barrier();                             // (not __syncthreads: that would drain the stores)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int row = 4 * k + (lane >> 4), c16 = lane & 15;
      const f32x4 v = *reinterpret_cast<const f32x4*>(st + row * W2_ST + 4 * c16);
      put4(((size_t)(3 * w + j) * 64 + 16 * c4 + row) * 64 + 4 * c16, v);
    }
    lds_barrier();
  }
  if (w < 4) {                                 // tap 24, co tile w
#pragma unroll
    for (int i = 0; i < 4; ++i) put1((size_t)(24 * 64 + 16 * c4 + 4 * g + i) * 64 + 16 * w + li, acc[12][i]);
  }
  DMLC_STAMP(DMLC_TK_W2, 3);
}

// ---------------------------------------------------------------------------------------------
// Single-GPU apply mode (DmlcWgradArgs::apply): the step's SGD runs inside this launch and no SGD
// launch follows (saves its ~7 us and the ~1.5 us dependent-launch gap).  Each slab family meets at a
// sub-grid barrier once its coherent slab stores are acknowledged -- the 32 conv2 blocks of an
// input-channel quarter, the g1 conv1 blocks -- and every block then reduces ITS share of the family's
// outputs in exactly the SGD kernel's order (split_sum: split sp sums slabs sp, sp+S, ... and the S
// partials are added in fixed order), so the weights are bit-identical to the two-launch path.
// Deadlock freedom: conv1 blocks (lowest ids, dispatched first) only wait for conv1 blocks, conv2
// blocks for the blocks of their quarter; one block per CU and g1, 4 * g2 <= the CU count (host
// check) -- if the chip cannot hold every block, the conv1 family still completes and frees CUs
// (the conv1 "helpers" of the conv2 reduction only ever join work they saw become ready, w2_chunk).
// sgd.mode 1 (data parallel, before the all-reduce): the same reductions write the flat gradient
// instead (the SGD kernel's mode 1); no update, no fc roles, stats or step counter.
DEV unsigned* wbar(unsigned* b, int k) { return b + 32 * k; }

// conv2 slab reduction of quarter c4, float4 outputs [f_begin, f_end) of its 6400 (25 taps x 16 ci
// x 16 co-float4), four threads per output (split sp = lane & 3 sums slabs sp, sp+4, ...: the SGD
// kernel's split_sum<4> order, combined ((s0 + s1) + s2) + s3), + SGD + shadows.
// fp8 (w2f8 set): also the e4m3 shadows (forward w2f8 and the dgrad's flipped w2d8) quantised with
// the delayed scale sw (as the SGD kernel does) and the maximum |w| of this range, stored to
// amax_w[nxt][slot] (every thread calls: one LDS reduction through red[8]).
struct W2Fp8 { float sw; int nxt, slot; float* red; };
DEV float w2_fp8_scale(const DmlcSgdArgs& s, int64_t step) {
  const float* src = s.amax_w + (size_t)(step & 1) * C2_BLOCKS;
  float m = 0.f;
  for (int i = threadIdx.x & 63; i < C2_BLOCKS; i += 64) m = fmaxf(m, src[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  return 224.f / fmaxf(m, 1e-20f);              // the SGD kernel's expression (cnn_sgd.hip conv2_rows)
}
DEV void w2_fp8_put(const DmlcWgradArgs& A, int slot, int nxt, float m, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = red[0];
    for (int k = 1; k < W2T / 64; ++k) t = fmaxf(t, red[k]);
    A.sgd.amax_w[(size_t)nxt * C2_BLOCKS + slot] = t;
  }
  __syncthreads();
}

DEV void conv2_reduce(const DmlcWgradArgs& A, int c4, int f_begin, int f_end, float lr, const W2Fp8& f8) {
  const DmlcSgdArgs& s = A.sgd;
  const int tid = threadIdx.x, sp = tid & 3, n = A.w2.g2;
  float wmax = 0.f;
  const rsrc_t part = buf_rsrc(A.w2.part2);
  for (int f0 = f_begin; f0 < f_end; f0 += W2T / 4) {
    const int f = f0 + (tid >> 2);
    const bool ok = f < f_end;
    const int fc = ok ? f : f_begin;
    const int krow = (fc >> 8) * 64 + 16 * c4 + ((fc >> 4) & 15), co = 4 * (fc & 15);
    const size_t e = (size_t)krow * 64 + co;
    const float4 w0 = *reinterpret_cast<const float4*>(s.master + s.off[2] + e);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = sp; q < n; q += 8 * C2_SPLIT) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = ld_sc1(part, (uint32_t)((size_t)(q + u * C2_SPLIT < n ? q + u * C2_SPLIT : 0) * 102400 + e) * 4);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = add4(acc, q + u * C2_SPLIT < n ? v[u] : make_float4(0.f, 0.f, 0.f, 0.f));
    }
    float4 o[3];                               // splits 1..3 from the next three lanes
#pragma unroll
    for (int j = 0; j < 3; ++j)
      o[j] = make_float4(__shfl_down(acc.x, j + 1), __shfl_down(acc.y, j + 1), __shfl_down(acc.z, j + 1),
                         __shfl_down(acc.w, j + 1));
    if (sp == 0 && ok) {
      const float4 t = add4(add4(add4(acc, o[0]), o[1]), o[2]);
      if (s.mode == 1) {
        grad_st4(s, s.off[2] + e, t);                          // reduce only (data parallel)
      } else {
        const float4 w = sgd4(s.master + s.off[2] + e, w0, t, lr, s.grad_scale, true);
        conv2_shadow4(s, krow, co, w);
        if (s.w2f8) {
          const float sw = f8.sw;
          const uint32_t q = pk_fp8x4(w.x * sw, w.y * sw, w.z * sw, w.w * sw);
          uint8_t* w8 = s.w2f8 + krow;
          w8[(co + 0) * 1600] = (uint8_t)q; w8[(co + 1) * 1600] = (uint8_t)(q >> 8);
          w8[(co + 2) * 1600] = (uint8_t)(q >> 16); w8[(co + 3) * 1600] = (uint8_t)(q >> 24);
          if (s.w2d8)
            *reinterpret_cast<uint32_t*>(s.w2d8 + (size_t)(krow & 63) * 1600 + (24 - (krow >> 6)) * 64 + co) = q;
          wmax = fmaxf(wmax, fmaxf(fmaxf(fabsf(w.x), fabsf(w.y)), fmaxf(fabsf(w.z), fabsf(w.w))));
        }
      }
    }
  }
  if (s.w2f8 && s.mode == 0) w2_fp8_put(A, f8.slot, f8.nxt, wmax, f8.red);
}

// Chunk of conv2 block (c4, grp): outputs [grp*per, min(grp*per + per, 6400)), per = ceil(6400 / g2).
// With helpers (g1 >= 4 * g2), conv1 block j -- its conv1 work done ~5 us before the conv2 blocks'
// -- helps conv2 block j: the chunk's second half goes to whoever CLAIMS it first after observing
// the quarter's barrier (atomicMax of the new generation into the chunk's claim word: the first
// caller sees an older value).  A helper that never observes the barrier (it started after it
// completed) just gives up; the conv2 block then claims and reduces the half itself -- no extra
// co-residency requirement, no wrong result in any schedule.
DEV bool w2_helpers(const DmlcWgradArgs& A) { return A.helpers && A.w1.g1 >= 4 * A.w2.g2; }
DEV void w2_chunk(const DmlcWgradArgs& A, int grp, int& b, int& m, int& e) {
  const int per = (6400 + A.w2.g2 - 1) / A.w2.g2;
  b = grp * per;
  e = min(b + per, 6400);
  m = w2_helpers(A) ? min(b + (per + 1) / 2, e) : e;
}
DEV unsigned* w2_claim(const DmlcWgradArgs& A, int c4, int grp) { return A.bar + 11 * 32 + c4 * A.w2.g2 + grp; }

DEV void conv2_apply(const DmlcWgradArgs& A, int c4, int grp, char* smem, unsigned g0, int64_t step) {
  const DmlcSgdArgs& s = A.sgd;
  const int tid = threadIdx.x, n = A.w2.g2;
  int* flag = reinterpret_cast<int*>(smem);
  wait_vm_all();                               // this thread's coherent slab stores are acknowledged
  __syncthreads();
  if (tid == 0) {
    bar_arrive(wbar(A.bar, 2 + c4), wbar(A.bar, 6 + c4), g0, (unsigned)n);
    bar_wait(wbar(A.bar, 6 + c4), g0, wbar(A.bar, 10));
  }
  __syncthreads();
  DMLC_STAMP(DMLC_TK_W2, 6);
  const float lr = lr_of(s, step);
  int b, m, e;
  w2_chunk(A, grp, b, m, e);
  // fp8: amax slots 2k / 2k+1 for the halves of chunk k = c4 * g2 + grp (whoever reduces a half
  // writes its slot); block (0, 0) also zeroes the unused slots and publishes the scale
  const int slot = 2 * (c4 * n + grp), nxt = (int)((step & 1) ^ 1);
  W2Fp8 f8 = {s.w2f8 ? w2_fp8_scale(s, step) : 0.f, nxt, slot, reinterpret_cast<float*>(smem + 64)};
  if (s.w2f8 && s.mode == 0 && c4 == 0 && grp == 0) {   // (reduce-only mode 1 touches no fp8 state)
    for (int i = 8 * n + tid; i < C2_BLOCKS; i += W2T) s.amax_w[(size_t)nxt * C2_BLOCKS + i] = 0.f;
    if (tid == 0) { s.scale_w[0] = f8.sw; s.scale_w[1] = f8.sw; }
  }
  conv2_reduce(A, c4, b, m, lr, f8);
  if (m < e) {                                 // the second half: claim it unless the helper did
    if (tid == 0)
      flag[0] = __hip_atomic_fetch_max(w2_claim(A, c4, grp), g0 + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < g0 + 1u;
    __syncthreads();
    f8.slot = slot + 1;
    if (flag[0]) DMLC_STAMP(DMLC_TK_HEAD, 6);    // (timing build: no helper took it; the HEAD row is
                                                 //  free for blocks >= 64 in this launch)
    if (flag[0]) conv2_reduce(A, c4, m, e, lr, f8);
    __syncthreads();                           // flag / LDS reused by the bias below
  } else if (s.w2f8 && s.mode == 0 && tid == 0) {
    s.amax_w[(size_t)nxt * C2_BLOCKS + slot + 1] = 0.f;   // no second half
  }
  if (c4 == 0 && grp == 0) conv_bias(s, 1, lr, reinterpret_cast<float4*>(smem), tid, true);
  DMLC_STAMP(DMLC_TK_W2, 7);
}

// conv1 block j < 4 * g2 helping conv2 block j (after its own work; hg0 = the quarter's generation
// read at kernel start)
DEV void conv2_help(const DmlcWgradArgs& A, int j, char* smem, unsigned hg0, int64_t step) {
  int c4, grp;
  w2_block_pos(A.w2, j, A.w1.g1, c4, grp);
  int* flag = reinterpret_cast<int*>(smem);
  __syncthreads();                             // the conv1 bias role may still read this LDS
  if (threadIdx.x == 0) {
    unsigned gen = hg0;
    // a short bound (~64 polls of ~1 us): the conv2 blocks normally pass the barrier ~3 us after the
    // helper gets here; if they are late (e.g. a concurrent comm kernel holds CUs) the helper leaves
    // rather than holding its CU, and the conv2 block claims the half itself
    for (int it = 0; it < 64 && (gen = bar_gen(wbar(A.bar, 6 + c4))) == hg0; ++it) __builtin_amdgcn_s_sleep(2);
    flag[0] = gen != hg0 &&
              __hip_atomic_fetch_max(w2_claim(A, c4, grp), gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gen;
  }
  __syncthreads();
  if (flag[0]) {
    DMLC_STAMP(DMLC_TK_SGD, 5);                // (timing build: this helper took the half)
    int b, m, e;
    w2_chunk(A, grp, b, m, e);
    const W2Fp8 f8 = {A.sgd.w2f8 ? w2_fp8_scale(A.sgd, step) : 0.f, (int)((step & 1) ^ 1),
                      2 * (c4 * A.w2.g2 + grp) + 1, reinterpret_cast<float*>(smem + 64)};
    conv2_reduce(A, c4, m, e, lr_of(A.sgd, step), f8);
  }
}

// conv1: arrive, run the slab-independent work (fc roles, stats + global_step, next batch rows),
// wait, then reduce float4 outputs [grp*per, grp*per+per) of the 75 x 16 (32 splits x 16 outputs
// per round of 512 threads, the SGD kernel's split_sum<32, 5> order) + shadows; one block: the bias.
DEV void conv1_arrive(const DmlcWgradArgs& A, unsigned g0) {
  wait_vm_all();
  __syncthreads();                             // also: w1_flush's LDS reads are done
  if (threadIdx.x == 0) bar_arrive(wbar(A.bar, 0), wbar(A.bar, 1), g0, (unsigned)A.w1.g1);
}
// arrived: the block already arrived at the conv1 barrier (conv1_arrive) and did other work since
DEV void conv1_apply(const DmlcWgradArgs& A, int grp, char* smem, unsigned g0, int64_t step, bool arrived = false) {
  const DmlcSgdArgs& s = A.sgd;
  const int tid = threadIdx.x, n = A.w1.g1;
  float4* lds = reinterpret_cast<float4*>(smem);
  if (!arrived) conv1_arrive(A, g0);
  else __syncthreads();                        // the previous role's LDS reads are done
  const float lr = lr_of(s, step);
  // reduce-only (data parallel): conv grads only; fc_in_launch: the fc parameters are updated in
  // the dW tiles' epilogues (below, after this function)
  const int nfc = s.mode == 1 || A.fc_in_launch || A.fc_done ? 0 : fc_role_count(s);
  for (int r = grp; r < nfc; r += n) {
    fc_role(s, r, lr, step, lds, tid);
    lds_barrier();                             // the fc2 transpose tile is reused by the next role
  }
  if (s.mode == 0 && grp == 0 && tid < 64) publish_step(s, step, lr, tid);
  if (s.mode == 0 && s.bidx) {                 // no block of this launch reads bidx (xraw is set)
    const int r = grp * W1T + tid;
    if (r < s.bidx_n) s.bidx[r] = order_row(s.next, step + 1, r);
  }
  DMLC_STAMP(DMLC_TK_SGD, 0);
  if (tid == 0) bar_wait(wbar(A.bar, 1), g0, wbar(A.bar, 10));
  __syncthreads();
  DMLC_STAMP(DMLC_TK_SGD, 1);
  const int per = (1200 + n - 1) / n, ol = tid & 15, sp = tid >> 4;
  const rsrc_t part1 = buf_rsrc(A.w1.part1);
  for (int f0 = 0; f0 < per; f0 += 16) {
    const int oo = f0 + ol, o = grp * per + oo;
    const bool ok = oo < per && o < 1200;
    const int oc = ok ? o : 0, row = oc >> 4, co = 4 * (oc & 15);   // HWIO row = (kh*5+kw)*3 + ci
    const int ci = row % 3, khw = row / 3, kh = khw / 5, kw = khw - kh * 5;
    const uint32_t p = (uint32_t)(kh * 16 + kw * 3 + ci) * 64 + co;   // slab row k'' (elements)
    const size_t e = (size_t)row * 64 + co;
    const float4 w0 = *reinterpret_cast<const float4*>(s.master + s.off[0] + e);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = sp; q < n; q += C1_LOADS * C1_SPLIT) {
      float4 v[C1_LOADS];
#pragma unroll
      for (int u = 0; u < C1_LOADS; ++u)
        v[u] = ld_sc1(part1, (p + (uint32_t)(q + u * C1_SPLIT < n ? q + u * C1_SPLIT : 0) * 80 * 64) * 4);
#pragma unroll
      for (int u = 0; u < C1_LOADS; ++u) acc = add4(acc, q + u * C1_SPLIT < n ? v[u] : make_float4(0.f, 0.f, 0.f, 0.f));
    }
    lds[tid] = acc;                            // [split sp][output ol]
    lds_barrier();
    if (tid < 16 && ok) {
      float4 t = lds[ol];
#pragma unroll
      for (int k = 1; k < C1_SPLIT; ++k) t = add4(t, lds[k * 16 + ol]);
      if (s.mode == 1) grad_st4(s, s.off[0] + e, t);                           // reduce only
      else conv1_shadow4(s, row, co, sgd4(s.master + s.off[0] + e, w0, t, lr, s.grad_scale, true));
    }
    lds_barrier();
  }
#ifndef DMLC_C1_BIAS_ON_1
  // the conv1 bias on the LAST conv1 block: the first ones also run the fc SGD roles (block 1, which
  // had both, ended the launch ~1 us after the rest at B=256, profiles/r5_ktiming_b256_wgrad_raw.json)
  if (grp == n - 1) conv_bias(s, 0, lr, lds, tid, true);
#else
  if (grp == (n > 1 ? 1 : 0)) conv_bias(s, 0, lr, lds, tid, true);
#endif
  DMLC_STAMP(DMLC_TK_SGD, 2);
}

// The late phases (fc dW tiles, reductions + SGD, helpers, next-batch copy) read their arguments
// through late_kernarg (common.h): the entry block loads only what the conv bodies need (same-box
// A/B, 300 steps: B=256 3.40 -> 3.55 M img/s, B=128 2.02 -> 2.11 M; profiles/r6_late_args_ab.txt).
#ifdef DMLC_EAGER_ARGS                         // A/B build: every field loaded in the entry block
#define late_args() a
#else
#define late_args() late_kernarg<DmlcWgradArgs>(0)
#endif

// Both weight gradients in ONE launch (no stream fork/join in the step graph): blocks [0, g1) run
// the conv1 body, the next 4 * g2 the conv2 body.  One block per CU (LDS): g1 + 4 * g2 <= 256 keeps
// every block resident in one wave of blocks.
constexpr size_t WG_LDS = W1_LDS > W2_LDS ? W1_LDS : W2_LDS;
static_assert(WG_LDS >= W8_LDS, "the fp8 conv2 body's double buffer fits the launch's LDS");
static_assert(WG_LDS >= (size_t)L_RED + 8 * 64 * 4 && WG_LDS >= 40960 + 64 * 136 * 2,
              "the fc dW tiles reuse the weight-gradient launch's LDS");
static_assert(W1T == FT, "the fc dW tiles run with the weight-gradient launch's block size");
static_assert(WG_LDS >= SGD_LDS4 * 16, "apply mode reuses the block's LDS for the SGD roles");
__global__ __launch_bounds__(W1T, 1) void k_wgrad(DmlcWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const bool conv1 = (int)blockIdx.x < a.w1.g1;
  int c4 = 0, grp = 0;
  if (!conv1) w2_block_pos(a.w2, blockIdx.x - a.w1.g1, a.w1.g1, c4, grp);
  unsigned g0 = 0, hg0 = 0;
  int64_t step = 0;
  const bool helper = a.apply && conv1 && w2_helpers(a) && (int)blockIdx.x < 4 * a.w2.g2;
  if (a.apply) {                               // read before this block can arrive
    if (threadIdx.x == 0) g0 = bar_gen(wbar(a.bar, conv1 ? 1 : 6 + c4));
    if (helper && threadIdx.x == 0) {
      int hc4, hgrp;
      w2_block_pos(a.w2, blockIdx.x, a.w1.g1, hc4, hgrp);
      hg0 = bar_gen(wbar(a.bar, 6 + hc4));
    }
    step = *a.sgd.step_rd;
  }
  if (conv1) {
    conv1_wgrad_block(a.w1, blockIdx.x, smem, a.apply != 0);
    const DmlcWgradArgs& L = late_args();
    if (a.apply && L.fc_in_launch) {
      // arrive at the conv1 barrier, then the fc weight gradients + their SGD (inputs from earlier
      // launches: no waits) while the rest of the family arrives, then the conv1 reduction + SGD;
      // the conv2 help comes last, when the conv2 slabs are ready anyway (running the fc tiles
      // after the help instead made the helpers late: the conv2 tail grew by ~3 us)
      // (the first task's operand loads go out before the slab stores are drained: the arrival
      // waits for both at once)
      const int parity = (int)(step & 1);
      if (blockIdx.x >= FC_DW_TASKS) conv1_arrive(L, g0);
      for (int d = blockIdx.x; d < FC_DW_TASKS; d += L.w1.g1) {
        const CTask T = dw_ctask(d);
        PreRegs R;
        pre_issue(L.fc, T, parity, R, threadIdx.x);
        const bool first = d == (int)blockIdx.x;
        dw_task<false>(L.fc, T, R, step, smem, threadIdx.x, [&]() {
          if (first) conv1_arrive(L, g0);
        });
      }
      DMLC_STAMP(DMLC_TK_SGD, 3);
      conv1_apply(L, blockIdx.x, smem, g0, step, true);
    } else if (a.apply) {
      conv1_apply(L, blockIdx.x, smem, g0, step);
    }
    if (helper) conv2_help(L, blockIdx.x, smem, hg0, step);
    // the next step's raw images over xraw: every conv1 block passed the conv1 barrier after its
    // image loop, so no block of this launch reads xraw any more
    if (a.apply && L.sgd.mode == 0 && L.sgd.xnext)
      for (int r = blockIdx.x; r < L.sgd.bidx_n; r += L.w1.g1) copy_next_row(L.sgd, step, r, threadIdx.x);
    DMLC_STAMP(DMLC_TK_SGD, 4);
  } else {
    conv2_wgrad_block(a.w2, blockIdx.x - a.w1.g1, a.w1.g1, smem, a.apply != 0);
    if (a.apply) conv2_apply(late_args(), c4, grp, smem, g0, step);
  }
}
static_assert(W1T == W2T, "k_wgrad runs both bodies with one block size");

}  // namespace dmlc

using namespace dmlc;

extern "C" {

hipError_t dmlc_wgrad(const DmlcWgradArgs* a, hipStream_t s) {
  DMLC_LDS_OPTIN(&k_wgrad, WG_LDS);
  const int blocks = a->w1.g1 + 4 * a->w2.g2;
  if (a->apply) {
    // every barrier family must fit on the chip at once (one block per CU), fp32 slabs, the step
    // read from the head's copy (a block bumps *step while others may not have read it yet), and
    // the forward's image copy (bidx is rewritten for the next step inside this launch)
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return hipErrorInvalidValue;
    }
    const DmlcSgdArgs& g = a->sgd;
    // mode 1 (data parallel): the reduced conv gradients go to the flat grad (nothing else runs)
    const bool ok_mode = g.mode == 0 ? (g.step_rd != g.step && g.fc1_fused && (!g.w2f8 || (g.amax_w && g.scale_w) ) &&
                                        8 * a->w2.g2 <= 400)
                                     : g.mode == 1;
    if (a->fc_in_launch && (g.mode != 0 || !g.fc1_fused || a->fc.fuse_sgd != 2 || a->fc.B < 16 || a->fc.B > 256 ||
                            !a->fc.p2 || !a->fc.dh1 || !a->fc.mw2 || !a->fc.fc2t))
      return hipErrorInvalidValue;
    if (a->w1.g1 < 1 || a->w1.g1 > cus || 4 * a->w2.g2 > cus || !a->bar || !a->w1.xraw ||
        !ok_mode || g.part1 != a->w1.part1 ||
        g.part2 != a->w2.part2 || g.g1 != a->w1.g1 || g.g2 != a->w2.g2 || g.bidx_n > a->w1.g1 * W1T)
      return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(k_wgrad, dim3(blocks), dim3(W1T), WG_LDS, s, *a);
  return hipGetLastError();
}

}  // extern "C"
