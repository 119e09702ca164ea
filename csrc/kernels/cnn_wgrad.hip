// Weight gradients of the two convolutions (TF Conv2DBackpropFilter + BiasAddGrad of
// /root/reference/cifar10cnn.py:107/:118 via the autodiff of :163; SURVEY.md §2.B N5/N7, §2.C
// conv5x5_wgrad).  Two kernels, launched on forked streams of the step graph so they run side by
// side on the chip:
//
//   k_conv1_wgrad  dW1[k''][co] = sum_{b,px} X[b,px][k''] dY1[b,px][co],  k'' = kh*16 + kw*3 + ci
//     * dY1 (the conv1 output gradient) is produced in LDS by the TF-SAME pool1 backward in "2x2
//       ownership" form from the staged pool1 gradient + argmax bytes (conv_common.h);
//     * X is kept as 15 channel-planar, column-shifted copies of the padded 28x24 crop (plane
//       kw*3+ci = Xpad[ci][y][x+kw]) so a K'' tile of 16 is one kernel row (15 taps + 1 zero plane)
//       and every B fragment is ONE aligned ds_read_b128 of 8 consecutive pixels: K'' = 80 instead
//       of the 160 a [pixel][4ch] image needs;
//     * the four waves split the 18 pixel k-steps of an image (not the output), each wave owns the
//       whole 64x80 tile (20 MFMA accumulators), reduced across waves once per block;
//   k_conv2_wgrad  dW2[(kh,kw,ci)][co] = sum_{b,px} Xpad[b][px+(kh,kw)][ci] dY2[b,px][co]
//     * one block per (kh, image group): wave w owns ci tile w x 5 kw x 4 co tiles (20 acc), so per
//       k-step it reads 10 A + 8 B transposed fragments (ds_read_b64_tr_b16) for 20 MFMAs.
// Both: the NEXT image's global data is prefetched into registers while the current image is being
// computed (one exposed memory latency per block instead of one per image); results are fp32
// split-K partial slabs, one per image group, reduced in fixed order by the SGD kernel.
#include "w1_common.h"

namespace dmlc {

// ---------------------------------------------------------------------------------------------
// dY1 | shifted planes | pool1 grad (bf16) | raw uint8 image [32][32][3] | argmax bytes | reduction
constexpr size_t W1_LDS = (size_t)(W1_DYT + W1_XS + 9216) * 2 + 3072 + 9216 + (W1T / 64) * 64 * 4;

DEV void conv1_wgrad_block(const DmlcConv1WgradArgs& a, const int grp, char* smem) {
  bf16* dyt = reinterpret_cast<bf16*>(smem);
  bf16* xs = dyt + W1_DYT;
  bf16* dps = xs + W1_XS;
  uint8_t* img = reinterpret_cast<uint8_t*>(dps + 9216);
  uint8_t* ams = img + 3072;
  float* red = reinterpret_cast<float*>(ams + 9216);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int ch = w & 1, ks = w >> 1;                     // MFMA: co tiles 2ch, 2ch+1; k-steps ks mod 4
  const int b0 = grp * a.B / a.g1, b1 = (grp + 1) * a.B / a.g1;
  DMLC_STAMP(DMLC_TK_W1, 0);

  w1_zero_plane15(xs, tid);

  f32x4 acc[2][5];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int t = 0; t < 5; ++t) acc[h][t] = zero4();
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  // Every load below is unconditional (image indices clamped to the block's last image, surplus
  // threads duplicating chunks): see PrefetchAll.  The dataset row of image b+1 is read one image
  // ahead of its pixels, so no index -> pixels dependency is exposed inside the loop.
  const int last = b1 > b0 ? b1 - 1 : b0;
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
  load(row_index(b0 < last ? b0 : last), b0);
  int nidx = row_index(b0 + 1 < last ? b0 + 1 : last);
  for (int b = b0; b < b1; ++b) {
    __syncthreads();                           // previous image's MFMA reads are done
    reinterpret_cast<uint4*>(img)[cI] = vI;
    reinterpret_cast<uint4*>(dps)[tid] = vD0;
    reinterpret_cast<uint4*>(dps)[tid + 512] = vD1;
    reinterpret_cast<uint4*>(dps)[cD2] = vD2;
    reinterpret_cast<uint4*>(ams)[tid] = vA0;
    reinterpret_cast<uint4*>(ams)[cA1] = vA1;
    load(nidx, b + 1 < last ? b + 1 : last);   // prefetch the next image while this one computes
    nidx = row_index(b + 2 < last ? b + 2 : last);
    __syncthreads();
    if (b == b0) DMLC_STAMP(DMLC_TK_W1, 1);
    w1_planes(xs, img, a.cy, a.cx, tid);
    w1_pool_bwd(dyt, dps, ams, bsum, tid);
    __syncthreads();
    if (b == b0) DMLC_STAMP(DMLC_TK_W1, 2);
    w1_mfma(dyt, xs, acc, ks, ch, g, li);
  }
  __syncthreads();
  DMLC_STAMP(DMLC_TK_W1, 3);
  w1_flush(smem, red, acc, bsum, a.part1 + (size_t)grp * 80 * 64, a.partb1 + grp * 64, ks, ch, lane, tid);
  DMLC_STAMP(DMLC_TK_W1, 4);
}

__global__ __launch_bounds__(W1T, 1) void k_conv1_wgrad(DmlcConv1WgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv1_wgrad_block(a, blockIdx.x, smem);
}

// ---------------------------------------------------------------------------------------------
constexpr int W2_LD = 72;                      // 144-B rows: tr reads of rows r / r+8 hit different banks
constexpr int W2_XT = 12 * 16 * W2_LD;         // rows kh..kh+11 of the padded input, 16 cols
constexpr int W2_DY = 160 * W2_LD;             // 144 pixels + 16 zero rows
constexpr size_t W2_LDS = (size_t)(W2_XT + W2_DY) * 2;

// HALVES = 1: one image group per 4-wave block (blk = kh + 5 * group).  HALVES = 2: an 8-wave block
// runs two independent 4-wave halves on groups 2*pair and 2*pair+1 (blk = kh + 5 * pair), each with
// its own LDS region; both halves step through max(#images) iterations so their barriers line up.
template <int HALVES>
DEV void conv2_wgrad_block(const DmlcConv2WgradArgs& a, const int blk, char* smem_all) {
  const int half = HALVES == 2 ? (int)(threadIdx.x >> 8) : 0;
  char* smem = smem_all + half * W2_LDS;
  bf16* xt = reinterpret_cast<bf16*>(smem);
  bf16* dyt = xt + W2_XT;
  const int tid = threadIdx.x & 255, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int kh = blk % 5, grp = (blk / 5) * HALVES + half;
  const bool valid = grp < a.g2;
  const int b0 = valid ? grp * a.B / a.g2 : 0, b1 = valid ? (grp + 1) * a.B / a.g2 : 0;
  int nmax = b1 - b0;
  if (HALVES == 2) {                            // both halves' image counts (uniform over the block)
    const int g0 = (blk / 5) * 2, gb = g0 + 1;
    const int n0 = g0 < a.g2 ? (g0 + 1) * a.B / a.g2 - g0 * a.B / a.g2 : 0;
    const int n1 = gb < a.g2 ? (gb + 1) * a.B / a.g2 - gb * a.B / a.g2 : 0;
    nmax = max(n0, n1);
  }
  DMLC_STAMP(DMLC_TK_W2, 0);

  // zero halo columns (xx = 0,1,14,15) and the 16 padding dY rows once
  for (int e = tid; e < 12 * 4 * 8; e += 256) {
    const int c = e & 7, r = e >> 3, yy = r >> 2, k = r & 3, xx = k < 2 ? k : 12 + k;
    *reinterpret_cast<bf16x8*>(xt + (yy * 16 + xx) * W2_LD + c * 8) = bf16x8{};
  }
  for (int e = tid; e < 16 * 8; e += 256)
    *reinterpret_cast<bf16x8*>(dyt + (144 + (e >> 3)) * W2_LD + (e & 7) * 8) = bf16x8{};

  f32x4 acc[5][4];
#pragma unroll
  for (int kw = 0; kw < 5; ++kw)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[kw][ct] = zero4();
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // conv2 bias grad (kh == 0 blocks)

  // prefetch: x rows iy = kh-2 .. kh+9 (1152 chunks, invalid rows -> 0) and dY (1152 chunks).  No
  // predicate on any load or store (PrefetchAll's reasoning): the image index is clamped to the
  // group's last image, and in the 5th round threads 128..255 duplicate the chunks of threads 0..127.
  constexpr int IT = 5;
  uint4 vx[IT], vd[IT];
  auto chunk = [&](int i) { return i < IT - 1 ? tid + i * 256 : 1024 + (tid & 127); };
  const int last = b1 > b0 ? b1 - 1 : b0;
  auto load = [&](int b) {
    const uint4* x = reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.p1) + (size_t)b * 9216);
    const uint4* d = reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.dy2) + (size_t)b * 9216);
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int k = chunk(i);
      const int yy = k / 96, iy = kh + yy - 2;
      vx[i] = load_sel(x + iy * 96 + (k - yy * 96), x, iy >= 0 && iy < 12);
      vd[i] = d[k];
    }
  };
  load(b0 < last ? b0 : last);
  for (int it = 0; it < nmax; ++it) {
    const int b = b0 + it;
    const bool act = b < b1;                   // uniform per half (waves of one half agree)
    __syncthreads();
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int k = chunk(i);
      const int yy = k / 96, rem = k - yy * 96, px = rem >> 3, c = rem & 7;
      *reinterpret_cast<uint4*>(xt + (yy * 16 + px + 2) * W2_LD + c * 8) = vx[i];
      *reinterpret_cast<uint4*>(dyt + (k >> 3) * W2_LD + (k & 7) * 8) = vd[i];
      if (kh == 0 && act && (i < IT - 1 || tid < 128)) {   // chunk k & 7 == tid & 7: channels 8c..8c+7
        const uint32_t d4[4] = {vd[i].x, vd[i].y, vd[i].z, vd[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) { bsum[2 * j] += bf16_lo(d4[j]); bsum[2 * j + 1] += bf16_hi(d4[j]); }
      }
    }
    load(b + 1 < last ? b + 1 : last);
    __syncthreads();
    if (it == 0) DMLC_STAMP(DMLC_TK_W2, 1);
    if (!act) continue;
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      const int rA = 32 * s + 8 * g + q, rB = rA + 4;
      bf16x8 bf[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        bf[ct] = tr_frag(dyt + rA * W2_LD + 16 * ct + 4 * p, dyt + rB * W2_LD + 16 * ct + 4 * p);
      const int cA = min(rA, 143), cB = min(rB, 143);
      const int yA = cA / 12, yB = cB / 12;
      const int pA = yA * 16 + cA - yA * 12, pB = yB * 16 + cB - yB * 12;
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) {
        const bf16x8 af = tr_frag(xt + (pA + kw) * W2_LD + 16 * w + 4 * p, xt + (pB + kw) * W2_LD + 16 * w + 4 * p);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[kw][ct] = mfma16(af, bf[ct], acc[kw][ct]);
      }
    }
  }
  DMLC_STAMP(DMLC_TK_W2, 2);
  // HALVES == 2: the two halves' partial sums are added in-block (half 0 + half 1, fixed order), so
  // one slab per PAIR leaves the kernel -- half the bytes for the SGD kernel to reduce.
  const int slab = HALVES == 2 ? blk / 5 : grp;
  const bool writer = HALVES == 2 ? half == 0 : valid;
  if (kh == 0) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);      // this half's region
    block_chunk_sum(bsum, red, tid);
    __syncthreads();
    if (writer && tid < 64) {
      float sb = (red[tid] + red[64 + tid]) + (red[128 + tid] + red[192 + tid]);
      if (HALVES == 2) {
        const float* r1 = reinterpret_cast<const float*>(smem_all + W2_LDS);
        sb += (r1[tid] + r1[64 + tid]) + (r1[128 + tid] + r1[192 + tid]);
      }
      a.partb2[slab * 64 + tid] = sb;
    }
  }
  if (HALVES == 2) {
    f32x4* xch = reinterpret_cast<f32x4*>(smem_all);  // 20 x 256 f32x4 = 80 KB
    __syncthreads();                                   // MFMA / bias reads of LDS are done
    if (half == 1) {
#pragma unroll
      for (int kw = 0; kw < 5; ++kw)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) xch[(kw * 4 + ct) * 256 + tid] = acc[kw][ct];
    }
    __syncthreads();
    if (half == 0) {
#pragma unroll
      for (int kw = 0; kw < 5; ++kw)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[kw][ct] += xch[(kw * 4 + ct) * 256 + tid];
    }
  }
  if (writer) {
    float* out = a.part2 + (size_t)slab * 1600 * 64;
#pragma unroll
    for (int kw = 0; kw < 5; ++kw)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int krow = (kh * 5 + kw) * 64 + 16 * w + 4 * g + i;
          out[krow * 64 + 16 * ct + li] = acc[kw][ct][i];
        }
  }
  DMLC_STAMP(DMLC_TK_W2, 3);
}

__global__ __launch_bounds__(256, 2) void k_conv2_wgrad(DmlcConv2WgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv2_wgrad_block<1>(a, blockIdx.x, smem);
}

// Both weight gradients in ONE launch (no stream fork/join in the step graph): blocks [0, g1) run
// the conv1 body (8 waves), the rest run the conv2 body as two 4-wave halves on image groups
// 2p, 2p+1 whose sums leave as ONE slab p (a.w2.g2 = image groups, slabs = ceil(g2 / 2)).  One block
// per CU (LDS): g1 + 5 * ceil(g2 / 2) <= 256 keeps every block resident in one wave of blocks.
constexpr size_t WG_LDS = W1_LDS > 2 * W2_LDS ? W1_LDS : 2 * W2_LDS;
__global__ __launch_bounds__(W1T, 1) void k_wgrad(DmlcWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if ((int)blockIdx.x < a.w1.g1) conv1_wgrad_block(a.w1, blockIdx.x, smem);
  else conv2_wgrad_block<2>(a.w2, blockIdx.x - a.w1.g1, smem);
}

}  // namespace dmlc

using namespace dmlc;

namespace {
bool g_w1 = false;
}

extern "C" {

hipError_t dmlc_conv1_wgrad(const DmlcConv1WgradArgs* a, hipStream_t s) {
  if (!g_w1) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_conv1_wgrad),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)W1_LDS);
    g_w1 = true;
  }
  hipLaunchKernelGGL(k_conv1_wgrad, dim3(a->g1), dim3(W1T), W1_LDS, s, *a);
  return hipGetLastError();
}

hipError_t dmlc_conv2_wgrad(const DmlcConv2WgradArgs* a, hipStream_t s) {
  hipLaunchKernelGGL(k_conv2_wgrad, dim3(5 * a->g2), dim3(256), W2_LDS, s, *a);
  return hipGetLastError();
}

hipError_t dmlc_wgrad(const DmlcWgradArgs* a, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_wgrad), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)WG_LDS);
    attr = true;
  }
  const int blocks = a->w1.g1 + 5 * ((a->w2.g2 + 1) / 2);
  hipLaunchKernelGGL(k_wgrad, dim3(blocks), dim3(W1T), WG_LDS, s, *a);
  return hipGetLastError();
}

}  // extern "C"
