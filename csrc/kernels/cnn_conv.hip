// Convolution kernels of the CIFAR-10 CNN for gfx950 (MI355X), one image per 256-thread workgroup.
//
// Replaces TF's Conv2D / BiasAdd / Relu / MaxPool (+ their gradients) used by
// /root/reference/cifar10cnn.py:106-123.
//
// Design (MI355X-first, not a cuDNN translation):
//   * implicit GEMM on MFMA 16x16x32 bf16 with the GEMM formulated TRANSPOSED (C[channel][pixel]):
//     the weight fragment comes from global/L2 (shared by every workgroup), the pixel fragment is read
//     straight out of an LDS image of the zero-padded input — no im2col buffer ever exists;
//     each lane then owns 4 consecutive channels of one pixel, i.e. an 8-byte NHWC store;
//   * bias + ReLU + TF-SAME 3x3/2 max-pool are fused into the epilogue: the whole conv output of an
//     image stays in LDS, the pool emits the pooled bf16 tensor plus a 1-byte argmax per output
//     (255 encodes "pooled <= 0", i.e. the ReLU mask), so the backward never re-reads activations;
//   * conv1 gathers its uint8 input directly from the device-resident dataset (index list + center
//     crop), so the input pipeline (N1-N3) costs no extra launch;
//   * conv1's K=75 (5x5x3) is laid out as k = kh*32 + kw*4 + ci (kw padded to 8, ci to 4) so that a
//     k-step of 32 is one kernel row and every fragment is 16 contiguous bytes of the LDS image;
//   * backward: pool/ReLU backward is a *gather* (each input pixel sums the <=4 windows whose argmax
//     points at it: deterministic, no atomics) fused into the staging of the dgrad/wgrad operands;
//     weight gradients read both operands from NHWC LDS images with ds_read_b64_tr_b16 (hardware
//     transpose) so no transposed copies are materialised; they are split-K over image groups with
//     fp32 partial slabs reduced deterministically by the SGD kernel.
#include "common.h"
#include "api.h"

namespace dmlc {

DEV int batch_index(const DmlcIndexSrc& s, int B, int b) {
  int row = 0;
  if (s.counter) row = (int)(*s.counter % (int64_t)s.period);
  return s.idx_base[row * B + b];
}

// ---------------------------------------------------------------------------------------------
// conv1 input image: 24x24 crop of the uint8 NHWC image at (cy,cx), zero halo of 2, stored as
// [28 rows][32 cols][4 ch] bf16 (col 28..31 and ch 3 zero).  Pixel (iy,ix) -> (iy+2, ix+2).
constexpr int C1_XIN = 28 * 32 * 4;        // 3584 bf16
constexpr int C1_OUT = 576 * 64;           // 36864 bf16

DEV void stage_conv1_input(bf16* xin, const uint8_t* src, int cy, int cx, int tid) {
  for (int p = tid; p < 28 * 32; p += 256) {
    const int r = p >> 5, c = p & 31;
    const int iy = r - 2, ix = c - 2;
    bf16x4 v = pack4(0.f, 0.f, 0.f, 0.f);
    if (iy >= 0 && iy < 24 && ix >= 0 && ix < 24) {
      const uint8_t* s = src + ((cy + iy) * 32 + (cx + ix)) * 3;
      v = pack4((float)s[0], (float)s[1], (float)s[2], 0.f);
    }
    *reinterpret_cast<bf16x4*>(xin + p * 4) = v;
  }
}

// Epilogue helper: acc (C[4g+i][px]) + bias -> ReLU -> bf16 -> LDS [px][64] swizzled.
DEV void store_relu_tile(bf16* cout, int px, int co_base, const f32x4& acc, const float* b4) {
  const bf16x4 v = pack4(fmaxf(acc[0] + b4[0], 0.f), fmaxf(acc[1] + b4[1], 0.f),
                         fmaxf(acc[2] + b4[2], 0.f), fmaxf(acc[3] + b4[3], 0.f));
  const int chunk = co_base >> 3, half = (co_base >> 2) & 1;
  *reinterpret_cast<bf16x4*>(cout + swz128(px, chunk) + half * 4) = v;
}

// TF-SAME 3x3/2 max-pool over an LDS image [H*W][64] (swizzled) -> global out [HO*WO][64] bf16 +
// argmax bytes.  Padding is bottom/right only (in = 2*out), padded cells never win.
template <int H>
DEV void pool_emit(const bf16* cout, bf16* out, uint8_t* am, int tid) {
  constexpr int HO = H / 2;
  for (int task = tid; task < HO * HO * 8; task += 256) {
    const int q = task >> 3, c = task & 7;
    const int py = q / HO, px = q - py * HO;
    float best[8];
    int arg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -1.f; arg[j] = 0; }
#pragma unroll
    for (int d = 0; d < 9; ++d) {
      const int y = 2 * py + d / 3, x = 2 * px + d % 3;
      if (y < H && x < H) {
        const bf16x8 v = lds_b128(cout + swz128(y * H + x, c));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = (float)v[j];
          if (f > best[j]) { best[j] = f; arg[j] = d; }
        }
      }
    }
    bf16x8 o;
    uint64_t a = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = (bf16)best[j];
      a |= (uint64_t)(best[j] > 0.f ? arg[j] : 255) << (8 * j);
    }
    *reinterpret_cast<bf16x8*>(out + q * 64 + c * 8) = o;
    *reinterpret_cast<uint64_t*>(am + q * 64 + c * 8) = a;
  }
}

// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void k_conv1_fwd(DmlcConv1FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xin = reinterpret_cast<bf16*>(smem);
  bf16* cout = xin + C1_XIN;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;

  const int img = batch_index(a.src, a.B, b);
  stage_conv1_input(xin, a.data + (size_t)img * 3072, a.cy, a.cx, tid);

  // A operand: weights [64 co][160 k]; this wave owns co = 16w .. 16w+15.
  const bf16* W = reinterpret_cast<const bf16*>(a.w) + (16 * w + li) * 160 + 8 * g;
  bf16x8 wa[5];
#pragma unroll
  for (int kh = 0; kh < 5; ++kh) wa[kh] = glb_b128(W + 32 * kh);
  float b4[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) b4[i] = a.bias[16 * w + 4 * g + i];
  __syncthreads();

#pragma unroll 1
  for (int ch = 0; ch < 3; ++ch) {        // 3 chunks x 12 pixel tiles of 16 = 576 pixels
    f32x4 acc[12];
#pragma unroll
    for (int t = 0; t < 12; ++t) acc[t] = zero4();
#pragma unroll
    for (int t = 0; t < 12; ++t) {
      const int px = (ch * 12 + t) * 16 + li;
      const int y = px / 24, x = px - (px / 24) * 24;
      const bf16* base = xin + (y * 32 + x + 2 * g) * 4;   // k = 8g..8g+7 -> kw = 2g,2g+1 ; ci 0..3
#pragma unroll
      for (int kh = 0; kh < 5; ++kh) {
        const bf16* p = base + kh * 128;
        const bf16x8 bx = cat44(*reinterpret_cast<const bf16x4*>(p), *reinterpret_cast<const bf16x4*>(p + 4));
        acc[t] = mfma16(wa[kh], bx, acc[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < 12; ++t) store_relu_tile(cout, (ch * 12 + t) * 16 + li, 16 * w + 4 * g, acc[t], b4);
  }
  __syncthreads();
  pool_emit<24>(cout, reinterpret_cast<bf16*>(a.out) + (size_t)b * 9216, a.am + (size_t)b * 9216, tid);
}

// ---------------------------------------------------------------------------------------------
// conv2-shaped implicit GEMM core shared by forward and dgrad:
//   C[c_out][px] = sum_{kh,kw,c_in} Wt[c_out][(kh*5+kw)*64 + c_in] * Xpad[(y+kh)*16 + x+kw][c_in]
// Xpad: LDS [16*16][64] bf16 (swizzled), wave w -> c_out tile 16w, 9 pixel tiles of 16.
constexpr int C2_XIN = 256 * 64;
constexpr int C2_OUT = 144 * 64;

DEV void conv2_core(const bf16* __restrict__ Wg, const bf16* xin, f32x4 (&acc)[9], int w, int g, int li) {
  const bf16* W = Wg + (16 * w + li) * 1600 + 8 * g;
  int pb[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int px = 16 * t + li;
    const int y = px / 12;
    pb[t] = y * 16 + (px - y * 12);
  }
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = zero4();
  bf16x8 wc[10], wn[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) wc[j] = glb_b128(W + j * 32);
#pragma unroll
  for (int kh = 0; kh < 5; ++kh) {
    if (kh < 4) {
#pragma unroll
      for (int j = 0; j < 10; ++j) wn[j] = glb_b128(W + (kh + 1) * 320 + j * 32);
    }
#pragma unroll
    for (int kw = 0; kw < 5; ++kw) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const bf16x8 bx = lds_b128(xin + swz128(pb[t] + kh * 16 + kw, 4 * s + g));
          acc[t] = mfma16(wc[kw * 2 + s], bx, acc[t]);
        }
      }
    }
    if (kh < 4) {
#pragma unroll
      for (int j = 0; j < 10; ++j) wc[j] = wn[j];
    }
  }
}

__global__ __launch_bounds__(256, 2) void k_conv2_fwd(DmlcConv2FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* xin = reinterpret_cast<bf16*>(smem);
  bf16* cout = xin + C2_XIN;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const bf16* in = reinterpret_cast<const bf16*>(a.in) + (size_t)b * 9216;

  for (int s = tid; s < 2048; s += 256) {
    const int pix = s >> 3, c = s & 7;
    const int iy = (pix >> 4) - 2, ix = (pix & 15) - 2;
    bf16x8 v = {};
    if (iy >= 0 && iy < 12 && ix >= 0 && ix < 12) v = glb_b128(in + (iy * 12 + ix) * 64 + c * 8);
    *reinterpret_cast<bf16x8*>(xin + swz128(pix, c)) = v;
  }
  float b4[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) b4[i] = a.bias[16 * w + 4 * g + i];
  __syncthreads();

  f32x4 acc[9];
  conv2_core(reinterpret_cast<const bf16*>(a.w), xin, acc, w, g, li);
#pragma unroll
  for (int t = 0; t < 9; ++t) store_relu_tile(cout, 16 * t + li, 16 * w + 4 * g, acc[t], b4);
  __syncthreads();
  pool_emit<12>(cout, reinterpret_cast<bf16*>(a.out) + (size_t)b * 2304, a.am + (size_t)b * 2304, tid);
}

// ---------------------------------------------------------------------------------------------
// Pool/ReLU backward as a gather: grad at conv pixel (y,x) = sum over the pool windows (py,px) that
// contain it and whose argmax is (y-2py, x-2px) of dpool[py][px].  HO = pooled size.
template <int HO>
DEV void pool_bwd_gather(const bf16* __restrict__ dp, const uint8_t* __restrict__ am, int y, int x, int c,
                         float (&accv)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) accv[j] = 0.f;
  const int py0 = max(0, (y - 1) >> 1), py1 = min(HO - 1, y >> 1);
  const int px0 = max(0, (x - 1) >> 1), px1 = min(HO - 1, x >> 1);
  for (int py = py0; py <= py1; ++py) {
    for (int px = px0; px <= px1; ++px) {
      const int d = (y - 2 * py) * 3 + (x - 2 * px);
      const int o = (py * HO + px) * 64 + c * 8;
      const uint64_t av = *reinterpret_cast<const uint64_t*>(am + o);
      const bf16x8 dv = glb_b128(dp + o);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if ((int)((av >> (8 * j)) & 0xff) == d) accv[j] += (float)dv[j];
    }
  }
}

// Reduce per-thread channel sums (thread's chunk = tid & 7) over the workgroup: red[64] result.
DEV void block_chunk_sum(float (&v)[8], float* red /*[4][64]*/, int tid) {
  const int lane = tid & 63, w = tid >> 6;
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

__global__ __launch_bounds__(256, 2) void k_conv2_dgrad(DmlcConv2DgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* dyp = reinterpret_cast<bf16*>(smem);
  bf16* outs = dyp + C2_XIN;
  float* red = reinterpret_cast<float*>(outs + C2_OUT);
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const bf16* dp2 = reinterpret_cast<const bf16*>(a.dp2) + (size_t)b * 2304;
  const uint8_t* am2 = a.am2 + (size_t)b * 2304;
  bf16* dy2 = reinterpret_cast<bf16*>(a.dy2) + (size_t)b * 9216;

  // halo of the padded 16x16 grad image
  for (int s = tid; s < 2048; s += 256) {
    const int pix = s >> 3, c = s & 7;
    const int r = pix >> 4, col = pix & 15;
    if (r < 2 || r >= 14 || col < 2 || col >= 14) *reinterpret_cast<bf16x8*>(dyp + swz128(pix, c)) = bf16x8{};
  }
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int task = tid; task < 1152; task += 256) {
    const int p = task >> 3, c = task & 7;
    const int y = p / 12, x = p - (p / 12) * 12;
    float accv[8];
    pool_bwd_gather<6>(dp2, am2, y, x, c, accv);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) { o[j] = (bf16)accv[j]; bsum[j] += (float)o[j]; }
    *reinterpret_cast<bf16x8*>(dyp + swz128((y + 2) * 16 + x + 2, c)) = o;
    *reinterpret_cast<bf16x8*>(dy2 + p * 64 + c * 8) = o;
  }
  block_chunk_sum(bsum, red, tid);
  __syncthreads();
  if (tid < 64) a.dbias_part[b * 64 + tid] = red[tid] + red[64 + tid] + red[128 + tid] + red[192 + tid];

  f32x4 acc[9];
  conv2_core(reinterpret_cast<const bf16*>(a.wd), dyp, acc, w, g, li);
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int px = 16 * t + li, cb = 16 * w + 4 * g;
    const bf16x4 v = pack4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
    *reinterpret_cast<bf16x4*>(outs + swz128(px, cb >> 3) + ((cb >> 2) & 1) * 4) = v;
  }
  __syncthreads();
  bf16* dp1 = reinterpret_cast<bf16*>(a.dp1) + (size_t)b * 9216;
  for (int s = tid; s < 1152; s += 256) {
    const int p = s >> 3, c = s & 7;
    *reinterpret_cast<bf16x8*>(dp1 + p * 64 + c * 8) = lds_b128(outs + swz128(p, c));
  }
}

// ---------------------------------------------------------------------------------------------
// Weight gradients.  Reduction index r = output pixel; both operands are NHWC LDS images read
// with the hardware transpose (lane 4q+p of a 16-lane group addresses row r = rb+q, cols 4p..4p+3).
constexpr int W2_XT = 12 * 16 * 32;     // conv2 x rows kh..kh+11, 16 cols, 32 ci (one half)
constexpr int W2_DY = 160 * 64;         // conv2 dy, 144 pixels + 16 zero rows
constexpr int WG_LDS_BYTES = (C1_XIN + C1_OUT) * 2 + 4 * 64 * 4;

DEV void conv2_wgrad_block(const DmlcConvWgradArgs& a, int blk, char* smem) {
  bf16* xt = reinterpret_cast<bf16*>(smem);
  bf16* dyt = xt + W2_XT;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int kh = blk % 5, hh = (blk / 5) & 1, grp = blk / 10;
  const int b0 = grp * a.B / a.g2, b1 = (grp + 1) * a.B / a.g2;

  f32x4 acc[5][2];
#pragma unroll
  for (int kw = 0; kw < 5; ++kw) { acc[kw][0] = zero4(); acc[kw][1] = zero4(); }

  for (int b = b0; b < b1; ++b) {
    const bf16* x = reinterpret_cast<const bf16*>(a.p1) + (size_t)b * 9216;
    const bf16* dy = reinterpret_cast<const bf16*>(a.dy2) + (size_t)b * 9216;
    for (int s = tid; s < 12 * 16 * 4; s += 256) {
      const int pix = s >> 2, c = s & 3;
      const int iy = kh + (pix >> 4) - 2, ix = (pix & 15) - 2;
      bf16x8 v = {};
      if (iy >= 0 && iy < 12 && ix >= 0 && ix < 12) v = glb_b128(x + (iy * 12 + ix) * 64 + hh * 32 + c * 8);
      *reinterpret_cast<bf16x8*>(xt + pix * 32 + c * 8) = v;
    }
    for (int s = tid; s < 160 * 8; s += 256) {
      const int pix = s >> 3, c = s & 7;
      bf16x8 v = {};
      if (pix < 144) v = glb_b128(dy + pix * 64 + c * 8);
      *reinterpret_cast<bf16x8*>(dyt + pix * 64 + c * 8) = v;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      const int rA = 32 * s + 8 * g + q, rB = rA + 4;
      const bf16x8 bf = tr_frag(dyt + rA * 64 + 16 * w + 4 * p, dyt + rB * 64 + 16 * w + 4 * p);
      const int cA = min(rA, 143), cB = min(rB, 143);
      const int yA = cA / 12, yB = cB / 12;
      const int pA = yA * 16 + cA - yA * 12, pB = yB * 16 + cB - yB * 12;
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const bf16x8 af = tr_frag(xt + (pA + kw) * 32 + 16 * mt + 4 * p, xt + (pB + kw) * 32 + 16 * mt + 4 * p);
          acc[kw][mt] = mfma16(af, bf, acc[kw][mt]);
        }
      }
    }
    __syncthreads();
  }
  float* out = a.part2 + (size_t)grp * 1600 * 64;
#pragma unroll
  for (int kw = 0; kw < 5; ++kw)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int krow = (kh * 5 + kw) * 64 + hh * 32 + 16 * mt + 4 * g + i;
        out[krow * 64 + 16 * w + li] = acc[kw][mt][i];
      }
}

DEV void conv1_wgrad_block(const DmlcConvWgradArgs& a, int grp, char* smem) {
  bf16* xin = reinterpret_cast<bf16*>(smem);
  bf16* dyt = xin + C1_XIN;
  float* red = reinterpret_cast<float*>(dyt + C1_OUT);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int b0 = grp * a.B / a.g1, b1 = (grp + 1) * a.B / a.g1;

  f32x4 acc[10];
#pragma unroll
  for (int mt = 0; mt < 10; ++mt) acc[mt] = zero4();
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  for (int b = b0; b < b1; ++b) {
    const int img = batch_index(a.src, a.B, b);
    stage_conv1_input(xin, a.data + (size_t)img * 3072, a.cy, a.cx, tid);
    const bf16* dp1 = reinterpret_cast<const bf16*>(a.dp1) + (size_t)b * 9216;
    const uint8_t* am1 = a.am1 + (size_t)b * 9216;
    for (int task = tid; task < 576 * 8; task += 256) {
      const int pp = task >> 3, c = task & 7;
      const int y = pp / 24, x = pp - (pp / 24) * 24;
      float accv[8];
      pool_bwd_gather<12>(dp1, am1, y, x, c, accv);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) { o[j] = (bf16)accv[j]; bsum[j] += (float)o[j]; }
      *reinterpret_cast<bf16x8*>(dyt + pp * 64 + c * 8) = o;
    }
    __syncthreads();
#pragma unroll 2
    for (int s = 0; s < 18; ++s) {
      const int rA = 32 * s + 8 * g + q, rB = rA + 4;
      const bf16x8 bf = tr_frag(dyt + rA * 64 + 16 * w + 4 * p, dyt + rB * 64 + 16 * w + 4 * p);
      const int yA = rA / 24, yB = rB / 24;
      const int xA = rA - yA * 24, xB = rB - yB * 24;
#pragma unroll
      for (int mt = 0; mt < 10; ++mt) {
        const int kh = mt >> 1, kw0 = 4 * (mt & 1);
        const bf16x8 af = tr_frag(xin + ((yA + kh) * 32 + xA + kw0 + p) * 4,
                                  xin + ((yB + kh) * 32 + xB + kw0 + p) * 4);
        acc[mt] = mfma16(af, bf, acc[mt]);
      }
    }
    __syncthreads();
  }
  float* out = a.part1 + (size_t)grp * 160 * 64;
#pragma unroll
  for (int mt = 0; mt < 10; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) out[(16 * mt + 4 * g + i) * 64 + 16 * w + li] = acc[mt][i];
  block_chunk_sum(bsum, red, tid);
  __syncthreads();
  if (tid < 64) a.partb1[grp * 64 + tid] = red[tid] + red[64 + tid] + red[128 + tid] + red[192 + tid];
}

__global__ __launch_bounds__(256, 2) void k_conv_wgrad(DmlcConvWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int blk = blockIdx.x;
  if (blk < 10 * a.g2) conv2_wgrad_block(a, blk, smem);
  else conv1_wgrad_block(a, blk - 10 * a.g2, smem);
}

}  // namespace dmlc

using namespace dmlc;

namespace {
// Kernels above 64 KiB of dynamic LDS must opt in once (gfx950 has 160 KiB per CU).
void allow_lds(const void* f, size_t bytes, bool& done) {
  if (!done) {
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    done = true;
  }
}
bool g_c1 = false, g_wg = false;
}  // namespace

extern "C" {

hipError_t dmlc_conv1_fwd(const DmlcConv1FwdArgs* a, hipStream_t s) {
  const size_t lds = (C1_XIN + C1_OUT) * 2;
  allow_lds(reinterpret_cast<const void*>(&k_conv1_fwd), lds, g_c1);
  hipLaunchKernelGGL(k_conv1_fwd, dim3(a->B), dim3(256), lds, s, *a);
  return hipGetLastError();
}

hipError_t dmlc_conv2_fwd(const DmlcConv2FwdArgs* a, hipStream_t s) {
  const size_t lds = (C2_XIN + C2_OUT) * 2;
  hipLaunchKernelGGL(k_conv2_fwd, dim3(a->B), dim3(256), lds, s, *a);
  return hipGetLastError();
}

hipError_t dmlc_conv2_dgrad(const DmlcConv2DgradArgs* a, hipStream_t s) {
  const size_t lds = (C2_XIN + C2_OUT) * 2 + 4 * 64 * 4;
  hipLaunchKernelGGL(k_conv2_dgrad, dim3(a->B), dim3(256), lds, s, *a);
  return hipGetLastError();
}

hipError_t dmlc_conv_wgrad(const DmlcConvWgradArgs* a, hipStream_t s) {
  static_assert((W2_XT + W2_DY) * 2 <= WG_LDS_BYTES, "conv2 wgrad staging must fit");
  allow_lds(reinterpret_cast<const void*>(&k_conv_wgrad), WG_LDS_BYTES, g_wg);
  hipLaunchKernelGGL(k_conv_wgrad, dim3(10 * a->g2 + a->g1), dim3(256), WG_LDS_BYTES, s, *a);
  return hipGetLastError();
}

}  // extern "C"
