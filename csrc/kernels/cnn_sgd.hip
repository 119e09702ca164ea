// Fused SGD step over the flat fp32 parameter buffer.
//
// Replaces TF's ApplyGradientDescent x10 + ExponentialDecay + AssignAdd(global_step)
// (/root/reference/cifar10cnn.py:159-164; SURVEY.md §2.B N13/N14, §2.C sgd_fused) and, on the way,
// finishes the split-K weight-gradient reductions of the conv kernels (deterministic fixed-order
// sums of the fp32 partial slabs) and refreshes the bf16 shadow copies of every weight in the
// layouts the MFMA kernels consume.  Everything it needs (step, LR schedule) lives in device memory,
// so the launch is graph-capturable; the LAST workgroup to arrive (agent-scope ticket) increments
// global_step and publishes {step, loss, accuracy, lr} into a device stats ring, so the host never
// has to synchronise for logging.
//
// Block roles (one launch, ranges of blockIdx.x in this order, all 256 threads):
//   conv1 rows  : half (32 co) of one of the 75 HWIO rows per block, g1 slabs split 32 ways.
//   conv biases : 2 blocks over the per-group partial rows of each conv.
//   conv2 rows  : 4 weight rows (k = (kh,kw,ci)) x 64 co per block (400 blocks); the g2 slabs are
//                 split over 4 thread groups (<= 8 loads in flight each) and combined in fixed order;
//                 shadows w2f (co-major) and w2d (flipped, ci-major).
//   fc1         : float4 groups of fc1 weight + bias (contiguous, 64-aligned), 4 per thread;
//   fc2         : 64 weight rows per block, transposed shadow through LDS;  fc tail: fc2 bias + fc3.
// modes: 0 = reduce + apply (single GPU), 1 = reduce only (conv grads -> flat grad, before the DP
// all-reduce; fc blocks are not launched), 2 = apply from the flat grad (after the all-reduce),
// 3 = refresh the shadows only (after init / checkpoint restore).
#include "common.h"
#include "api.h"

namespace dmlc {

constexpr int SEG_NUMEL[10] = {4800, 64, 102400, 64, 884736, 384, 73728, 192, 1920, 10};
constexpr int C2_SPLIT = 4, C2_ROWS = 256 / C2_SPLIT / 16;   // 4 rows x 64 co per block
constexpr int C2_BLOCKS = 1600 / C2_ROWS;                     // 400
constexpr int C1_SPLIT = 32;                                  // 1 row x 32 co per block
constexpr int C1_LOADS = 5;                                   // g1 <= 160 slabs: one round of loads
constexpr int C1_BLOCKS = 150;
constexpr int FC_F4_PER_THREAD = 4;
constexpr int FC2_ROWS = 64, FC2_COLS = 48;                  // fc2 weight tile (k x n) per block
constexpr int FC2_BLOCKS = (384 / FC2_ROWS) * (192 / FC2_COLS);   // 24
constexpr int FC_TAIL = 192 + 1920 + 10;                      // fc2 bias, fc3 weight + bias
constexpr int FC_TAIL_BLOCKS = (FC_TAIL + 255) / 256;         // one element per thread

// fc1 weight + bias (contiguous float4 range, same-layout shadow): blocks of 1024 float4; with
// fc1_fused only the bias (the weights were updated by the dW1 GEMM epilogue)
__host__ __device__ inline int fc1_first(const DmlcSgdArgs& a) { return a.fc1_fused ? a.off[5] : a.off[4]; }
__host__ __device__ inline int fc1_blocks(const DmlcSgdArgs& a) {
  return ((a.off[6] - fc1_first(a)) / 4 + 256 * FC_F4_PER_THREAD - 1) / (256 * FC_F4_PER_THREAD);
}

DEV float lr_of(const DmlcSgdArgs& a, int64_t step) {
  return lr_sched(a.lr0, a.decay, a.decay_steps, a.staircase, a.warmup, step);
}

DEV float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

// Deterministic split reduction of n fp32 slabs (float4 at p + q*stride).  The block's threads are
// S splits x (256/S) outputs; split sp sums slabs sp, sp+S, ... with up to 8 loads in flight, then
// split 0 adds the S partial sums in fixed order.  Returns the total on split-0 threads.
template <int S, int U = 8>
DEV float4 split_sum(const float* __restrict__ p, size_t stride, int n, float4* lds) {
  constexpr int T = 256 / S;
  const int sp = threadIdx.x / T, idx = threadIdx.x % T;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  // U branch-free loads in flight per round (out-of-range slabs read slab 0 and add zero): a
  // remainder loop here would serialise one memory latency per slab
  for (int q = sp; q < n; q += U * S) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = load_sel(reinterpret_cast<const float4*>(p + (size_t)(q + u * S) * stride),
                      reinterpret_cast<const float4*>(p), q + u * S < n);
#pragma unroll
    for (int u = 0; u < U; ++u) s = add4(s, v[u]);
  }
  lds[threadIdx.x] = s;
  __syncthreads();
  float4 t = lds[idx];
#pragma unroll
  for (int k = 1; k < S; ++k) t = add4(t, lds[k * T + idx]);
  return t;
}

// The same over bf16 slabs (4 bf16 = 8 bytes per slab and thread), summed in fp32 in the same order.
DEV float4 bf4(uint2 u) {
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}
template <int S, int U = 8>
DEV float4 split_sum_bf16(const bf16* __restrict__ p, size_t stride, int n, float4* lds) {
  constexpr int T = 256 / S;
  const int sp = threadIdx.x / T, idx = threadIdx.x % T;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int q = sp; q < n; q += U * S) {
    uint2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = load_sel(reinterpret_cast<const uint2*>(p + (size_t)(q + u * S) * stride), reinterpret_cast<const uint2*>(p),
                      q + u * S < n);
#pragma unroll
    for (int u = 0; u < U; ++u) s = add4(s, bf4(v[u]));
  }
  lds[threadIdx.x] = s;
  __syncthreads();
  float4 t = lds[idx];
#pragma unroll
  for (int k = 1; k < S; ++k) t = add4(t, lds[k * T + idx]);
  return t;
}

// w: the master value, loaded by the caller BEFORE the slab reduction so that its memory latency
// overlaps the slab loads instead of adding a second dependent round trip
DEV float4 sgd4(float* m, float4 w, float4 g, float lr, float scale, bool apply) {
  if (apply) {
    const float f = lr * scale;
    w.x -= f * g.x; w.y -= f * g.y; w.z -= f * g.z; w.w -= f * g.w;
    *reinterpret_cast<float4*>(m) = w;
  }
  return w;
}

DEV void conv2_rows(const DmlcSgdArgs& a, int blk, float lr, float4* lds) {
  constexpr int T = 256 / C2_SPLIT;
  const int idx = threadIdx.x % T, r = idx >> 4, co = (idx & 15) * 4;
  const int krow = blk * C2_ROWS + r;                 // (kh*5+kw)*64 + ci
  const size_t e = (size_t)krow * 64 + co;
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f), w0 = g;
  if (a.mode != 1 && threadIdx.x < T) w0 = *reinterpret_cast<const float4*>(a.master + a.off[2] + e);
  // fp8: the previous weights' amax = max of the C2_BLOCKS per-block maxima the last launch stored
  // (plain stores, no same-address atomics), loaded by wave 0 beside the slab loads
  float am[(C2_BLOCKS + 63) / 64];
  if (a.w2f8 && a.mode != 1 && threadIdx.x < T) {
    const float* src = a.amax_w + (size_t)(*a.step_rd & 1) * C2_BLOCKS;
#pragma unroll
    for (int u = 0; u < (C2_BLOCKS + 63) / 64; ++u) {
      const int i = threadIdx.x + 64 * u;
      am[u] = src[i < C2_BLOCKS ? i : 0];
    }
  }
  if (a.mode == 0 || a.mode == 1)
    g = a.part2_bf16 ? split_sum_bf16<C2_SPLIT>(reinterpret_cast<const bf16*>(a.part2) + e, 1600 * 64, a.g2, lds)
                     : split_sum<C2_SPLIT>(reinterpret_cast<const float*>(a.part2) + e, 1600 * 64, a.g2, lds);
  if (threadIdx.x >= T) return;
  if (a.mode == 2) g = *reinterpret_cast<const float4*>(a.grad + a.off[2] + e);
  if (a.mode == 1) { *reinterpret_cast<float4*>(a.grad + a.off[2] + e) = g; return; }
  const float4 w = sgd4(a.master + a.off[2] + e, w0, g, lr, a.grad_scale, a.mode != 3);
  const int ci = krow & 63, khw = krow >> 6;
  if (a.w2f8) {                                       // fp8 shadow for the fp8 conv2 forward
    const int64_t step = *a.step_rd;
    const int cur = (int)(step & 1), nxt = a.mode == 3 ? cur : cur ^ 1;
    float amax = am[0];
#pragma unroll
    for (int u = 1; u < (C2_BLOCKS + 63) / 64; ++u) amax = fmaxf(amax, am[u]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
    const float sw = 224.f / fmaxf(amax, 1e-20f);
    const uint32_t q = pk_fp8x4(w.x * sw, w.y * sw, w.z * sw, w.w * sw);
    uint8_t* w8 = a.w2f8 + krow;
    w8[(co + 0) * 1600] = (uint8_t)q; w8[(co + 1) * 1600] = (uint8_t)(q >> 8);
    w8[(co + 2) * 1600] = (uint8_t)(q >> 16); w8[(co + 3) * 1600] = (uint8_t)(q >> 24);
    // the fp8 dgrad's flipped ci-major copy: the same 4 bytes, contiguous in co
    if (a.w2d8) *reinterpret_cast<uint32_t*>(a.w2d8 + (size_t)ci * 1600 + (24 - khw) * 64 + co) = q;
    // identical value from every block, into BOTH slots: the training forward runs without a step
    // counter (slot 0) and must dequantise with the scale this launch quantised w2f8 with
    if (threadIdx.x == 0) { a.scale_w[0] = sw; a.scale_w[1] = sw; }
    if (a.mode != 3) {
      float m = fmaxf(fmaxf(fabsf(w.x), fabsf(w.y)), fmaxf(fabsf(w.z), fabsf(w.w)));
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
      if (threadIdx.x == 0) a.amax_w[(size_t)nxt * C2_BLOCKS + blk] = m;
    }
  }
  // w2d[ci][((4-kh)*5 + (4-kw))*64 + co] : contiguous in co
  *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.w2d) + (size_t)ci * 1600 + (24 - khw) * 64 + co) =
      pack4(w.x, w.y, w.z, w.w);
  if (!a.w2f8) {                                      // the bf16 forward's shadow (fp8: not read)
    bf16* w2f = reinterpret_cast<bf16*>(a.w2f) + krow;  // w2f[co][krow]
    w2f[(co + 0) * 1600] = (bf16)w.x; w2f[(co + 1) * 1600] = (bf16)w.y;
    w2f[(co + 2) * 1600] = (bf16)w.z; w2f[(co + 3) * 1600] = (bf16)w.w;
  }
}

DEV void conv1_rows(const DmlcSgdArgs& a, int blk, float lr, float4* lds) {
  constexpr int T = 256 / C1_SPLIT;
  const int row = blk >> 1, co = (blk & 1) * 32 + (threadIdx.x % T) * 4;   // HWIO row = (kh*5+kw)*3 + ci
  const int ci = row % 3, khw = row / 3, kh = khw / 5, kw = khw - kh * 5;
  const size_t e = (size_t)row * 64 + co;
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f), w0 = g;
  if (a.mode != 1 && threadIdx.x < T) w0 = *reinterpret_cast<const float4*>(a.master + a.off[0] + e);
  if (a.mode == 0 || a.mode == 1)                     // slab row k'' = kh*16 + kw*3 + ci
    g = split_sum<C1_SPLIT, C1_LOADS>(a.part1 + (size_t)(kh * 16 + kw * 3 + ci) * 64 + co, 80 * 64, a.g1, lds);
  if (threadIdx.x >= T) return;
  if (a.mode == 2) g = *reinterpret_cast<const float4*>(a.grad + a.off[0] + e);
  if (a.mode == 1) { *reinterpret_cast<float4*>(a.grad + a.off[0] + e) = g; return; }
  const float4 w = sgd4(a.master + a.off[0] + e, w0, g, lr, a.grad_scale, a.mode != 3);
  const int k = kh * 32 + kw * 4 + ci;                // forward shadow layout w1f[co][160]
  bf16* w1f = reinterpret_cast<bf16*>(a.w1f);
  w1f[(co + 0) * 160 + k] = (bf16)w.x;
  w1f[(co + 1) * 160 + k] = (bf16)w.y;
  w1f[(co + 2) * 160 + k] = (bf16)w.z;
  w1f[(co + 3) * 160 + k] = (bf16)w.w;
}

// conv biases: block 0 -> conv1 bias (g1 group partials), block 1 -> conv2 bias (g2 group partials)
DEV void conv_bias(const DmlcSgdArgs& a, int which, float lr, float4* lds) {
  const int c = (threadIdx.x % 16) * 4;
  const int seg = which == 0 ? 1 : 3;
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f), w0 = g;
  if (a.mode != 1 && threadIdx.x < 16) w0 = *reinterpret_cast<const float4*>(a.master + a.off[seg] + c);
  if (a.mode == 0 || a.mode == 1)
    g = split_sum<16>((which == 0 ? a.partb1 : a.partb2) + c, 64, which == 0 ? a.g1 : a.g2, lds);
  if (threadIdx.x >= 16) return;
  float* gp = a.grad + a.off[seg] + c;
  if (a.mode == 1) { *reinterpret_cast<float4*>(gp) = g; return; }
  if (a.mode == 2) g = *reinterpret_cast<const float4*>(gp);
  sgd4(a.master + a.off[seg] + c, w0, g, lr, a.grad_scale, a.mode != 3);
}

DEV void fc1_block(const DmlcSgdArgs& a, int blk, float lr, int64_t step) {
  const int base4 = fc1_first(a) >> 2, end4 = a.off[6] >> 2;
  // the shadow the NEXT step's kernels read (mode 3: this step's)
  bf16* shadow = reinterpret_cast<bf16*>(a.fc1n) + ((((a.mode == 3 ? step : step + 1) & 1) != 0) ? 884736 : 0);
  const bool apply = a.mode != 3;
  const float f = lr * a.grad_scale;
  int i4[FC_F4_PER_THREAD];
  float4 w[FC_F4_PER_THREAD], g[FC_F4_PER_THREAD];
#pragma unroll
  for (int u = 0; u < FC_F4_PER_THREAD; ++u) {
    i4[u] = base4 + (blk * FC_F4_PER_THREAD + u) * 256 + threadIdx.x;
    const int ic = i4[u] < end4 ? i4[u] : base4;             // branch-free loads (clamped)
    w[u] = reinterpret_cast<const float4*>(a.master)[ic];
    g[u] = reinterpret_cast<const float4*>(a.grad)[ic];
  }
#pragma unroll
  for (int u = 0; u < FC_F4_PER_THREAD; ++u) {
    const int i = i4[u] * 4;
    if (i4[u] >= end4) continue;
    float4 v = w[u];
    if (apply) {
      v.x -= f * g[u].x; v.y -= f * g[u].y; v.z -= f * g[u].z; v.w -= f * g[u].w;
      reinterpret_cast<float4*>(a.master)[i4[u]] = v;
    }
    if (i < a.off[5])                                 // fc1 weight [2304][384]: same layout shadow
      *reinterpret_cast<bf16x4*>(shadow + (i - a.off[4])) = pack4(v.x, v.y, v.z, v.w);
  }
}

// fc2 weight [384 k][192 n], one FC2_ROWS x FC2_COLS tile per block: shadows fc2n[k][n] (same
// layout) and fc2t[n][k].  The transposed copy goes through LDS so every global store is a 16-B chunk
// of a whole 128-B fc2t row segment (2-byte stores scattered over 192 rows made these blocks the
// SGD's tail); tiles keep each block's bytes near the other roles' (the launch is bandwidth-bound:
// a block that moves 3x the average bytes finishes 2-3x later).
DEV void fc2_block(const DmlcSgdArgs& a, int blk, float lr, bf16* tl /*[FC2_COLS][FC2_ROWS + 8]*/) {
  constexpr int LD = FC2_ROWS + 8, C4 = FC2_COLS / 4;
  constexpr int F4 = FC2_ROWS * C4 / 256;                      // float4 per thread (3)
  const bool apply = a.mode != 3;
  const float f = lr * a.grad_scale;
  const int k0 = (blk / (192 / FC2_COLS)) * FC2_ROWS, n0 = (blk % (192 / FC2_COLS)) * FC2_COLS;
  float4 w[F4], g[F4];
#pragma unroll
  for (int u = 0; u < F4; ++u) {
    const int j4 = u * 256 + threadIdx.x, kk = j4 / C4, n = n0 + 4 * (j4 - kk * C4);
    const size_t e = (size_t)a.off[6] + (size_t)(k0 + kk) * 192 + n;
    w[u] = *reinterpret_cast<const float4*>(a.master + e);
    g[u] = *reinterpret_cast<const float4*>(a.grad + e);
  }
#pragma unroll
  for (int u = 0; u < F4; ++u) {
    const int j4 = u * 256 + threadIdx.x, kk = j4 / C4, nn = 4 * (j4 - kk * C4);
    float4 v = w[u];
    if (apply) {
      v.x -= f * g[u].x; v.y -= f * g[u].y; v.z -= f * g[u].z; v.w -= f * g[u].w;
      *reinterpret_cast<float4*>(a.master + a.off[6] + (size_t)(k0 + kk) * 192 + n0 + nn) = v;
    }
    *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.fc2n) + (size_t)(k0 + kk) * 192 + n0 + nn) =
        pack4(v.x, v.y, v.z, v.w);
    tl[(nn + 0) * LD + kk] = (bf16)v.x; tl[(nn + 1) * LD + kk] = (bf16)v.y;
    tl[(nn + 2) * LD + kk] = (bf16)v.z; tl[(nn + 3) * LD + kk] = (bf16)v.w;
  }
  lds_barrier();
  for (int c = threadIdx.x; c < FC2_COLS * (FC2_ROWS / 8); c += 256) {
    const int nn = c / (FC2_ROWS / 8), k8 = c - nn * (FC2_ROWS / 8);
    *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(a.fc2t) + (size_t)(n0 + nn) * 384 + k0 + 8 * k8) =
        *reinterpret_cast<const bf16x8*>(tl + nn * LD + 8 * k8);
  }
}

// fc2 bias, fc3 weight [192][10] (shadows fc3t[n][k], fc3d[k][n]) and fc3 bias: one scalar per thread
DEV void fc_tail_block(const DmlcSgdArgs& a, int blk, float lr) {
  const int j = blk * 256 + threadIdx.x;
  if (j >= FC_TAIL) return;
  const int i = a.off[7] + j;
  float v = a.master[i];
  if (a.mode != 3) {
    v -= lr * a.grad_scale * a.grad[i];
    a.master[i] = v;
  }
  if (i >= a.off[8] && i < a.off[8] + 1920) {
    const int q = i - a.off[8], k = q / 10, n = q - k * 10;
    reinterpret_cast<bf16*>(a.fc3t)[n * 192 + k] = (bf16)v;
    reinterpret_cast<bf16*>(a.fc3d)[k * 32 + n] = (bf16)v;
  }
}

__global__ __launch_bounds__(256) void k_sgd(DmlcSgdArgs a) {
  constexpr int LDS4 = FC2_COLS * (FC2_ROWS + 8) * 2 / 16 > 256 ? FC2_COLS * (FC2_ROWS + 8) * 2 / 16 : 256;
  __shared__ float4 lds[LDS4];                                // split sums (4 KB), fc2 transpose (6.8 KB)
  DMLC_STAMP(DMLC_TK_SGD, 0);
  const int64_t step = *a.step_rd;
  const float lr = lr_of(a, step);
  const int nfc1 = fc1_blocks(a);
  int blk = blockIdx.x + (a.roles == 2 ? C2_BLOCKS + C1_BLOCKS + 2 : 0);
  // the slowest role (conv1 rows: 128 slabs per output) takes the lowest block ids, dispatched first
  // (conv2 rows first measured 0.9 % slower per step: the late conv1 blocks were the launch's tail)
  if (blk < C1_BLOCKS) conv1_rows(a, blk, lr, lds);
  else if ((blk -= C1_BLOCKS) < 2) conv_bias(a, blk, lr, lds);
  else if ((blk -= 2) < C2_BLOCKS) conv2_rows(a, blk, lr, lds);
  else if ((blk -= C2_BLOCKS) < nfc1) fc1_block(a, blk, lr, step);
  else if ((blk -= nfc1) < FC2_BLOCKS) fc2_block(a, blk, lr, reinterpret_cast<bf16*>(lds));
  else fc_tail_block(a, blk - FC2_BLOCKS, lr);
  DMLC_STAMP(DMLC_TK_SGD, 1);

  if (!(a.mode == 0 || a.mode == 2) || !a.finalize) return;
  // the next step's batch rows (no kernel of this step reads bidx any more: they all ran before)
  if (a.bidx && (int)blockIdx.x * 256 < a.bidx_n) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r < a.bidx_n) a.bidx[r] = order_row(a.next, step + 1, r);
  }
  if (a.step_rd != a.step) {
    // the step was read from the head's copy: no block of this launch reads *a.step, so workgroup 0
    // alone sums the head's partials (an earlier launch), publishes the stats and bumps the counter
    // -- no arrival ticket (two dependent atomic round trips on the launch's critical path)
    if (blockIdx.x == 0 && threadIdx.x < 64) {
      float loss = 0.f, corr = 0.f;
      for (int q = threadIdx.x; q < a.nhead; q += 64) { loss += a.loss_part[q]; corr += (float)a.correct_part[q]; }
      loss = wave_sum(loss);
      corr = wave_sum(corr);
      if (threadIdx.x == 0) {
        float* st = a.stats + (size_t)(step % a.stats_len) * 4;
        st[0] = (float)(step + 1);
        st[1] = loss / (float)a.B;
        st[2] = corr / (float)a.B;
        st[3] = lr;
        *a.step = step + 1;
      }
    }
    DMLC_STAMP(DMLC_TK_SGD, 2);
    return;
  }
  // last arriver: bump global_step, publish stats, re-arm the ticket for the next launch (the engine
  // zeroes it once at creation; every launch that starts also completes, so it stays consistent).
  // Nothing is published THROUGH the ticket (loss/accuracy partials come from an earlier launch and
  // the step/stats are consumed by later launches), so no release/acquire fences: an agent-scope
  // release is an L2 write-back on every XCD, which 700 blocks would pay for nothing.  The only
  // ordering needed -- every block has read *a.step before the last one bumps it -- holds once every
  // wave of the block is past its update code, which consumed lr (hence *a.step): an LDS-only
  // barrier (its lgkmcnt(0) also retires the scalar load) instead of __syncthreads(), whose vmcnt(0)
  // would hold the ticket until every store of the block had been acknowledged.
  lds_barrier();
  if (threadIdx.x < 64) {                              // wave 0: ticket, then (last) the stats
    // the head's per-workgroup partials (an earlier launch), loaded by EVERY block's wave 0 together
    // with its ticket: the last arriver then has them in registers instead of paying one more memory
    // round trip on the launch's critical path (802 x 512 B of L2 reads, nothing)
    // (branch-free, clamped: no wait between these loads and the ticket atomic, which then share
    // one memory latency; partials beyond 256 -- per-GPU batch > 1024 -- are summed by the last only)
    float lv[4];
    int cv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = threadIdx.x + 64 * u, qc = q < a.nhead ? q : 0;
      lv[u] = a.loss_part[qc];
      cv[u] = a.correct_part[qc];
    }
    int last = 0;
    if (threadIdx.x == 0) last = last_arrival(a.ticket, blockIdx.x, gridDim.x) ? 1 : 0;
    if (__shfl(last, 0)) {
      float loss = 0.f, corr = 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (threadIdx.x + 64 * u < a.nhead) { loss += lv[u]; corr += (float)cv[u]; }
      for (int q = threadIdx.x + 256; q < a.nhead; q += 64) { loss += a.loss_part[q]; corr += (float)a.correct_part[q]; }
      loss = wave_sum(loss);
      corr = wave_sum(corr);
      if (threadIdx.x == 0) {
        float* st = a.stats + (size_t)(step % a.stats_len) * 4;
        st[0] = (float)(step + 1);
        st[1] = loss / (float)a.B;
        st[2] = corr / (float)a.B;
        st[3] = lr;
        *a.step = step + 1;
      }
    }
  }
  DMLC_STAMP(DMLC_TK_SGD, 2);
}

}  // namespace dmlc

using namespace dmlc;

extern "C" hipError_t dmlc_sgd(DmlcSgdArgs* a, hipStream_t s) {
  if (a->off[5] - a->off[4] != 884736 || a->off[6] % 4 || a->off[6] - a->off[4] != 884736 + 384 ||
      a->off[7] - a->off[6] != 73728 || a->off[8] - a->off[7] != 192 || a->off[9] - a->off[8] != 1920)
    return hipErrorInvalidValue;                      // the fc segments must be contiguous, float4-aligned
  const int fc_blocks = fc1_blocks(*a) + FC2_BLOCKS + FC_TAIL_BLOCKS;
  const int conv_blocks = C2_BLOCKS + C1_BLOCKS + 2;
  int blocks = conv_blocks + (a->mode == 1 ? 0 : fc_blocks);
  if (a->roles == 1) blocks = conv_blocks;
  if (a->roles == 2) blocks = a->mode == 1 ? 0 : fc_blocks;
  if (blocks == 0) return hipSuccess;
  a->nblocks = blocks;
  hipLaunchKernelGGL(k_sgd, dim3(blocks), dim3(256), 0, s, *a);
  return hipGetLastError();
}
