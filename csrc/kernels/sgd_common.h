// SGD building blocks shared by the stand-alone SGD launch (cnn_sgd.hip) and the weight-gradient
// launch that applies the conv updates itself on a single GPU (cnn_wgrad.hip, DmlcWgradArgs::apply).
// Both paths must produce bit-identical weights, so the reduction orders and the update expression
// live here once (TF ApplyGradientDescent + ExponentialDecay, /root/reference/cifar10cnn.py:159-164).
//
// Every role function takes the block's thread index `tid` and works with threads tid < 256 (the
// SGD launch has exactly 256; the 512-thread wgrad blocks idle their upper half).  Functions that
// contain a workgroup barrier must be called by EVERY thread of the block.
#pragma once
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
// LDS (float4) the roles need: split sums over 512 threads (8 KB) or the fc2 transpose (6.8 KB)
constexpr int SGD_LDS4 = 512;
static_assert(FC2_COLS * (FC2_ROWS + 8) * 2 / 16 <= SGD_LDS4, "fc2 transpose tile exceeds the role LDS");

// fc1 weight + bias (contiguous float4 range, same-layout shadow): blocks of 1024 float4; with
// fc1_fused only the bias (the weights were updated by the dW1 GEMM epilogue)
__host__ __device__ inline int fc1_first(const DmlcSgdArgs& a) { return a.fc1_fused ? a.off[5] : a.off[4]; }
__host__ __device__ inline int fc1_blocks(const DmlcSgdArgs& a) {
  return ((a.off[6] - fc1_first(a)) / 4 + 256 * FC_F4_PER_THREAD - 1) / (256 * FC_F4_PER_THREAD);
}
// fc roles (fc1 bias / weights, fc2 tiles, fc tail) in launch order
__host__ __device__ inline int fc_role_count(const DmlcSgdArgs& a) { return fc1_blocks(a) + FC2_BLOCKS + FC_TAIL_BLOCKS; }

// The flat gradient, element e: fp32 `grad`, or bf16 `grad16` on the RCCL bf16 wire (api.h).
DEV float4 grad_ld4(const DmlcSgdArgs& a, size_t e) {
  if (a.grad16) {
    const bf16x4 v = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const bf16*>(a.grad16) + e);
    return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
  }
  return *reinterpret_cast<const float4*>(a.grad + e);
}
DEV void grad_st4(const DmlcSgdArgs& a, size_t e, const float4& g) {
  if (a.grad16) *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.grad16) + e) = pack4(g.x, g.y, g.z, g.w);
  else *reinterpret_cast<float4*>(a.grad + e) = g;
}
DEV float grad_ld1(const DmlcSgdArgs& a, size_t e) {
  return a.grad16 ? (float)reinterpret_cast<const bf16*>(a.grad16)[e] : a.grad[e];
}

DEV float lr_of(const DmlcSgdArgs& a, int64_t step) {
  return lr_sched(a.lr0, a.decay, a.decay_steps, a.staircase, a.warmup, step);
}

DEV float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }

// Deterministic split reduction of n fp32 slabs (float4 at p + q*stride).  Threads tid < 256 are
// S splits x (256/S) outputs; split sp sums slabs sp, sp+S, ... with up to U loads in flight, then
// split 0 adds the S partial sums in fixed order.  Returns the total on split-0 threads (tid < 256/S).
// Call with every thread of the block (one barrier); lds: >= 256 float4.
// coh: the slabs were written by other blocks of the SAME launch (agent-coherent sc1 loads from the
// wave-uniform base `cb`, p = cb + a per-lane offset); otherwise plain loads.
template <int S, int U = 8>
DEV float4 split_sum(const float* __restrict__ p, size_t stride, int n, float4* lds, int tid, bool coh = false,
                     const float* cb = nullptr) {
  constexpr int T = 256 / S;
  const int sp = tid / T, idx = tid % T;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  // U branch-free loads in flight per round (out-of-range slabs read slab 0 and add zero): a
  // remainder loop here would serialise one memory latency per slab
  if (tid < 256) {
    for (int q = sp; q < n; q += U * S) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u] = coh ? (q + u * S < n ? ld_sc1(buf_rsrc(cb), (uint32_t)((p - cb) + (size_t)(q + u * S) * stride) * 4)
                                    : make_float4(0.f, 0.f, 0.f, 0.f))
                   : load_sel(reinterpret_cast<const float4*>(p + (size_t)(q + u * S) * stride),
                              reinterpret_cast<const float4*>(p), q + u * S < n);
#pragma unroll
      for (int u = 0; u < U; ++u) s = add4(s, v[u]);
    }
    lds[tid] = s;
  }
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

// bf16 shadows of 4 updated conv2 weights W2[krow][co..co+3] (krow = (kh*5+kw)*64 + ci): the dgrad's
// flipped ci-major copy w2d and (bf16 forward) the co-major w2f
DEV void conv2_shadow4(const DmlcSgdArgs& a, int krow, int co, const float4& w) {
  const int ci = krow & 63, khw = krow >> 6;
  // w2d[ci][((4-kh)*5 + (4-kw))*64 + co] : contiguous in co
  *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.w2d) + (size_t)ci * 1600 + (24 - khw) * 64 + co) =
      pack4(w.x, w.y, w.z, w.w);
  if (!a.w2f8) {                                      // the bf16 forward's shadow (fp8: not read)
    bf16* w2f = reinterpret_cast<bf16*>(a.w2f) + krow;  // w2f[co][krow]
    w2f[(co + 0) * 1600] = (bf16)w.x; w2f[(co + 1) * 1600] = (bf16)w.y;
    w2f[(co + 2) * 1600] = (bf16)w.z; w2f[(co + 3) * 1600] = (bf16)w.w;
  }
}

// bf16 forward shadow w1f[co][96] (k = kh*16 + kw*3 + ci; conv_common.h C1_K) of 4 updated conv1 weights of HWIO row
// `row` = (kh*5+kw)*3 + ci, channels co..co+3
DEV void conv1_shadow4(const DmlcSgdArgs& a, int row, int co, const float4& w) {
  const int ci = row % 3, khw = row / 3, kh = khw / 5, kw = khw - kh * 5;
  const int k = kh * 16 + kw * 3 + ci;
  bf16* w1f = reinterpret_cast<bf16*>(a.w1f);
  w1f[(co + 0) * 96 + k] = (bf16)w.x;
  w1f[(co + 1) * 96 + k] = (bf16)w.y;
  w1f[(co + 2) * 96 + k] = (bf16)w.z;
  w1f[(co + 3) * 96 + k] = (bf16)w.w;
}

// conv biases: which 0 -> conv1 bias (g1 group partials), 1 -> conv2 bias (g2 group partials).
// Every thread of the block calls (split_sum barrier).
DEV void conv_bias(const DmlcSgdArgs& a, int which, float lr, float4* lds, int tid, bool coh = false) {
  const int c = (tid % 16) * 4;
  const int seg = which == 0 ? 1 : 3;
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f), w0 = g;
  if (a.mode != 1 && tid < 16) w0 = *reinterpret_cast<const float4*>(a.master + a.off[seg] + c);
  if (a.mode == 0 || a.mode == 1)
    g = split_sum<16>((which == 0 ? a.partb1 : a.partb2) + c, 64, which == 0 ? a.g1 : a.g2, lds, tid, coh,
                      which == 0 ? a.partb1 : a.partb2);
  if (tid >= 16) return;
  const size_t ge = (size_t)a.off[seg] + c;
  if (a.mode == 1) { grad_st4(a, ge, g); return; }
  if (a.mode == 2) g = grad_ld4(a, ge);
  sgd4(a.master + a.off[seg] + c, w0, g, lr, a.grad_scale, a.mode != 3);
}

DEV void fc1_block(const DmlcSgdArgs& a, int blk, float lr, int64_t step, int tid) {
  if (tid >= 256) return;
  const int base4 = fc1_first(a) >> 2, end4 = a.off[6] >> 2;
  // the shadow the NEXT step's kernels read (mode 3: this step's)
  bf16* shadow = reinterpret_cast<bf16*>(a.fc1n) + ((((a.mode == 3 ? step : step + 1) & 1) != 0) ? 884736 : 0);
  const bool apply = a.mode != 3;
  const float f = lr * a.grad_scale;
  int i4[FC_F4_PER_THREAD];
  float4 w[FC_F4_PER_THREAD], g[FC_F4_PER_THREAD];
#pragma unroll
  for (int u = 0; u < FC_F4_PER_THREAD; ++u) {
    i4[u] = base4 + (blk * FC_F4_PER_THREAD + u) * 256 + tid;
    const int ic = i4[u] < end4 ? i4[u] : base4;             // branch-free loads (clamped)
    w[u] = reinterpret_cast<const float4*>(a.master)[ic];
    g[u] = grad_ld4(a, (size_t)ic * 4);
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
// a block that moves 3x the average bytes finishes 2-3x later).  Every thread calls (one barrier).
DEV void fc2_block(const DmlcSgdArgs& a, int blk, float lr, bf16* tl /*[FC2_COLS][FC2_ROWS + 8]*/, int tid) {
  constexpr int LD = FC2_ROWS + 8, C4 = FC2_COLS / 4;
  constexpr int F4 = FC2_ROWS * C4 / 256;                      // float4 per thread (3)
  const bool apply = a.mode != 3, act = tid < 256;
  const float f = lr * a.grad_scale;
  const int k0 = (blk / (192 / FC2_COLS)) * FC2_ROWS, n0 = (blk % (192 / FC2_COLS)) * FC2_COLS;
  if (act) {
    float4 w[F4], g[F4];
#pragma unroll
    for (int u = 0; u < F4; ++u) {
      const int j4 = u * 256 + tid, kk = j4 / C4, n = n0 + 4 * (j4 - kk * C4);
      const size_t e = (size_t)a.off[6] + (size_t)(k0 + kk) * 192 + n;
      w[u] = *reinterpret_cast<const float4*>(a.master + e);
      g[u] = grad_ld4(a, e);
    }
#pragma unroll
    for (int u = 0; u < F4; ++u) {
      const int j4 = u * 256 + tid, kk = j4 / C4, nn = 4 * (j4 - kk * C4);
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
  }
  lds_barrier();
  if (!act) return;
  for (int c = tid; c < FC2_COLS * (FC2_ROWS / 8); c += 256) {
    const int nn = c / (FC2_ROWS / 8), k8 = c - nn * (FC2_ROWS / 8);
    *reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(a.fc2t) + (size_t)(n0 + nn) * 384 + k0 + 8 * k8) =
        *reinterpret_cast<const bf16x8*>(tl + nn * LD + 8 * k8);
  }
}

// fc2 bias, fc3 weight [192][10] (shadows fc3t[n][k], fc3d[k][n]) and fc3 bias: one scalar per thread
DEV void fc_tail_block(const DmlcSgdArgs& a, int blk, float lr, int tid) {
  if (tid >= 256) return;
  const int j = blk * 256 + tid;
  if (j >= FC_TAIL) return;
  const int i = a.off[7] + j;
  float v = a.master[i];
  if (a.mode != 3) {
    v -= lr * a.grad_scale * grad_ld1(a, i);
    a.master[i] = v;
  }
  if (i >= a.off[8] && i < a.off[8] + 1920) {
    const int q = i - a.off[8], k = q / 10, n = q - k * 10;
    reinterpret_cast<bf16*>(a.fc3t)[n * 192 + k] = (bf16)v;
    reinterpret_cast<bf16*>(a.fc3d)[k * 32 + n] = (bf16)v;
  }
}

// fc role r of fc_role_count(a) (fc1, then the fc2 tiles, then the fc tail).  Every thread calls.
DEV void fc_role(const DmlcSgdArgs& a, int r, float lr, int64_t step, float4* lds, int tid) {
  const int nfc1 = fc1_blocks(a);
  if (r < nfc1) fc1_block(a, r, lr, step, tid);
  else if ((r -= nfc1) < FC2_BLOCKS) fc2_block(a, r, lr, reinterpret_cast<bf16*>(lds), tid);
  else fc_tail_block(a, r - FC2_BLOCKS, lr, tid);
}

// The next step's raw image of batch row `row` into xnext[row] (192 16-B chunks; threads tid < 192 of
// the caller copy one each).  Called once every reader of the current xnext contents is done.
DEV void copy_next_row(const DmlcSgdArgs& a, int64_t step, int row, int tid) {
  if (tid >= 192) return;
  const int src = order_row(a.next, step + 1, row);
  reinterpret_cast<uint4*>(a.xnext + (size_t)row * 3072)[tid] =
      reinterpret_cast<const uint4*>(a.xdata + (size_t)src * 3072)[tid];
}

// Publish the step's stats into the ring and bump the device global_step (one wave, lanes < 64).
// loss / accuracy partials come from the head (an earlier launch).
DEV void publish_step(const DmlcSgdArgs& a, int64_t step, float lr, int lane) {
  float loss = 0.f, corr = 0.f;
  for (int q = lane; q < a.nhead; q += 64) { loss += a.loss_part[q]; corr += (float)a.correct_part[q]; }
  loss = wave_sum(loss);
  corr = wave_sum(corr);
  if (lane == 0) {
    float* st = a.stats + (size_t)(step % a.stats_len) * 4;
    st[0] = (float)(step + 1);
    st[1] = loss / (float)a.B;
    st[2] = corr / (float)a.B;
    st[3] = lr;
    *a.step = step + 1;
  }
}

}  // namespace dmlc
