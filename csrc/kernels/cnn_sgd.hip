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
#include "sgd_common.h"

namespace dmlc {

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
    g = split_sum<C2_SPLIT>(reinterpret_cast<const float*>(a.part2) + e, 1600 * 64, a.g2, lds, threadIdx.x);
  if (threadIdx.x >= T) return;
  if (a.mode == 2) g = grad_ld4(a, a.off[2] + e);
  if (a.mode == 1) { grad_st4(a, a.off[2] + e, g); return; }
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
  conv2_shadow4(a, krow, co, w);
}

DEV void conv1_rows(const DmlcSgdArgs& a, int blk, float lr, float4* lds) {
  constexpr int T = 256 / C1_SPLIT;
  const int row = blk >> 1, co = (blk & 1) * 32 + (threadIdx.x % T) * 4;   // HWIO row = (kh*5+kw)*3 + ci
  const int ci = row % 3, khw = row / 3, kh = khw / 5, kw = khw - kh * 5;
  const size_t e = (size_t)row * 64 + co;
  float4 g = make_float4(0.f, 0.f, 0.f, 0.f), w0 = g;
  if (a.mode != 1 && threadIdx.x < T) w0 = *reinterpret_cast<const float4*>(a.master + a.off[0] + e);
  if (a.mode == 0 || a.mode == 1)                     // slab row k'' = kh*16 + kw*3 + ci
    g = split_sum<C1_SPLIT, C1_LOADS>(a.part1 + (size_t)(kh * 16 + kw * 3 + ci) * 64 + co, 80 * 64, a.g1, lds, threadIdx.x);
  if (threadIdx.x >= T) return;
  if (a.mode == 2) g = grad_ld4(a, a.off[0] + e);
  if (a.mode == 1) { grad_st4(a, a.off[0] + e, g); return; }
  conv1_shadow4(a, row, co, sgd4(a.master + a.off[0] + e, w0, g, lr, a.grad_scale, a.mode != 3));
}

__global__ __launch_bounds__(256) void k_sgd(DmlcSgdArgs a) {
  __shared__ float4 lds[SGD_LDS4];                            // split sums, fc2 transpose
  DMLC_STAMP(DMLC_TK_SGD, 0);
  const int64_t step = *a.step_rd;
  const float lr = lr_of(a, step);
  int blk = blockIdx.x + (a.roles == 2 ? C2_BLOCKS + C1_BLOCKS + 2 : 0);
  // the slowest role (conv1 rows: 128 slabs per output) takes the lowest block ids, dispatched first
  // (conv2 rows first measured 0.9 % slower per step: the late conv1 blocks were the launch's tail)
  if (blk < C1_BLOCKS) conv1_rows(a, blk, lr, lds);
  else if ((blk -= C1_BLOCKS) < 2) conv_bias(a, blk, lr, lds, threadIdx.x);
  else if ((blk -= 2) < C2_BLOCKS) conv2_rows(a, blk, lr, lds);
  else fc_role(a, blk - C2_BLOCKS, lr, step, lds, threadIdx.x);
  DMLC_STAMP(DMLC_TK_SGD, 1);

  if (!(a.mode == 0 || a.mode == 2) || !a.finalize) return;
  // the next step's batch rows (no kernel of this step reads bidx any more: they all ran before)
  if (a.bidx && (int)blockIdx.x * 256 < a.bidx_n) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r < a.bidx_n) a.bidx[r] = order_row(a.next, step + 1, r);
  }
  // ... and their raw images (the wgrad launch, the last reader of xnext, has completed)
  if (a.xnext)
    for (int r = blockIdx.x; r < a.bidx_n; r += gridDim.x) copy_next_row(a, step, r, threadIdx.x);
  if (a.step_rd != a.step) {
    // the step was read from the head's copy: no block of this launch reads *a.step, so workgroup 0
    // alone sums the head's partials (an earlier launch), publishes the stats and bumps the counter
    // -- no arrival ticket (two dependent atomic round trips on the launch's critical path)
    if (blockIdx.x == 0 && threadIdx.x < 64) publish_step(a, step, lr, threadIdx.x);
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
  const int fc_blocks = fc_role_count(*a);
  const int conv_blocks = C2_BLOCKS + C1_BLOCKS + 2;
  int blocks = conv_blocks + (a->mode == 1 ? 0 : fc_blocks);
  if (a->roles == 1) blocks = conv_blocks;
  if (a->roles == 2) blocks = a->mode == 1 ? 0 : fc_blocks;
  if (blocks == 0) return hipSuccess;
  a->nblocks = blocks;
  hipLaunchKernelGGL(k_sgd, dim3(blocks), dim3(256), 0, s, *a);
  return hipGetLastError();
}
