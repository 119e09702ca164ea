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
// modes: 0 = reduce + apply (single GPU), 1 = reduce only (conv grads -> flat grad, before the DP
// all-reduce), 2 = apply from the flat grad (after the all-reduce, grad_scale = 1/world),
// 3 = refresh the shadows only (after init / checkpoint restore).
#include "common.h"
#include "api.h"

namespace dmlc {

constexpr int SEG_NUMEL[10] = {4800, 64, 102400, 64, 884736, 384, 73728, 192, 1920, 10};

DEV float conv_bias_grad(const float* __restrict__ part, int n, int co, int tid, float* red) {
  // deterministic sum over n partial rows [n][64] by the whole workgroup (4 threads per channel)
  (void)co;
  const int c = tid & 63, qd = tid >> 6;
  float s = 0.f;
  for (int i = qd; i < n; i += 4) s += part[i * 64 + c];
  red[tid] = s;
  __syncthreads();
  float r = 0.f;
  if (tid < 64) r = red[tid] + red[tid + 64] + red[tid + 128] + red[tid + 192];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void k_sgd(DmlcSgdArgs a) {
  __shared__ float red[256];
  const int tid = threadIdx.x;
  const int64_t step = *a.step;
  float lr = a.lr0;
  if (a.staircase) lr = a.lr0 * powf(a.decay, floorf((float)step / a.decay_steps));
  const bool apply = a.mode == 0 || a.mode == 2;
  const bool reduce = a.mode == 0 || a.mode == 1;
  const float scale = a.grad_scale;
  bf16* w1f = reinterpret_cast<bf16*>(a.w1f);
  bf16* w2f = reinterpret_cast<bf16*>(a.w2f);
  bf16* w2d = reinterpret_cast<bf16*>(a.w2d);
  const int end = a.off[9] + 10;

  for (int i = blockIdx.x * 256 + tid; i < end; i += gridDim.x * 256) {
    int seg = 9;
    while (seg > 0 && i < a.off[seg]) --seg;
    const int j = i - a.off[seg];
    if (j >= SEG_NUMEL[seg]) continue;       // alignment padding
    if (seg == 1 || seg == 3) continue;      // conv biases: block 0 below
    float gv = 0.f;
    if (seg == 0) {
      const int co = j & 63, t = j >> 6, ci = t % 3, kw = (t / 3) % 5, kh = t / 15;
      const int k = kh * 32 + kw * 4 + ci;
      if (reduce) for (int q = 0; q < a.g1; ++q) gv += a.part1[((size_t)q * 160 + k) * 64 + co];
      else gv = a.grad[i];
      if (a.mode == 1) { a.grad[i] = gv; continue; }
      float wv = a.master[i];
      if (apply) { wv -= lr * gv * scale; a.master[i] = wv; }
      w1f[co * 160 + k] = (bf16)wv;
    } else if (seg == 2) {
      const int co = j & 63, krow = j >> 6, ci = krow & 63, khw = krow >> 6;
      const int kh = khw / 5, kw = khw - kh * 5;
      if (reduce) for (int q = 0; q < a.g2; ++q) gv += a.part2[((size_t)q * 1600 + krow) * 64 + co];
      else gv = a.grad[i];
      if (a.mode == 1) { a.grad[i] = gv; continue; }
      float wv = a.master[i];
      if (apply) { wv -= lr * gv * scale; a.master[i] = wv; }
      w2f[co * 1600 + krow] = (bf16)wv;
      w2d[ci * 1600 + ((4 - kh) * 5 + (4 - kw)) * 64 + co] = (bf16)wv;
    } else {
      if (a.mode == 1) continue;             // fc grads are already complete in a.grad
      float wv = a.master[i];
      if (apply) { wv -= lr * a.grad[i] * scale; a.master[i] = wv; }
      const bf16 bv = (bf16)wv;
      if (seg == 4) {
        reinterpret_cast<bf16*>(a.fc1n)[j] = bv;
      } else if (seg == 6) {
        const int k = j / 192, n = j - k * 192;
        reinterpret_cast<bf16*>(a.fc2n)[j] = bv;
        reinterpret_cast<bf16*>(a.fc2t)[n * 384 + k] = bv;
      } else if (seg == 8) {
        const int k = j / 10, n = j - k * 10;
        reinterpret_cast<bf16*>(a.fc3t)[n * 192 + k] = bv;
        reinterpret_cast<bf16*>(a.fc3d)[k * 32 + n] = bv;
      }
    }
  }

  if (blockIdx.x == 0) {   // conv biases: cooperative deterministic reductions
    float g1 = 0.f, g3 = 0.f;
    if (reduce) {
      g1 = conv_bias_grad(a.partb1, a.g1, 0, tid, red);
      g3 = conv_bias_grad(a.partb2, a.B, 0, tid, red);
    }
    if (tid < 64) {
      const int i1 = a.off[1] + tid, i3 = a.off[3] + tid;
      if (a.mode == 1) {
        a.grad[i1] = g1;
        a.grad[i3] = g3;
      } else if (apply) {
        if (a.mode == 2) { g1 = a.grad[i1]; g3 = a.grad[i3]; }
        a.master[i1] -= lr * g1 * scale;
        a.master[i3] -= lr * g3 * scale;
      }
    }
  }

  if (!apply) return;
  // last-arriver: bump global_step, publish stats, reset the ticket for the next launch
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned t = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (unsigned)gridDim.x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      float loss = 0.f;
      int corr = 0;
      for (int q = 0; q < a.nhead; ++q) { loss += a.loss_part[q]; corr += a.correct_part[q]; }
      float* st = a.stats + (size_t)(step % a.stats_len) * 4;
      st[0] = (float)(step + 1);
      st[1] = loss / (float)a.B;
      st[2] = (float)corr / (float)a.B;
      st[3] = lr;
      *a.step = step + 1;
      __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace dmlc

using namespace dmlc;

extern "C" hipError_t dmlc_sgd(DmlcSgdArgs* a, hipStream_t s) {
  const int end = a->off[9] + 10;
  int blocks = (end + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  a->nblocks = blocks;
  hipLaunchKernelGGL(k_sgd, dim3(blocks), dim3(256), 0, s, *a);
  return hipGetLastError();
}
