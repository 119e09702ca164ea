// MLP head of the CIFAR-10 CNN, one launch for forward AND backward of the small layers:
//   fc1 split-K reduction + bias + ReLU (prologue), fc2 + ReLU, fc3 (+ ReLU on the logits, D4),
//   sparse softmax cross-entropy + batch accuracy, then dlogits -> dh2 -> dh1 (with ReLU masks).
// Replaces /root/reference/cifar10cnn.py:130-176 (full1..full3, cifar_loss, batch_accuracy) and the
// corresponding autodiff ops (SURVEY.md §2.B N7/N8/N10-N12, §2.C xent10_fwd_bwd + linear_bwd_dx).
//
// Rows-parallel: 16 batch rows per 256-thread workgroup; everything per row stays in LDS.  Every
// product is computed TRANSPOSED (C[feature][row]) so the weight fragment streams from L2 and each
// lane ends up with 4 consecutive features of one row.  Weight *gradients* of fc1/fc2/fc3 are NOT
// computed here (they need a reduction over the whole batch): the grouped GEMM kernel does them.
#include "common.h"
#include "api.h"

namespace dmlc {

constexpr int H1_LD = 392;   // 784-B rows: 16-B aligned, rows land on distinct bank slots
constexpr int H2_LD = 200;   // 400-B rows
constexpr int DL_LD = 40;    // 80-B rows (k padded to 32 with zeros)

DEV int head_index(const DmlcIndexSrc& s, int B, int b) {
  int row = 0;
  if (s.counter) row = (int)(*s.counter % (int64_t)s.period);
  return s.idx_base[row * B + b];
}

__global__ __launch_bounds__(256) void k_head(DmlcHeadArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 h1s[16 * H1_LD];
  __shared__ __attribute__((aligned(16))) bf16 h2s[16 * H2_LD];
  __shared__ __attribute__((aligned(16))) bf16 dh2s[16 * H2_LD];
  __shared__ __attribute__((aligned(16))) bf16 dls[16 * DL_LD];
  __shared__ float lg[16][17];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int r0 = blockIdx.x * 16;

  // (a) h1 = relu(sum_s part[s] + b1)
  for (int e = tid; e < 16 * 96; e += 256) {
    const int r = e / 96, n = (e - r * 96) * 4;
    float4 s = *reinterpret_cast<const float4*>(a.b1 + n);
    for (int sp = 0; sp < a.nsplit; ++sp) {
      const float4 v = *reinterpret_cast<const float4*>(a.h1part + ((size_t)sp * a.B + r0 + r) * 384 + n);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    const bf16x4 o = pack4(fmaxf(s.x, 0.f), fmaxf(s.y, 0.f), fmaxf(s.z, 0.f), fmaxf(s.w, 0.f));
    *reinterpret_cast<bf16x4*>(h1s + r * H1_LD + n) = o;
    if (a.train) *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.h1) + (size_t)(r0 + r) * 384 + n) = o;
  }
  __syncthreads();

  // (b) h2 = relu(h1 W2 + b2): C[n][r] = sum_k W2t[n][k] h1[r][k]; wave w: n-tiles w, w+4, w+8
  {
    const bf16* W = reinterpret_cast<const bf16*>(a.w2t);
    f32x4 acc[3] = {zero4(), zero4(), zero4()};
#pragma unroll
    for (int ks = 0; ks < 12; ++ks) {
      const bf16x8 bx = lds_b128(h1s + li * H1_LD + ks * 32 + 8 * g);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int nt = w + 4 * j;
        acc[j] = mfma16(glb_b128(W + (16 * nt + li) * 384 + ks * 32 + 8 * g), bx, acc[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int n = 16 * (w + 4 * j) + 4 * g;
      const bf16x4 o = pack4(fmaxf(acc[j][0] + a.b2[n], 0.f), fmaxf(acc[j][1] + a.b2[n + 1], 0.f),
                             fmaxf(acc[j][2] + a.b2[n + 2], 0.f), fmaxf(acc[j][3] + a.b2[n + 3], 0.f));
      *reinterpret_cast<bf16x4*>(h2s + li * H2_LD + n) = o;
      if (a.train) *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.h2) + (size_t)(r0 + li) * 192 + n) = o;
    }
  }
  __syncthreads();

  // (c) logits = [relu](h2 W3 + b3): wave 0, one 16x16 tile, K = 192
  if (w == 0) {
    const bf16* W = reinterpret_cast<const bf16*>(a.w3t);
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 6; ++ks)
      acc = mfma16(glb_b128(W + li * 192 + ks * 32 + 8 * g), lds_b128(h2s + li * H2_LD + ks * 32 + 8 * g), acc);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = 4 * g + i;
      if (n < 10) {
        float v = acc[i] + a.b3[n];
        if (a.relu_logits) v = fmaxf(v, 0.f);
        lg[li][n] = v;
      }
    }
  }
  __syncthreads();

  // (d) softmax cross-entropy, accuracy, dlogits (wave 0, lanes 0..15 = rows)
  if (w == 0) {
    float loss = 0.f, corr = 0.f;
    if (lane < 16) {
      const int b = r0 + lane;
      const int label = a.labels[head_index(a.src, a.B, b)];
      float m = lg[lane][0];
      int am = 0;
#pragma unroll
      for (int j = 1; j < 10; ++j) if (lg[lane][j] > m) { m = lg[lane][j]; am = j; }
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < 10; ++j) se += __expf(lg[lane][j] - m);
      const float lse = m + __logf(se);
      loss = lse - lg[lane][label];
      corr = am == label ? 1.f : 0.f;
      if (a.logits_out) {
#pragma unroll
        for (int j = 0; j < 10; ++j) a.logits_out[b * 10 + j] = lg[lane][j];
      }
      if (a.train) {
        bf16* dlg = reinterpret_cast<bf16*>(a.dl) + (size_t)b * 16;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          float d = 0.f;
          if (j < 10) {
            d = (__expf(lg[lane][j] - lse) - (j == label ? 1.f : 0.f)) * a.inv_batch;
            if (a.relu_logits && !(lg[lane][j] > 0.f)) d = 0.f;
          }
          dls[lane * DL_LD + j] = (bf16)d;
          if (j < 16) dlg[j] = (bf16)d;
        }
      }
    }
    loss = wave_sum(loss);
    corr = wave_sum(corr);
    if (lane == 0) {
      a.loss_part[blockIdx.x] = loss;
      a.correct_part[blockIdx.x] = (int)(corr + 0.5f);
    }
  }
  if (!a.train) return;
  __syncthreads();

  // (e) dh2 = (dl W3^T) * (h2 > 0): C[n][r] = sum_k W3d[n][k] dl[r][k], K = 32 (one step)
  {
    const bf16* W = reinterpret_cast<const bf16*>(a.w3d);
    const bf16x8 bx = lds_b128(dls + li * DL_LD + 8 * g);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int nt = w + 4 * j;
      const f32x4 acc = mfma16(glb_b128(W + (16 * nt + li) * 32 + 8 * g), bx, zero4());
      const int n = 16 * nt + 4 * g;
      const bf16x4 hv = *reinterpret_cast<const bf16x4*>(h2s + li * H2_LD + n);
      const bf16x4 o = pack4((float)hv[0] > 0.f ? acc[0] : 0.f, (float)hv[1] > 0.f ? acc[1] : 0.f,
                             (float)hv[2] > 0.f ? acc[2] : 0.f, (float)hv[3] > 0.f ? acc[3] : 0.f);
      *reinterpret_cast<bf16x4*>(dh2s + li * H2_LD + n) = o;
      *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.dh2) + (size_t)(r0 + li) * 192 + n) = o;
    }
  }
  __syncthreads();

  // (f) dh1 = (dh2 W2^T) * (h1 > 0): C[n][r] = sum_k W2n[n][k] dh2[r][k], n < 384, K = 192
  {
    const bf16* W = reinterpret_cast<const bf16*>(a.w2d);
    f32x4 acc[6] = {zero4(), zero4(), zero4(), zero4(), zero4(), zero4()};
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) {
      const bf16x8 bx = lds_b128(dh2s + li * H2_LD + ks * 32 + 8 * g);
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int nt = w + 4 * j;
        acc[j] = mfma16(glb_b128(W + (16 * nt + li) * 192 + ks * 32 + 8 * g), bx, acc[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int n = 16 * (w + 4 * j) + 4 * g;
      const bf16x4 hv = *reinterpret_cast<const bf16x4*>(h1s + li * H1_LD + n);
      const bf16x4 o = pack4((float)hv[0] > 0.f ? acc[j][0] : 0.f, (float)hv[1] > 0.f ? acc[j][1] : 0.f,
                             (float)hv[2] > 0.f ? acc[j][2] : 0.f, (float)hv[3] > 0.f ? acc[j][3] : 0.f);
      *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.dh1) + (size_t)(r0 + li) * 384 + n) = o;
    }
  }
}

}  // namespace dmlc

using namespace dmlc;

extern "C" hipError_t dmlc_head(const DmlcHeadArgs* a, hipStream_t s) {
  hipLaunchKernelGGL(k_head, dim3(a->B / 16), dim3(256), 0, s, *a);
  return hipGetLastError();
}
