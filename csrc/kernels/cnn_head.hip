// MLP head of the CIFAR-10 CNN, one launch for forward AND backward of the small layers:
//   fc1 split-K reduction + bias + ReLU (prologue), fc2 + ReLU, fc3 (+ ReLU on the logits, D4),
//   sparse softmax cross-entropy + batch accuracy, then dlogits -> dh2 -> dh1 (with ReLU masks).
// Replaces /root/reference/cifar10cnn.py:130-176 (full1..full3, cifar_loss, batch_accuracy) and the
// corresponding autodiff ops (SURVEY.md §2.B N7/N8/N10-N12, §2.C xent10_fwd_bwd + linear_bwd_dx).
//
// Rows-parallel: RB (4/8/16) batch rows per workgroup of 16 waves; everything per row stays in LDS.
// The MFMA tiles keep 16 row columns (columns >= RB compute on zeros and are never stored): the head
// is bound by how fast each CU pulls the ~300 KB of fc2 weights (both layouts), not by MFMA, so more
// workgroups with fewer rows -- 8 per XCD sharing one L2 copy of the weights -- finish sooner.  Every
// product is computed TRANSPOSED (C[feature][row]) so the weight fragment streams from L2 and each
// lane ends up with 4 consecutive features of one row.  The weight fragments of a wave's output
// tiles are loaded up front (fc2 at entry, behind the fc1 reduction; fc2^T right after the fc2
// MFMAs, behind the loss phase), so each phase pays at most one exposed L2 latency.  Weight
// *gradients* of fc1/fc2/fc3 need a reduction over the whole batch: the grouped GEMM kernel does them.
#include "common.h"
#include "api.h"

namespace dmlc {

constexpr int HT = 1024;     // 16 waves
constexpr int H1_LD = 392;   // 784-B rows: 16-B aligned, rows land on distinct bank slots
constexpr int H2_LD = 200;   // 400-B rows
constexpr int DL_LD = 40;    // 80-B rows (k padded to 32 with zeros)

DEV int head_index(const DmlcIndexSrc& s, int B, int b) {
  int row = 0;
  if (s.counter) row = (int)(*s.counter % (int64_t)s.period);
  return s.idx_base[row * B + b];
}

DEV bf16x4 relu_mask4(const f32x4& acc, const bf16x4& h) {
  return pack4((float)h[0] > 0.f ? acc[0] : 0.f, (float)h[1] > 0.f ? acc[1] : 0.f,
               (float)h[2] > 0.f ? acc[2] : 0.f, (float)h[3] > 0.f ? acc[3] : 0.f);
}

template <int RB>
__global__ __launch_bounds__(HT, 1) void k_head(DmlcHeadArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 h1s[16 * H1_LD];
  __shared__ __attribute__((aligned(16))) bf16 h2s[16 * H2_LD];
  __shared__ __attribute__((aligned(16))) bf16 dh2s[16 * H2_LD];
  __shared__ __attribute__((aligned(16))) bf16 dls[16 * DL_LD];
  __shared__ float lg[16][17];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int r0 = blockIdx.x * RB;
  const bool rv = li < RB;                      // this lane's row column is a real batch row
  DMLC_STAMP(DMLC_TK_HEAD, 0);

  // the loss wave's labels (counter -> index -> label chain) are fetched at entry
  int label = 0;
  if (w == 12 && lane < RB) label = a.labels[head_index(a.src, a.B, r0 + lane)];

  // fc2 weight fragments of this wave's output tile (waves 0..11: features 16w..16w+15), in flight
  // while the fc1 partial sums are reduced
  bf16x8 w2f[12];
  if (w < 12) {
    const bf16* W = reinterpret_cast<const bf16*>(a.w2t) + (16 * w + li) * 384 + 8 * g;
#pragma unroll
    for (int ks = 0; ks < 12; ++ks) w2f[ks] = glb_b128(W + ks * 32);
  }

  // (a) h1 = relu(sum_s part[s] + b1): RB x 96 float4, at most 2 per thread; rows RB..15 of the LDS
  // tile are zeroed (their MFMA columns then compute on zeros).
  {
    constexpr int U = (RB * 96 + HT - 1) / HT;
    float4 acc[U];
    int e[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      e[u] = tid + u * HT;
      const int ec = e[u] < RB * 96 ? e[u] : 0;               // branch-free: clamp, discard later
      const int r = ec / 96, n = (ec - r * 96) * 4;
      acc[u] = *reinterpret_cast<const float4*>(a.b1 + n);
      const float* hp = a.h1part + (size_t)(r0 + r) * 384 + n;
      const size_t sstride = (size_t)a.B * 384;
      int sp = 0;
      for (; sp + 4 <= a.nsplit; sp += 4) {
        float4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<const float4*>(hp + (sp + k) * sstride);
#pragma unroll
        for (int k = 0; k < 4; ++k) { acc[u].x += v[k].x; acc[u].y += v[k].y; acc[u].z += v[k].z; acc[u].w += v[k].w; }
      }
      for (; sp < a.nsplit; ++sp) {
        const float4 v = *reinterpret_cast<const float4*>(hp + sp * sstride);
        acc[u].x += v.x; acc[u].y += v.y; acc[u].z += v.z; acc[u].w += v.w;
      }
    }
    if (RB < 16) {
      for (int z = tid; z < (16 - RB) * 96; z += HT)
        *reinterpret_cast<bf16x4*>(h1s + (RB + z / 96) * H1_LD + (z % 96) * 4) = pack4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (e[u] < RB * 96) {
        const int r = e[u] / 96, n = (e[u] - r * 96) * 4;
        const bf16x4 o = pack4(fmaxf(acc[u].x, 0.f), fmaxf(acc[u].y, 0.f), fmaxf(acc[u].z, 0.f), fmaxf(acc[u].w, 0.f));
        *reinterpret_cast<bf16x4*>(h1s + r * H1_LD + n) = o;
        if (a.train) *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.h1) + (size_t)(r0 + r) * 384 + n) = o;
      }
    }
  }
  lds_barrier();
  DMLC_STAMP(DMLC_TK_HEAD, 1);

  // (b) h2 = relu(h1 W2 + b2): C[n][r] = sum_k W2t[n][k] h1[r][k]
  if (w < 12) {
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 12; ++ks) acc = mfma16(w2f[ks], lds_b128(h1s + li * H1_LD + ks * 32 + 8 * g), acc);
    const int n = 16 * w + 4 * g;
    const bf16x4 o = pack4(fmaxf(acc[0] + a.b2[n], 0.f), fmaxf(acc[1] + a.b2[n + 1], 0.f),
                           fmaxf(acc[2] + a.b2[n + 2], 0.f), fmaxf(acc[3] + a.b2[n + 3], 0.f));
    *reinterpret_cast<bf16x4*>(h2s + li * H2_LD + n) = o;
    if (a.train && rv) *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.h2) + (size_t)(r0 + li) * 192 + n) = o;
  }
  // fc2^T fragments for (f): tiles w and w+16 (w < 8) of the 24 dh1 feature tiles, K = 192
  bf16x8 w2d[2][6];
  if (a.train) {
    const bf16* W = reinterpret_cast<const bf16*>(a.w2d);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j == 0 || w < 8) {
        const bf16* Wr = W + (16 * (w + 16 * j) + li) * 192 + 8 * g;
#pragma unroll
        for (int ks = 0; ks < 6; ++ks) w2d[j][ks] = glb_b128(Wr + ks * 32);
      }
    }
  }
  lds_barrier();
  DMLC_STAMP(DMLC_TK_HEAD, 2);

  // (c) logits = [relu](h2 W3 + b3): wave 12, one 16x16 tile, K = 192
  if (w == 12) {
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
  lds_barrier();

  // (d) softmax cross-entropy, accuracy, dlogits (wave 12, lanes 0..15 = rows)
  if (w == 12) {
    float loss = 0.f, corr = 0.f;
    if (lane >= RB && lane < 16 && a.train) {
#pragma unroll
      for (int j = 0; j < 32; ++j) dls[lane * DL_LD + j] = (bf16)0.f;
    }
    if (lane < RB) {
      const int b = r0 + lane;
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
  lds_barrier();
  DMLC_STAMP(DMLC_TK_HEAD, 3);

  // (e) dh2 = (dl W3^T) * (h2 > 0): C[n][r] = sum_k W3d[n][k] dl[r][k], K = 32 (one step), waves 0..11
  if (w < 12) {
    const bf16* W = reinterpret_cast<const bf16*>(a.w3d);
    const f32x4 acc = mfma16(glb_b128(W + (16 * w + li) * 32 + 8 * g), lds_b128(dls + li * DL_LD + 8 * g), zero4());
    const int n = 16 * w + 4 * g;
    const bf16x4 o = relu_mask4(acc, *reinterpret_cast<const bf16x4*>(h2s + li * H2_LD + n));
    *reinterpret_cast<bf16x4*>(dh2s + li * H2_LD + n) = o;
    if (rv) *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.dh2) + (size_t)(r0 + li) * 192 + n) = o;
  }
  lds_barrier();
  DMLC_STAMP(DMLC_TK_HEAD, 4);

  // (f) dh1 = (dh2 W2^T) * (h1 > 0): tiles w and w+16, K = 192
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j == 1 && w >= 8) break;
    f32x4 acc = zero4();
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) acc = mfma16(w2d[j][ks], lds_b128(dh2s + li * H2_LD + ks * 32 + 8 * g), acc);
    const int n = 16 * (w + 16 * j) + 4 * g;
    const bf16x4 o = relu_mask4(acc, *reinterpret_cast<const bf16x4*>(h1s + li * H1_LD + n));
    if (rv) *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(a.dh1) + (size_t)(r0 + li) * 384 + n) = o;
  }
  DMLC_STAMP(DMLC_TK_HEAD, 5);
}

}  // namespace dmlc

using namespace dmlc;

extern "C" hipError_t dmlc_head(const DmlcHeadArgs* a, hipStream_t s) {
  switch (a->rows) {
    case 4: hipLaunchKernelGGL(k_head<4>, dim3(a->B / 4), dim3(HT), 0, s, *a); break;
    case 8: hipLaunchKernelGGL(k_head<8>, dim3(a->B / 8), dim3(HT), 0, s, *a); break;
    case 16: hipLaunchKernelGGL(k_head<16>, dim3(a->B / 16), dim3(HT), 0, s, *a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
