// Which lane's scale byte scales which (row / column, 32-K block) of v_mfma_scale_f32_16x16x128_f8f6f4:
// for every lane L, scale_a (then scale_b) of lane L alone is 2^1 (byte 128, opsel 0); the change of C
// against the all-2^0 product is matched against the per-block partial products.  Prints
// "A lane L -> row r kblock j" / "B lane L -> col c kblock j" (or "unmatched").
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef int fp8x32 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ float av(int r, int k) { return (float)(((r * 7 + k * 3) % 11) - 5) * 0.25f + 0.01f * (r + 1); }
__device__ float bv(int k, int c) { return (float)(((k * 5 + c * 13) % 9) - 4) * 0.125f + 0.003f * (c + 1); }

__global__ void k(float* out /*[129][256]*/, float* part /*[16][16][16]*/) {
  const int l = threadIdx.x, rc = l & 15, g = l >> 4;
  unsigned char a8[32], b8[32];
  for (int j = 0; j < 32; j += 2) {
    int wa = __builtin_amdgcn_cvt_pk_fp8_f32(av(rc, 32 * g + j), av(rc, 32 * g + j + 1), 0, false);
    int wb = __builtin_amdgcn_cvt_pk_fp8_f32(bv(32 * g + j, rc), bv(32 * g + j + 1, rc), 0, false);
    a8[j] = wa & 255; a8[j + 1] = (wa >> 8) & 255;
    b8[j] = wb & 255; b8[j + 1] = (wb >> 8) & 255;
  }
  fp8x32 A, B;
  for (int d = 0; d < 8; ++d) {
    A[d] = a8[4 * d] | (a8[4 * d + 1] << 8) | (a8[4 * d + 2] << 16) | (a8[4 * d + 3] << 24);
    B[d] = b8[4 * d] | (b8[4 * d + 1] << 8) | (b8[4 * d + 2] << 16) | (b8[4 * d + 3] << 24);
  }
  for (int t = 0; t < 129; ++t) {           // t = 0: no change; 1..64: A lane t-1; 65..128: B lane t-65
    const int sa = (t >= 1 && t <= 64 && l == t - 1) ? 128 : 127;
    const int sb = (t >= 65 && l == t - 65) ? 128 : 127;
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A, B, c, 0, 0, 0, sa, 0, sb);
    for (int i = 0; i < 4; ++i) out[t * 256 + (4 * g + i) * 16 + rc] = c[i];
  }
  if (l < 16) {
    for (int r = 0; r < 16; ++r)
      for (int j = 0; j < 16; ++j) {
        float s = 0.f;
        for (int k = 8 * j; k < 8 * j + 8; ++k) {
          int wa = __builtin_amdgcn_cvt_pk_fp8_f32(av(r, k), 0.f, 0, false);
          int wb = __builtin_amdgcn_cvt_pk_fp8_f32(bv(k, l), 0.f, 0, false);
          s += __builtin_amdgcn_cvt_f32_fp8(wa, 0) * __builtin_amdgcn_cvt_f32_fp8(wb, 0);
        }
        part[(r * 16 + l) * 16 + j] = s;
      }
  }
}

int main() {
  float *o, *pp;
  if (hipMalloc(&o, 129 * 256 * 4) || hipMalloc(&pp, 4096 * 4)) return 1;
  hipLaunchKernelGGL(k, 1, 64, 0, 0, o, pp);
  static float h[129 * 256], P[4096];
  if (hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost) || hipMemcpy(P, pp, sizeof(P), hipMemcpyDeviceToHost)) return 2;
  // every lane: the set of 4 sub-blocks of 8 K (k = 8m .. 8m+7) its scale covers, searched over all
  // 4-subsets of the 16 sub-blocks against the change of its row (A) / column (B)
  for (int t = 1; t < 129; ++t) {
    const bool isA = t <= 64;
    const int L = isA ? t - 1 : t - 65, x = L & 15;
    int best = -1;
    for (int S = 0; S < (1 << 16) && best < 0; ++S) {
      if (__builtin_popcount(S) != 4) continue;
      bool ok = true;
      for (int y = 0; y < 16 && ok; ++y) {
        const int r = isA ? x : y, c = isA ? y : x;
        float want = 0.f;
        for (int m = 0; m < 16; ++m) if (S >> m & 1) want += P[(r * 16 + c) * 16 + m];
        const float d = h[t * 256 + r * 16 + c] - h[r * 16 + c];
        if (fabsf(d - want) > 2e-3f) ok = false;
      }
      if (ok) best = S;
    }
    printf("%s lane %2d (%s %2d) -> sub-blocks", isA ? "A" : "B", L, isA ? "row" : "col", x);
    if (best < 0) printf(" none");
    for (int m = 0; m < 16; ++m) if (best >= 0 && (best >> m & 1)) printf(" %d", m);
    printf("\n");
  }
  return 0;
}
