// Probes for the fp8 conv2 weight gradient (round 6): (1) the lane map of ds_read_b64_tr_b8 and
// (2) v_mfma_scale_f32_16x16x128_f8f6f4 with an e4m3 A operand and an e5m2 (bf8) B operand -- the
// MFMA result against an fp32 sum of the dequantised operands.  Prints "tr8 lane .." lines and
// "mfma max_abs_err ..".
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef int v2i __attribute__((ext_vector_type(2)));
typedef int fp8x32 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k_tr8(unsigned* out) {
  __shared__ unsigned char s[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) s[i] = (unsigned char)(i & 255);
  __syncthreads();
  const int l = threadIdx.x, gi = l & 15, grp = l >> 4;
  const int q = gi >> 1, p = gi & 1;           // guess: lane 2q+p -> row q, bytes 8p..8p+7
  const int row = grp * 8 + q;                 // 16-B rows, each group its own 8 rows
  v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(s + row * 16 + p * 8));
  out[2 * l] = r.x; out[2 * l + 1] = r.y;
}

__device__ float av(int r, int k) { return (float)(((r * 7 + k * 3) % 11) - 5) * 0.25f; }
__device__ float bv(int k, int c) { return (float)(((k * 5 + c * 13) % 9) - 4) * 0.125f; }

__global__ void k_mfma(float* out, float* ref) {
  const int l = threadIdx.x, rc = l & 15, g = l >> 4;
  unsigned char a8[32], b8[32];
  for (int j = 0; j < 32; j += 2) {
    int wa = __builtin_amdgcn_cvt_pk_fp8_f32(av(rc, 32 * g + j), av(rc, 32 * g + j + 1), 0, false);
    int wb = __builtin_amdgcn_cvt_pk_bf8_f32(bv(32 * g + j, rc), bv(32 * g + j + 1, rc), 0, false);
    a8[j] = wa & 255; a8[j + 1] = (wa >> 8) & 255;
    b8[j] = wb & 255; b8[j + 1] = (wb >> 8) & 255;
  }
  fp8x32 A, B;
  for (int d = 0; d < 8; ++d) {
    A[d] = a8[4 * d] | (a8[4 * d + 1] << 8) | (a8[4 * d + 2] << 16) | (a8[4 * d + 3] << 24);
    B[d] = b8[4 * d] | (b8[4 * d + 1] << 8) | (b8[4 * d + 2] << 16) | (b8[4 * d + 3] << 24);
  }
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A, B, c, 0, 1, 0, 127, 0, 127);
  for (int i = 0; i < 4; ++i) out[(4 * g + i) * 16 + rc] = c[i];
  if (l < 16) {                                // fp32 reference from the dequantised values
    for (int r = 0; r < 16; ++r) {
      float s = 0.f;
      for (int k = 0; k < 128; ++k) {
        int wa = __builtin_amdgcn_cvt_pk_fp8_f32(av(r, k), 0.f, 0, false);
        int wb = __builtin_amdgcn_cvt_pk_bf8_f32(bv(k, l), 0.f, 0, false);
        s += __builtin_amdgcn_cvt_f32_fp8(wa, 0) * __builtin_amdgcn_cvt_f32_bf8(wb, 0);
      }
      ref[r * 16 + l] = s;
    }
  }
}

// (3) per-lane E8M0 block scales: lane (row/col, K block g) scales its 32 K values by 2^(s - 127)
__global__ void k_mfma_scaled(float* out, float* ref) {
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
  const int sa = 127 + (g & 1) + (rc & 1), sb = 127 - g;
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A, B, c, 0, 0, 0, sa, 0, sb);
  for (int i = 0; i < 4; ++i) out[(4 * g + i) * 16 + rc] = c[i];
  if (l < 16) {
    for (int r = 0; r < 16; ++r) {
      float s = 0.f;
      for (int k = 0; k < 128; ++k) {
        int wa = __builtin_amdgcn_cvt_pk_fp8_f32(av(r, k), 0.f, 0, false);
        int wb = __builtin_amdgcn_cvt_pk_fp8_f32(bv(k, l), 0.f, 0, false);
        const int kb = k >> 5;
        s += __builtin_amdgcn_cvt_f32_fp8(wa, 0) * exp2f((float)((kb & 1) + (r & 1))) *
             __builtin_amdgcn_cvt_f32_fp8(wb, 0) * exp2f(-(float)kb);
      }
      ref[r * 16 + l] = s;
    }
  }
}

int main() {
  unsigned* d; float *o, *rf;
  if (hipMalloc(&d, 512) || hipMalloc(&o, 1024) || hipMalloc(&rf, 1024)) return 1;
  hipLaunchKernelGGL(k_tr8, 1, 64, 0, 0, d);
  hipLaunchKernelGGL(k_mfma, 1, 64, 0, 0, o, rf);
  unsigned h[128]; float ho[256], hr[256];
  if (hipMemcpy(h, d, 512, hipMemcpyDeviceToHost) || hipMemcpy(ho, o, 1024, hipMemcpyDeviceToHost) ||
      hipMemcpy(hr, rf, 1024, hipMemcpyDeviceToHost)) return 2;
  for (int l = 0; l < 64; ++l) {
    unsigned char* b = (unsigned char*)&h[2 * l];
    printf("tr8 lane %2d:", l); for (int j = 0; j < 8; ++j) printf(" %3d", b[j]); printf("\n");
  }
  float e = 0.f, m = 0.f;
  for (int i = 0; i < 256; ++i) { e = fmaxf(e, fabsf(ho[i] - hr[i])); m = fmaxf(m, fabsf(hr[i])); }
  printf("mfma max_abs_err %g max_ref %g c00 %g r00 %g c_1_2 %g r_1_2 %g\n", e, m, ho[0], hr[0], ho[18], hr[18]);
  hipLaunchKernelGGL(k_mfma_scaled, 1, 64, 0, 0, o, rf);
  if (hipMemcpy(ho, o, 1024, hipMemcpyDeviceToHost) || hipMemcpy(hr, rf, 1024, hipMemcpyDeviceToHost)) return 3;
  e = 0.f; m = 0.f;
  for (int i = 0; i < 256; ++i) { e = fmaxf(e, fabsf(ho[i] - hr[i])); m = fmaxf(m, fabsf(hr[i])); }
  printf("mfma_scaled max_abs_err %g max_ref %g c00 %g r00 %g c_1_2 %g r_1_2 %g\n", e, m, ho[0], hr[0], ho[18], hr[18]);
  return 0;
}
