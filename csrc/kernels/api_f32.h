// Host-side API of the fp32 kernels (csrc/kernels/f32_gemm.hip): the fp32-accurate path of the
// reference CNN (every reference variable and op is tf.float32, /root/reference/cifar10cnn.py:97-145).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {

// C[M,N] = op(A)[M,K] . op(B)[K,N] (+ bias[N]) (ReLU), fp32 in, fp32 MFMA (v_mfma_f32_16x16x4_f32),
// fp32 out.  op(A) = A stored [M,K] (row stride lda) or, with ta, A stored [K,M]; likewise op(B) =
// B stored [K,N] (ldb) or, with tb, B stored [N,K].  splits > 1: K is cut into `splits` chunks of
// `kc` (multiple of 16) whose partial products go to ws[splits][M][N] and are summed in slice order
// by a second kernel (deterministic).  ws may be null when splits == 1.
// conv = 1 / 2: A is an NHWC activation and op(A) its implicit im2col matrix (no tb): geometry 1 =
// [B][24][24][3], geometry 2 = [B][12][12][64], 5x5 taps, pad 2; rows = pixels (B*HW*HW), columns
// (kh*5 + kw)*C + c, and column 25*C (if K or M reaches it) is the constant 1 (bias-gradient row).
// With ta the product is im2col(A)^T op(B) (weight gradient); lda is unused.
hipError_t dmlc_f32_gemm(const float* A, const float* B, const float* bias, float* C, float* ws, int M, int N,
                         int K, int lda, int ldb, bool ta, bool tb, bool relu, int splits, int kc, int conv,
                         hipStream_t s);

// im2col of a stride-1, zero-padded KHxKW convolution (TF 'SAME' for odd kernels: pad = k/2):
// x NHWC [B,H,W,C] -> cols [B*H*W][KH*KW*C], column (kh*KW + kw)*C + c (the row order of an HWIO
// weight viewed as [KH*KW*C][CO]).
hipError_t dmlc_f32_im2col(const float* x, float* cols, int B, int H, int W, int C, int KH, int KW, int pad,
                           hipStream_t s);
// Its adjoint, as a gather (fixed summation order, deterministic): dx[b,y,x,c] = sum over the
// (kh,kw) taps of dcols[(b, y-kh+pad, x-kw+pad)][(kh*KW + kw)*C + c].
hipError_t dmlc_f32_col2im(const float* dcols, float* dx, int B, int H, int W, int C, int KH, int KW, int pad,
                           hipStream_t s);
// out[N] = sum over the M rows of x[M][N], in a fixed order (ws: >= splits * N floats).
hipError_t dmlc_f32_colsum(const float* x, float* out, float* ws, int M, int N, int splits, hipStream_t s);

}  // extern "C"
