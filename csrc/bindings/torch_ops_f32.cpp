// torch.ops.dmlc.f32_* bindings of the fp32 kernels (csrc/kernels/f32_gemm.hip): the building blocks
// of the fp32-accurate CNN path (ops/f32.py).  Functional ops (they allocate their outputs on the
// caching allocator and launch on the current HIP stream, so they compose with autograd and are
// capturable into HIP graphs); every launch is preceded by a full shape / dtype / layout check.
#include <c10/core/DeviceGuard.h>

#include <algorithm>

#include "../kernels/api_f32.h"
#include "check.h"

namespace {

using namespace dmlc_bind;

void f32_in(const Tensor& t, const char* n, int64_t dim) {
  dev(t, n);
  TORCH_CHECK(t.scalar_type() == at::kFloat, n, " must be fp32, got ", t.scalar_type());
  TORCH_CHECK(t.dim() == dim, n, " must be ", dim, "-D, got ", t.sizes());
}

// split-K so that the launch has >= ~512 workgroups (256 CUs x 2) when the output tile grid alone is
// small; each slice keeps >= 256 of K (4 k-steps), and at most 128 slices (the reduction reads them
// in order)
void pick_split(int64_t M, int64_t N, int64_t K, int* splits, int* kc) {
  const int64_t tiles = ((M + 63) / 64) * ((N + 63) / 64);
  int64_t s = tiles >= 256 ? 1 : std::min<int64_t>(std::min<int64_t>((512 + tiles - 1) / tiles, 128), std::max<int64_t>(1, K / 256));
  int64_t c = ((K + s - 1) / s + 63) / 64 * 64;   // multiple of the kernel's 64-deep k-step
  s = (K + c - 1) / c;
  *splits = (int)s;
  *kc = (int)c;
}

Tensor f32_gemm(const Tensor& a, const Tensor& b, const c10::optional<Tensor>& bias, bool ta, bool tb, bool relu) {
  f32_in(a, "a", 2);
  f32_in(b, "b", 2);
  const int64_t M = ta ? a.size(1) : a.size(0), K = ta ? a.size(0) : a.size(1);
  const int64_t Kb = tb ? b.size(1) : b.size(0), N = tb ? b.size(0) : b.size(1);
  TORCH_CHECK(K == Kb, "f32_gemm: inner dimensions differ (", K, " vs ", Kb, ")");
  TORCH_CHECK(M > 0 && N > 0 && K > 0 && M < (1 << 30) && N < (1 << 30) && K < (1 << 30), "f32_gemm: bad sizes");
  TORCH_CHECK(b.device() == a.device(), "f32_gemm: a and b on different devices");
  const float* bp = nullptr;
  if (bias.has_value()) {
    check(*bias, "bias", at::kFloat, {N});
    bp = bias->data_ptr<float>();
  }
  const c10::DeviceGuard g(a.device());
  auto out = at::empty({M, N}, a.options());
  int splits, kc;
  pick_split(M, N, K, &splits, &kc);
  Tensor ws;
  if (splits > 1) ws = at::empty({splits, M, N}, a.options());
  CHECK_HIP(dmlc_f32_gemm(a.data_ptr<float>(), b.data_ptr<float>(), bp, out.data_ptr<float>(),
                          splits > 1 ? ws.data_ptr<float>() : nullptr, (int)M, (int)N, (int)K, (int)a.size(1),
                          (int)b.size(1), ta, tb, relu, splits, kc, 0, stream_of(a)));
  return out;
}

// implicit-im2col convolution GEMM (geometries of the reference CNN at the 24x24 crop):
//   ta = false: out[B*HW*HW][N] = im2col(x) . w   (w [25*C][N]; forward, or data gradient with the
//               flipped / transposed weight)
//   ta = true : out[25*C (+1)][N] = im2col(x)^T . w  (w = dY [B*HW*HW][N]; weight gradient, and with
//               ones the bias gradient as the last row)
Tensor f32_conv_gemm(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, bool ta, bool ones) {
  f32_in(x, "x", 4);
  f32_in(w, "w", 2);
  const int64_t B = x.size(0), H = x.size(1), C = x.size(3);
  TORCH_CHECK(x.size(2) == H, "f32_conv_gemm: square images expected");
  int geom = 0;
  if (H == 24 && C == 3) geom = 1;
  else if (H == 12 && C == 64) geom = 2;
  TORCH_CHECK(geom != 0, "f32_conv_gemm: no implicit geometry for [", H, "x", H, "x", C, "] (use im2col)");
  TORCH_CHECK(!ones || ta, "f32_conv_gemm: the ones column is a weight-gradient option");
  TORCH_CHECK(w.device() == x.device(), "f32_conv_gemm: x and w on different devices");
  const int64_t pix = B * H * H, kc = 25 * C;
  TORCH_CHECK(pix > 0 && pix < (1 << 30), "f32_conv_gemm: bad batch");
  const int64_t M = ta ? kc + (ones ? 1 : 0) : pix, K = ta ? pix : kc, N = w.size(1);
  TORCH_CHECK(w.size(0) == K, "f32_conv_gemm: w has ", w.size(0), " rows, expected ", K);
  const float* bp = nullptr;
  if (bias.has_value()) {
    check(*bias, "bias", at::kFloat, {N});
    bp = bias->data_ptr<float>();
  }
  const c10::DeviceGuard g(x.device());
  auto out = at::empty({M, N}, x.options());
  int splits, kcs;
  pick_split(M, N, K, &splits, &kcs);
  Tensor ws;
  if (splits > 1) ws = at::empty({splits, M, N}, x.options());
  CHECK_HIP(dmlc_f32_gemm(x.data_ptr<float>(), w.data_ptr<float>(), bp, out.data_ptr<float>(),
                          splits > 1 ? ws.data_ptr<float>() : nullptr, (int)M, (int)N, (int)K, 0, (int)N, ta, false,
                          false, splits, kcs, geom, stream_of(x)));
  return out;
}

Tensor f32_im2col(const Tensor& x, int64_t kh, int64_t kw, int64_t pad) {
  f32_in(x, "x", 4);
  TORCH_CHECK(kh > 0 && kw > 0 && pad >= 0 && pad < kh && pad < kw, "f32_im2col: bad kernel/pad");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(B * H * W * kh * kw * C < ((int64_t)1 << 40), "f32_im2col: too large");
  const c10::DeviceGuard g(x.device());
  auto cols = at::empty({B * H * W, kh * kw * C}, x.options());
  CHECK_HIP(dmlc_f32_im2col(x.data_ptr<float>(), cols.data_ptr<float>(), (int)B, (int)H, (int)W, (int)C, (int)kh,
                            (int)kw, (int)pad, stream_of(x)));
  return cols;
}

Tensor f32_col2im(const Tensor& dcols, int64_t B, int64_t H, int64_t W, int64_t C, int64_t kh, int64_t kw,
                  int64_t pad) {
  check(dcols, "dcols", at::kFloat, {B * H * W, kh * kw * C});
  TORCH_CHECK(pad >= 0 && pad < kh && pad < kw, "f32_col2im: bad kernel/pad");
  const c10::DeviceGuard g(dcols.device());
  auto dx = at::empty({B, H, W, C}, dcols.options());
  CHECK_HIP(dmlc_f32_col2im(dcols.data_ptr<float>(), dx.data_ptr<float>(), (int)B, (int)H, (int)W, (int)C, (int)kh,
                            (int)kw, (int)pad, stream_of(dcols)));
  return dx;
}

Tensor f32_colsum(const Tensor& x) {
  f32_in(x, "x", 2);
  const int64_t M = x.size(0), N = x.size(1);
  TORCH_CHECK(M > 0 && N > 0 && M < (1 << 30) && N < (1 << 30), "f32_colsum: bad sizes");
  const c10::DeviceGuard g(x.device());
  const int splits = (int)std::min<int64_t>(std::min<int64_t>(std::max<int64_t>(1, M / 32), 128),
                                            std::max<int64_t>(1, 2048 / ((N + 63) / 64)));
  auto ws = at::empty({splits, N}, x.options());
  auto out = at::empty({N}, x.options());
  CHECK_HIP(dmlc_f32_colsum(x.data_ptr<float>(), out.data_ptr<float>(), ws.data_ptr<float>(), (int)M, (int)N, splits,
                            stream_of(x)));
  return out;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(dmlc, m) {
  m.def("f32_gemm(Tensor a, Tensor b, Tensor? bias, bool ta, bool tb, bool relu) -> Tensor");
  m.def("f32_conv_gemm(Tensor x, Tensor w, Tensor? bias, bool ta, bool ones) -> Tensor");
  m.def("f32_im2col(Tensor x, int kh, int kw, int pad) -> Tensor");
  m.def("f32_col2im(Tensor dcols, int B, int H, int W, int C, int kh, int kw, int pad) -> Tensor");
  m.def("f32_colsum(Tensor x) -> Tensor");
}

TORCH_LIBRARY_IMPL(dmlc, CUDA, m) {
  m.impl("f32_gemm", &f32_gemm);
  m.impl("f32_conv_gemm", &f32_conv_gemm);
  m.impl("f32_im2col", &f32_im2col);
  m.impl("f32_col2im", &f32_col2im);
  m.impl("f32_colsum", &f32_colsum);
}
