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
// small; each slice keeps >= 64 of K, and at most 128 slices (the reduction reads them in order)
void pick_split(int64_t M, int64_t N, int64_t K, int* splits, int* kc) {
  const int64_t tiles = ((M + 63) / 64) * ((N + 63) / 64);
  int64_t s = tiles >= 256 ? 1 : std::min<int64_t>(std::min<int64_t>((512 + tiles - 1) / tiles, 128), std::max<int64_t>(1, K / 64));
  int64_t c = ((K + s - 1) / s + 15) / 16 * 16;
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
                          (int)b.size(1), ta, tb, relu, splits, kc, stream_of(a)));
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
  const int splits = (int)std::min<int64_t>(std::min<int64_t>(std::max<int64_t>(1, M / 256), 128),
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
  m.def("f32_im2col(Tensor x, int kh, int kw, int pad) -> Tensor");
  m.def("f32_col2im(Tensor dcols, int B, int H, int W, int C, int kh, int kw, int pad) -> Tensor");
  m.def("f32_colsum(Tensor x) -> Tensor");
}

TORCH_LIBRARY_IMPL(dmlc, CUDA, m) {
  m.impl("f32_gemm", &f32_gemm);
  m.impl("f32_im2col", &f32_im2col);
  m.impl("f32_col2im", &f32_col2im);
  m.impl("f32_colsum", &f32_colsum);
}
