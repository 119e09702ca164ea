// torch.ops.dmlc.* bindings of the HIP CNN kernels (csrc/kernels/*.hip).
//
// Every op validates device, dtype, contiguity and the exact shapes the kernel's indexing and grid
// assume BEFORE launching (a mis-shaped launch on MI355X can fault the GPU), then launches on the
// current HIP stream, so the ops compose with torch streams and are capturable into HIP graphs.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>

#include <vector>

#include "../kernels/api.h"
#include "../kernels/api_comm.h"
#include "check.h"

namespace {

using namespace dmlc_bind;

// optional [B, 3072] uint8 raw-image copy (forward writes it, the conv1 weight gradient reads it)
uint8_t* xraw_ptr(const c10::optional<Tensor>& xraw, int64_t B) {
  if (!xraw.has_value()) return nullptr;
  check(*xraw, "xraw", at::kByte, {B, 3072});
  return xraw->data_ptr<uint8_t>();
}


void conv1_fwd(const Tensor& data, const Tensor& idx, const c10::optional<Tensor>& counter, int64_t period,
               int64_t cy, int64_t cx, const Tensor& w1f, const Tensor& b1, const Tensor& out, const Tensor& am,
               const c10::optional<Tensor>& amax, const c10::optional<Tensor>& xraw) {
  const int64_t B = out.size(0);
  check_data(data);
  TORCH_CHECK(cy >= 0 && cy <= 8 && cx >= 0 && cx <= 8, "crop offsets must be in [0,8]");
  check(w1f, "w1f", at::kBFloat16, {64, 96});
  check_numel(b1, "b1", at::kFloat, 64);
  check(out, "out", at::kBFloat16, {B, 12, 12, 64});
  check(am, "am", at::kByte, {B, 12, 12, 64});
  c10::DeviceGuard guard(out.device());
  DmlcConv1FwdArgs a;
  a.data = data.data_ptr<uint8_t>();
  a.src = index_src(idx, counter, period, B);
  check_order_fits(a.src, data.size(0));
  a.B = (int)B; a.cy = (int)cy; a.cx = (int)cx;
  a.w = w1f.data_ptr(); a.bias = b1.data_ptr<float>();
  a.out = out.data_ptr(); a.am = am.data_ptr<uint8_t>();
  a.amax = nullptr;
  a.xraw = xraw_ptr(xraw, B);
  a.xraw_in = 0;
  if (amax.has_value()) {
    check_numel(*amax, "amax", at::kFloat, B);
    a.amax = amax->data_ptr<float>();
  }
  CHECK_HIP(dmlc_conv1_fwd(&a, stream_of(out)));
}

void conv2_fwd_fp8(const Tensor& in, const Tensor& w8, const Tensor& b2, const Tensor& amax_x, const Tensor& scale_w,
                   const c10::optional<Tensor>& counter, const Tensor& out, const Tensor& am,
                   const c10::optional<Tensor>& x8out, const c10::optional<Tensor>& sx_out) {
  const int64_t B = in.size(0);
  check(in, "in", at::kBFloat16, {B, 12, 12, 64});
  check(w8, "w8", at::kByte, {64, 1600});
  check_numel(b2, "b2", at::kFloat, 64);
  check_numel(amax_x, "amax_x", at::kFloat, B);
  check_numel(scale_w, "scale_w", at::kFloat, 2);
  check(out, "out", at::kBFloat16, {B, 6, 6, 64});
  check(am, "am", at::kByte, {B, 6, 6, 64});
  c10::DeviceGuard guard(in.device());
  DmlcConv2FwdFp8Args a;
  a.in = in.data_ptr(); a.w8 = w8.data_ptr<uint8_t>(); a.bias = b2.data_ptr<float>();
  a.amax_x = amax_x.data_ptr<float>(); a.scale_w = scale_w.data_ptr<float>();
  a.counter = nullptr;
  if (counter.has_value()) {
    check_numel(*counter, "counter", at::kLong, 1);
    a.counter = counter->data_ptr<int64_t>();
  }
  a.out = out.data_ptr(); a.am = am.data_ptr<uint8_t>(); a.B = (int)B;
  TORCH_CHECK(x8out.has_value() == sx_out.has_value(), "conv2_fwd_fp8: x8out and sx_out go together");
  a.x8out = nullptr; a.sx_out = nullptr;
  if (x8out.has_value()) {
    check(*x8out, "x8out", at::kByte, {B, 144, 64});
    check_numel(*sx_out, "sx_out", at::kFloat, 1);
    a.x8out = x8out->data_ptr<uint8_t>(); a.sx_out = sx_out->data_ptr<float>();
  }
  CHECK_HIP(dmlc_conv2_fwd_fp8(&a, stream_of(in)));
}

void fp8_roundtrip(const Tensor& x, const Tensor& y, double scale) {
  check_numel(x, "x", at::kFloat, x.numel());
  check_numel(y, "y", at::kFloat, x.numel());
  c10::DeviceGuard guard(x.device());
  CHECK_HIP(dmlc_fp8_roundtrip(x.data_ptr<float>(), y.data_ptr<float>(), (int)x.numel(), (float)scale, stream_of(x)));
}

void conv12_fwd(const Tensor& data, const Tensor& idx, const c10::optional<Tensor>& counter, int64_t period,
                int64_t cy, int64_t cx, const Tensor& w1f, const Tensor& b1, const Tensor& p1, const Tensor& am1,
                const Tensor& w2f, const Tensor& b2, const Tensor& p2, const Tensor& am2,
                const c10::optional<Tensor>& xraw, bool xraw_in, const c10::optional<Tensor>& split_flags,
                const c10::optional<Tensor>& err) {
  const int64_t B = p1.size(0);
  TORCH_CHECK(!xraw_in || xraw.has_value(), "conv12_fwd: xraw_in needs the prefetched images");
  const bool split = split_flags.has_value();
  TORCH_CHECK(!split || (err.has_value() && !xraw_in && B <= 128),
              "conv12_fwd split (two workgroups per image): B <= 128, the error word, no prefetched images");
  check_data(data);
  TORCH_CHECK(cy >= 0 && cy <= 8 && cx >= 0 && cx <= 8, "crop offsets must be in [0,8]");
  check(w1f, "w1f", at::kBFloat16, {64, 96});
  check_numel(b1, "b1", at::kFloat, 64);
  check(p1, "p1", at::kBFloat16, {B, 12, 12, 64});
  check(am1, "am1", at::kByte, {B, 12, 12, 64});
  check(w2f, "w2f", at::kBFloat16, {64, 1600});
  check_numel(b2, "b2", at::kFloat, 64);
  check(p2, "p2", at::kBFloat16, {B, 6, 6, 64});
  check(am2, "am2", at::kByte, {B, 6, 6, 64});
  c10::DeviceGuard guard(p1.device());
  DmlcConv1FwdArgs a1;
  a1.data = data.data_ptr<uint8_t>(); a1.src = index_src(idx, counter, period, B);
  check_order_fits(a1.src, data.size(0));
  a1.B = (int)B; a1.cy = (int)cy; a1.cx = (int)cx;
  a1.w = w1f.data_ptr(); a1.bias = b1.data_ptr<float>(); a1.out = p1.data_ptr(); a1.am = am1.data_ptr<uint8_t>();
  a1.amax = nullptr;
  a1.xraw = xraw_ptr(xraw, B);
  a1.xraw_in = xraw_in ? 1 : 0;
  DmlcConv2FwdArgs a2;
  a2.in = p1.data_ptr(); a2.w = w2f.data_ptr(); a2.bias = b2.data_ptr<float>();
  a2.out = p2.data_ptr(); a2.am = am2.data_ptr<uint8_t>(); a2.B = (int)B;
  if (split) {
    check_min(*split_flags, "split_flags", at::kInt, 32 * 2 * B);
    check_numel(*err, "err", at::kInt, 1);
    CHECK_HIP(dmlc_conv12_fwd_split(&a1, &a2, reinterpret_cast<unsigned*>(split_flags->data_ptr<int>()),
                                    reinterpret_cast<unsigned*>(err->data_ptr<int>()), stream_of(p1)));
  } else {
    CHECK_HIP(dmlc_conv12_fwd(&a1, &a2, stream_of(p1)));
  }
}

void conv2_fwd(const Tensor& in, const Tensor& w2f, const Tensor& b2, const Tensor& out, const Tensor& am) {
  const int64_t B = in.size(0);
  check(in, "in", at::kBFloat16, {B, 12, 12, 64});
  check(w2f, "w2f", at::kBFloat16, {64, 1600});
  check_numel(b2, "b2", at::kFloat, 64);
  check(out, "out", at::kBFloat16, {B, 6, 6, 64});
  check(am, "am", at::kByte, {B, 6, 6, 64});
  c10::DeviceGuard guard(in.device());
  DmlcConv2FwdArgs a;
  a.in = in.data_ptr(); a.w = w2f.data_ptr(); a.bias = b2.data_ptr<float>();
  a.out = out.data_ptr(); a.am = am.data_ptr<uint8_t>(); a.B = (int)B;
  CHECK_HIP(dmlc_conv2_fwd(&a, stream_of(in)));
}

void conv2_dgrad(const Tensor& dp2, const Tensor& am2, const Tensor& w2d, const Tensor& dp1, const Tensor& dy2) {
  const int64_t B = dp2.size(0);
  check(dp2, "dp2", at::kBFloat16, {B, 6, 6, 64});
  check(am2, "am2", at::kByte, {B, 6, 6, 64});
  check(w2d, "w2d", at::kBFloat16, {64, 1600});
  check(dp1, "dp1", at::kBFloat16, {B, 12, 12, 64});
  check(dy2, "dy2", at::kBFloat16, {B, 144, 64});
  c10::DeviceGuard guard(dp2.device());
  DmlcConv2DgradArgs a;
  a.dp2 = dp2.data_ptr(); a.am2 = am2.data_ptr<uint8_t>(); a.wd = w2d.data_ptr();
  a.dp1 = dp1.data_ptr(); a.dy2 = dy2.data_ptr(); a.B = (int)B; a.split = 0;
  CHECK_HIP(dmlc_conv2_dgrad(&a, stream_of(dp2)));
}

// channel-split forward / input gradient (cnn_split.hip): same tensors as conv1_fwd / conv2_fwd /
// conv2_dgrad; the kernel batch must be a multiple of 8 (the engine pads it to 16)
void conv1_fwd_split(const Tensor& data, const Tensor& idx, const c10::optional<Tensor>& counter, int64_t period,
                     int64_t cy, int64_t cx, const Tensor& w1f, const Tensor& b1, const Tensor& out, const Tensor& am,
                     const c10::optional<Tensor>& xraw, int64_t nsplit) {
  const int64_t B = out.size(0);
  TORCH_CHECK(B % 8 == 0, "split kernels need a batch multiple of 8");
  TORCH_CHECK(nsplit == 2 || nsplit == 4, "conv1 split must be 2 or 4");
  check_data(data);
  TORCH_CHECK(cy >= 0 && cy <= 8 && cx >= 0 && cx <= 8, "crop offsets must be in [0,8]");
  check(w1f, "w1f", at::kBFloat16, {64, 96});
  check_numel(b1, "b1", at::kFloat, 64);
  check(out, "out", at::kBFloat16, {B, 12, 12, 64});
  check(am, "am", at::kByte, {B, 12, 12, 64});
  c10::DeviceGuard guard(out.device());
  DmlcConv1FwdArgs a;
  a.data = data.data_ptr<uint8_t>();
  a.src = index_src(idx, counter, period, B);
  check_order_fits(a.src, data.size(0));
  a.B = (int)B; a.cy = (int)cy; a.cx = (int)cx;
  a.w = w1f.data_ptr(); a.bias = b1.data_ptr<float>();
  a.out = out.data_ptr(); a.am = am.data_ptr<uint8_t>();
  a.amax = nullptr;
  a.xraw = xraw_ptr(xraw, B);
  a.xraw_in = 0;
  CHECK_HIP(dmlc_conv1_fwd_split(&a, (int)nsplit, stream_of(out)));
}

void conv2_fwd_split(const Tensor& in, const Tensor& w2f, const Tensor& b2, const Tensor& out, const Tensor& am) {
  const int64_t B = in.size(0);
  TORCH_CHECK(B % 8 == 0, "split kernels need a batch multiple of 8");
  check(in, "in", at::kBFloat16, {B, 12, 12, 64});
  check(w2f, "w2f", at::kBFloat16, {64, 1600});
  check_numel(b2, "b2", at::kFloat, 64);
  check(out, "out", at::kBFloat16, {B, 6, 6, 64});
  check(am, "am", at::kByte, {B, 6, 6, 64});
  c10::DeviceGuard guard(in.device());
  DmlcConv2FwdArgs a;
  a.in = in.data_ptr(); a.w = w2f.data_ptr(); a.bias = b2.data_ptr<float>();
  a.out = out.data_ptr(); a.am = am.data_ptr<uint8_t>(); a.B = (int)B;
  CHECK_HIP(dmlc_conv2_fwd_split(&a, stream_of(in)));
}

void conv2_dgrad_split(const Tensor& dp2, const Tensor& am2, const Tensor& w2d, const Tensor& dp1, const Tensor& dy2) {
  const int64_t B = dp2.size(0);
  TORCH_CHECK(B % 8 == 0, "split kernels need a batch multiple of 8");
  check(dp2, "dp2", at::kBFloat16, {B, 6, 6, 64});
  check(am2, "am2", at::kByte, {B, 6, 6, 64});
  check(w2d, "w2d", at::kBFloat16, {64, 1600});
  check(dp1, "dp1", at::kBFloat16, {B, 12, 12, 64});
  check(dy2, "dy2", at::kBFloat16, {B, 144, 64});
  c10::DeviceGuard guard(dp2.device());
  DmlcConv2DgradArgs a;
  a.dp2 = dp2.data_ptr(); a.am2 = am2.data_ptr<uint8_t>(); a.wd = w2d.data_ptr();
  a.dp1 = dp1.data_ptr(); a.dy2 = dy2.data_ptr(); a.B = (int)B; a.split = 0;
  CHECK_HIP(dmlc_conv2_dgrad_split(&a, stream_of(dp2)));
}

void conv2_dgrad_fp8(const Tensor& dp2, const Tensor& am2, const Tensor& w2d8, const Tensor& scale_w, const Tensor& dp1,
                     const Tensor& dy2, const c10::optional<Tensor>& dy8out, const c10::optional<Tensor>& sy_img) {
  const int64_t B = dp2.size(0);
  check(dp2, "dp2", at::kBFloat16, {B, 6, 6, 64});
  check(am2, "am2", at::kByte, {B, 6, 6, 64});
  check(w2d8, "w2d8", at::kByte, {64, 1600});
  check_numel(scale_w, "scale_w", at::kFloat, 2);
  check(dp1, "dp1", at::kBFloat16, {B, 12, 12, 64});
  check(dy2, "dy2", at::kBFloat16, {B, 144, 64});
  c10::DeviceGuard guard(dp2.device());
  DmlcConv2DgradFp8Args a;
  a.dp2 = dp2.data_ptr(); a.am2 = am2.data_ptr<uint8_t>(); a.w8 = w2d8.data_ptr<uint8_t>();
  a.scale_w = scale_w.data_ptr<float>(); a.dp1 = dp1.data_ptr(); a.dy2 = dy2.data_ptr(); a.B = (int)B;
  TORCH_CHECK(dy8out.has_value() == sy_img.has_value(), "conv2_dgrad_fp8: dy8out and sy_img go together");
  a.dy8out = nullptr; a.sy_img = nullptr;
  if (dy8out.has_value()) {
    check(*dy8out, "dy8out", at::kByte, {B, 144, 64});
    check_numel(*sy_img, "sy_img", at::kFloat, B);
    a.dy8out = dy8out->data_ptr<uint8_t>(); a.sy_img = sy_img->data_ptr<float>();
  }
  CHECK_HIP(dmlc_conv2_dgrad_fp8(&a, stream_of(dp2)));
}

// conv2 weight-gradient slabs: [g2][1600][64] fp32
static DmlcWgradArgs make_wgrad(const Tensor& data, const Tensor& idx, const c10::optional<Tensor>& counter,
                                int64_t period, int64_t cy, int64_t cx, const Tensor& dp1, const Tensor& am1,
                                const Tensor& part1, const Tensor& partb1, const Tensor& p1, const Tensor& dy2,
                                const Tensor& part2, const Tensor& partb2, int64_t groups2,
                                const c10::optional<Tensor>& xraw,
                                const c10::optional<at::TensorList>& fp8 = c10::nullopt) {
  const int64_t B = p1.size(0), g1 = part1.size(0), g2 = groups2;
  check_data(data);
  TORCH_CHECK(cy >= 0 && cy <= 8 && cx >= 0 && cx <= 8, "crop offsets must be in [0,8]");
  TORCH_CHECK(g1 >= 1 && g1 <= B && g2 >= 1 && g2 <= B, "split-K groups must be in [1,B]");
  TORCH_CHECK(part2.size(0) == g2, "wgrad: one conv2 slab per image group");
  TORCH_CHECK(g1 + 4 * g2 <= 1024, "wgrad: too many workgroups");
  check(dp1, "dp1", at::kBFloat16, {B, 12, 12, 64});
  check(am1, "am1", at::kByte, {B, 12, 12, 64});
  check(part1, "part1", at::kFloat, {g1, 80, 64});
  check(partb1, "partb1", at::kFloat, {g1, 64});
  check(p1, "p1", at::kBFloat16, {B, 12, 12, 64});
  check(dy2, "dy2", at::kBFloat16, {B, 144, 64});
  check(part2, "part2", at::kFloat, {g2, 1600, 64});
  check(partb2, "partb2", at::kFloat, {g2, 64});
  DmlcWgradArgs a;
  memset(&a, 0, sizeof(a));                      // (fc_in_launch off unless wgrad_sgd sets it)
  a.w1.data = data.data_ptr<uint8_t>(); a.w1.src = index_src(idx, counter, period, B);
  check_order_fits(a.w1.src, data.size(0));
  a.w1.cy = (int)cy; a.w1.cx = (int)cx;
  a.w1.dp1 = dp1.data_ptr(); a.w1.am1 = am1.data_ptr<uint8_t>();
  a.w1.part1 = part1.data_ptr<float>(); a.w1.partb1 = partb1.data_ptr<float>(); a.w1.g1 = (int)g1; a.w1.B = (int)B;
  a.w1.xraw = xraw_ptr(xraw, B);
  a.w2.p1 = p1.data_ptr(); a.w2.dy2 = dy2.data_ptr(); a.w2.part2 = part2.data_ptr();
  a.w2.partb2 = partb2.data_ptr<float>(); a.w2.g2 = (int)g2; a.w2.B = (int)B;
  if (fp8.has_value()) {
    // the fp8 conv2 weight gradient's operands: {x8 [B][144][64] e4m3, y8 (same), sx [1], sy_img [B]}
    const at::TensorList f = *fp8;
    TORCH_CHECK(f.size() == 4, "wgrad: fp8 = {x8, y8, sx, sy_img}");
    check(f[0], "x8", at::kByte, {B, 144, 64});
    check(f[1], "y8", at::kByte, {B, 144, 64});
    check_numel(f[2], "sx", at::kFloat, 1);
    check_numel(f[3], "sy_img", at::kFloat, B);
    a.w2.x8 = f[0].data_ptr<uint8_t>(); a.w2.y8 = f[1].data_ptr<uint8_t>();
    a.w2.sx = f[2].data_ptr<float>(); a.w2.sy_img = f[3].data_ptr<float>();
  }
  a.apply = 0; a.bar = nullptr; a.helpers = 0; a.fc_done = 0;
  memset(&a.sgd, 0, sizeof(a.sgd));
  return a;
}

void wgrad(const Tensor& data, const Tensor& idx, const c10::optional<Tensor>& counter, int64_t period, int64_t cy,
           int64_t cx, const Tensor& dp1, const Tensor& am1, const Tensor& part1, const Tensor& partb1,
           const Tensor& p1, const Tensor& dy2, const Tensor& part2, const Tensor& partb2, int64_t groups2,
           const c10::optional<Tensor>& xraw, const c10::optional<at::TensorList> fp8) {
  DmlcWgradArgs a = make_wgrad(data, idx, counter, period, cy, cx, dp1, am1, part1, partb1, p1, dy2, part2, partb2,
                               groups2, xraw, fp8);
  c10::DeviceGuard guard(dp1.device());
  CHECK_HIP(dmlc_wgrad(&a, stream_of(dp1)));
}

// params per problem (14 ints): M, N, K, lda, a_kmajor, ldb, b_kmajor, ldc, c_mode, ksplit, relu, nvalid,
// b_par, s_par.  c_mode 0 fp32 C, 1 bf16 C, 2 split-K fp32 slabs, 3 column sums, 4 fused SGD (C = fp32
// master weights updated in place, bf16 shadow into `shadow` at parity offset s_par; needs `step` and
// sched = {lr0, decay, decay_steps, staircase, warmup, grad_scale}).  b_par != 0: the B operand of odd
// steps lives b_par elements further on (double-buffered shadow; needs `step`).
void gemm_grouped(at::TensorList A, at::TensorList Bm, at::TensorList C, const c10::List<c10::optional<Tensor>>& bias,
                  at::IntArrayRef params, const c10::optional<Tensor>& step, const c10::optional<Tensor>& shadow,
                  at::ArrayRef<double> sched) {
  const int n = (int)A.size();
  TORCH_CHECK(n >= 1 && n <= DMLC_MAX_GEMM, "1..8 problems per group");
  TORCH_CHECK((int)Bm.size() == n && (int)C.size() == n && (int)bias.size() == n, "list lengths differ");
  TORCH_CHECK((int)params.size() == 14 * n, "params must hold 14 ints per problem");
  DmlcGemmGroup G;
  memset(&G, 0, sizeof(G));
  G.nprob = n;
  static const int xcd_map = 1;    // XCD-aware tile order (cnn_gemm.hip)
  G.xcd_map = xcd_map;
  if (step.has_value()) {
    check_numel(*step, "step", at::kLong, 1);
    G.step = step->data_ptr<int64_t>();
  }
  for (int i = 0; i < n; ++i) {
    const int64_t* q = params.data() + 14 * i;
    DmlcGemmProblem& P = G.p[i];
    P.M = (int)q[0]; P.N = (int)q[1]; P.K = (int)q[2];
    P.lda = (int)q[3]; P.a_kmajor = (int)q[4]; P.ldb = (int)q[5]; P.b_kmajor = (int)q[6];
    P.ldc = (int)q[7]; P.c_mode = (int)q[8]; P.ksplit = (int)q[9]; P.relu = (int)q[10]; P.nvalid = (int)q[11];
    P.b_par = q[12]; P.s_par = q[13];
    TORCH_CHECK(P.c_mode >= 0 && P.c_mode <= 4, "gemm ", i, ": c_mode must be 0..4");
    TORCH_CHECK(P.b_par >= 0 && P.s_par >= 0, "gemm ", i, ": negative parity offset");
    TORCH_CHECK(P.b_par == 0 || G.step, "gemm ", i, ": a parity-buffered B needs the step counter");
    TORCH_CHECK(P.M > 0 && P.K > 0 && P.M % 8 == 0 && P.K % 8 == 0, "gemm ", i, ": M,K must be positive multiples of 8");
    TORCH_CHECK(P.lda % 8 == 0, "gemm ", i, ": lda must be a multiple of 8 (16-byte rows)");
    check_min(A[i], "A", at::kBFloat16, P.a_kmajor ? (int64_t)(P.M - 1) * P.lda + P.K : (int64_t)(P.K - 1) * P.lda + P.M);
    TORCH_CHECK(P.a_kmajor ? P.lda >= P.K : P.lda >= P.M, "gemm ", i, ": lda too small");
    if (P.c_mode == 3) {
      TORCH_CHECK(P.a_kmajor == 0, "gemm ", i, ": column sums need an m-major A");
      TORCH_CHECK(P.b_par == 0, "gemm ", i, ": column sums read no B");
      check_min(C[i], "C", at::kFloat, std::min(P.M, P.nvalid));
      P.ksplit = 1;
      continue;
    }
    TORCH_CHECK(P.N > 0 && P.N % 8 == 0, "gemm ", i, ": N must be a positive multiple of 8");
    TORCH_CHECK(P.ldb % 8 == 0, "gemm ", i, ": ldb must be a multiple of 8");
    TORCH_CHECK(P.b_kmajor ? P.ldb >= P.K : P.ldb >= P.N, "gemm ", i, ": ldb too small");
    check_min(Bm[i], "B", at::kBFloat16,
              P.b_par + (P.b_kmajor ? (int64_t)(P.N - 1) * P.ldb + P.K : (int64_t)(P.K - 1) * P.ldb + P.N));
    TORCH_CHECK(P.ksplit >= 1 && (P.ksplit == 1 || P.c_mode == 2), "gemm ", i, ": split-K needs c_mode 2");
    TORCH_CHECK(P.nvalid >= 1 && P.nvalid <= P.N && P.ldc >= P.nvalid, "gemm ", i, ": bad nvalid/ldc");
    const int64_t cneed = (int64_t)(P.c_mode == 2 ? P.ksplit : 1) * P.M * P.ldc;
    check_min(C[i], "C", P.c_mode == 1 ? at::kBFloat16 : at::kFloat, cneed);
    P.S = nullptr;
    if (P.c_mode == 4) {
      TORCH_CHECK(G.step && shadow.has_value() && sched.size() == 6, "gemm ", i,
                  ": the fused SGD epilogue needs step, shadow and sched = {lr0, decay, decay_steps, staircase, warmup, grad_scale}");
      TORCH_CHECK(P.ksplit == 1 && P.nvalid == P.N && P.N % 4 == 0 && P.ldc % 4 == 0 && !P.bias && !P.relu,
                  "gemm ", i, ": the fused SGD epilogue needs ksplit 1, full 16-B rows, no bias / ReLU");
      TORCH_CHECK(!bias.get(i).has_value(), "gemm ", i, ": the fused SGD epilogue takes no bias");
      check_min(*shadow, "shadow", at::kBFloat16, P.s_par + (int64_t)P.M * P.ldc);
      P.S = shadow->data_ptr();
      G.lr0 = (float)sched[0]; G.decay = (float)sched[1]; G.decay_steps = (float)sched[2];
      G.staircase = sched[3] != 0.0; G.warmup = (float)sched[4]; G.grad_scale = (float)sched[5];
    }
    P.A = A[i].data_ptr(); P.B = Bm[i].data_ptr(); P.C = C[i].data_ptr();
    P.bias = nullptr;
    const c10::optional<Tensor> bo = bias.get(i);
    if (bo.has_value()) {
      check_min(*bo, "bias", at::kFloat, P.nvalid);
      P.bias = bo->data_ptr<float>();
    }
  }
  for (int i = 0; i < n; ++i) {
    if (G.p[i].c_mode == 3) { G.p[i].A = A[i].data_ptr(); G.p[i].C = C[i].data_ptr(); G.p[i].bias = nullptr; }
  }
  c10::DeviceGuard guard(A[0].device());
  CHECK_HIP(dmlc_gemm_grouped(&G, stream_of(A[0])));
}

void head(const Tensor& h1part, const Tensor& b1, const Tensor& w2t, const Tensor& b2, const Tensor& w3t,
          const Tensor& b3, const Tensor& w3d, const Tensor& w2d, const Tensor& labels, const Tensor& idx,
          const c10::optional<Tensor>& counter, int64_t period, double inv_batch, bool relu_logits, bool train,
          const Tensor& h1, const Tensor& h2, const Tensor& dl, const Tensor& dh1, const Tensor& dh2,
          const Tensor& loss_part, const Tensor& correct_part, const c10::optional<Tensor>& logits_out,
          int64_t nvalid, const c10::optional<Tensor>& step, const c10::optional<Tensor>& step_copy) {
  TORCH_CHECK(h1part.dim() == 3 && h1part.size(2) == 384, "h1part must be [nsplit,B,384]");
  const int64_t nsplit = h1part.size(0), B = h1part.size(1);
  TORCH_CHECK(B % 16 == 0 && B > 0, "head: batch must be a positive multiple of 16");
  TORCH_CHECK(loss_part.numel() >= 1 && B % loss_part.numel() == 0, "head: loss partials must divide the batch");
  const int64_t rows = B / loss_part.numel();      // rows per workgroup, picked by the caller
  TORCH_CHECK(rows == 2 || rows == 4, "head: B / loss_part.numel() (rows per workgroup) must be 2 or 4");
  check(h1part, "h1part", at::kFloat, {nsplit, B, 384});
  check_numel(b1, "b1", at::kFloat, 384);
  check(w2t, "w2t", at::kBFloat16, {192, 384});
  check_numel(b2, "b2", at::kFloat, 192);
  check(w3t, "w3t", at::kBFloat16, {16, 192});
  check_numel(b3, "b3", at::kFloat, 10);
  check(w3d, "w3d", at::kBFloat16, {192, 32});
  check(w2d, "w2d", at::kBFloat16, {384, 192});
  dev(labels, "labels");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.dim() == 1, "labels must be int32 [N]");
  check(loss_part, "loss_part", at::kFloat, {B / rows});
  check(correct_part, "correct_part", at::kInt, {B / rows});
  if (train) {
    check(h1, "h1", at::kBFloat16, {B, 384});
    check(h2, "h2", at::kBFloat16, {B, 192});
    check(dl, "dl", at::kBFloat16, {B, 16});
    check(dh1, "dh1", at::kBFloat16, {B, 384});
    check(dh2, "dh2", at::kBFloat16, {B, 192});
  }
  c10::DeviceGuard guard(h1part.device());
  DmlcHeadArgs a;
  a.h1part = h1part.data_ptr<float>(); a.nsplit = (int)nsplit;
  a.b1 = b1.data_ptr<float>(); a.w2t = w2t.data_ptr(); a.b2 = b2.data_ptr<float>();
  a.w3t = w3t.data_ptr(); a.b3 = b3.data_ptr<float>(); a.w3d = w3d.data_ptr(); a.w2d = w2d.data_ptr();
  a.labels = labels.data_ptr<int>(); a.src = index_src(idx, counter, period, B);
  check_order_fits(a.src, labels.size(0));
  if (nvalid < 0) nvalid = B;
  TORCH_CHECK(nvalid >= 1 && nvalid <= B, "head: nvalid must be in [1, B]");
  a.nvalid = (int)nvalid;
  a.B = (int)B; a.rows = (int)rows; a.inv_batch = (float)inv_batch; a.relu_logits = relu_logits; a.train = train;
  a.h1 = train ? h1.data_ptr() : nullptr; a.h2 = train ? h2.data_ptr() : nullptr; a.dl = train ? dl.data_ptr() : nullptr;
  a.dh1 = train ? dh1.data_ptr() : nullptr; a.dh2 = train ? dh2.data_ptr() : nullptr;
  a.loss_part = loss_part.data_ptr<float>(); a.correct_part = correct_part.data_ptr<int>();
  a.logits_out = nullptr;
  if (logits_out.has_value()) {
    check(*logits_out, "logits_out", at::kFloat, {B, 10});
    a.logits_out = logits_out->data_ptr<float>();
  }
  a.step = nullptr; a.step_copy = nullptr;
  TORCH_CHECK(step.has_value() == step_copy.has_value(), "head: step and step_copy go together");
  if (step.has_value()) {
    check_numel(*step, "step", at::kLong, 1);
    check_numel(*step_copy, "step_copy", at::kLong, 1);
    a.step = step->data_ptr<int64_t>(); a.step_copy = step_copy->data_ptr<int64_t>();
  }
  CHECK_HIP(dmlc_head(&a, stream_of(h1part)));
}

// the whole fc chain of a training step, one persistent launch (cnn_fc.hip)
void fc_chain(const Tensor& p2, const Tensor& fc1n, const Tensor& h1part, const Tensor& b1, const Tensor& w2t,
              const Tensor& b2, const Tensor& w3t, const Tensor& b3, const Tensor& w3d, const Tensor& labels,
              const Tensor& idx, const c10::optional<Tensor>& counter, int64_t period, double inv_batch,
              bool relu_logits, const Tensor& h1, const Tensor& h2, const Tensor& dl, const Tensor& dh1,
              const Tensor& dh2, const Tensor& loss_part, const Tensor& correct_part, const Tensor& dp2,
              const Tensor& gw1, const Tensor& gw2, const Tensor& gw3, const Tensor& gb1, const Tensor& gb2,
              const Tensor& gb3, bool fuse_sgd, at::ArrayRef<double> sched, int64_t nvalid, const Tensor& step,
              const c10::optional<Tensor>& step_copy, const Tensor& sync, const Tensor& err, bool dw_tasks,
              const c10::optional<Tensor>& am2, const c10::optional<Tensor>& w2d, const c10::optional<Tensor>& dp1,
              const c10::optional<Tensor>& dy2, const c10::optional<Tensor>& fc2n) {
  const int64_t B = p2.size(0);
  TORCH_CHECK(B >= 16 && B <= 256 && B % 16 == 0, "fc_chain: batch must be a multiple of 16 in [16, 256]");
  check(p2, "p2", at::kBFloat16, {B, 2304});
  check(fc1n, "fc1n", at::kBFloat16, {2, 2304, 384});
  check(h1part, "h1part", at::kFloat, {8, B, 384});
  check_numel(b1, "b1", at::kFloat, 384);
  check(w2t, "w2t", at::kBFloat16, {192, 384});
  check_numel(b2, "b2", at::kFloat, 192);
  check(w3t, "w3t", at::kBFloat16, {16, 192});
  check_numel(b3, "b3", at::kFloat, 10);
  check(w3d, "w3d", at::kBFloat16, {192, 32});
  dev(labels, "labels");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.dim() == 1, "labels must be int32 [N]");
  check(h1, "h1", at::kBFloat16, {B, 384});
  check(h2, "h2", at::kBFloat16, {B, 192});
  check(dl, "dl", at::kBFloat16, {B, 16});
  check(dh1, "dh1", at::kBFloat16, {B, 384});
  check(dh2, "dh2", at::kBFloat16, {B, 192});
  check(loss_part, "loss_part", at::kFloat, {B / 4});
  check(correct_part, "correct_part", at::kInt, {B / 4});
  check(dp2, "dp2", at::kBFloat16, {B, 2304});
  // the fc gradients: fp32 views of the flat gradient, or bf16 views (the RCCL bf16 wire, no fused SGD)
  const bool g16 = gw1.scalar_type() == at::kBFloat16;
  TORCH_CHECK(!g16 || !fuse_sgd, "fc_chain: bf16 gradient views only without the fused SGD");
  const auto gt = g16 ? at::kBFloat16 : at::kFloat;
  check_numel(gw1, "gw1", gt, 2304 * 384);
  check_numel(gw2, "gw2", gt, 384 * 192);
  check_numel(gw3, "gw3", gt, 192 * 10);
  check_numel(gb1, "gb1", gt, 384);
  check_numel(gb2, "gb2", gt, 192);
  check_numel(gb3, "gb3", gt, 10);
  check_numel(step, "step", at::kLong, 1);
  check_min(sync, "sync", at::kInt, 212 * 32);   // fc_common.h SY_END
  check_min(err, "err", at::kInt, 1);
  TORCH_CHECK(sched.size() == 6, "fc_chain: sched = {lr0, decay, decay_steps, staircase, warmup, grad_scale}");
  if (nvalid < 0) nvalid = B;
  TORCH_CHECK(nvalid >= 1 && nvalid <= B, "fc_chain: nvalid must be in [1, B]");
  c10::DeviceGuard guard(p2.device());
  DmlcFcArgs a;
  memset(&a, 0, sizeof(a));
  a.B = (int)B; a.nvalid = (int)nvalid; a.mtiles = (int)((B + 63) / 64);
  a.p2 = p2.data_ptr(); a.w1 = fc1n.data_ptr(); a.h1part = h1part.data_ptr<float>();
  a.b1 = b1.data_ptr<float>(); a.w2t = w2t.data_ptr(); a.b2 = b2.data_ptr<float>();
  a.w3t = w3t.data_ptr(); a.b3 = b3.data_ptr<float>(); a.w3d = w3d.data_ptr();
  a.labels = labels.data_ptr<int>(); a.src = index_src(idx, counter, period, B);
  check_order_fits(a.src, labels.size(0));
  a.inv_batch = (float)inv_batch; a.relu_logits = relu_logits;
  a.h1 = h1.data_ptr(); a.h2 = h2.data_ptr(); a.dl = dl.data_ptr(); a.dh1 = dh1.data_ptr(); a.dh2 = dh2.data_ptr();
  a.loss_part = loss_part.data_ptr<float>(); a.correct_part = correct_part.data_ptr<int>();
  a.dp2 = dp2.data_ptr();
  a.gw1 = (float*)gw1.data_ptr(); a.gw2 = (float*)gw2.data_ptr(); a.gw3 = (float*)gw3.data_ptr();
  a.gb1 = (float*)gb1.data_ptr(); a.gb2 = (float*)gb2.data_ptr(); a.gb3 = (float*)gb3.data_ptr();
  a.grad_bf16 = g16 ? 1 : 0;
  a.fuse_sgd = fuse_sgd ? 1 : 0;
  a.dw_tasks = dw_tasks ? 1 : 0;
  if (fc2n.has_value()) {
    // every fc parameter's SGD in the dW tiles' epilogues (fuse_sgd 2, as the wgrad launch runs them):
    // gw2 / gw3 / gb1..3 are then the fp32 MASTER views and w2t / w3t / w3d + fc2n the bf16 shadows the
    // epilogues rewrite (the head has read them before the dW tiles' seam)
    TORCH_CHECK(fuse_sgd && dw_tasks, "fc_chain: the fc SGD in the chain needs fuse_sgd and the dW tiles");
    check(*fc2n, "fc2n", at::kBFloat16, {384, 192});
    a.fuse_sgd = 2;
    a.mw2 = gw2.data_ptr<float>(); a.mw3 = gw3.data_ptr<float>();
    a.mb1 = gb1.data_ptr<float>(); a.mb2 = gb2.data_ptr<float>(); a.mb3 = gb3.data_ptr<float>();
    a.fc2n = fc2n->data_ptr(); a.fc2t = w2t.data_ptr(); a.fc3t = w3t.data_ptr(); a.fc3d = w3d.data_ptr();
  }
  a.lr0 = (float)sched[0]; a.decay = (float)sched[1]; a.decay_steps = (float)sched[2];
  a.staircase = sched[3] != 0.0; a.warmup = (float)sched[4]; a.grad_scale = (float)sched[5];
  a.step = step.data_ptr<int64_t>();
  a.step_copy = nullptr;
  if (step_copy.has_value()) {
    check_numel(*step_copy, "step_copy", at::kLong, 1);
    a.step_copy = step_copy->data_ptr<int64_t>();
  }
  a.sync = reinterpret_cast<unsigned int*>(sync.data_ptr<int>());
  a.err = reinterpret_cast<unsigned int*>(err.data_ptr<int>());
  // am2 / w2d / dp1 / dy2: the conv2 input gradient runs in the same launch (one image per workgroup)
  const bool dg_on = am2.has_value();
  TORCH_CHECK(dg_on == w2d.has_value() && dg_on == dp1.has_value() && dg_on == dy2.has_value(),
              "fc_chain: am2, w2d, dp1, dy2 come together");
  DmlcConv2DgradArgs g;
  memset(&g, 0, sizeof(g));
  if (dg_on) {
    check(*am2, "am2", at::kByte, {B, 6, 6, 64});
    check(*w2d, "w2d", at::kBFloat16, {64, 1600});
    check(*dp1, "dp1", at::kBFloat16, {B, 12, 12, 64});
    check(*dy2, "dy2", at::kBFloat16, {B, 144, 64});
    g.dp2 = dp2.data_ptr(); g.am2 = am2->data_ptr<uint8_t>(); g.wd = w2d->data_ptr();
    g.dp1 = dp1->data_ptr(); g.dy2 = dy2->data_ptr(); g.B = (int)B;
    g.split = B <= 128 ? 1 : 0;          // the chain's 256 workgroups: two per image at B <= 128
  }
  CHECK_HIP(dmlc_fc_chain(&a, dg_on ? &g : nullptr, stream_of(p2)));
}

static DmlcSgdArgs make_sgd(const Tensor& master, const Tensor& grad, int64_t mode, double grad_scale, at::IntArrayRef off,
         const Tensor& part1, const Tensor& partb1, const Tensor& part2, const Tensor& partb2, const Tensor& w1f,
         const Tensor& w2f, const Tensor& w2d, const Tensor& fc1n, const Tensor& fc2t, const Tensor& fc2n,
         const Tensor& fc3t, const Tensor& fc3d, const Tensor& step, double lr0, double decay, double decay_steps,
         bool staircase, const Tensor& ticket, const Tensor& loss_part, const Tensor& correct_part,
         const Tensor& stats, const c10::optional<Tensor>& w2f8, const c10::optional<Tensor>& amax_w,
         const c10::optional<Tensor>& scale_w, int64_t roles, bool finalize, int64_t batch,
         const c10::optional<Tensor>& bidx, const c10::optional<Tensor>& order, double warmup, bool fc1_fused,
         const c10::optional<Tensor>& step_rd, const c10::optional<Tensor>& xnext,
         const c10::optional<Tensor>& xdata) {
  TORCH_CHECK(roles >= 0 && roles <= 2, "sgd roles must be 0..2");
  TORCH_CHECK(warmup >= 0.0, "sgd: warmup must be >= 0");
  TORCH_CHECK(mode >= 0 && mode <= 3, "sgd mode must be 0..3");
  TORCH_CHECK(off.size() == 10, "off must have 10 entries");
  static const int64_t numel[10] = {4800, 64, 102400, 64, 884736, 384, 73728, 192, 1920, 10};
  for (int i = 0; i < 10; ++i) {
    TORCH_CHECK(off[i] >= 0 && (i == 0 || off[i] >= off[i - 1] + numel[i - 1]), "bad param offsets");
  }
  const int64_t end = off[9] + 10;
  check_min(master, "master", at::kFloat, end);
  // the flat gradient: fp32, or bf16 (DmlcSgdArgs::grad16: the RCCL bf16 wire, modes 1 / 2 only)
  const bool g16 = grad.scalar_type() == at::kBFloat16;
  check_min(grad, "grad", g16 ? at::kBFloat16 : at::kFloat, end);
  TORCH_CHECK(!g16 || mode == 1 || mode == 2, "sgd: a bf16 gradient only in modes 1 / 2 (data parallel)");
  const int64_t g1 = part1.size(0), g2 = part2.size(0);
  check(part1, "part1", at::kFloat, {g1, 80, 64});
  check(partb1, "partb1", at::kFloat, {g1, 64});
  check(part2, "part2", at::kFloat, {g2, 1600, 64});
  check(partb2, "partb2", at::kFloat, {g2, 64});
  TORCH_CHECK(loss_part.numel() >= 1, "loss partials missing");
  const int64_t B = batch;
  TORCH_CHECK(B >= 1 && B <= 4 * loss_part.numel(), "sgd: batch (valid rows) exceeds the head's rows");
  check(w1f, "w1f", at::kBFloat16, {64, 96});
  check(w2f, "w2f", at::kBFloat16, {64, 1600});
  check(w2d, "w2d", at::kBFloat16, {64, 1600});
  check(fc1n, "fc1n", at::kBFloat16, {2, 2304, 384});          // step-parity double buffer
  TORCH_CHECK(!fc1_fused || mode == 0, "sgd: fc1_fused only in mode 0 (single GPU)");
  check(fc2t, "fc2t", at::kBFloat16, {192, 384});
  check(fc2n, "fc2n", at::kBFloat16, {384, 192});
  check(fc3t, "fc3t", at::kBFloat16, {16, 192});
  check(fc3d, "fc3d", at::kBFloat16, {192, 32});
  check_numel(step, "step", at::kLong, 1);
  check_numel(ticket, "ticket", at::kInt, DMLC_TICKET_WORDS);
  dev(loss_part, "loss_part"); dev(correct_part, "correct_part");
  TORCH_CHECK(loss_part.scalar_type() == at::kFloat && correct_part.scalar_type() == at::kInt &&
                  loss_part.numel() == correct_part.numel(), "loss/correct partials mismatch");
  dev(stats, "stats");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.dim() == 2 && stats.size(1) == 4, "stats must be [R,4] fp32");
  DmlcSgdArgs a;
  a.master = master.data_ptr<float>();
  a.grad = g16 ? nullptr : grad.data_ptr<float>();
  a.grad16 = g16 ? grad.data_ptr() : nullptr;
  a.mode = (int)mode; a.grad_scale = (float)grad_scale;
  for (int i = 0; i < 10; ++i) a.off[i] = (int)off[i];
  a.part1 = part1.data_ptr<float>(); a.partb1 = partb1.data_ptr<float>(); a.g1 = (int)g1;
  a.part2 = part2.data_ptr(); a.g2 = (int)g2;
  a.partb2 = partb2.data_ptr<float>(); a.B = (int)B;
  a.w1f = w1f.data_ptr(); a.w2f = w2f.data_ptr(); a.w2d = w2d.data_ptr(); a.fc1n = fc1n.data_ptr();
  a.fc2t = fc2t.data_ptr(); a.fc2n = fc2n.data_ptr(); a.fc3t = fc3t.data_ptr(); a.fc3d = fc3d.data_ptr();
  a.step = step.data_ptr<int64_t>(); a.lr0 = (float)lr0;
  a.step_rd = a.step;
  if (step_rd.has_value()) {
    check_numel(*step_rd, "step_rd", at::kLong, 1);
    a.step_rd = step_rd->data_ptr<int64_t>();
  } a.decay = (float)decay;
  a.decay_steps = (float)decay_steps; a.staircase = staircase; a.warmup = (float)warmup; a.fc1_fused = fc1_fused ? 1 : 0;
  a.ticket = reinterpret_cast<unsigned int*>(ticket.data_ptr<int>());
  a.loss_part = loss_part.data_ptr<float>(); a.correct_part = correct_part.data_ptr<int>();
  a.nhead = (int)loss_part.numel();
  a.stats = stats.data_ptr<float>(); a.stats_len = (int)stats.size(0);
  a.w2f8 = nullptr; a.w2d8 = nullptr; a.amax_w = nullptr; a.scale_w = nullptr;
  a.roles = (int)roles; a.finalize = finalize ? 1 : 0;
  if (w2f8.has_value()) {
    TORCH_CHECK(amax_w.has_value() && scale_w.has_value(), "fp8 shadow needs amax_w and scale_w");
    // [64][1600] = the forward shadow only; [2][64][1600] = forward + the fp8 dgrad's flipped copy
    if (w2f8->dim() == 3) check(*w2f8, "w2f8", at::kByte, {2, 64, 1600});
    else check(*w2f8, "w2f8", at::kByte, {64, 1600});
    check_numel(*amax_w, "amax_w", at::kFloat, 2 * 400);   // [2 slots][400 conv2-row blocks]
    check_numel(*scale_w, "scale_w", at::kFloat, 2);
    a.w2f8 = w2f8->data_ptr<uint8_t>(); a.amax_w = amax_w->data_ptr<float>(); a.scale_w = scale_w->data_ptr<float>();
    if (w2f8->dim() == 3) a.w2d8 = a.w2f8 + 64 * 1600;
  }
  a.bidx = nullptr; a.bidx_n = 0;
  memset(&a.next, 0, sizeof(a.next));
  if (bidx.has_value()) {
    TORCH_CHECK(order.has_value(), "sgd: bidx needs the order descriptor");
    dev(*bidx, "bidx");
    TORCH_CHECK(bidx->scalar_type() == at::kInt && bidx->dim() == 1 && bidx->numel() >= 1 &&
                    bidx->numel() <= 4096, "bidx must be int32 [Bpad <= 4096]");
    TORCH_CHECK(!order->is_cuda() && order->scalar_type() == at::kLong && order->numel() == 6,
                "sgd: order must be the host int64 [6] descriptor");
    const int64_t* d = order->data_ptr<int64_t>();
    TORCH_CHECK(d[2] >= 1 && d[4] >= 1, "sgd: bad order descriptor");
    a.next = index_src(*order, step, d[0] / (d[2] * d[4]), bidx->numel());   // validates it
    TORCH_CHECK(a.next.idx_base == nullptr, "sgd: order must be the host descriptor");
    a.bidx = bidx->data_ptr<int>(); a.bidx_n = (int)bidx->numel();
  }
  a.xnext = nullptr; a.xdata = nullptr;
  if (xnext.has_value()) {
    TORCH_CHECK(xdata.has_value() && a.bidx, "sgd: xnext needs the dataset and bidx");
    check(*xnext, "xnext", at::kByte, {a.bidx_n, 3072});
    check_data(*xdata);
    TORCH_CHECK(a.next.n <= xdata->size(0), "sgd: the order's rows exceed the dataset");
    a.xnext = xnext->data_ptr<uint8_t>(); a.xdata = xdata->data_ptr<uint8_t>();
  }
  return a;
}

#define DMLC_SGD_PARAMS                                                                                  \
  const Tensor &master, const Tensor &grad, int64_t mode, double grad_scale, at::IntArrayRef off,          \
      const Tensor &part1, const Tensor &partb1, const Tensor &part2, const Tensor &partb2, const Tensor &w1f, \
      const Tensor &w2f, const Tensor &w2d, const Tensor &fc1n, const Tensor &fc2t, const Tensor &fc2n,     \
      const Tensor &fc3t, const Tensor &fc3d, const Tensor &step, double lr0, double decay, double decay_steps, \
      bool staircase, const Tensor &ticket, const Tensor &loss_part, const Tensor &correct_part,            \
      const Tensor &stats, const c10::optional<Tensor> &w2f8, const c10::optional<Tensor> &amax_w,          \
      const c10::optional<Tensor> &scale_w, int64_t roles, bool finalize, int64_t batch,                    \
      const c10::optional<Tensor> &bidx, const c10::optional<Tensor> &order, double warmup, bool fc1_fused,  \
      const c10::optional<Tensor> &step_rd, const c10::optional<Tensor> &xnext, const c10::optional<Tensor> &xdata
#define DMLC_SGD_ARGS                                                                                     \
  master, grad, mode, grad_scale, off, part1, partb1, part2, partb2, w1f, w2f, w2d, fc1n, fc2t, fc2n, fc3t, fc3d, \
      step, lr0, decay, decay_steps, staircase, ticket, loss_part, correct_part, stats, w2f8, amax_w, scale_w,  \
      roles, finalize, batch, bidx, order, warmup, fc1_fused, step_rd, xnext, xdata

// data parallel: the xGMI exchange of the whole flat gradient with the SGD update in its epilogue
// (xgmi_allreduce.hip); `grad` must be the xGMI context's buffer
void xgmi_allreduce_sgd(int64_t ctx, int64_t blocks, bool bf16_wire, DMLC_SGD_PARAMS) {
  TORCH_CHECK(blocks >= 0 && blocks <= DMLC_XGMI_MAX_BLOCKS, "xgmi_allreduce_sgd: blocks must be in [0,512]");
  TORCH_CHECK(mode == 2 && roles == 0 && finalize && !fc1_fused && !w2f8.has_value() && step_rd.has_value(),
              "xgmi_allreduce_sgd: apply mode (2) over every role, bf16 shadows, the head's step copy");
  DmlcSgdArgs a = make_sgd(DMLC_SGD_ARGS);
  TORCH_CHECK(!a.grad16, "xgmi_allreduce_sgd: the exchange buffer is fp32");
  c10::DeviceGuard guard(master.device());
  CHECK_HIP(dmlc_xgmi_allreduce_sgd((int)ctx, (int)blocks, bf16_wire ? 1 : 0, &a, stream_of(master)));
}

void sgd(DMLC_SGD_PARAMS) {
  DmlcSgdArgs a = make_sgd(DMLC_SGD_ARGS);
  c10::DeviceGuard guard(master.device());
  CHECK_HIP(dmlc_sgd(&a, stream_of(master)));
}

// Single GPU: the weight gradients AND the whole SGD step in one launch (cnn_wgrad.hip apply mode).
// The wgrad arguments come first (data .. xraw), then the barrier words, then sgd()'s arguments
// (whose slab tensors must be the wgrad's).
void wgrad_sgd(const Tensor& data, const Tensor& idx, const c10::optional<Tensor>& counter, int64_t period, int64_t cy,
               int64_t cx, const Tensor& dp1, const Tensor& am1, const Tensor& p1, const Tensor& dy2,
               int64_t groups2, const Tensor& xraw, const Tensor& bar, DMLC_SGD_PARAMS,
               const c10::optional<at::TensorList> fc_acts, bool fc_sgd_done, const c10::optional<at::TensorList> fp8) {
  DmlcWgradArgs a = make_wgrad(data, idx, counter, period, cy, cx, dp1, am1, part1, partb1, p1, dy2, part2, partb2,
                               groups2, xraw, fp8);
  TORCH_CHECK((mode == 0 && fc1_fused && step_rd.has_value() && roles == 0 && finalize &&
               grad_scale == 1.0) || (mode == 1 && roles == 0),
              "wgrad_sgd: the single-GPU mode-0 step (fc1 epilogue, the head's step copy) or mode 1 (reduce only)");
  check_numel(bar, "bar", at::kInt, DMLC_WBAR_WORDS);
  a.sgd = make_sgd(DMLC_SGD_ARGS);
  a.apply = 1;
  a.bar = reinterpret_cast<unsigned int*>(bar.data_ptr<int>());
  // conv1 blocks help reduce the conv2 slabs unless they also carry the fc dW tiles at B <= 128 (then
  // they arrive too late: 65.8 vs 67.2 us at B=128 without helpers, profiles/r5_wgrad_helpers_ab.txt;
  // with helpers 75.0 vs 75.7 at B=256)
  a.helpers = (a.w1.B > 128 || !fc_acts.has_value()) ? 1 : 0;
  a.fc_in_launch = 0;
  a.fc_done = fc_sgd_done ? 1 : 0;             // the fc chain applied every fc SGD: no fc roles here
  TORCH_CHECK(!fc_sgd_done || (mode == 0 && !fc_acts.has_value()), "wgrad_sgd: fc_sgd_done is the chain's mode-0 step");
  memset(&a.fc, 0, sizeof(a.fc));
  if (fc_acts.has_value()) {
    // the fc weight-gradient tiles + every fc SGD run in this launch (fc_common.h): fc_acts = the fc
    // chain's activations {p2 [B][2304], h1, h2, dl, dh1, dh2}; masters / shadows from the SGD args
    const at::TensorList t = *fc_acts;
    TORCH_CHECK(t.size() == 6 && mode == 0 && fc1_fused, "wgrad_sgd: fc_acts = {p2, h1, h2, dl, dh1, dh2} in mode 0");
    const int64_t B = t[0].size(0);
    TORCH_CHECK(B >= 16 && B <= 256 && B % 16 == 0, "wgrad_sgd: fc tiles need a batch in [16, 256]");
    check(t[0], "p2", at::kBFloat16, {B, 2304});
    check(t[1], "h1", at::kBFloat16, {B, 384});
    check(t[2], "h2", at::kBFloat16, {B, 192});
    check(t[3], "dl", at::kBFloat16, {B, 16});
    check(t[4], "dh1", at::kBFloat16, {B, 384});
    check(t[5], "dh2", at::kBFloat16, {B, 192});
    check(fc2n, "fc2n", at::kBFloat16, {384, 192});
    check(fc2t, "fc2t", at::kBFloat16, {192, 384});
    DmlcFcArgs& f = a.fc;
    f.B = (int)B; f.nvalid = (int)B; f.mtiles = (int)((B + 63) / 64);
    f.p2 = t[0].data_ptr(); f.w1 = fc1n.data_ptr();
    f.h1 = t[1].data_ptr(); f.h2 = t[2].data_ptr(); f.dl = t[3].data_ptr(); f.dh1 = t[4].data_ptr();
    f.dh2 = t[5].data_ptr();
    float* m = master.data_ptr<float>();
    f.gw1 = m + off[4]; f.mb1 = m + off[5]; f.mw2 = m + off[6]; f.mb2 = m + off[7]; f.mw3 = m + off[8];
    f.mb3 = m + off[9];
    f.fc2n = fc2n.data_ptr(); f.fc2t = fc2t.data_ptr(); f.fc3t = fc3t.data_ptr(); f.fc3d = fc3d.data_ptr();
    f.fuse_sgd = 2; f.dw_tasks = 1;
    f.lr0 = (float)lr0; f.decay = (float)decay; f.decay_steps = (float)decay_steps; f.staircase = staircase;
    f.warmup = (float)warmup; f.grad_scale = (float)grad_scale;
    f.err = a.bar + 10 * 32;
    a.fc_in_launch = 1;
  }
  c10::DeviceGuard guard(dp1.device());
  CHECK_HIP(dmlc_wgrad(&a, stream_of(dp1)));
}

}  // namespace

TORCH_LIBRARY(dmlc, m) {
  m.def("conv1_fwd(Tensor data, Tensor idx, Tensor? counter, int period, int cy, int cx, Tensor w1f, Tensor b1, "
        "Tensor(a!) out, Tensor(b!) am, Tensor(c!)? amax=None, Tensor(d!)? xraw=None) -> ()");
  m.def("conv2_fwd_fp8(Tensor inp, Tensor w8, Tensor b2, Tensor amax_x, Tensor scale_w, Tensor? counter, "
        "Tensor(a!) out, Tensor(b!) am, Tensor(c!)? x8out=None, Tensor(d!)? sx_out=None) -> ()");
  m.def("fp8_roundtrip(Tensor x, Tensor(a!) y, float scale) -> ()");
  m.def("conv2_fwd(Tensor inp, Tensor w2f, Tensor b2, Tensor(a!) out, Tensor(b!) am) -> ()");
  m.def("conv12_fwd(Tensor data, Tensor idx, Tensor? counter, int period, int cy, int cx, Tensor w1f, Tensor b1, "
        "Tensor(a!) p1, Tensor(b!) am1, Tensor w2f, Tensor b2, Tensor(c!) p2, Tensor(d!) am2, "
        "Tensor(e!)? xraw=None, bool xraw_in=False, Tensor(f!)? split_flags=None, Tensor(g!)? err=None) -> ()");
  m.def("conv2_dgrad(Tensor dp2, Tensor am2, Tensor w2d, Tensor(a!) dp1, Tensor(b!) dy2) -> ()");
  m.def("conv1_fwd_split(Tensor data, Tensor idx, Tensor? counter, int period, int cy, int cx, Tensor w1f, Tensor b1, "
        "Tensor(a!) out, Tensor(b!) am, Tensor(c!)? xraw, int nsplit) -> ()");
  m.def("conv2_fwd_split(Tensor inp, Tensor w2f, Tensor b2, Tensor(a!) out, Tensor(b!) am) -> ()");
  m.def("conv2_dgrad_split(Tensor dp2, Tensor am2, Tensor w2d, Tensor(a!) dp1, Tensor(b!) dy2) -> ()");
  m.def("conv2_dgrad_fp8(Tensor dp2, Tensor am2, Tensor w2d8, Tensor scale_w, Tensor(a!) dp1, Tensor(b!) dy2, "
        "Tensor(c!)? dy8out=None, Tensor(d!)? sy_img=None) -> ()");
  m.def("wgrad(Tensor data, Tensor idx, Tensor? counter, int period, int cy, int cx, Tensor dp1, Tensor am1, "
        "Tensor(a!) part1, Tensor(b!) partb1, Tensor p1, Tensor dy2, Tensor(c!) part2, Tensor(d!) partb2, "
        "int groups2, Tensor? xraw=None, Tensor[]? fp8=None) -> ()");
  m.def("gemm_grouped(Tensor[] A, Tensor[] B, Tensor(a!)[] C, Tensor?[] bias, int[] params, Tensor? step=None, "
        "Tensor(b!)? shadow=None, float[] sched=[]) -> ()");
  m.def("head(Tensor h1part, Tensor b1, Tensor w2t, Tensor b2, Tensor w3t, Tensor b3, Tensor w3d, Tensor w2d, "
        "Tensor labels, Tensor idx, Tensor? counter, int period, float inv_batch, bool relu_logits, bool train, "
        "Tensor(a!) h1, Tensor(b!) h2, Tensor(c!) dl, Tensor(d!) dh1, Tensor(e!) dh2, Tensor(f!) loss_part, "
        "Tensor(g!) correct_part, Tensor(h!)? logits_out, int nvalid=-1, Tensor? step=None, Tensor(i!)? step_copy=None) -> ()");
  m.def("fc_chain(Tensor p2, Tensor(a!) fc1n, Tensor(b!) h1part, Tensor b1, Tensor w2t, Tensor b2, Tensor w3t, "
        "Tensor b3, Tensor w3d, Tensor labels, Tensor idx, Tensor? counter, int period, float inv_batch, "
        "bool relu_logits, Tensor(c!) h1, Tensor(d!) h2, Tensor(e!) dl, Tensor(f!) dh1, Tensor(g!) dh2, "
        "Tensor(h!) loss_part, Tensor(i!) correct_part, Tensor(j!) dp2, Tensor(k!) gw1, Tensor(l!) gw2, "
        "Tensor(m!) gw3, Tensor(n!) gb1, Tensor(o!) gb2, Tensor(p!) gb3, bool fuse_sgd, float[] sched, "
        "int nvalid, Tensor step, Tensor(q!)? step_copy, Tensor(r!) sync, Tensor(s!) err, bool dw_tasks=True, "
        "Tensor? am2=None, Tensor? w2d=None, Tensor(t!)? dp1=None, Tensor(u!)? dy2=None, Tensor(v!)? fc2n=None) -> ()");
  m.def("wgrad_sgd(Tensor data, Tensor idx, Tensor? counter, int period, int cy, int cx, Tensor dp1, Tensor am1, "
        "Tensor p1, Tensor dy2, int groups2, Tensor xraw, Tensor(z!) bar, "
        "Tensor(a!) master, Tensor(b!) grad, int mode, float grad_scale, int[] off, Tensor(r!) part1, Tensor(s!) partb1, "
        "Tensor(t!) part2, Tensor(u!) partb2, Tensor(c!) w1f, Tensor(d!) w2f, Tensor(e!) w2d, Tensor(f!) fc1n, "
        "Tensor(g!) fc2t, Tensor(h!) fc2n, Tensor(i!) fc3t, Tensor(j!) fc3d, Tensor(k!) step, float lr0, float decay, "
        "float decay_steps, bool staircase, Tensor(l!) ticket, Tensor loss_part, Tensor correct_part, "
        "Tensor(m!) stats, Tensor(n!)? w2f8, Tensor(o!)? amax_w, Tensor(p!)? scale_w, int roles, "
        "bool finalize, int batch, Tensor(q!)? bidx=None, Tensor? order=None, float warmup=0.0, "
        "bool fc1_fused=False, Tensor? step_rd=None, Tensor(v!)? xnext=None, Tensor? xdata=None, "
        "Tensor[]? fc_acts=None, bool fc_sgd_done=False, Tensor[]? fp8=None) -> ()");
  m.def("sgd(Tensor(a!) master, Tensor(b!) grad, int mode, float grad_scale, int[] off, Tensor part1, Tensor partb1, "
        "Tensor part2, Tensor partb2, Tensor(c!) w1f, Tensor(d!) w2f, Tensor(e!) w2d, Tensor(f!) fc1n, "
        "Tensor(g!) fc2t, Tensor(h!) fc2n, Tensor(i!) fc3t, Tensor(j!) fc3d, Tensor(k!) step, float lr0, float decay, "
        "float decay_steps, bool staircase, Tensor(l!) ticket, Tensor loss_part, Tensor correct_part, "
        "Tensor(m!) stats, Tensor(n!)? w2f8, Tensor(o!)? amax_w, Tensor(p!)? scale_w, int roles, "
        "bool finalize, int batch, Tensor(q!)? bidx=None, Tensor? order=None, float warmup=0.0, "
        "bool fc1_fused=False, Tensor? step_rd=None, Tensor(v!)? xnext=None, Tensor? xdata=None) -> ()");
  m.def("xgmi_allreduce_sgd(int ctx, int blocks, bool bf16_wire, Tensor(a!) master, Tensor(b!) grad, int mode, "
        "float grad_scale, int[] off, Tensor part1, Tensor partb1, "
        "Tensor part2, Tensor partb2, Tensor(c!) w1f, Tensor(d!) w2f, Tensor(e!) w2d, Tensor(f!) fc1n, "
        "Tensor(g!) fc2t, Tensor(h!) fc2n, Tensor(i!) fc3t, Tensor(j!) fc3d, Tensor(k!) step, float lr0, float decay, "
        "float decay_steps, bool staircase, Tensor(l!) ticket, Tensor loss_part, Tensor correct_part, "
        "Tensor(m!) stats, Tensor(n!)? w2f8, Tensor(o!)? amax_w, Tensor(p!)? scale_w, int roles, "
        "bool finalize, int batch, Tensor(q!)? bidx=None, Tensor? order=None, float warmup=0.0, "
        "bool fc1_fused=False, Tensor? step_rd=None, Tensor(v!)? xnext=None, Tensor? xdata=None) -> ()");
}

TORCH_LIBRARY_IMPL(dmlc, CUDA, m) {
  m.impl("conv1_fwd", &conv1_fwd);
  m.impl("conv2_fwd", &conv2_fwd);
  m.impl("conv12_fwd", &conv12_fwd);
  m.impl("conv2_fwd_fp8", &conv2_fwd_fp8);
  m.impl("fp8_roundtrip", &fp8_roundtrip);
  m.impl("conv2_dgrad", &conv2_dgrad);
  m.impl("conv1_fwd_split", &conv1_fwd_split);
  m.impl("conv2_fwd_split", &conv2_fwd_split);
  m.impl("conv2_dgrad_split", &conv2_dgrad_split);
  m.impl("conv2_dgrad_fp8", &conv2_dgrad_fp8);
  m.impl("wgrad", &wgrad);
  m.impl("gemm_grouped", &gemm_grouped);
  m.impl("head", &head);
  m.impl("fc_chain", &fc_chain);
  m.impl("sgd", &sgd);
  m.impl("xgmi_allreduce_sgd", &xgmi_allreduce_sgd);
  m.impl("wgrad_sgd", &wgrad_sgd);
}
