// torch.ops.dmlc.rn_* bindings of the fused ResNet-20 kernels (csrc/kernels/resnet.hip).
//
// Same contract as torch_ops.cpp: every launch is preceded by a full check of device, dtype,
// contiguity and the exact shapes implied by the layer geometry (one of the six ResNet-20 conv
// shapes), so a mis-wired engine raises instead of faulting the GPU.
#include <c10/core/DeviceGuard.h>

#include "../kernels/api_resnet.h"
#include "check.h"

namespace {

using namespace dmlc_bind;

struct Geom {
  int64_t cin, cout, hin, stride;
  int64_t cinp() const { return cin < 8 ? 8 : cin; }
  int64_t hout() const { return hin / stride; }
  int64_t kp() const { return (9 * cinp() + 31) / 32 * 32; }
  int64_t kpd() const { return (9 * cout + 31) / 32 * 32; }
  DmlcRnLayerGeom c() const { return DmlcRnLayerGeom{(int)cin, (int)cout, (int)hin, (int)stride}; }
};

Geom geom(int64_t cin, int64_t cout, int64_t hin, int64_t stride) {
  static const int64_t ok[6][4] = {{3, 16, 32, 1}, {16, 16, 32, 1}, {16, 32, 32, 2},
                                   {32, 32, 16, 1}, {32, 64, 16, 2}, {64, 64, 8, 1}};
  for (const auto& g : ok)
    if (g[0] == cin && g[1] == cout && g[2] == hin && g[3] == stride) return Geom{cin, cout, hin, stride};
  TORCH_CHECK(false, "rn: unsupported conv geometry cin=", cin, " cout=", cout, " hin=", hin, " stride=", stride);
}

// per-layer statistics accumulators: fixed-point int64 [NSLOT][256] (integer parts of sum / sum of
// squares or R1 / R2 at [0, 128), their 48-bit fractions at [128, 256); resnet.hip fx_add)
void check_stat(const Tensor& t, const char* n) { check_numel(t, n, at::kLong, DMLC_RN_NSLOT * 256); }
#define STAT_PTR(t) reinterpret_cast<long long*>((t).data_ptr<int64_t>())

// nvalid: the first nvalid images are real, the rest batch padding (0: all B); every BatchNorm mean is
// over the real images only
int64_t valid_count(int64_t nvalid, int64_t B) {
  const int64_t nv = nvalid > 0 ? nvalid : B;
  TORCH_CHECK(nv >= 1 && nv <= B, "nvalid must be in [1, B]");
  return nv;
}

void rn_fwd(int64_t cin, int64_t cout, int64_t hin, int64_t stride, const c10::optional<Tensor>& data,
            const c10::optional<Tensor>& idx, const c10::optional<Tensor>& counter, int64_t period, int64_t cy,
            int64_t cx, const c10::optional<Tensor>& z_prev, const c10::optional<Tensor>& stat_prev,
            const c10::optional<Tensor>& gamma_prev, const c10::optional<Tensor>& beta_prev,
            const c10::optional<Tensor>& sc_src, int64_t sc_mode, const c10::optional<Tensor>& a_out, const Tensor& w,
            const Tensor& z, const Tensor& stat, int64_t nvalid) {
  const Geom g = geom(cin, cout, hin, stride);
  const int64_t B = z.size(0), nv = valid_count(nvalid, B);
  check(w, "w", at::kBFloat16, {g.cout, g.kp()});
  check(z, "z", at::kBFloat16, {B, g.hout(), g.hout(), g.cout});
  check_stat(stat, "stat");
  DmlcRnFwdArgs a{};
  a.B = (int)B;
  a.nvalid = (int)nv;
  if (cin == 3) {
    TORCH_CHECK(data.has_value() && idx.has_value(), "rn_fwd stem needs data and idx");
    check_data(*data);
    TORCH_CHECK(cy == 0 && cx == 0, "the ResNet stem consumes full 32x32 images (crop offsets 0)");
    a.data = data->data_ptr<uint8_t>();
    a.src = index_src(*idx, counter, period, B);
    check_order_fits(a.src, data->size(0));
  } else {
    TORCH_CHECK(z_prev && stat_prev && gamma_prev && beta_prev && a_out, "rn_fwd needs the previous layer's tensors");
    check(*z_prev, "z_prev", at::kBFloat16, {B, hin, hin, cin});
    check_stat(*stat_prev, "stat_prev");
    check_numel(*gamma_prev, "gamma_prev", at::kFloat, cin);
    check_numel(*beta_prev, "beta_prev", at::kFloat, cin);
    check(*a_out, "a_out", at::kBFloat16, {B, hin, hin, cin});
    TORCH_CHECK(sc_mode >= 0 && sc_mode <= 2, "sc_mode must be 0..2");
    if (sc_mode == 1) {
      TORCH_CHECK(sc_src.has_value(), "sc_mode 1 needs sc_src");
      check(*sc_src, "sc_src", at::kBFloat16, {B, hin, hin, cin});
    } else if (sc_mode == 2) {
      TORCH_CHECK(sc_src.has_value(), "sc_mode 2 needs sc_src");
      check(*sc_src, "sc_src", at::kBFloat16, {B, 2 * hin, 2 * hin, cin / 2});
    }
    a.z_prev = z_prev->data_ptr(); a.stat_prev = STAT_PTR(*stat_prev);
    a.gamma_prev = gamma_prev->data_ptr<float>(); a.beta_prev = beta_prev->data_ptr<float>();
    a.sc_src = sc_mode ? sc_src->data_ptr() : nullptr; a.sc_mode = (int)sc_mode;
    a.a_out = a_out->data_ptr(); a.inv_n_prev = 1.f / (float)(nv * hin * hin);
  }
  a.w = w.data_ptr(); a.z = z.data_ptr(); a.stat = STAT_PTR(stat);
  c10::DeviceGuard guard(z.device());
  const DmlcRnLayerGeom gc = g.c();
  CHECK_HIP(dmlc_rn_fwd(&gc, &a, stream_of(z)));
}

DmlcRnDgradArgs dgrad_args(const Geom& g, int64_t cin, int64_t cout, int64_t hin, const Tensor& gy, const Tensor& z,
                           const Tensor& stat, const Tensor& red, const Tensor& gamma, const Tensor& wd,
                           const Tensor& a_prev, const Tensor& z_prev, const Tensor& stat_prev,
                           const c10::optional<Tensor>& gy_sc, int64_t sc_mode, const Tensor& gy_prev,
                           const Tensor& red_prev, int64_t nvalid) {
  TORCH_CHECK(cin >= 16, "rn_dgrad: the stem has no input gradient");
  const int64_t B = gy.size(0), ho = g.hout(), nv = valid_count(nvalid, B);
  check(gy, "gy", at::kBFloat16, {B, ho, ho, cout});
  check(z, "z", at::kBFloat16, {B, ho, ho, cout});
  check_stat(stat, "stat"); check_stat(red, "red"); check_stat(stat_prev, "stat_prev"); check_stat(red_prev, "red_prev");
  check_numel(gamma, "gamma", at::kFloat, cout);
  check(wd, "wd", at::kBFloat16, {cin, g.kpd()});
  check(a_prev, "a_prev", at::kBFloat16, {B, hin, hin, cin});
  check(z_prev, "z_prev", at::kBFloat16, {B, hin, hin, cin});
  check(gy_prev, "gy_prev", at::kBFloat16, {B, hin, hin, cin});
  TORCH_CHECK(sc_mode >= 0 && sc_mode <= 2, "sc_mode must be 0..2");
  if (sc_mode == 1) {
    TORCH_CHECK(gy_sc.has_value(), "sc_mode 1 needs gy_sc");
    check(*gy_sc, "gy_sc", at::kBFloat16, {B, hin, hin, cin});
  } else if (sc_mode == 2) {
    TORCH_CHECK(gy_sc.has_value(), "sc_mode 2 needs gy_sc");
    check(*gy_sc, "gy_sc", at::kBFloat16, {B, hin / 2, hin / 2, 2 * cin});
  }
  DmlcRnDgradArgs a{};
  a.gy = gy.data_ptr(); a.z = z.data_ptr(); a.stat = STAT_PTR(stat); a.red = STAT_PTR(red);
  a.gamma = gamma.data_ptr<float>(); a.inv_n = 1.f / (float)(nv * ho * ho);
  a.wd = wd.data_ptr();
  a.a_prev = a_prev.data_ptr(); a.z_prev = z_prev.data_ptr(); a.stat_prev = STAT_PTR(stat_prev);
  a.inv_n_prev = 1.f / (float)(nv * hin * hin);
  a.nvalid = (int)nv;
  a.gy_sc = sc_mode ? gy_sc->data_ptr() : nullptr; a.sc_mode = (int)sc_mode;
  a.gy_prev = gy_prev.data_ptr(); a.red_prev = STAT_PTR(red_prev); a.B = (int)B;
  return a;
}

void rn_dgrad(int64_t cin, int64_t cout, int64_t hin, int64_t stride, const Tensor& gy, const Tensor& z,
              const Tensor& stat, const Tensor& red, const Tensor& gamma, const Tensor& wd, const Tensor& a_prev,
              const Tensor& z_prev, const Tensor& stat_prev, const c10::optional<Tensor>& gy_sc, int64_t sc_mode,
              const Tensor& gy_prev, const Tensor& red_prev, int64_t nvalid) {
  const Geom g = geom(cin, cout, hin, stride);
  const DmlcRnDgradArgs a = dgrad_args(g, cin, cout, hin, gy, z, stat, red, gamma, wd, a_prev, z_prev, stat_prev,
                                       gy_sc, sc_mode, gy_prev, red_prev, nvalid);
  c10::DeviceGuard guard(gy.device());
  const DmlcRnLayerGeom gc = g.c();
  CHECK_HIP(dmlc_rn_dgrad(&gc, &a, stream_of(gy)));
}

DmlcRnWgradArgs wgrad_args(const Geom& g, int64_t cin, int64_t cout, int64_t hin,
                           const c10::optional<Tensor>& data, const c10::optional<Tensor>& idx,
                           const c10::optional<Tensor>& counter, int64_t period, int64_t cy, int64_t cx,
                           const c10::optional<Tensor>& x, const Tensor& gy, const Tensor& z, const Tensor& stat,
                           const Tensor& red, const Tensor& gamma, const Tensor& part, int64_t nvalid) {
  const int64_t B = gy.size(0), ho = g.hout(), G = part.size(0), nv = valid_count(nvalid, B);
  check(gy, "gy", at::kBFloat16, {B, ho, ho, cout});
  check(z, "z", at::kBFloat16, {B, ho, ho, cout});
  check_stat(stat, "stat"); check_stat(red, "red");
  check_numel(gamma, "gamma", at::kFloat, cout);
  check(part, "part", at::kFloat, {G, g.kp(), cout});
  TORCH_CHECK(G >= 1 && G <= B, "rn_wgrad: 1 <= groups <= batch");
  DmlcRnWgradArgs a{};
  if (cin == 3) {
    TORCH_CHECK(data.has_value() && idx.has_value(), "rn_wgrad stem needs data and idx");
    check_data(*data);
    TORCH_CHECK(cy == 0 && cx == 0, "the ResNet stem consumes full 32x32 images (crop offsets 0)");
    a.data = data->data_ptr<uint8_t>();
    a.src = index_src(*idx, counter, period, B);
    check_order_fits(a.src, data->size(0));
  } else {
    TORCH_CHECK(x.has_value(), "rn_wgrad needs x");
    check(*x, "x", at::kBFloat16, {B, hin, hin, cin});
    a.x = x->data_ptr();
  }
  a.gy = gy.data_ptr(); a.z = z.data_ptr(); a.stat = STAT_PTR(stat); a.red = STAT_PTR(red);
  a.gamma = gamma.data_ptr<float>(); a.inv_n = 1.f / (float)(nv * ho * ho);
  a.part = part.data_ptr<float>(); a.G = (int)G; a.B = (int)B; a.nvalid = (int)nv;
  return a;
}

void rn_wgrad(int64_t cin, int64_t cout, int64_t hin, int64_t stride, const c10::optional<Tensor>& data,
              const c10::optional<Tensor>& idx, const c10::optional<Tensor>& counter, int64_t period, int64_t cy,
              int64_t cx, const c10::optional<Tensor>& x, const Tensor& gy, const Tensor& z, const Tensor& stat,
              const Tensor& red, const Tensor& gamma, const Tensor& part, int64_t nvalid) {
  const Geom g = geom(cin, cout, hin, stride);
  const DmlcRnWgradArgs a = wgrad_args(g, cin, cout, hin, data, idx, counter, period, cy, cx, x, gy, z, stat, red,
                                       gamma, part, nvalid);
  c10::DeviceGuard guard(gy.device());
  const DmlcRnLayerGeom gc = g.c();
  CHECK_HIP(dmlc_rn_wgrad(&gc, &a, stream_of(gy)));
}

// dgrad + wgrad of one (non-stem) layer in one launch; the wgrad's input is the dgrad's a_prev
void rn_bwd(int64_t cin, int64_t cout, int64_t hin, int64_t stride, const Tensor& gy, const Tensor& z,
            const Tensor& stat, const Tensor& red, const Tensor& gamma, const Tensor& wd, const Tensor& a_prev,
            const Tensor& z_prev, const Tensor& stat_prev, const c10::optional<Tensor>& gy_sc, int64_t sc_mode,
            const Tensor& gy_prev, const Tensor& red_prev, const Tensor& part, int64_t nvalid,
            bool per_image) {
  const Geom g = geom(cin, cout, hin, stride);
  const DmlcRnDgradArgs d = dgrad_args(g, cin, cout, hin, gy, z, stat, red, gamma, wd, a_prev, z_prev, stat_prev,
                                       gy_sc, sc_mode, gy_prev, red_prev, nvalid);
  const DmlcRnWgradArgs w = wgrad_args(g, cin, cout, hin, c10::nullopt, c10::nullopt, c10::nullopt, 1, 0, 0, a_prev, gy,
                                       z, stat, red, gamma, part, nvalid);
  TORCH_CHECK(!per_image || (((cin == 16 && hin == 32) || (cin == 32 && hin == 16)) && cout == cin && stride == 1 &&
                              w.G == w.B),
              "rn_bwd per_image: 16->16 / 32->32 stride-1 layers with one split-K group per image only");
  c10::DeviceGuard guard(gy.device());
  DmlcRnLayerGeom gc = g.c();
  gc.per_image = per_image ? 1 : 0;
  CHECK_HIP(dmlc_rn_bwd(&gc, &d, &w, stream_of(gy)));
}

void rn_head(const Tensor& z, const Tensor& stat, const Tensor& gamma, const Tensor& beta, const Tensor& sc,
             const Tensor& fcw, const Tensor& fcb, const Tensor& labels, const Tensor& idx,
             const c10::optional<Tensor>& counter, int64_t period, double inv_batch, const Tensor& gy,
             const Tensor& red, const Tensor& fc_part, const Tensor& loss_img, const Tensor& correct_img,
             const c10::optional<Tensor>& logits, int64_t nvalid,
             const c10::optional<Tensor>& step, const c10::optional<Tensor>& step_copy) {
  const int64_t B = z.size(0), nv = valid_count(nvalid, B);
  check(z, "z", at::kBFloat16, {B, 8, 8, 64});
  check_stat(stat, "stat"); check_stat(red, "red");
  check_numel(gamma, "gamma", at::kFloat, 64);
  check_numel(beta, "beta", at::kFloat, 64);
  check(sc, "sc", at::kBFloat16, {B, 8, 8, 64});
  check_numel(fcw, "fcw", at::kFloat, 640);
  check_numel(fcb, "fcb", at::kFloat, 10);
  dev(labels, "labels");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.numel() >= 1, "labels must be int32");
  check(gy, "gy", at::kBFloat16, {B, 8, 8, 64});
  check(fc_part, "fc_part", at::kFloat, {B, 656});
  check_numel(loss_img, "loss_img", at::kFloat, B);
  check_numel(correct_img, "correct_img", at::kInt, B);
  DmlcRnHeadArgs a{};
  a.z = z.data_ptr(); a.stat = STAT_PTR(stat); a.gamma = gamma.data_ptr<float>();
  a.beta = beta.data_ptr<float>(); a.inv_n = 1.f / (float)(nv * 64);
  a.sc = sc.data_ptr(); a.fcw = fcw.data_ptr<float>(); a.fcb = fcb.data_ptr<float>();
  a.labels = labels.data_ptr<int>(); a.src = index_src(idx, counter, period, B);
  check_order_fits(a.src, labels.size(0));
  a.inv_batch = (float)inv_batch;
  a.gy = gy.data_ptr(); a.red = STAT_PTR(red); a.fc_part = fc_part.data_ptr<float>();
  a.loss_img = loss_img.data_ptr<float>(); a.correct_img = correct_img.data_ptr<int>();
  a.logits_out = nullptr;
  if (logits.has_value()) {
    check(*logits, "logits", at::kFloat, {B, 10});
    a.logits_out = logits->data_ptr<float>();
  }
  a.B = (int)B;
  a.nvalid = (int)nv;
  TORCH_CHECK(step.has_value() == step_copy.has_value(), "rn_head: step and step_copy go together");
  if (step.has_value()) {
    check_numel(*step, "step", at::kLong, 1);
    check_numel(*step_copy, "step_copy", at::kLong, 1);
    a.step = step->data_ptr<int64_t>(); a.step_copy = step_copy->data_ptr<int64_t>();
  }
  c10::DeviceGuard guard(z.device());
  CHECK_HIP(dmlc_rn_head(&a, stream_of(z)));
}

// layer table of ResNet-20 (cin, cout, hin, stride) in execution order
const int64_t kLayers[DMLC_RN_LAYERS][4] = {
    {3, 16, 32, 1},  {16, 16, 32, 1}, {16, 16, 32, 1}, {16, 16, 32, 1}, {16, 16, 32, 1}, {16, 16, 32, 1},
    {16, 16, 32, 1}, {16, 32, 32, 2}, {32, 32, 16, 1}, {32, 32, 16, 1}, {32, 32, 16, 1}, {32, 32, 16, 1},
    {32, 32, 16, 1}, {32, 64, 16, 2}, {64, 64, 8, 1},  {64, 64, 8, 1},  {64, 64, 8, 1},  {64, 64, 8, 1},
    {64, 64, 8, 1}};

void rn_sgd(const Tensor& master, const c10::optional<Tensor>& grad, double grad_scale, const Tensor& state,
            at::IntArrayRef conv_off, at::IntArrayRef gamma_off, at::IntArrayRef beta_off, at::IntArrayRef mm_off,
            at::IntArrayRef mv_off, int64_t fcw_off, int64_t fcb_off, at::TensorList part, at::TensorList wf,
            at::TensorList wd, const Tensor& stat, const Tensor& red, const Tensor& fc_part, const Tensor& loss_img,
            const Tensor& correct_img, const Tensor& step, const Tensor& ticket, const Tensor& stats, int64_t mode,
            double lr0, double decay, double decay_steps, bool staircase, double bn_momentum, double warmup,
            int64_t layer_lo, int64_t layer_hi, bool tail, int64_t nvalid, const c10::optional<Tensor>& step_rd) {
  constexpr int L = DMLC_RN_LAYERS;
  TORCH_CHECK(layer_lo >= 0 && layer_lo <= layer_hi && layer_hi <= L, "rn_sgd: bad layer range");
  TORCH_CHECK(tail || mode == 0, "rn_sgd: a partial (tail=False) launch is mode 0 only");
  TORCH_CHECK(mode >= 0 && mode <= 3, "rn_sgd mode must be 0..3");
  TORCH_CHECK(conv_off.size() == L && gamma_off.size() == L && beta_off.size() == L && mm_off.size() == L &&
                  mv_off.size() == L, "rn_sgd: 19 offsets per table");
  TORCH_CHECK(part.size() == L && wf.size() == L && wd.size() == L, "rn_sgd: 19 slabs / shadows");
  const int64_t B = loss_img.numel(), nv = valid_count(nvalid, B);
  dev(master, "master"); dev(state, "state");
  TORCH_CHECK(master.scalar_type() == at::kFloat && state.scalar_type() == at::kFloat, "master/state must be fp32");
  const int64_t np = master.numel(), ns = state.numel();
  check(stat, "stat", at::kLong, {L, DMLC_RN_NSLOT, 256});
  check(red, "red", at::kLong, {L, DMLC_RN_NSLOT, 256});
  check(fc_part, "fc_part", at::kFloat, {B, 656});
  check_numel(correct_img, "correct_img", at::kInt, B);
  check_numel(loss_img, "loss_img", at::kFloat, B);
  check_numel(step, "step", at::kLong, 1);
  check_numel(ticket, "ticket", at::kInt, DMLC_TICKET_WORDS);
  dev(stats, "stats");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.dim() == 2 && stats.size(1) == 4, "stats must be [R,4] fp32");
  TORCH_CHECK(fcw_off >= 0 && fcw_off % 4 == 0 && fcw_off + 640 <= np && fcb_off >= 0 && fcb_off + 10 <= np,
              "bad fc offsets");
  if (mode == 1 || mode == 2) {
    TORCH_CHECK(grad.has_value(), "rn_sgd modes 1/2 need grad");
    check_numel(*grad, "grad", at::kFloat, np);
  }
  DmlcRnSgdArgs a{};
  a.master = master.data_ptr<float>(); a.nparams = (int)np;
  a.grad = grad.has_value() ? grad->data_ptr<float>() : nullptr; a.grad_scale = (float)grad_scale;
  for (int l = 0; l < L; ++l) {
    const Geom g = geom(kLayers[l][0], kLayers[l][1], kLayers[l][2], kLayers[l][3]);
    TORCH_CHECK(conv_off[l] >= 0 && conv_off[l] % 4 == 0 && conv_off[l] + 9 * g.cin * g.cout <= np, "bad conv offset ", l);
    TORCH_CHECK(gamma_off[l] >= 0 && gamma_off[l] + g.cout <= np && beta_off[l] >= 0 && beta_off[l] + g.cout <= np,
                "bad BN offset ", l);
    TORCH_CHECK(mm_off[l] >= 0 && mm_off[l] + g.cout <= ns && mv_off[l] >= 0 && mv_off[l] + g.cout <= ns,
                "bad BN state offset ", l);
    const int64_t G = part[l].size(0);
    check(part[l], "part", at::kFloat, {G, g.kp(), g.cout});
    check(wf[l], "wf", at::kBFloat16, {g.cout, g.kp()});
    a.conv_off[l] = (int)conv_off[l]; a.gamma_off[l] = (int)gamma_off[l]; a.beta_off[l] = (int)beta_off[l];
    a.mm_off[l] = (int)mm_off[l]; a.mv_off[l] = (int)mv_off[l];
    a.cin[l] = (int)g.cin; a.cout[l] = (int)g.cout;
    a.part[l] = part[l].data_ptr<float>(); a.G[l] = (int)G;
    a.wf[l] = wf[l].data_ptr();
    a.wd[l] = nullptr;
    if (l > 0) {
      check(wd[l], "wd", at::kBFloat16, {g.cin, g.kpd()});
      a.wd[l] = wd[l].data_ptr();
    }
    a.inv_n[l] = 1.f / (float)(nv * g.hout() * g.hout());
  }
  a.stat = STAT_PTR(stat); a.red = STAT_PTR(red);
  a.state = state.data_ptr<float>(); a.bn_momentum = (float)bn_momentum;
  a.fcw_off = (int)fcw_off; a.fcb_off = (int)fcb_off; a.fc_part = fc_part.data_ptr<float>(); a.B = (int)B;
  a.mode = (int)mode;
  a.layer_lo = (int)layer_lo; a.layer_hi = (int)layer_hi; a.tail = tail ? 1 : 0;
  a.step = step.data_ptr<int64_t>();
  a.step_rd = a.step;
  if (step_rd.has_value()) {
    check_numel(*step_rd, "step_rd", at::kLong, 1);
    a.step_rd = step_rd->data_ptr<int64_t>();
  }
  a.lr0 = (float)lr0; a.decay = (float)decay; a.decay_steps = (float)decay_steps;
  a.staircase = staircase ? 1 : 0;
  a.warmup = (float)warmup;
  a.ticket = reinterpret_cast<unsigned int*>(ticket.data_ptr<int>());
  a.loss_img = loss_img.data_ptr<float>(); a.correct_img = correct_img.data_ptr<int>();
  a.stats = stats.data_ptr<float>(); a.stats_len = (int)stats.size(0);
  a.nvalid = (int)nv;
  c10::DeviceGuard guard(master.device());
  CHECK_HIP(dmlc_rn_sgd(&a, stream_of(master)));
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(dmlc, m) {
  m.def("rn_fwd(int cin, int cout, int hin, int stride, Tensor? data, Tensor? idx, Tensor? counter, int period, "
        "int cy, int cx, Tensor? z_prev, Tensor? stat_prev, Tensor? gamma_prev, Tensor? beta_prev, Tensor? sc_src, "
        "int sc_mode, Tensor(a!)? a_out, Tensor w, Tensor(b!) z, Tensor(c!) stat, "
        "int nvalid=0) -> ()");
  m.def("rn_dgrad(int cin, int cout, int hin, int stride, Tensor gy, Tensor z, Tensor stat, Tensor red, "
        "Tensor gamma, Tensor wd, Tensor a_prev, Tensor z_prev, Tensor stat_prev, Tensor? gy_sc, int sc_mode, "
        "Tensor(a!) gy_prev, Tensor(b!) red_prev, int nvalid=0) -> ()");
  m.def("rn_wgrad(int cin, int cout, int hin, int stride, Tensor? data, Tensor? idx, Tensor? counter, int period, "
        "int cy, int cx, Tensor? x, Tensor gy, Tensor z, Tensor stat, Tensor red, Tensor gamma, "
        "Tensor(a!) part, int nvalid=0) -> ()");
  m.def("rn_bwd(int cin, int cout, int hin, int stride, Tensor gy, Tensor z, Tensor stat, Tensor red, "
        "Tensor gamma, Tensor wd, Tensor a_prev, Tensor z_prev, Tensor stat_prev, Tensor? gy_sc, int sc_mode, "
        "Tensor(a!) gy_prev, Tensor(b!) red_prev, Tensor(c!) part, int nvalid=0, "
        "bool per_image=False) -> ()");
  m.def("rn_head(Tensor z, Tensor stat, Tensor gamma, Tensor beta, Tensor sc, Tensor fcw, Tensor fcb, "
        "Tensor labels, Tensor idx, Tensor? counter, int period, float inv_batch, Tensor(a!) gy, Tensor(b!) red, "
        "Tensor(c!) fc_part, Tensor(d!) loss_img, Tensor(e!) correct_img, Tensor(f!)? logits, "
        "int nvalid=0, Tensor? step=None, Tensor(h!)? step_copy=None) -> ()");
  m.def("rn_sgd(Tensor(a!) master, Tensor(b!)? grad, float grad_scale, Tensor(c!) state, int[] conv_off, "
        "int[] gamma_off, int[] beta_off, int[] mm_off, int[] mv_off, int fcw_off, int fcb_off, Tensor[] part, "
        "Tensor(d!)[] wf, Tensor(e!)[] wd, Tensor stat, Tensor red, Tensor fc_part, Tensor loss_img, "
        "Tensor correct_img, Tensor(f!) step, Tensor(g!) ticket, Tensor(h!) stats, int mode, float lr0, "
        "float decay, float decay_steps, bool staircase, float bn_momentum, float warmup=0.0, int layer_lo=0, "
        "int layer_hi=19, bool tail=True, int nvalid=0, Tensor? step_rd=None) -> ()");
}

TORCH_LIBRARY_IMPL(dmlc, CUDA, m) {
  m.impl("rn_fwd", &rn_fwd);
  m.impl("rn_dgrad", &rn_dgrad);
  m.impl("rn_wgrad", &rn_wgrad);
  m.impl("rn_bwd", &rn_bwd);
  m.impl("rn_head", &rn_head);
  m.impl("rn_sgd", &rn_sgd);
}
