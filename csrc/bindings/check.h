// Shared argument validation of the torch.ops.dmlc.* bindings (torch_ops.cpp, torch_ops_resnet.cpp).
#pragma once
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <vector>

#include "../kernels/api.h"

namespace dmlc_bind {

using at::Tensor;

#define CHECK_HIP(expr)                                                                       \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    TORCH_CHECK(_e == hipSuccess, "dmlc HIP launch failed: ", hipGetErrorString(_e));         \
  } while (0)

inline void dev(const Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda(), n, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), n, " must be contiguous");
}
inline void check(const Tensor& t, const char* n, at::ScalarType st, std::vector<int64_t> shape) {
  dev(t, n);
  TORCH_CHECK(t.scalar_type() == st, n, " has dtype ", t.scalar_type(), ", expected ", st);
  TORCH_CHECK(t.sizes().vec() == shape, n, " has shape ", t.sizes(), ", expected ", at::IntArrayRef(shape));
}
inline void check_numel(const Tensor& t, const char* n, at::ScalarType st, int64_t numel) {
  dev(t, n);
  TORCH_CHECK(t.scalar_type() == st, n, " has dtype ", t.scalar_type(), ", expected ", st);
  TORCH_CHECK(t.numel() == numel, n, " has ", t.numel(), " elements, expected ", numel);
}
inline void check_min(const Tensor& t, const char* n, at::ScalarType st, int64_t numel) {
  dev(t, n);
  TORCH_CHECK(t.scalar_type() == st, n, " has dtype ", t.scalar_type(), ", expected ", st);
  TORCH_CHECK(t.numel() >= numel, n, " has ", t.numel(), " elements, need at least ", numel);
}

// `idx` is either a device int32 index list [period * B] or, for the generated training order, a
// HOST int64 descriptor [n, half_bits, world, rank, bvalid, seed] (dmlc/data/order.py
// OrderSpec.descriptor(); read here at launch/capture time, so no device sync) -- see api.h.
inline DmlcIndexSrc index_src(const Tensor& idx, const c10::optional<Tensor>& counter, int64_t period, int64_t B) {
  TORCH_CHECK(period >= 1, "period must be >= 1");
  DmlcIndexSrc s;
  memset(&s, 0, sizeof(s));
  s.counter = nullptr;
  if (counter.has_value()) {
    check_numel(*counter, "counter", at::kLong, 1);
    s.counter = counter->data_ptr<int64_t>();
  }
  s.period = (int)period;
  if (!idx.is_cuda()) {
    TORCH_CHECK(idx.scalar_type() == at::kLong && idx.numel() == 6 && idx.is_contiguous(),
                "a host idx must be the int64 [6] order descriptor");
    TORCH_CHECK(s.counter != nullptr, "the generated order needs the device step counter");
    const int64_t* d = idx.data_ptr<int64_t>();
    const int64_t n = d[0], hb = d[1], world = d[2], rank = d[3], bvalid = d[4], seed = d[5];
    TORCH_CHECK(n >= 1 && n < (1ll << 30), "order: dataset size out of range");
    TORCH_CHECK(hb >= 1 && hb <= 15 && (1ll << (2 * hb)) >= n && (1ll << (2 * (hb - 1))) < std::max<int64_t>(n, 2),
                "order: half_bits must be the smallest h with 4^h >= n");
    TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "order: bad rank/world");
    TORCH_CHECK(bvalid >= 1 && bvalid <= B, "order: bvalid must be in [1, B]");
    TORCH_CHECK(period == n / (world * bvalid), "order: period must be n / (world * bvalid) steps per epoch");
    TORCH_CHECK(seed >= 0 && seed <= 0xffffffffll, "order: seed must be a uint32");
    s.idx_base = nullptr;
    s.n = (int)n; s.half_bits = (int)hb; s.world = (int)world; s.rank = (int)rank; s.bvalid = (int)bvalid;
    s.seed = (uint32_t)seed;
    return s;
  }
  check_numel(idx, "idx", at::kInt, period * B);
  s.idx_base = idx.data_ptr<int>();
  s.bvalid = (int)B;
  return s;
}

// generated order: every index it yields is < n, which must address rows of the dataset
inline void check_order_fits(const DmlcIndexSrc& s, int64_t rows) {
  TORCH_CHECK(s.idx_base != nullptr || s.n <= rows, "order: dataset size ", s.n, " exceeds the ", rows, " rows given");
}

inline hipStream_t stream_of(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

inline void check_data(const Tensor& data) {
  dev(data, "data");
  TORCH_CHECK(data.scalar_type() == at::kByte && data.dim() == 4 && data.size(1) == 32 && data.size(2) == 32 &&
                  data.size(3) == 3,
              "data must be uint8 [N,32,32,3], got ", data.sizes());
}

}  // namespace dmlc_bind
