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

inline DmlcIndexSrc index_src(const Tensor& idx, const c10::optional<Tensor>& counter, int64_t period, int64_t B) {
  TORCH_CHECK(period >= 1, "period must be >= 1");
  check_numel(idx, "idx", at::kInt, period * B);
  DmlcIndexSrc s;
  s.idx_base = idx.data_ptr<int>();
  s.counter = nullptr;
  if (counter.has_value()) {
    check_numel(*counter, "counter", at::kLong, 1);
    s.counter = counter->data_ptr<int64_t>();
  }
  s.period = (int)period;
  return s;
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
