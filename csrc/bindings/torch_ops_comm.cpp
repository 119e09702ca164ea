// torch.ops.dmlc.xgmi_* — bindings of the xGMI peer-to-peer all-reduce (csrc/kernels/xgmi_allreduce.hip).
//
// Life cycle (driven by dmlc/parallel/xgmi.py):
//   ctx = xgmi_create(rank, world, numel)     device buffer + signal block on the current GPU
//   h   = xgmi_handles(ctx)                   uint8[192] IPC handles, exchanged over the process group
//   xgmi_open(ctx, all_h)                     map every peer's buffer + signals (hipIpcOpenMemHandle)
//   buf = xgmi_buffer(ctx)                    fp32 [numel] tensor view of this rank's buffer
//   xgmi_allreduce(ctx, buf, offset, numel, blocks, bf16_wire)   in place, on the current stream (capturable)
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>

#include "../kernels/api_comm.h"
#include "check.h"

namespace {

using namespace dmlc_bind;

int64_t xgmi_create(int64_t rank, int64_t world, int64_t numel) {
  const int id = dmlc_xgmi_create((int)rank, (int)world, numel);
  TORCH_CHECK(id >= 0, "xgmi_create failed: ", dmlc_xgmi_last_error());
  return id;
}

Tensor xgmi_buffer(int64_t ctx) {
  float* p = dmlc_xgmi_buffer((int)ctx);
  TORCH_CHECK(p != nullptr, "xgmi_buffer: bad context");
  int dev = 0;
  CHECK_HIP(hipPointerGetAttribute(&dev, HIP_POINTER_ATTRIBUTE_DEVICE_ORDINAL, reinterpret_cast<hipDeviceptr_t>(p)));
  // no deleter: the context owns the allocation (xgmi_destroy frees it)
  return torch::from_blob(p, {dmlc_xgmi_numel((int)ctx)},
                          torch::TensorOptions().dtype(at::kFloat).device(at::Device(at::kCUDA, (int8_t)dev)));
}

Tensor xgmi_handles(int64_t ctx) {
  Tensor out = torch::empty({DMLC_XGMI_HANDLES * DMLC_XGMI_HANDLE_BYTES}, torch::TensorOptions().dtype(at::kByte));
  TORCH_CHECK(dmlc_xgmi_handles((int)ctx, out.data_ptr<uint8_t>()) == 0, "xgmi_handles failed: ",
              dmlc_xgmi_last_error());
  return out;
}

void xgmi_open(int64_t ctx, const Tensor& all) {
  TORCH_CHECK(!all.is_cuda() && all.scalar_type() == at::kByte && all.is_contiguous() && all.dim() == 2 &&
                  all.size(1) == DMLC_XGMI_HANDLES * DMLC_XGMI_HANDLE_BYTES,
              "xgmi_open: handles must be a contiguous CPU uint8 [world, 192] tensor");
  TORCH_CHECK(dmlc_xgmi_open((int)ctx, all.data_ptr<uint8_t>()) == 0, "xgmi_open failed: ", dmlc_xgmi_last_error());
}

void xgmi_allreduce(int64_t ctx, const Tensor& buf, int64_t offset, int64_t numel, int64_t blocks, bool bf16_wire) {
  dev(buf, "buf");
  TORCH_CHECK(buf.scalar_type() == at::kFloat, "xgmi_allreduce: buf must be fp32");
  TORCH_CHECK(buf.data_ptr<float>() == dmlc_xgmi_buffer((int)ctx), "xgmi_allreduce: buf is not the context's buffer");
  TORCH_CHECK(offset >= 0 && numel > 0 && offset % 4 == 0 && numel % 4 == 0 && offset + numel <= buf.numel(),
              "xgmi_allreduce: range must be 16-byte aligned and inside the buffer");
  TORCH_CHECK(blocks >= 0 && blocks <= DMLC_XGMI_MAX_BLOCKS, "xgmi_allreduce: blocks must be in [0,512]");
  c10::DeviceGuard guard(buf.device());
  CHECK_HIP(dmlc_xgmi_allreduce((int)ctx, offset, numel, (int)blocks, bf16_wire ? 1 : 0, stream_of(buf)));
}

int64_t xgmi_error(int64_t ctx) { return dmlc_xgmi_error((int)ctx); }

void xgmi_destroy(int64_t ctx) { dmlc_xgmi_destroy((int)ctx); }

}  // namespace

TORCH_LIBRARY_FRAGMENT(dmlc, m) {
  m.def("xgmi_create(int rank, int world, int numel) -> int", &xgmi_create);
  m.def("xgmi_buffer(int ctx) -> Tensor", &xgmi_buffer);
  m.def("xgmi_handles(int ctx) -> Tensor", &xgmi_handles);
  m.def("xgmi_open(int ctx, Tensor handles) -> ()", &xgmi_open);
  m.def("xgmi_error(int ctx) -> int", &xgmi_error);
  m.def("xgmi_destroy(int ctx) -> ()", &xgmi_destroy);
  m.def("xgmi_allreduce(int ctx, Tensor(a!) buf, int offset, int numel, int blocks=0, bool bf16_wire=False) -> ()");
}

TORCH_LIBRARY_IMPL(dmlc, CUDA, m) {
  m.impl("xgmi_allreduce", &xgmi_allreduce);
}
