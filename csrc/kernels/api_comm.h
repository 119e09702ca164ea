// Host-side API of the xGMI peer-to-peer all-reduce (csrc/kernels/xgmi_allreduce.hip).
//
// One context per process (= per GPU rank).  It owns a device data buffer that every peer maps
// through HIP IPC, plus a small signal block (uncached device memory) used for the cross-GPU
// barriers.  The all-reduce is an ordinary kernel launch on the caller's stream: its barrier epochs
// live in device memory, so the launch can be captured into a HIP graph and replayed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DMLC_XGMI_MAX_RANKS 8
#define DMLC_XGMI_MAX_BLOCKS 512
#define DMLC_XGMI_HANDLE_BYTES 64   // sizeof(hipIpcMemHandle_t)
#define DMLC_XGMI_HANDLES 3         // per rank: data buffer, signal block, bf16 wire buffer

extern "C" {

// Create the context: allocate `numel` fp32 elements (zeroed), a bf16 wire buffer of `numel` and the
// signal block.
// Returns a context id >= 0, or -1 (error string via dmlc_xgmi_last_error()).
int dmlc_xgmi_create(int rank, int world, int64_t numel);
float* dmlc_xgmi_buffer(int ctx);
int64_t dmlc_xgmi_numel(int ctx);
// DMLC_XGMI_HANDLES * DMLC_XGMI_HANDLE_BYTES bytes: IPC handles of the data buffer, the signal block
// and the wire buffer.
int dmlc_xgmi_handles(int ctx, uint8_t* out);
// all_handles: world * DMLC_XGMI_HANDLES * DMLC_XGMI_HANDLE_BYTES bytes in rank order (own entry ignored).
int dmlc_xgmi_open(int ctx, const uint8_t* all_handles);
// Sum-all-reduce elements [offset, offset + numel) of the buffer across the ranks, in place.
// offset and numel must be multiples of 4 (16-byte vectors).  Deterministic: element i's sum is
// computed by one owner rank in fixed rank order and pushed to every peer, so replicas stay
// bit-identical.  bf16_wire: the values cross the links as bf16 (sums in fp32, result bf16-rounded).
hipError_t dmlc_xgmi_allreduce(int ctx, int64_t offset, int64_t numel, int blocks, int bf16_wire, hipStream_t s);
// The same exchange over the whole flat gradient (the context's buffer) with the SGD update in its
// epilogue: every thread applies the step (mode 2 of the SGD launch: master, every bf16 shadow, the
// next batch rows; workgroup 0 publishes the stats and bumps global_step) to the elements it owns in
// the exchange.  Replaces all-reduce + SGD launch in the data-parallel step (bf16 shadows only).
struct DmlcSgdArgs;
hipError_t dmlc_xgmi_allreduce_sgd(int ctx, int blocks, int bf16_wire, const DmlcSgdArgs* sgd, hipStream_t s);
// Sticky error word of the context (device memory): bit 0 = a barrier timed out.
int dmlc_xgmi_error(int ctx);
void dmlc_xgmi_destroy(int ctx);
const char* dmlc_xgmi_last_error();

}  // extern "C"
