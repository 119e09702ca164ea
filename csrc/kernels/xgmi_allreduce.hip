// Two-shot peer-to-peer all-reduce over xGMI for the data-parallel gradient buckets
// (replaces the reference's worker->PS gradient push / PS->worker variable
// pull over gRPC, /root/reference/cifar10cnn.py:188-196, :222, :230).
//
// Why not only RCCL: an MI355X node is 8 GPUs fully connected by point-to-point xGMI links (7 per
// GPU).  A ring all-reduce drives one link per GPU per ring step and pays 2(W-1) latency-bound
// steps; the gradient buckets here are small (3.84 MB fc + 0.43 MB conv per step), the regime where
// that latency dominates.  This kernel is the xGMI-shaped alternative:
//   * every rank maps every peer's gradient buffer (HIP IPC) -> loads/stores go straight over the
//     link to that peer, all 7 links busy at once;
//   * reduce-scatter: rank r owns 1/W of the bucket and READS its slice from all W buffers (fixed
//     rank order -> deterministic), then PUSHES the sum into all W buffers (all-gather by stores);
//   * two cross-GPU barriers per launch (data ready / pushes landed), one flag slot per
//     (workgroup, peer) in uncached device memory; epochs are per-workgroup counters in device
//     memory, so the launch is graph-capturable and replays need no host involvement;
//   * optional bf16 wire format: each rank first packs its fp32 bucket into a bf16 wire buffer
//     (also peer-mapped), the owners read bf16, sum in fp32 in rank order and push bf16(sum); every
//     rank then unpacks the whole bucket from its own wire buffer -- half the link bytes, and every
//     replica ends with the same bf16-rounded sums (the semantics of an all-reduce of bf16 tensors);
//   * every spin is bounded (s_memrealtime deadline): a missing peer sets a sticky error word and
//     the kernel drains instead of hanging the GPU.  The word is mirrored into mapped pinned host
//     memory, so the training loop polls it with a plain load (no HIP call, no sync) and exits for
//     a restart; once it is set, later launches skip their barriers (drain at once).
// Memory model: writer side = every wave drains its stores, then ONE wave per workgroup issues the
// system-scope release fence (writes back the L2 of this XCD) before the flag stores; reader side =
// that wave's system-scope acquire after the flag wait (invalidates this CU's non-local lines), then a
// workgroup barrier before any load -- per the AMDGPU memory model for multi-L2 agents.  (r5 fenced
// in every wave: 4x the write-backs per workgroup; the world-1 DP step paid +16 us for the exchange.)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "api_comm.h"
#include "sgd_common.h"

namespace dmlc {

struct XgmiSignal {
  uint32_t flag[2][DMLC_XGMI_MAX_BLOCKS][DMLC_XGMI_MAX_RANKS];   // [start|end][workgroup][peer]
  uint32_t epoch[DMLC_XGMI_MAX_BLOCKS];
  uint32_t err;
};

struct XgmiArgs {
  float4* bufs[DMLC_XGMI_MAX_RANKS];
  uint2* wires[DMLC_XGMI_MAX_RANKS];   // bf16 wire buffers (4 bf16 per float4 of the data buffer)
  XgmiSignal* sigs[DMLC_XGMI_MAX_RANKS];
  uint32_t* host_err; // mapped pinned host word (device pointer), or null
  int rank;
  int64_t off4, n4;   // bucket, in float4 units
};

constexpr int XT = 256;
constexpr uint64_t TIMEOUT_TICKS = 500000000ull;   // 5 s of the 100 MHz s_memrealtime clock

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Cross-GPU barrier of workgroup b: lane p < W publishes epoch e into peer p's slot [which][b][rank]
// and waits for peer p's epoch in its own slot [which][b][p].  Every wave drains its own stores
// (s_waitcnt vmcnt(0)), the workgroup meets, and ONE wave releases at system scope (writes back this
// XCD's L2) before its lanes signal; after the waits that wave alone acquires (invalidates this CU's
// caches) and the workgroup meets again before any thread loads peer data -- one fence pair per
// workgroup instead of one per wave (MI355X_MICROARCH.md, Valid forms: producer / consumer).
template <int W>
__device__ __forceinline__ void peer_barrier(const XgmiArgs& a, int which, uint32_t e) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x, b = blockIdx.x;
  if (t < 64) {                        // wave 0: one release for the whole workgroup's stores
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the write-back completes before any flag
  }
  if (t < W) {
    st_sys(&a.sigs[t]->flag[which][b][a.rank], e);
    XgmiSignal* self = a.sigs[a.rank];
    const uint32_t* mine = &self->flag[which][b][t];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // a sticky error (an earlier launch lost a peer) drains this launch without waiting
    while (ld_sys(&self->err) == 0u && (int32_t)(ld_sys(mine) - e) < 0) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > TIMEOUT_TICKS) {
        __hip_atomic_fetch_or(&self->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (a.host_err) __hip_atomic_fetch_or(a.host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  if (t < 64) {                        // wave 0 (the pollers): one acquire for the workgroup's CU
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

__device__ __forceinline__ uint2 pack_bf16x4(float4 v) {
  typedef __bf16 b4 __attribute__((ext_vector_type(4)));
  const b4 r = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
  return __builtin_bit_cast(uint2, r);
}
__device__ __forceinline__ float4 unpack_bf16x4(uint2 u) {
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}

// The exchange of one launch: returns once every element this thread owns (element i belongs to
// thread (i - off4) % stride in EVERY phase) holds the sum over ranks in this rank's buffer.
template <int W, bool BF16>
__device__ __forceinline__ void xgmi_exchange(const XgmiArgs& a, uint32_t e, int64_t t0, int64_t stride) {
  if (BF16)                            // my whole bucket -> my wire buffer (read by the owners)
    for (int64_t i = a.off4 + t0; i < a.off4 + a.n4; i += stride) a.wires[a.rank][i] = pack_bf16x4(a.bufs[a.rank][i]);

  peer_barrier<W>(a, 0, e);            // every rank's gradients are complete

  // reduce-scatter of this rank's slice + push of the sums to every rank
  // Element i belongs to thread (i - off4) % stride in EVERY phase (pack, reduce/push, unpack): the
  // barriers are per workgroup, so a workgroup may only touch peer elements that the same workgroup
  // of the peer produced before its barrier signal.  (Walking the slice from `lo` instead hands
  // element i to another workgroup than the one that packed / unpacks it: a race in the bf16 path.)
  const int64_t lo = a.off4 + a.n4 * a.rank / W, hi = a.off4 + a.n4 * (a.rank + 1) / W;
  int64_t i0 = a.off4 + t0;
  if (i0 < lo) i0 += (lo - i0 + stride - 1) / stride * stride;
  for (int64_t i = i0; i < hi; i += stride) {
    float4 v[W];
#pragma unroll
    for (int p = 0; p < W; ++p) v[p] = BF16 ? unpack_bf16x4(a.wires[p][i]) : a.bufs[p][i];
    float4 s = v[0];
#pragma unroll
    for (int p = 1; p < W; ++p) { s.x += v[p].x; s.y += v[p].y; s.z += v[p].z; s.w += v[p].w; }
    if (BF16) {
      const uint2 r = pack_bf16x4(s);
#pragma unroll
      for (int p = 0; p < W; ++p) a.wires[(a.rank + p) % W][i] = r;   // staggered start: links evenly loaded
    } else {
#pragma unroll
      for (int p = 0; p < W; ++p) a.bufs[(a.rank + p) % W][i] = s;
    }
  }

  peer_barrier<W>(a, 1, e);            // every rank's pushes into my buffer landed
  if (BF16)                            // every slice, mine included, from the bf16 sums
    for (int64_t i = a.off4 + t0; i < a.off4 + a.n4; i += stride) a.bufs[a.rank][i] = unpack_bf16x4(a.wires[a.rank][i]);
}

template <int W, bool BF16>
__global__ __launch_bounds__(XT) void k_xgmi_allreduce(XgmiArgs a) {
  XgmiSignal* self = a.sigs[a.rank];
  __shared__ uint32_t s_e;
  if (threadIdx.x == 0) s_e = ld_sys(&self->epoch[blockIdx.x]) + 1u;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * XT, t0 = (int64_t)blockIdx.x * XT + threadIdx.x;
  xgmi_exchange<W, BF16>(a, s_e, t0, stride);
  if (threadIdx.x == 0) st_sys(&self->epoch[blockIdx.x], s_e);
}

// ------------------------------------------------------------------------------------------------
// Exchange + SGD in ONE launch (data parallel, r5): the step's optimizer update runs in the
// all-reduce kernel's epilogue instead of a separate SGD launch.  After the second peer barrier each
// thread owns a fixed set of float4s of the flat gradient (the exchange's element -> thread map), so
// it applies SGD to exactly those: master -= lr * grad_scale * sum, plus every bf16 shadow of those
// four weights in the layout its kernel reads -- the SGD launch's mode-2 expressions
// (sgd_common.h), so the weights are bit-identical to all-reduce + SGD launch
// (tests/test_fused_dp_gpu.py::test_xgmi_sgd_epilogue_is_bit_identical).  Workgroup 0 then publishes
// the step's stats and bumps global_step (the LR came from the head's step copy); every thread
// writes its next-step batch row.  bf16 shadows only: the fp8 path keeps its SGD launch.
__device__ __forceinline__ void sgd_apply4(const DmlcSgdArgs& s, int64_t q, float lr, int64_t step) {
  const int e0 = (int)(4 * q), end = s.off[9] + 10;
  if (e0 >= end) return;
  const float f = lr * s.grad_scale;
  if (e0 + 4 > end) {                  // the fc3 bias tail: master is exactly `end` floats long
    for (int e = e0; e < end; ++e) s.master[e] -= f * s.grad[e];
    return;
  }
  float4 w = *reinterpret_cast<const float4*>(s.master + e0);
  const float4 g = *reinterpret_cast<const float4*>(s.grad + e0);
  w.x -= f * g.x; w.y -= f * g.y; w.z -= f * g.z; w.w -= f * g.w;
  *reinterpret_cast<float4*>(s.master + e0) = w;
  if (e0 < s.off[1]) {                                  // conv1 kernel HWIO [5,5,3,64]
    const int r = e0 - s.off[0];
    conv1_shadow4(s, r >> 6, r & 63, w);
  } else if (e0 >= s.off[2] && e0 < s.off[3]) {         // conv2 kernel [5,5,64,64]
    const int r = e0 - s.off[2];
    conv2_shadow4(s, r >> 6, r & 63, w);
  } else if (e0 >= s.off[4] && e0 < s.off[5]) {         // fc1 weight: same-layout shadow, next step's slot
    bf16* shadow = reinterpret_cast<bf16*>(s.fc1n) + (((step + 1) & 1) ? 884736 : 0);
    *reinterpret_cast<bf16x4*>(shadow + (e0 - s.off[4])) = pack4(w.x, w.y, w.z, w.w);
  } else if (e0 >= s.off[6] && e0 < s.off[7]) {         // fc2 weight [384 k][192 n]
    const int r = e0 - s.off[6], k = r / 192, n = r - k * 192;
    *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(s.fc2n) + r) = pack4(w.x, w.y, w.z, w.w);
    bf16* t = reinterpret_cast<bf16*>(s.fc2t) + (size_t)n * 384 + k;
    t[0] = (bf16)w.x; t[384] = (bf16)w.y; t[2 * 384] = (bf16)w.z; t[3 * 384] = (bf16)w.w;
  } else if (e0 >= s.off[8] && e0 < s.off[9]) {         // fc3 weight [192 k][10 n]
    const float v[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = e0 - s.off[8] + j, k = r / 10, n = r - k * 10;
      reinterpret_cast<bf16*>(s.fc3t)[n * 192 + k] = (bf16)v[j];
      reinterpret_cast<bf16*>(s.fc3d)[k * 32 + n] = (bf16)v[j];
    }
  }                                                      // biases: no shadow
}

template <int W, bool BF16>
__global__ __launch_bounds__(XT) void k_xgmi_allreduce_sgd(XgmiArgs a, DmlcSgdArgs s) {
  XgmiSignal* self = a.sigs[a.rank];
  __shared__ uint32_t s_e;
  if (threadIdx.x == 0) s_e = ld_sys(&self->epoch[blockIdx.x]) + 1u;
  const int64_t step = *s.step_rd;                       // the head's copy: nobody bumps it here
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * XT, t0 = (int64_t)blockIdx.x * XT + threadIdx.x;
  xgmi_exchange<W, BF16>(a, s_e, t0, stride);
  // the SGD's arguments through late_kernarg (common.h): not loaded before the exchange starts
#ifdef DMLC_EAGER_ARGS
  const DmlcSgdArgs& S = s;
#else
  const DmlcSgdArgs& S = late_kernarg<DmlcSgdArgs>(kernarg_second<XgmiArgs, DmlcSgdArgs>());
#endif
  const float lr = lr_of(S, step);
  for (int64_t i = a.off4 + t0; i < a.off4 + a.n4; i += stride) sgd_apply4(S, i, lr, step);
  if (S.bidx && t0 < S.bidx_n) S.bidx[t0] = order_row(S.next, step + 1, (int)t0);
  if (S.xnext)
    for (int r = blockIdx.x; r < S.bidx_n; r += gridDim.x) copy_next_row(S, step, r, threadIdx.x);
  if (blockIdx.x == 0 && threadIdx.x < 64) publish_step(S, step, lr, threadIdx.x);
  if (threadIdx.x == 0) st_sys(&self->epoch[blockIdx.x], s_e);
}

// ------------------------------------------------------------------------------------------------
struct XgmiCtx {
  int rank = 0, world = 1, device = 0;
  int64_t numel = 0;
  float* buf = nullptr;
  uint16_t* wire = nullptr;          // bf16 wire buffer (numel)
  XgmiSignal* sig = nullptr;
  uint32_t* host_err = nullptr;      // pinned, mapped (host view)
  uint32_t* host_err_dev = nullptr;  // the same word as the kernels address it
  float* peer_buf[DMLC_XGMI_MAX_RANKS] = {};
  uint16_t* peer_wire[DMLC_XGMI_MAX_RANKS] = {};
  XgmiSignal* peer_sig[DMLC_XGMI_MAX_RANKS] = {};
  bool opened = false;
};

std::mutex g_mu;
std::vector<XgmiCtx*> g_ctx;
std::string g_err;

XgmiCtx* get(int id) {
  std::lock_guard<std::mutex> l(g_mu);
  return (id >= 0 && id < (int)g_ctx.size()) ? g_ctx[id] : nullptr;
}

void fail(const std::string& what, hipError_t e) { g_err = what + ": " + hipGetErrorString(e); }

}  // namespace dmlc

using namespace dmlc;

extern "C" {

const char* dmlc_xgmi_last_error() { return g_err.c_str(); }

int dmlc_xgmi_create(int rank, int world, int64_t numel) {
  if (world < 1 || world > DMLC_XGMI_MAX_RANKS || rank < 0 || rank >= world || numel <= 0 || numel % 4) {
    g_err = "xgmi_create: bad rank/world/numel";
    return -1;
  }
  auto* c = new XgmiCtx();
  c->rank = rank; c->world = world; c->numel = numel;
  hipError_t e = hipGetDevice(&c->device);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&c->buf), (size_t)numel * sizeof(float));
  if (e == hipSuccess) e = hipMemset(c->buf, 0, (size_t)numel * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&c->wire), (size_t)numel * sizeof(uint16_t));
  if (e == hipSuccess) e = hipMemset(c->wire, 0, (size_t)numel * sizeof(uint16_t));
  if (e == hipSuccess) {
    // flags in uncached device memory: every poll and every remote flag store goes to memory
    e = hipExtMallocWithFlags(reinterpret_cast<void**>(&c->sig), sizeof(XgmiSignal), hipDeviceMallocUncached);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      e = hipMalloc(reinterpret_cast<void**>(&c->sig), sizeof(XgmiSignal));
    }
  }
  if (e == hipSuccess) e = hipMemset(c->sig, 0, sizeof(XgmiSignal));
  if (e == hipSuccess) {
    // host mirror of the error word: optional (without it dmlc_xgmi_error copies from the device)
    if (hipHostMalloc(reinterpret_cast<void**>(&c->host_err), sizeof(uint32_t),
                      hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
      *c->host_err = 0u;
      if (hipHostGetDevicePointer(reinterpret_cast<void**>(&c->host_err_dev), c->host_err, 0) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(c->host_err);
        c->host_err = nullptr;
        c->host_err_dev = nullptr;
      }
    } else {
      (void)hipGetLastError();
      c->host_err = nullptr;
    }
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    fail("xgmi_create", e);
    if (c->buf) (void)hipFree(c->buf);
    if (c->wire) (void)hipFree(c->wire);
    if (c->sig) (void)hipFree(c->sig);
    delete c;
    return -1;
  }
  c->peer_buf[rank] = c->buf;
  c->peer_wire[rank] = c->wire;
  c->peer_sig[rank] = c->sig;
  std::lock_guard<std::mutex> l(g_mu);
  g_ctx.push_back(c);
  return (int)g_ctx.size() - 1;
}

float* dmlc_xgmi_buffer(int id) {
  XgmiCtx* c = get(id);
  return c ? c->buf : nullptr;
}

int64_t dmlc_xgmi_numel(int id) {
  XgmiCtx* c = get(id);
  return c ? c->numel : 0;
}

int dmlc_xgmi_handles(int id, uint8_t* out) {
  XgmiCtx* c = get(id);
  if (!c) { g_err = "xgmi_handles: bad context"; return -1; }
  static_assert(sizeof(hipIpcMemHandle_t) == DMLC_XGMI_HANDLE_BYTES, "IPC handle size");
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, c->buf);
  if (e != hipSuccess) { fail("hipIpcGetMemHandle(buf)", e); return -1; }
  memcpy(out, &h, DMLC_XGMI_HANDLE_BYTES);
  e = hipIpcGetMemHandle(&h, c->sig);
  if (e != hipSuccess) { fail("hipIpcGetMemHandle(sig)", e); return -1; }
  memcpy(out + DMLC_XGMI_HANDLE_BYTES, &h, DMLC_XGMI_HANDLE_BYTES);
  e = hipIpcGetMemHandle(&h, c->wire);
  if (e != hipSuccess) { fail("hipIpcGetMemHandle(wire)", e); return -1; }
  memcpy(out + 2 * DMLC_XGMI_HANDLE_BYTES, &h, DMLC_XGMI_HANDLE_BYTES);
  return 0;
}

int dmlc_xgmi_open(int id, const uint8_t* all) {
  XgmiCtx* c = get(id);
  if (!c) { g_err = "xgmi_open: bad context"; return -1; }
  if (c->opened) return 0;
  for (int p = 0; p < c->world; ++p) {
    if (p == c->rank) continue;
    hipIpcMemHandle_t h;
    void* ptr = nullptr;
    const uint8_t* hp = all + (size_t)p * DMLC_XGMI_HANDLES * DMLC_XGMI_HANDLE_BYTES;
    memcpy(&h, hp, DMLC_XGMI_HANDLE_BYTES);
    hipError_t e = hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) { fail("hipIpcOpenMemHandle(buf of rank " + std::to_string(p) + ")", e); return -1; }
    c->peer_buf[p] = static_cast<float*>(ptr);
    memcpy(&h, hp + DMLC_XGMI_HANDLE_BYTES, DMLC_XGMI_HANDLE_BYTES);
    e = hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) { fail("hipIpcOpenMemHandle(sig of rank " + std::to_string(p) + ")", e); return -1; }
    c->peer_sig[p] = static_cast<XgmiSignal*>(ptr);
    memcpy(&h, hp + 2 * DMLC_XGMI_HANDLE_BYTES, DMLC_XGMI_HANDLE_BYTES);
    e = hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) { fail("hipIpcOpenMemHandle(wire of rank " + std::to_string(p) + ")", e); return -1; }
    c->peer_wire[p] = static_cast<uint16_t*>(ptr);
  }
  c->opened = true;
  return 0;
}

hipError_t dmlc_xgmi_allreduce(int id, int64_t offset, int64_t numel, int blocks, int bf16_wire, hipStream_t s) {
  XgmiCtx* c = get(id);
  if (!c || !c->opened) return hipErrorInvalidValue;
  if (offset < 0 || numel <= 0 || offset % 4 || numel % 4 || offset + numel > c->numel) return hipErrorInvalidValue;
  XgmiArgs a;
  for (int p = 0; p < DMLC_XGMI_MAX_RANKS; ++p) {
    a.bufs[p] = reinterpret_cast<float4*>(c->peer_buf[p]);
    a.wires[p] = reinterpret_cast<uint2*>(c->peer_wire[p]);
    a.sigs[p] = c->peer_sig[p];
  }
  a.rank = c->rank;
  a.host_err = c->host_err_dev;
  a.off4 = offset / 4;
  a.n4 = numel / 4;
  const int64_t shard4 = (a.n4 + c->world - 1) / c->world;
  if (blocks <= 0) blocks = (int)std::min<int64_t>(64, std::max<int64_t>(4, (shard4 + 2 * XT - 1) / (2 * XT)));
  blocks = std::min(blocks, DMLC_XGMI_MAX_BLOCKS);
  switch (c->world) {
#define DMLC_XGMI_CASE(W)                                                                   \
    case W:                                                                                 \
      if (bf16_wire) hipLaunchKernelGGL((k_xgmi_allreduce<W, true>), dim3(blocks), dim3(XT), 0, s, a); \
      else hipLaunchKernelGGL((k_xgmi_allreduce<W, false>), dim3(blocks), dim3(XT), 0, s, a);         \
      break;
    DMLC_XGMI_CASE(1) DMLC_XGMI_CASE(2) DMLC_XGMI_CASE(3) DMLC_XGMI_CASE(4)
    DMLC_XGMI_CASE(5) DMLC_XGMI_CASE(6) DMLC_XGMI_CASE(7) DMLC_XGMI_CASE(8)
#undef DMLC_XGMI_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t dmlc_xgmi_allreduce_sgd(int id, int blocks, int bf16_wire, const DmlcSgdArgs* sgd, hipStream_t s) {
  XgmiCtx* c = get(id);
  if (!c || !c->opened || !sgd) return hipErrorInvalidValue;
  // the whole flat buffer, apply from the summed gradient (mode 2), the head's step copy, bf16 shadows
  const int64_t end = (int64_t)sgd->off[9] + 10;
  if (sgd->mode != 2 || sgd->w2f8 || sgd->step_rd == sgd->step || sgd->grad != c->buf || end > c->numel ||
      sgd->fc1_fused || sgd->roles != 0 || !sgd->finalize)
    return hipErrorInvalidValue;
  XgmiArgs a;
  for (int p = 0; p < DMLC_XGMI_MAX_RANKS; ++p) {
    a.bufs[p] = reinterpret_cast<float4*>(c->peer_buf[p]);
    a.wires[p] = reinterpret_cast<uint2*>(c->peer_wire[p]);
    a.sigs[p] = c->peer_sig[p];
  }
  a.rank = c->rank;
  a.host_err = c->host_err_dev;
  a.off4 = 0;
  a.n4 = (end + 3) / 4;
  // the epilogue streams the whole buffer (master, gradient, shadows: ~15 MB at this model's size):
  // two workgroups per CU, as many as the SGD launch it replaces keeps busy (128 measured 2x slower)
  if (blocks <= 0) blocks = DMLC_XGMI_MAX_BLOCKS;
  blocks = std::min(blocks, DMLC_XGMI_MAX_BLOCKS);
  if ((int64_t)blocks * XT < sgd->bidx_n) return hipErrorInvalidValue;   // one batch row per thread
  switch (c->world) {
#define DMLC_XGMI_SGD_CASE(W)                                                                          \
    case W:                                                                                            \
      if (bf16_wire) hipLaunchKernelGGL((k_xgmi_allreduce_sgd<W, true>), dim3(blocks), dim3(XT), 0, s, a, *sgd); \
      else hipLaunchKernelGGL((k_xgmi_allreduce_sgd<W, false>), dim3(blocks), dim3(XT), 0, s, a, *sgd);         \
      break;
    DMLC_XGMI_SGD_CASE(1) DMLC_XGMI_SGD_CASE(2) DMLC_XGMI_SGD_CASE(3) DMLC_XGMI_SGD_CASE(4)
    DMLC_XGMI_SGD_CASE(5) DMLC_XGMI_SGD_CASE(6) DMLC_XGMI_SGD_CASE(7) DMLC_XGMI_SGD_CASE(8)
#undef DMLC_XGMI_SGD_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

int dmlc_xgmi_error(int id) {
  XgmiCtx* c = get(id);
  if (!c) return -1;
  if (c->host_err) return (int)__atomic_load_n(c->host_err, __ATOMIC_ACQUIRE);   // no HIP call, no sync
  uint32_t v = 0;
  if (hipMemcpy(&v, &c->sig->err, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int)v;
}

void dmlc_xgmi_destroy(int id) {
  XgmiCtx* c = get(id);
  if (!c) return;
  (void)hipDeviceSynchronize();
  for (int p = 0; p < c->world; ++p) {
    if (p == c->rank) continue;
    if (c->peer_buf[p]) (void)hipIpcCloseMemHandle(c->peer_buf[p]);
    if (c->peer_sig[p]) (void)hipIpcCloseMemHandle(c->peer_sig[p]);
    if (c->peer_wire[p]) (void)hipIpcCloseMemHandle(c->peer_wire[p]);
  }
  (void)hipFree(c->buf);
  (void)hipFree(c->wire);
  (void)hipFree(c->sig);
  if (c->host_err) (void)hipHostFree(c->host_err);
  std::lock_guard<std::mutex> l(g_mu);
  g_ctx[id] = nullptr;
  delete c;
}

}  // extern "C"
