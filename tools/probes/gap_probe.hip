// Inter-kernel gap probe: a HIP graph of back-to-back 256-workgroup kernels, each stamping
// s_memrealtime (100 MHz) at entry and exit of every workgroup.  gap = first entry of kernel k+1 -
// last exit of kernel k.  Variants: what the kernel leaves behind (nothing / dirty L2 lines from plain
// stores / write-through stores), its LDS size and its kernel-argument size.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/gap_probe.hip -o gap_probe && ./gap_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Big { uint64_t pad[120]; };
typedef float f4v __attribute__((ext_vector_type(4)));   // ~1 KB of kernel arguments (the fused step's kernels pass 0.5-1.3 KB)

template <int MODE>   // 0: nothing; 32 KB stores per workgroup: 1 plain, 2 nontemporal, 3 write-through (sc1)
__global__ __launch_bounds__(512) void k_stamp(uint64_t* st, int k, float* buf, Big big) {
  extern __shared__ char lds[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (MODE == 1 || MODE == 2) {
    float4* p = reinterpret_cast<float4*>(buf) + (size_t)blockIdx.x * 2048;
    const float4 v = make_float4((float)k, 1.f, 2.f, (float)big.pad[0]);
    for (int i = threadIdx.x; i < 2048; i += 512) {
      if (MODE == 1) p[i] = v;
      else if (MODE == 2) __builtin_nontemporal_store(__builtin_bit_cast(f4v, v), reinterpret_cast<f4v*>(&p[i]));
      else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                  __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7fffffff, 0x00020000),
                                                  i * 16, 0, 16);
    }
  }
  if (threadIdx.x == 0) lds[0] = 1;
  __syncthreads();
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { st[(k * 256 + blockIdx.x) * 2] = t0; st[(k * 256 + blockIdx.x) * 2 + 1] = t1; }
}

template <int MODE>
int run(const char* name, size_t lds, int nk) {
  uint64_t* st; float* buf;
  CK(hipMalloc(&st, (size_t)nk * 256 * 2 * 8));
  CK(hipMalloc(&buf, (size_t)256 * 2048 * 16));
  CK(hipFuncSetAttribute((const void*)k_stamp<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipStream_t s; CK(hipStreamCreate(&s));
  Big big = {};
  hipGraph_t g; hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int k = 0; k < nk; ++k) hipLaunchKernelGGL(k_stamp<MODE>, dim3(256), dim3(512), lds, s, st, k, buf, big);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int it = 0; it < 3; ++it) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  std::vector<uint64_t> h((size_t)nk * 256 * 2);
  CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> gaps, spans;
  for (int k = 0; k + 1 < nk; ++k) {
    uint64_t mx = 0, mn = UINT64_MAX, e0 = UINT64_MAX;
    for (int b = 0; b < 256; ++b) {
      mx = std::max(mx, h[(k * 256 + b) * 2 + 1]);
      e0 = std::min(e0, h[(k * 256 + b) * 2]);
      mn = std::min(mn, h[((k + 1) * 256 + b) * 2]);
    }
    gaps.push_back((double)((int64_t)mn - (int64_t)mx) / 100.0);
    spans.push_back((double)(mx - e0) / 100.0);
  }
  std::sort(gaps.begin(), gaps.end());
  std::sort(spans.begin(), spans.end());
  printf("%-34s lds %6zu  gap us: min %.2f med %.2f max %.2f   kernel span med %.2f\n", name, lds, gaps.front(),
         gaps[gaps.size() / 2], gaps.back(), spans[spans.size() / 2]);
  CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g)); CK(hipStreamDestroy(s)); CK(hipFree(st)); CK(hipFree(buf));
  return 0;
}

int main() {
  const int nk = 32;
  if (run<0>("empty", 0, nk)) return 1;
  if (run<0>("empty, 150 KB LDS", 150 * 1024, nk)) return 1;
  if (run<1>("8 MB plain stores", 0, nk)) return 1;
  if (run<2>("8 MB nontemporal stores", 0, nk)) return 1;
  if (run<3>("8 MB write-through (sc1) stores", 0, nk)) return 1;
  if (run<1>("8 MB plain stores, 150 KB LDS", 150 * 1024, nk)) return 1;
  return 0;
}
