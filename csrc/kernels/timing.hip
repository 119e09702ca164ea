// Storage + host access of the diagnostic phase-timing buffer (only populated in DMLC_TIMING builds).
#include "common.h"

#ifdef DMLC_TIMING
__device__ unsigned long long dmlc_timing_buf[DMLC_TK_N * DMLC_TK_BLOCKS * DMLC_TK_SLOTS];
#endif

extern "C" int dmlc_timing_enabled() {
#ifdef DMLC_TIMING
  return 1;
#else
  return 0;
#endif
}

// Copies the buffer (DMLC_TK_N * DMLC_TK_BLOCKS * DMLC_TK_SLOTS uint64) to host memory.
extern "C" hipError_t dmlc_timing_read(unsigned long long* host) {
#ifdef DMLC_TIMING
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(dmlc_timing_buf), sizeof(dmlc_timing_buf), 0, hipMemcpyDeviceToHost);
#else
  (void)host;
  return hipErrorNotSupported;
#endif
}

extern "C" hipError_t dmlc_timing_clear() {
#ifdef DMLC_TIMING
  static unsigned long long zeros[DMLC_TK_N * DMLC_TK_BLOCKS * DMLC_TK_SLOTS];
  return hipMemcpyToSymbol(HIP_SYMBOL(dmlc_timing_buf), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
#else
  return hipErrorNotSupported;
#endif
}
