// Shared device helpers for the CDNA4 (gfx950) CNN kernels.
//
// Conventions (see docs in cnn_conv.hip):
//   * activations are NHWC bf16; accumulation is fp32 (MFMA 16x16x32 bf16);
//   * MFMA lane maps (v_mfma_f32_16x16x32_bf16, wave64):
//       A frag: lane l holds A[row = l&15][k = 8*(l>>4) + j], j = 0..7
//       B frag: lane l holds B[k = 8*(l>>4) + j][col = l&15]
//       C/D   : lane l holds C[row = 4*(l>>4) + i][col = l&15], i = 0..3
//   * every kernel is launched with 256 threads = 4 waves.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dmlc {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define DEV static __device__ __forceinline__
#define MDEV __device__ __forceinline__   // member functions
#define LDS_AS __attribute__((address_space(3)))

DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

DEV f32x4 zero4() { f32x4 z = {0.f, 0.f, 0.f, 0.f}; return z; }

// the wave's index in its workgroup as a wave-uniform (SGPR) value: the compiler cannot prove
// threadIdx.x >> 6 uniform, and everything derived from it would otherwise be VALU work
DEV int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// A launch argument read through an opaque pointer into the kernarg segment, made where a kernel's
// late phase starts.  hipcc loads every field a kernel ever reads in its entry block, and with ~100
// SGPRs live it serialises them (k_wgrad: ~45 scalar-load round trips, 3.4 us, before the first
// body instruction); loads through this reference cannot be hoisted above the asm.  The kernarg
// segment pointer, not &param: taking a by-value parameter's address copies it to scratch.
// (The opaque value is the 32-bit offset, made uniform again by readfirstlane: an "s"-constrained
// pointer is an illegal VGPR-to-SGPR copy wherever the compiler's divergence analysis loses it.)
template <class T> DEV const T& late_kernarg(unsigned off) {
  typedef __attribute__((address_space(4))) const char* cptr;
  asm volatile("" : "+v"(off));
  off = __builtin_amdgcn_readfirstlane(off);
  return *(const T*)((cptr)__builtin_amdgcn_kernarg_segment_ptr() + off);
}
// byte offset of a kernel's second by-value argument (arguments are laid out in order, each at its
// own alignment)
template <class A, class B> constexpr unsigned kernarg_second() {
  return (unsigned)((sizeof(A) + alignof(B) - 1) / alignof(B) * alignof(B));
}

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p supplies the address of row q, columns 4p..4p+3
// of a 4x16 block of 16-bit elements; lane i of the group receives column i (row q in element q).
// Two reads (rows kb..kb+3 and kb+4..kb+7) give the 8-element MFMA fragment of one column.
// EXEC must be all ones around these reads (no divergence).
DEV bf16x8 tr_frag(const bf16* p0, const bf16* p1) {
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(p0));
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(p1));
  s16x8 r = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, r);
}

// s_waitcnt lgkmcnt(0) as a real instruction the waitcnt pass accounts for (vmcnt / expcnt left at
// their maxima).  Software-pipelined loops use it to retire the PREVIOUS chunk's LDS reads before
// issuing the next chunk's: the compiler would otherwise wait lgkmcnt(0) right before an MFMA, i.e.
// also for the reads just issued for the next chunk, exposing one LDS latency per chunk.
DEV void wait_lds() { __builtin_amdgcn_s_waitcnt(0xC07F); }

DEV bf16x8 lds_b128(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
DEV bf16x8 glb_b128(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

DEV bf16x8 cat44(const bf16x4& a, const bf16x4& b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

DEV bf16x4 pack4(float a, float b, float c, float d) {
  bf16x4 r = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
  return r;
}

// Workgroup barrier that orders LDS only.  __syncthreads() is a release/acquire fence + s_barrier,
// and the release waits vmcnt(0) -- on gfx950 vmcnt counts loads AND stores, so a __syncthreads()
// placed after global stores also drains every prefetch load in flight.  When the barrier only
// publishes LDS writes, waiting lgkmcnt(0) is enough and global traffic keeps flowing across it.
DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// 4 floats -> 4 OCP e4m3fn bytes (saturated to +-448; gfx950's converter is the OCP format).
DEV uint32_t pk_fp8x4(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -448.f), 448.f); b = fminf(fmaxf(b, -448.f), 448.f);
  c = fminf(fmaxf(c, -448.f), 448.f); d = fminf(fmaxf(d, -448.f), 448.f);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

// staircase (or constant) decay, times a linear warm-up ramp (step + 1) / warmup over the first
// `warmup` steps (large-batch recipe, BASELINE config 5).  The SGD kernel and the fused-SGD GEMM
// epilogue evaluate the SAME expression, so both see bit-identical rates.
DEV float lr_sched(float lr0, float decay, float decay_steps, int staircase, float warmup, int64_t step) {
  const float lr = staircase ? lr0 * powf(decay, floorf((float)step / decay_steps)) : lr0;
  return warmup > 0.f && (float)step < warmup ? lr * ((float)step + 1.f) / warmup : lr;
}

// Producer -> next-launch stores: plain, or streaming (nt: the lines do not stay dirty in this XCD's
// L2, so the kernel-boundary write-back has less to flush; the consumers run on other XCDs anyway).
// Same-session A/B at B=256 (r3): 79.3 us/step all plain, 78.8 with the conv2 slabs + dgrad outputs
// streaming, 77.8-78.2 with conv12's pooled outputs, the conv1 slabs and the GEMM fp32 outputs too.
// -DDMLC_NO_NT builds every site plain.
#ifdef DMLC_NO_NT
constexpr bool kNtDefault = false;
#else
constexpr bool kNtDefault = true;
#endif
template <bool NT, class T>
DEV void st_maybe_nt(T* p, const T& v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <bool NT>
DEV void st_maybe_nt(uint4* p, const uint4& v) {
  st_maybe_nt<NT>(reinterpret_cast<u32x4*>(p), __builtin_bit_cast(u32x4, v));
}
template <bool NT>
DEV void st_maybe_nt(uint2* p, const uint2& v) {
  st_maybe_nt<NT>(reinterpret_cast<u32x2*>(p), __builtin_bit_cast(u32x2, v));
}
constexpr bool kNtFwd = kNtDefault;
constexpr bool kNtX = kNtDefault;   // the channel-split kernels' outputs, the fused-SGD epilogue (-0.4 us)
constexpr bool kNtW1 = kNtDefault;
constexpr bool kNtDg = kNtDefault;
constexpr bool kNtGemm = kNtDefault;

// Agent-coherent (sc1) buffer stores / loads through compiler-visible builtins (aux bit 4 = sc1;
// inline-asm memory ops are invisible to the compiler's vmcnt accounting: an asm store issued while
// compiler loads are in flight made it wait too little -- wrong data, seen in r3).  Written through
// this XCD's L2, so once acknowledged (s_waitcnt vmcnt(0)) every XCD reads the value; sc1 loads read
// at agent coherence whatever this XCD's L2 holds.  For data OTHER blocks of the same launch read
// after a sub-grid barrier.  `base` must be wave-uniform (a buffer resource lives in SGPRs), offsets
// in bytes (< 2 GiB).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
DEV rsrc_t buf_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
constexpr int kSC1 = 16;
// (the builtins take / return unsigned data: every value goes through an explicit bit cast -- an
// implicit float -> uint conversion would convert the VALUE)
DEV void st_sc1(rsrc_t r, uint32_t off, const f32x4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, kSC1);
}
DEV void st_sc1(rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, kSC1);
}
#ifdef DMLC_RED_PLAIN_LOADS
constexpr int kLdPol = 0;     // A/B variant: plain (non-coherent) reduction loads
#else
constexpr int kLdPol = kSC1;
#endif
DEV float4 ld_sc1(rsrc_t r, uint32_t off) {
  const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kLdPol));
  return make_float4(v[0], v[1], v[2], v[3]);
}
DEV void wait_vm_all() { __builtin_amdgcn_s_waitcnt(0x0F70); }   // s_waitcnt vmcnt(0)

// Producer -> next-launch activation stores (the conv kernels' pooled outputs / argmax bytes, the
// dgrad's dY2 / dP1): write-through (sc1) buffer stores, which leave no dirty lines in this XCD's L2
// for the kernel boundary's write-back (r5 same-box A/B at B=256: 79.1 / 79.4 vs 79.8 / 80.4 us per
// step with streaming nt stores, profiles/r5_ab_wt_pool_prefetch.txt).  -DDMLC_NO_WT_STORES builds
// the streaming form.  `base` must be wave-uniform.
#ifdef DMLC_NO_WT_STORES
constexpr bool kWtStores = false;
#else
constexpr bool kWtStores = true;
#endif
// A pointer the compiler cannot prove wave-uniform, made so (buffer descriptors live in SGPRs; a
// VGPR descriptor makes hipcc wrap every buffer op in a waterfall loop -- guide T20)
DEV const void* uni(const void* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  // (through uint32_t: readfirstlane returns int, which would sign-extend into the high word)
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<const void*>(((uint64_t)hi << 32) | lo);
}
DEV void st_out16(void* base, uint32_t byte_off, const uint4& v) {
  if constexpr (kWtStores)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), buf_rsrc(base), byte_off, 0, kSC1);
  else
    st_maybe_nt<kNtDefault>(reinterpret_cast<uint4*>(reinterpret_cast<char*>(base) + byte_off), v);
}
DEV void st_out8(void* base, uint32_t byte_off, const uint2& v) {
  if constexpr (kWtStores)
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), buf_rsrc(base), byte_off, 0, kSC1);
  else
    st_maybe_nt<kNtDefault>(reinterpret_cast<uint2*>(reinterpret_cast<char*>(base) + byte_off), v);
}

// Spin bound of every in-launch wait (sub-grid barriers, hand-off seams, split-forward flags): past it
// the waiter sets the sticky error word and goes on.  A diagnostic build with -DDMLC_SPIN_LIMIT=0
// (DMLC_VARIANT="spin0:-DDMLC_SPIN_LIMIT=0") gives up at the first unsatisfied poll, which forces the
// timeout paths on purpose (tests/test_health.py::test_forced_spin_timeouts_name_kernel_and_switch).
#ifndef DMLC_SPIN_LIMIT
#define DMLC_SPIN_LIMIT (1u << 20)
#endif

// Sub-grid barrier among the n co-resident blocks sharing (cnt, gen) (each on its own 128-B line,
// zero-initialised; they re-arm themselves).  Thread 0 reads the generation BEFORE its block can
// arrive (bar_gen), arrives once the block's coherent stores are acknowledged (bar_arrive) and spins
// (bar_wait).  The spin is bounded: a block that is never scheduled (co-residency violated) sets the
// sticky error word instead of hanging the GPU.
DEV unsigned bar_gen(unsigned* gen) { return __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DEV void bar_arrive(unsigned* cnt, unsigned* gen, unsigned g0, unsigned n) {
  if (__hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n - 1) {
    __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(gen, g0 + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
DEV void bar_wait(unsigned* gen, unsigned g0, unsigned* err) {
  for (unsigned it = 0; bar_gen(gen) == g0; ++it) {
    if (it >= DMLC_SPIN_LIMIT) {
      __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Last-arrival detection over a whole grid, two levels: workgroup b adds to the counter of group
// b % 8 (each counter on its own 128-B line), the last of each group adds to a top counter, and the
// last of those is the grid's last arriver.  One counter taking ~800 atomics in a row serialised
// them at the memory side (~4-5 us at the end of the SGD launch); 8 groups + 8 top arrivals cut the
// queue by ~90x.  Counters re-arm themselves (every member has arrived when its group's last one
// resets it), so a zeroed buffer of DMLC_TICKET_WORDS (api.h) uints serves every later launch.
// Relaxed atomics, no fences: nothing is published THROUGH the ticket (callers order their own
// data).  Call from ONE thread per workgroup; returns true in exactly one workgroup.
DEV bool last_arrival(unsigned int* tk, int blk, int nblk) {
  const int g = blk & 7;
  const unsigned gsize = (unsigned)((nblk - g + 7) >> 3);
  unsigned int* gc = tk + g * 32;
  if (__hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gsize - 1) return false;
  __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned ngroups = (unsigned)(nblk < 8 ? nblk : 8);
  unsigned int* top = tk + 8 * 32;
  if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ngroups - 1) return false;
  __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// A hand-off seam of n counters 128 B apart (p, p + 32, ...), each of which must reach `target`.
// Many producers adding to ONE word serialise at the memory side (r5 phase stamps: ~2.4 us for the 48
// arrivals on one fc1-forward tile counter), so a seam's arrivals are spread over several words and
// the consumer's lanes 0..n-1 of wave 0 poll them side by side.  Bounded; on give-up the sticky error
// word gets `errbit`.  Call with every lane of wave 0 (tid < 64); the caller then barriers.
// (lane_target: this lane's word target, for seams whose words differ -- default s.target)
struct Seam { unsigned* p; int n; unsigned target; };
DEV void seam_wait(const Seam& s, int lane, unsigned* err, unsigned errbit, int lane_target = -1) {
  const bool on = lane < s.n;
  unsigned* q = s.p + 32 * (on ? lane : 0);
  const unsigned t = lane_target >= 0 ? (unsigned)lane_target : s.target;
  for (unsigned it = 0;; ++it) {
    const bool ok = !on || __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= t;
    if (__all(ok)) break;
    if (it >= DMLC_SPIN_LIMIT) {
      if (lane == 0) __hip_atomic_fetch_or(err, errbit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// 32-bit integer mixer (a bijective avalanche hash): the round function of the data-order Feistel
// network below.  Host twin: dmlc/data/order.py (_mix32).
DEV uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du;
  x ^= x >> 15; x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Dataset row of position `pos` in the epoch's permutation of [0, n): a 4-round balanced Feistel
// network on 2*half_bits bits keyed by (seed, epoch), cycle-walked back into [0, n) (the walk ends:
// pos < n lies on its own cycle).  Expected walks: 2^(2*half_bits) / n < 4.
DEV uint32_t order_perm(uint32_t pos, uint32_t n, int half_bits, uint32_t seed, uint32_t epoch) {
  const uint32_t ek = mix32(mix32(seed ^ 0x5bd1e995u) ^ mix32(epoch * 0x85ebca77u + 0x632be5abu));
  const uint32_t mask = (1u << half_bits) - 1u;
  uint32_t x = pos;
  do {
    uint32_t l = x >> half_bits, r = x & mask;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t t = l ^ (mix32(r ^ (ek + (uint32_t)k * 0x9e3779b9u)) & mask);
      l = r;
      r = t;
    }
    x = (l << half_bits) | r;
  } while (x >= n);
  return x;
}

// Generated-order dataset row of batch row b at global step `step` (api.h DmlcIndexSrc).
template <class Src>
DEV int order_row(const Src& s, int64_t step, int b) {
  const uint32_t epoch = (uint32_t)(step / s.period);
  const int64_t j = step - (int64_t)epoch * s.period;
  const int bb = b < s.bvalid ? b : s.bvalid - 1;
  const uint32_t pos = (uint32_t)((j * s.world + s.rank) * s.bvalid + bb);
  return (int)order_perm(pos, (uint32_t)s.n, s.half_bits, s.seed, epoch);
}

// Sample index of batch row b (api.h DmlcIndexSrc: explicit list or generated epoch order).
template <class Src>
DEV int batch_index(const Src& s, int B, int b) {
  if (s.idx_base) {
    int row = 0;
    if (s.counter) row = (int)(*s.counter % (int64_t)s.period);
    return s.idx_base[row * B + b];
  }
  return order_row(s, *s.counter, b);
}

// 16-byte chunk swizzle for [pixel][64 x bf16] LDS images (128-B rows): chunk c of pixel p is
// stored at chunk slot c ^ (p & 7), spreading 16 consecutive pixels over all bank slots.
DEV int swz128(int pix, int chunk) { return pix * 64 + ((chunk ^ (pix & 7)) << 3); }
// Swizzle of the zero-padded 16x16-pixel conv2 input images (pixel = 16*y + x): the XOR key also
// folds in the row (4*y), so the 16 pixels of an MFMA B tile -- which wrap from x = 11 back to
// x = 0 of the next row -- hit distinct bank groups: 4 LDS cycles per ds_read_b128 instead of 8
// with the plain (pix & 7) key (modelled per lane group, tools/lds_banks.py).
DEV int swzpad(int pix, int chunk) { return pix * 64 + ((chunk ^ ((pix + 4 * (pix >> 4)) & 7)) << 3); }

// Kernels above 64 KiB of dynamic LDS opt in once per kernel (gfx950: 160 KiB per CU).  The
// attribute's status is returned to the launcher, so a refused opt-in reports itself instead of
// surfacing later as a generic launch failure; it is retried on the next launch until it succeeds.
inline hipError_t lds_optin(const void* f, size_t bytes, bool& done) {
  if (done) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  done = e == hipSuccess;
  return e;
}
#define DMLC_LDS_OPTIN(fn, bytes)                                                                   \
  do {                                                                                              \
    static bool optin_done_ = false;                                                                \
    const hipError_t optin_e_ = ::dmlc::lds_optin(reinterpret_cast<const void*>(fn), (bytes), optin_done_); \
    if (optin_e_ != hipSuccess) return optin_e_;                                                    \
  } while (0)

}  // namespace dmlc

// ---- diagnostic phase timing (build with DMLC_TIMING=1: separate library, never the default) ----
// DMLC_STAMP(kernel, slot): thread 0 of the block records s_memrealtime (100 MHz) into
// dmlc_timing_buf[kernel][block][slot]; tools/ktiming.py reads it back.
#define DMLC_TK_CONV1_FWD 0
#define DMLC_TK_CONV2_FWD 1
#define DMLC_TK_GEMM 2
#define DMLC_TK_HEAD 3
#define DMLC_TK_DGRAD 4
#define DMLC_TK_W1 5
#define DMLC_TK_W2 6
#define DMLC_TK_SGD 7
#define DMLC_TK_N 8
#define DMLC_TK_BLOCKS 1024
#define DMLC_TK_SLOTS 8
#ifdef DMLC_TIMING
extern __device__ unsigned long long dmlc_timing_buf[DMLC_TK_N * DMLC_TK_BLOCKS * DMLC_TK_SLOTS];
#define DMLC_STAMP(k, slot)                                                                          \
  do {                                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < DMLC_TK_BLOCKS)                                             \
      dmlc_timing_buf[((k) * DMLC_TK_BLOCKS + blockIdx.x) * DMLC_TK_SLOTS + (slot)] =               \
          __builtin_amdgcn_s_memrealtime();                                                          \
  } while (0)
#else
#define DMLC_STAMP(k, slot) do {} while (0)
#endif
// DMLC_STAMP_T(kernel, slot, thread): the same, recorded by thread `thread` (another wave's view)
#ifdef DMLC_TIMING
#define DMLC_STAMP_T(k, slot, t)                                                                     \
  do {                                                                                               \
    if (threadIdx.x == (t) && blockIdx.x < DMLC_TK_BLOCKS)                                           \
      dmlc_timing_buf[((k) * DMLC_TK_BLOCKS + blockIdx.x) * DMLC_TK_SLOTS + (slot)] =               \
          __builtin_amdgcn_s_memrealtime();                                                          \
  } while (0)
#else
#define DMLC_STAMP_T(k, slot, t) do {} while (0)
#endif

// ---- branch-free guarded loads --------------------------------------------------------------------
// `if (ok) v = *p;` makes hipcc branch around the load and wait vmcnt(0) inside the branch, which
// serialises every load of an unrolled prefetch.  These load unconditionally from `ok ? p : safe`
// (a valid address of the same buffer) and select afterwards, so all loads stay in flight together.
template <class T>
DEV T load_sel(const T* p, const T* safe, bool ok) {
  const T v = *(ok ? p : safe);
  return ok ? v : T{};
}
DEV uint4 load_sel(const uint4* p, const uint4* safe, bool ok) {
  const uint4 v = *(ok ? p : safe);
  return ok ? v : make_uint4(0, 0, 0, 0);
}
DEV float4 load_sel(const float4* p, const float4* safe, bool ok) {
  const float4 v = *(ok ? p : safe);
  return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}
