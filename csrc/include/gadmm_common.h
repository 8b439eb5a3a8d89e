// Common definitions for the gfx950 (MI355X / CDNA4) kernels of gadmm_amd.
//
// All arithmetic is IEEE float64: the reference's stopping rule is an absolute objective gap of
// 1e-4 .. 1e-8 on objectives of O(1e2), i.e. ~5e-11 relative, which rules out any
// f32/bf16 path on the iterate.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GADMM_WAVE 64

typedef double f64x4 __attribute__((ext_vector_type(4)));

#define GADMM_CHECK(expr)                                                              \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess) {                                                            \
      gadmm_set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr, hipGetErrorString(_e)); \
      return (int)_e;                                                                  \
    }                                                                                  \
  } while (0)

// Return code of every RCCL-backed entry point whose communicator its watchdog aborted (a deadline
// passed): the caller falls back to another data plane (Python: native.RcclDead).
#define GADMM_RCCL_DEAD (-77)
// Return code of a bounded host wait of the chain engine whose deadline passed (Python: NativeTimeout).
#define GADMM_ENGINE_TIMEOUT (-78)
// A watchdog abort after which the stream still did not drain: no fallback, the process must exit.
#define GADMM_RCCL_WEDGED (-79)

#ifdef __cplusplus
extern "C" {
#endif
void gadmm_set_error(const char* fmt, ...);
// Compute units of the current device (hipDeviceGetAttribute, cached per device: a full
// hipGetDeviceProperties costs tens of microseconds and sat on every persistent launch's path).
int gadmm_cu_count(void);
const char* gadmm_last_error(void);
#ifdef __cplusplus
}
#endif

// Wave-level f64 sum (64 lanes) using cross-lane shuffles.
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Workgroup barrier that orders LDS only. __syncthreads() also waits for every outstanding global
// store (s_waitcnt vmcnt(0)) - a write-through granule store takes ~1 us to complete, which a
// persistent kernel would then pay at every barrier. Global hand-offs in this code base are
// data-is-flag granules (self-validating), so the workgroup barrier only has to cover LDS.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Block-level f64 sum; `scratch` must hold >= blockDim.x/64 doubles. Result valid on all threads.
__device__ __forceinline__ double block_sum_f64(double v, double* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum_f64(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < nw; ++i) t += scratch[i];  // fixed order -> deterministic
  return t;
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5, T1): blocks that
// the dispatcher deals to the same XCD (b % 8 equal) get consecutive logical ids, so neighbouring
// tiles share that XCD's L2. Placement only changes speed, never results.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}
