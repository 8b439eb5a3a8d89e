// Debug aid for the GPU test tier: fill every CU's LDS (and optionally a device buffer) with NaN
// bit patterns, so a kernel that reads LDS it never wrote sees a NaN instead of whatever finite data
// the previous kernel on that CU happened to leave behind.
//
// Why: a padded 64-wide vector that is written only for j < d and then multiplied by an exact zero
// (identity padding of an inverse, a zero weight) is harmless only while the stale word is finite:
// 0 * NaN = NaN. The GPU tier runs many kernels in one process, so the LDS content a kernel starts
// with depends on test order; this kernel makes it deterministic (and hostile) -- see
// tests/test_gpu.py (autouse poison fixture) and VERDICT r02 "weak #1".
//
// The NaNs are quiet NaNs with a recognisable payload (0x7ff8_dead_0000_0000 | slot), so a trace
// that picks one up can be told apart from a NaN produced by arithmetic.
#include "gadmm_common.h"

namespace {

constexpr int POISON_THREADS = 1024;
constexpr unsigned long long POISON_BITS = 0x7ff8dead00000000ull;

__global__ void __launch_bounds__(POISON_THREADS) lds_poison_kernel(int words, unsigned long long* sink) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long plds[];
  for (int i = threadIdx.x; i < words; i += POISON_THREADS) plds[i] = POISON_BITS | (unsigned)i;
  __syncthreads();
  // one read back so the stores cannot be dropped as dead; the sink is written only on a mismatch
  // (never, unless LDS is broken), i.e. the kernel's only global effect is nothing
  const unsigned long long v = plds[(threadIdx.x * 7) % words];
  if ((v >> 32) != (POISON_BITS >> 32) && sink) sink[blockIdx.x] = v;
}

__global__ void buffer_poison_kernel(unsigned long long* p, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    p[i] = POISON_BITS | (unsigned long long)(i & 0xffffffff);
}

// Reads LDS it never wrote (deliberately): the test tier uses it to check that the poison landed.
__global__ void __launch_bounds__(256) lds_probe_kernel(unsigned long long* out, int words) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long plds[];
  for (int i = threadIdx.x; i < words; i += 256) out[(long)blockIdx.x * words + i] = plds[i];
}

}  // namespace

// One wave that keeps its stream busy for `ticks` of the 100 MHz s_memrealtime clock, then exits: a
// bounded stand-in for a stalled peer in the watchdog tests (tests/test_gpu.py), never unbounded.
__global__ void __launch_bounds__(64) busy_wait_kernel(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

extern "C" {

// Occupy `st` for `seconds` (at most 30 s): see busy_wait_kernel.
int gadmm_debug_busy_wait(double seconds, hipStream_t st) {
  if (!(seconds > 0.0) || seconds > 30.0) {
    gadmm_set_error("debug_busy_wait: %g s out of (0, 30]", seconds);
    return -1;
  }
  hipLaunchKernelGGL(busy_wait_kernel, dim3(1), dim3(64), 0, st, (unsigned long long)(seconds * 1e8));
  GADMM_CHECK(hipGetLastError());
  return 0;
}


// out: [blocks][words] u64, the LDS content each probe workgroup found at start.
int gadmm_lds_probe(void* out, int blocks, int words, hipStream_t st) {
  if (!out || blocks < 1 || words < 1 || words > 8192) {
    gadmm_set_error("lds_probe: bad arguments");
    return -1;
  }
  hipLaunchKernelGGL(lds_probe_kernel, dim3(blocks), dim3(256), (size_t)words * 8, st, (unsigned long long*)out, words);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// Fill the LDS of every CU with NaN patterns: `lds_bytes` per workgroup (0: the device maximum),
// `waves` workgroups per CU (several, so every CU gets at least one whatever the dispatcher does).
int gadmm_poison_lds(long lds_bytes, int per_cu, hipStream_t st) {
  int dev = 0, maxlds = 0;
  GADMM_CHECK(hipGetDevice(&dev));
  GADMM_CHECK(hipDeviceGetAttribute(&maxlds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
  long bytes = lds_bytes > 0 ? lds_bytes : (long)maxlds;
  if (bytes > maxlds) bytes = maxlds;
  bytes &= ~7L;
  if (bytes < 8) {
    gadmm_set_error("poison_lds: no LDS (%ld B)", bytes);
    return -1;
  }
  if (bytes > 65536)
    GADMM_CHECK(hipFuncSetAttribute((const void*)lds_poison_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)bytes));
  const int blocks = gadmm_cu_count() * (per_cu > 0 ? per_cu : 4);
  hipLaunchKernelGGL(lds_poison_kernel, dim3(blocks), dim3(POISON_THREADS), (size_t)bytes, st, (int)(bytes / 8),
                     (unsigned long long*)nullptr);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// Fill `bytes` (multiple of 8) of device memory at `p` with the same NaN patterns.
int gadmm_poison_buffer(void* p, long bytes, hipStream_t st) {
  if (!p || bytes < 8) return 0;
  const long n = bytes / 8;
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(buffer_poison_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (unsigned long long*)p, n);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"

extern "C" int gadmm_memset_async(void* p, int v, long bytes, hipStream_t st) {
  if (!p || bytes <= 0) return 0;
  GADMM_CHECK(hipMemsetAsync(p, v, (size_t)bytes, st));
  return 0;
}
