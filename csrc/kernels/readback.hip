// Read-back of a persistent solve's result block (control words, objective trace, clock) into the
// engine's pinned host buffer by a small kernel's vector stores over the host link, queued right
// behind the solve kernel on the same stream.
//
// The SDMA copy it replaces (hipMemcpyAsync device -> host) started ~10 us after the solve kernel
// ended and took ~5 us more on the GPU timeline of every D-GADMM and E1 solve (rocprofv3 kernel + copy
// trace, profiles/r06_dgadmm/trace): all of it on the solve's critical path, since the host waits for
// exactly this block. A dependent kernel launch on the same queue starts within a few us, and a 48 KB
// block is ~1 us of host-link writes.
#include "gadmm_common.h"

#include <stdint.h>

namespace {

__global__ void __launch_bounds__(256) readback_kernel(double2* __restrict__ dst, const double2* __restrict__ src,
                                                       long n2) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256) dst[i] = src[i];
  // system-scope release: the host reads the block as soon as the stream reports the kernel done, and
  // the end-of-kernel release does not cover stores to non-coherent pinned memory (a stale control
  // word read as a timed-out hand-off in tests/test_gpu.py::test_postfence_stress without it)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

}  // namespace

extern "C" {

// Device -> pinned host copy of `bytes` on `st` by readback_kernel; a plain hipMemcpyAsync when the
// block is not 16-byte shaped or the host buffer has no device mapping.
int gadmm_readback_d2h(void* dst_host, const void* src, size_t bytes, hipStream_t st) {
  void* dd = nullptr;
  if (bytes % 16 == 0 && ((uintptr_t)dst_host % 16) == 0 && ((uintptr_t)src % 16) == 0 &&
      (hipHostGetDevicePointer(&dd, dst_host, 0) != hipSuccess || !dd)) {
    (void)hipGetLastError();  // not a mapped pinned buffer: the copy engine path below
    dd = nullptr;
  }
  if (!dd) {
    GADMM_CHECK(hipMemcpyAsync(dst_host, src, bytes, hipMemcpyDeviceToHost, st));
    return 0;
  }
  const long n2 = (long)(bytes / 16);
  if (n2 == 0) return 0;
  long blocks = (n2 + 255) / 256;
  if (blocks > 64) blocks = 64;
  readback_kernel<<<dim3((unsigned)blocks), dim3(256), 0, st>>>((double2*)dd, (const double2*)src, n2);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"
