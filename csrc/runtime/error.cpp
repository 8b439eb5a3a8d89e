// Thread-local last-error string shared by every C entry point of libgadmm_native.
#include <stdarg.h>
#include <stdio.h>
#include <hip/hip_runtime.h>

#include <atomic>

static thread_local char g_err[1024] = {0};
static std::atomic<int> g_cus[64];

extern "C" int gadmm_cu_count(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 0;
  if (dev < 64) {
    const int c = g_cus[dev].load(std::memory_order_relaxed);
    if (c > 0) return c;
  }
  int c = 0;
  if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) return 0;
  if (dev < 64) g_cus[dev].store(c, std::memory_order_relaxed);
  return c;
}

extern "C" void gadmm_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* gadmm_last_error(void) { return g_err; }

extern "C" int gadmm_native_version(void) { return 1; }

// Device properties the Python side wants without initialising torch.cuda first.
extern "C" int gadmm_device_info(int dev, char* name, int name_len, int* cus, long long* mem_bytes, int* arch_major,
                                 int* arch_minor) {
  hipDeviceProp_t p;
  hipError_t e = hipGetDeviceProperties(&p, dev);
  if (e != hipSuccess) {
    gadmm_set_error("hipGetDeviceProperties: %s", hipGetErrorString(e));
    return (int)e;
  }
  snprintf(name, name_len, "%s (%s)", p.name, p.gcnArchName);
  *cus = p.multiProcessorCount;
  *mem_bytes = (long long)p.totalGlobalMem;
  *arch_major = p.major;
  *arch_minor = p.minor;
  return 0;
}
