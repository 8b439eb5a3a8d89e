// Cross-workgroup hand-off latency on one MI355X: two workgroups ping-pong a 64-granule row (one
// wave, 16-B {tag, lo, tag, hi} granules, the persistent kernels' θ-row format) through device memory
// with system-scope (sc0 sc1) stores and sc1 polls, and time N round trips with s_memrealtime.
// Poll variants: D = loads in flight per lane (1 = load -> wait -> check, the kernels' current
// poll; 2 / 4 = a staggered pipeline: each check waits only for the OLDEST load, a new one is issued
// right after), optional s_sleep between polls. Placement: the two workgroups on one XCD or on two.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pingpong.hip -o build/pingpong && build/pingpong
// Prints one line per variant: ns per one-way hop (median of 5 runs).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                              \
    }                                                                        \
  } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ unsigned long long ticks() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void put(__amdgpu_buffer_rsrc_t rs, int off, unsigned tag, unsigned v) {
  u32x4 g = {tag, v, tag, v};
  __builtin_amdgcn_raw_buffer_store_b128(g, rs, off, 0, 17);
}
__device__ __forceinline__ bool ok(const u32x4& g, unsigned tag) { return g.x == tag && g.z == tag; }

// sc1 poll load issued by inline asm: the buffer-load builtin's loads of one address are merged by
// the compiler (its volatile aux bit does not stop that), so a pipeline of D loads in flight needs
// asm loads and explicit `s_waitcnt vmcnt(k)`s that take the loaded registers as operands (no use
// of a register moves above its wait, no register is reused while a load into it is in flight).
__device__ __forceinline__ u32x4 aload(const u32x4* p) {
  u32x4 g;
  asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(g) : "v"(p) : "memory");
  return g;
}
#define VMWAIT(n, g) asm volatile("s_waitcnt vmcnt(" #n ")" : "+v"(g))

// wait until every lane's granule carries `tag`; returns false after `limit` ticks
template <int D, int SLEEP>
__device__ __forceinline__ bool wait_row(const u32x4* p, unsigned tag, unsigned long long limit) {
  if constexpr (D == 1) {
    for (int spin = 0;; ++spin) {
      u32x4 g = aload(p);
      VMWAIT(0, g);
      if (__all(ok(g, tag))) return true;
      if ((spin & 63) == 63 && ticks() > limit) return false;
      if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    }
  } else if constexpr (D == 2) {
    u32x4 g0 = aload(p);
    if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    u32x4 g1 = aload(p);
    bool r = false;
    for (int spin = 0;; ++spin) {
      VMWAIT(1, g0);
      if (__all(ok(g0, tag))) { r = true; break; }
      g0 = aload(p);
      VMWAIT(1, g1);
      if (__all(ok(g1, tag))) { r = true; break; }
      g1 = aload(p);
      if ((spin & 31) == 31 && ticks() > limit) break;
      if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(g0), "+v"(g1));  // drain before the registers are reused
    return r;
  } else {
    u32x4 g0 = aload(p), g1, g2, g3;
    if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    g1 = aload(p);
    if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    g2 = aload(p);
    if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    g3 = aload(p);
    bool r = false;
    for (int spin = 0;; ++spin) {
      VMWAIT(3, g0);
      if (__all(ok(g0, tag))) { r = true; break; }
      g0 = aload(p);
      VMWAIT(3, g1);
      if (__all(ok(g1, tag))) { r = true; break; }
      g1 = aload(p);
      VMWAIT(3, g2);
      if (__all(ok(g2, tag))) { r = true; break; }
      g2 = aload(p);
      VMWAIT(3, g3);
      if (__all(ok(g3, tag))) { r = true; break; }
      g3 = aload(p);
      if ((spin & 15) == 15 && ticks() > limit) break;
      if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(g0), "+v"(g1), "+v"(g2), "+v"(g3));
    return r;
  }
}

// grid: `stride` + 1 blocks; block 0 and block `stride` play, the rest exit (stride 8: same XCD,
// stride 1: neighbouring XCDs under round-robin dispatch). buf: 2 rows of 64 granules.
template <int D, int SLEEP>
__global__ void __launch_bounds__(64) pingpong(u32x4* buf, int n, int stride, unsigned salt,
                                               unsigned long long* out) {
  const int b = blockIdx.x;
  if (b != 0 && b != stride) return;
  const __amdgpu_buffer_rsrc_t rs = rsrc(buf);
  const int lane = threadIdx.x;
  const int row_ab = lane * 16, row_ba = (64 + lane) * 16;
  const unsigned long long limit = ticks() + 200000000ull;  // 2 s
  const unsigned long long t0 = ticks();
  bool good = true;
  for (int i = 1; i <= n && good; ++i) {
    const unsigned tag = (salt << 20) | (unsigned)i;
    if (b == 0) {
      put(rs, row_ab, tag, i);
      good = wait_row<D, SLEEP>(buf + 64 + lane, tag, limit);
    } else {
      good = wait_row<D, SLEEP>(buf + lane, tag, limit);
      put(rs, row_ba, tag, i);
    }
  }
  const unsigned long long t1 = ticks();
  if (b == 0 && lane == 0) {
    out[0] = good ? t1 - t0 : 0ull;
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    out[1] = x;
  }
  if (b == stride && lane == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    out[2] = x;
  }
}

template <int D, int SLEEP>
static int run(const char* name, u32x4* buf, unsigned long long* out, int stride, unsigned& salt) {
  const int n = 20000;
  std::vector<double> ns;
  unsigned long long h[3] = {0, 0, 0};
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipMemset(buf, 0, 2 * 64 * 16));
    CHECK(hipMemset(out, 0, 3 * 8));
    ++salt;
    hipLaunchKernelGGL((pingpong<D, SLEEP>), dim3(stride + 1), dim3(64), 0, 0, buf, n, stride, salt & 0xfff, out);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
    if (h[0] == 0) {
      printf("%-28s stride %d: TIMED OUT\n", name, stride);
      return 0;
    }
    ns.push_back(h[0] * 10.0 / (2.0 * n));  // s_memrealtime: 100 MHz
  }
  std::sort(ns.begin(), ns.end());
  printf("%-28s %s (XCC %llu -> %llu): %7.1f ns per hop (min %.1f, max %.1f)\n", name,
         stride == 8 ? "same XCD " : "cross XCD", h[1], h[2], ns[2], ns[0], ns[4]);
  return 0;
}

int main() {
  u32x4* buf;
  unsigned long long* out;
  CHECK(hipMalloc(&buf, 2 * 64 * 16));
  CHECK(hipMalloc(&out, 3 * 8));
  unsigned salt = 0;
  for (int stride : {8, 1}) {
    if (run<1, 1>("D=1 sleep 1 (current)", buf, out, stride, salt)) return 1;
    if (run<1, 0>("D=1 no sleep", buf, out, stride, salt)) return 1;
    if (run<2, 0>("D=2 pipelined", buf, out, stride, salt)) return 1;
    if (run<4, 0>("D=4 pipelined", buf, out, stride, salt)) return 1;
    if (run<2, 1>("D=2 pipelined sleep 1", buf, out, stride, salt)) return 1;
    if (run<4, 1>("D=4 pipelined sleep 1", buf, out, stride, salt)) return 1;
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
