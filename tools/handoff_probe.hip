// Hand-off latency probe: the one-way store -> poll latency between two persistent waves, the unit
// cost behind every cross-workgroup hand-off of the chain kernels (a per-worker phase waits for one,
// the blocked kernel's halo exchange is one per k iterations, an xGMI boundary hop is one between
// GPUs). Two single-wave workgroups ping-pong a counter `rounds` times; one-way = round trip / 2.
//
// Placement: workgroup b of a launch lands on XCD b mod 8 (round-robin dispatch; checked with
// HW_REG_XCC_ID and reported). Pairs: blocks (0, 8) share XCD 0, blocks (0, 1) sit on XCDs 0 and 1.
// Store flavours (vector stores by all 64 lanes, one 256-B line):
//   mode 0: workgroup-scope stores (sc0; the line stays in the writer's L2: visible on the same XCD)
//   mode 1: sc1 stores (write-through past L2, what the chain kernels use across XCDs)
// Loads are sc1 (L1-bypassing) polls. Every poll has a deadline, so a run never hangs.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/handoff_probe tools/handoff_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ unsigned long long now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void put(int* p, int v, int mode) {
  if (mode == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int get(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// line[0..63]: ping (a -> b), line[64..127]: pong (b -> a); out: [0] ticks, [1] rounds done, [2..3] XCC ids
__global__ void __launch_bounds__(64) probe(int* line, long long* out, int a, int b, int rounds, int mode) {
  const int bid = blockIdx.x, lane = threadIdx.x;
  if (bid != a && bid != b) return;
  const int xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // HW_REG_XCC_ID[3:0]
  if (lane == 0) out[bid == a ? 2 : 3] = xcc;
  int* ping = line + lane;
  int* pong = line + 64 + lane;
  const unsigned long long deadline = now_ticks() + 200000000ull;  // 2 s at 100 MHz
  const unsigned long long t0 = now_ticks();
  int done = 0;
  bool ok = true;
  for (int r = 1; r <= rounds && ok; ++r) {
    if (bid == a) {
      put(ping, r, mode);
      while (!__all(get(pong) == r)) {
        if (now_ticks() > deadline) { ok = false; break; }
      }
    } else {
      while (!__all(get(ping) == r)) {
        if (now_ticks() > deadline) { ok = false; break; }
      }
      if (ok) put(pong, r, mode);
    }
    if (ok) done = r;
  }
  if (bid == a && lane == 0) {
    out[0] = (long long)(now_ticks() - t0);
    out[1] = done;
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 20000;
  int* line;
  long long* out;
  if (hipMalloc(&line, 128 * sizeof(int)) != hipSuccess || hipMalloc(&out, 4 * sizeof(long long)) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  struct Case { int a, b, mode; const char* what; };
  const Case cases[] = {{0, 8, 0, "same XCD, wg-scope stores"},
                        {0, 8, 1, "same XCD, sc1 stores"},
                        {0, 1, 1, "across XCDs, sc1 stores"}};
  int rc = 0;
  for (const Case& c : cases) {
    for (int rep = 0; rep < 2; ++rep) {
      hipMemset(line, 0, 128 * sizeof(int));
      hipMemset(out, 0, 4 * sizeof(long long));
      hipLaunchKernelGGL(probe, dim3(16), dim3(64), 0, 0, line, out, c.a, c.b, rounds, c.mode);
      if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 1;
      }
      long long h[4];
      hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
      if (rep == 0) continue;  // warm-up
      const double us = h[1] > 0 ? (double)h[0] * 1e-2 / (2.0 * h[1]) : -1.0;  // 100 MHz ticks -> us
      printf("%-30s blocks (%d, %d) on XCC %lld / %lld: %lld rounds, one-way %.3f us\n", c.what, c.a, c.b, h[2], h[3],
             h[1], us);
      if (h[1] != rounds) rc = 2;
    }
  }
  return rc;
}
