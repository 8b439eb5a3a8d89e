// MFMA issue-rate probe: cycles per instruction (s_memtime, per wave) of back-to-back independent MFMAs
// with register operands, for the shapes the Gram kernels use -- v_mfma_i32_32x32x32_i8 (Ozaki digit
// pairs), v_mfma_f32_32x32x16_bf16 (the reference rate) and v_mfma_f64_16x16x4_f64 (the f64 Gram) --
// at 1 and 2 waves per SIMD. Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_rate.hip -o mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef double v4d __attribute__((ext_vector_type(4)));

constexpr int ITERS = 4096;

template <int KIND>
__global__ void __launch_bounds__(256) probe(const int* seed, long long* cyc, int* sink) {
  const int l = threadIdx.x;
  long long t0 = 0, t1 = 0;
  if constexpr (KIND == 0) {
    v4i a = {seed[l & 7], seed[(l + 1) & 7], seed[(l + 2) & 7], seed[(l + 3) & 7]}, b = a;
    v16i c0 = {}, c1 = {}, c2 = {}, c3 = {};
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
      c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c3, 0, 0, 0);
    }
    t1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * 256 + l] = c0[0] + c1[1] + c2[2] + c3[3];
  } else if constexpr (KIND == 3) {  // one dependent i8 accumulation chain
    v4i a = {seed[l & 7], seed[(l + 1) & 7], seed[(l + 2) & 7], seed[(l + 3) & 7]}, b = a;
    v16i c0 = {};
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
      for (int k = 0; k < 4; ++k) c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
    }
    t1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * 256 + l] = c0[0];
  } else if constexpr (KIND == 4) {  // the Ozaki level pattern: 28 digit pairs into 7 level accumulators
    v4i f[7];
#pragma unroll
    for (int p = 0; p < 7; ++p) f[p] = v4i{seed[(l + p) & 7], seed[(l + p + 1) & 7], seed[(l + 2) & 7], p};
    v16i acc[7] = {};
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS / 7; ++i) {
#pragma unroll
      for (int p = 0; p < 7; ++p)
#pragma unroll
        for (int q = 0; q < 7 - p; ++q) acc[p + q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(f[p], f[q], acc[p + q], 0, 0, 0);
    }
    t1 = __builtin_amdgcn_s_memtime();
    int v = 0;
#pragma unroll
    for (int p = 0; p < 7; ++p) v += acc[p][p];
    sink[blockIdx.x * 256 + l] = v;
  } else if constexpr (KIND == 1) {
    v8bf a, b;
    for (int j = 0; j < 8; ++j) a[j] = b[j] = (__bf16)(float)(seed[(l + j) & 7] & 3);
    v16f c0 = {}, c1 = {}, c2 = {}, c3 = {};
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
    }
    t1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * 256 + l] = (int)(c0[0] + c1[1] + c2[2] + c3[3]);
  } else {
    double a = seed[l & 7] * 0.5, b = a;
    v4d c0 = {}, c1 = {}, c2 = {}, c3 = {};
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    t1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * 256 + l] = (int)(c0[0] + c1[1] + c2[2] + c3[3]);
  }
  if (l % 64 == 0) cyc[blockIdx.x * 4 + l / 64] = t1 - t0;
}

template <int KIND>
void run(const char* name, double ops_per_mfma, int blocks_per_cu) {
  int dev = 0, ncu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int nb = ncu * blocks_per_cu;
  int* seed;
  long long* cyc;
  int* sink;
  (void)hipMalloc(&seed, 8 * sizeof(int));
  (void)hipMalloc(&cyc, (size_t)nb * 4 * sizeof(long long));
  (void)hipMalloc(&sink, (size_t)nb * 256 * sizeof(int));
  std::vector<int> h = {1, 2, 3, 4, 5, 6, 7, 8};
  if (getenv("RATE_RANDOM")) {  // full-toggle operands (random bytes): the power-limited rate
    unsigned x = 12345;
    for (int& v : h) {
      x = x * 1664525u + 1013904223u;
      v = (int)(x ^ (x >> 13)) | 0x01010101;
    }
  }
  (void)hipMemcpy(seed, h.data(), 32, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  probe<KIND><<<nb, 256>>>(seed, cyc, sink);  // warm-up (clock ramp)
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) probe<KIND><<<nb, 256>>>(seed, cyc, sink);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> c(nb * 4);
  (void)hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
  double avg = 0;
  for (long long v : c) avg += (double)v;
  avg /= c.size();
  const double mfmas = KIND == 4 ? 28.0 * (ITERS / 7) : 4.0 * ITERS;
  const double tops = 5.0 * nb * 4 * mfmas * ops_per_mfma / (ms * 1e-3) / 1e12;
  printf("%-28s waves/SIMD %d: %.1f memtime ticks per MFMA per wave, %.0f TOPS (%.3f ms / 5 launches)\n", name,
         blocks_per_cu, avg / mfmas, tops, ms);
  (void)hipFree(seed);
  (void)hipFree(cyc);
  (void)hipFree(sink);
}

int main() {
  for (int w = 1; w <= 2; ++w) {
    run<0>("i32_32x32x32_i8", 2.0 * 32 * 32 * 32, w);
    run<1>("f32_32x32x16_bf16", 2.0 * 32 * 32 * 16, w);
    run<2>("f64_16x16x4_f64", 2.0 * 16 * 16 * 4, w);
    run<3>("i8 one dependent chain", 2.0 * 32 * 32 * 32, w);
    run<4>("i8 Ozaki 28-pair pattern", 2.0 * 32 * 32 * 32, w);
  }
  return 0;
}
