// Probe: do f64 MFMA (v_mfma_f64_16x16x4_f64) and f64 VALU FMA (v_fma_f64) issue concurrently on
// gfx950? Each 512-thread workgroup runs 8 waves (two per SIMD); mode 0: every wave runs MFMA
// chains, mode 1: every wave runs VALU FMA chains, mode 2: waves 0-3 MFMA + waves 4-7 VALU (one of
// each per SIMD). If mode 2's combined flop rate exceeds both single-pipe rates, a Gram kernel can
// put part of each tile on the VALU. Build: hipcc --offload-arch=gfx950 -O3 -o build/f64_pipe_probe
// tools/f64_pipe_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(512) probe(double* out, int iters, double s) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool mfma = MODE == 0 || (MODE == 2 && wid < 4);
  double acc_out = 0.0;
  if (mfma) {
    f64x4 c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = f64x4{0.0, 0.0, 0.0, 0.0};
    double a = s + lane * 1e-3, b = s - lane * 1e-3;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc_out += c[k][0] + c[k][1] + c[k][2] + c[k][3];
  } else {
    double v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = lane * 1e-3 + k;
    const double a = s, b = 1.0 - s;
    // 16 FMAs per MFMA (1024 FMAs) / 64 lanes: one MFMA-equivalent of work = 16 wave FMAs
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = fma(v[k], a, b);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) acc_out += v[k];
  }
  out[blockIdx.x * 512 + threadIdx.x] = acc_out;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4096;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int blocks = cus * 2;
  double* out;
  hipMalloc(&out, (size_t)blocks * 512 * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 3; ++mode) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(512), 0, 0, out, iters, 0.5);
      if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(512), 0, 0, out, iters, 0.5);
      if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(512), 0, 0, out, iters, 0.5);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0 && ms < best) best = ms;
    }
    // every wave does iters * 8 MFMA-equivalents = iters * 8 * 2048 flops
    const double flops = (double)blocks * 8 * iters * 8 * 2048.0;
    printf("mode %d (%s): %.3f ms, %.1f TF/s\n", mode, mode == 0 ? "all MFMA" : mode == 1 ? "all VALU" : "MFMA+VALU",
           best, flops / (best * 1e-3) / 1e12);
  }
  hipError_t err = hipGetLastError();
  printf("status: %s\n", hipGetErrorString(err));
  return err == hipSuccess ? 0 : 1;
}
