// Probe: latency of one dependent quad GEMV step (the d <= 64 register GEMV of every persistent chain
// kernel, quad_gemv.h) with the iterate broadcast through LDS (quad_gemv: one ds_write + T/2
// ds_read_b128) against a DPP broadcast (v_mov_b64_dpp row_newbcast: the iterate kept in the permuted
// lane layout "element c + 4 t in lane 16 c + t", the matrix rows permuted so the reduced result lands
// in that layout again: no LDS at all). One wave runs `iters` dependent steps x <- s * (M x); the
// probe prints ns per step from s_memrealtime and checks both variants produce the same bits.
// Build: hipcc --offload-arch=gfx950 -O3 -I csrc/include -o build/gemv_bcast_probe tools/gemv_bcast_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "quad_gemv.h"

constexpr int T = 13;
constexpr int D = 50;

template <int t>
__device__ __forceinline__ double bcast(double x) {
  return __builtin_amdgcn_update_dpp(0.0, x, 0x150 + t, 0xf, 0xf, false);
}
template <int t>
__device__ __forceinline__ void fma_col(const double (&m)[4][T], double x, double (&p)[4]) {
  if constexpr (t < T) {
    const double xb = bcast<t>(x);
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = fma(m[r][t], xb, p[r]);
    fma_col<t + 1>(m, x, p);
  }
}

__global__ void __launch_bounds__(64) probe(const double* M, const double* x0, double* out, long long* ticks,
                                            int iters, int mode, double s) {
  __shared__ double st[QSTAGE];
  const int lane = threadIdx.x, i = lane & 15, c = lane >> 4;
  double m[4][T];
  // mode 0: quad layout (lane (i, c): rows i + 16 r, columns c + 4 t), natural vector layout
  // mode 1: rows r + 4 i (the reduced sum of slot i + 16 g lands in lane 16 g + i = element g + 4 i)
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int row = mode != 1 ? i + 16 * r : r + 4 * i, col = c + 4 * t;
      m[r][t] = (row < D && col < D) ? M[row * D + col] : 0.0;
    }
  const int e = mode != 1 ? lane : (lane >> 4) + 4 * (lane & 15);  // this lane's element
  double x = e < D ? x0[e] : 0.0;
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  if (mode == 0) {
    for (int k = 0; k < iters; ++k) x = s * quad_gemv<T>(m, x, st);
  } else if (mode == 2) {  // LDS broadcast, two accumulators per row (even / odd columns): half the chain depth
    const int cc = lane >> 4;
    for (int k = 0; k < iters; ++k) {
      st[(lane & 3) * QX + (lane >> 2)] = x;
      asm volatile("" ::: "memory");
      const double* xs = st + cc * QX;
      double p[4] = {0.0, 0.0, 0.0, 0.0}, q[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int t = 0; t < T; t += 2) {
        const double2 xp = *reinterpret_cast<const double2*>(xs + t);
#pragma unroll
        for (int r = 0; r < 4; ++r) p[r] = fma(m[r][t], xp.x, p[r]);
        if (t + 1 < T) {
#pragma unroll
          for (int r = 0; r < 4; ++r) q[r] = fma(m[r][t + 1], xp.y, q[r]);
        }
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int r = 0; r < 4; ++r) p[r] += q[r];
      x = s * quad_reduce(p);
    }
  } else {
    for (int k = 0; k < iters; ++k) {
      double p[4] = {0.0, 0.0, 0.0, 0.0};
      fma_col<0>(m, x, p);
      x = s * quad_reduce(p);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memrealtime();
  if (e < D) out[e] = x;
  if (lane == 0) ticks[0] = t1 - t0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 100000;
  double hM[D * D], hx[D];
  srand(1);
  for (int k = 0; k < D * D; ++k) hM[k] = (rand() / (double)RAND_MAX - 0.5) * 0.2;
  for (int k = 0; k < D; ++k) hx[k] = rand() / (double)RAND_MAX;
  double *dM, *dx, *dout;
  long long* dt;
  hipMalloc(&dM, sizeof(hM));
  hipMalloc(&dx, sizeof(hx));
  hipMalloc(&dout, 3 * D * sizeof(double));
  hipMalloc(&dt, sizeof(long long));
  hipMemcpy(dM, hM, sizeof(hM), hipMemcpyHostToDevice);
  hipMemcpy(dx, hx, sizeof(hx), hipMemcpyHostToDevice);
  double res[3][D];
  for (int mode = 0; mode < 3; ++mode) {
    double best = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dM, dx, dout + mode * D, dt, iters, mode, 0.9);
      long long tk = 0;
      hipMemcpy(&tk, dt, sizeof(tk), hipMemcpyDeviceToHost);
      const double ns = tk * 10.0 / iters;  // s_memrealtime: 100 MHz
      if (ns < best) best = ns;
    }
    hipMemcpy(res[mode], dout + mode * D, sizeof(res[mode]), hipMemcpyDeviceToHost);
    printf("%s: %.1f ns per dependent GEMV step (d = %d)\n",
           mode == 0 ? "LDS broadcast (quad_gemv)" : mode == 1 ? "DPP row_newbcast" : "LDS, 2 accumulators per row",
           best, D);
  }
  printf("DPP bit-identical to quad_gemv: %s\n", memcmp(res[0], res[1], sizeof(res[0])) == 0 ? "yes" : "NO");
  double mx = 0.0;
  for (int k = 0; k < D; ++k) mx = fmax(mx, fabs(res[2][k] - res[0][k]) / (fabs(res[0][k]) + 1e-300));
  printf("2-accumulator max rel diff vs quad_gemv: %.2e\n", mx);
  return 0;
}
