// Row-per-wave HBM-streaming f64 GEMV shared by the large-d kernels (d > 256: the 10M x 10k
// "LinearRegression_Real-shaped" config): chain_big.hip (GADMM phases) and star_big.hip (star ADMM).
// Each wave owns RPW consecutive rows of a row-major d x d matrix and streams them with 16-byte loads
// (one contiguous 1-KiB wave access per row chunk); the reduction stays inside the wave (no split-K),
// so results are deterministic and identical between the kernels that share it.
#pragma once
#include "gadmm_common.h"
#include "sym_gemv.h"

namespace biggemv {

constexpr int NT = 256;
constexpr int RPW = 2;  // rows per wave
constexpr int ROWS_PER_WG = RPW * (NT / 64);

// A worker's r-buffer (large-d kernels): [ r, zero padded to symv::padded(d) | one objective partial per
// row-GEMV workgroup + 1 | two partials per symmetric-GEMV block row (objective, primal residual: the
// reduce kernels' fused elementwise tails) | the symmetric GEMV's partial table P (symv::part_doubles) ].
// The padding stays zero (allocated zeroed, only r[0, d) is ever written): the packed GEMV reads whole
// blocks of r.
__device__ __host__ __forceinline__ long obj_off(int d) { return symv::padded(d); }
__device__ __host__ __forceinline__ long fz_off(int d) { return obj_off(d) + (d + ROWS_PER_WG - 1) / ROWS_PER_WG + 1; }
__device__ __host__ __forceinline__ long part_off(int d) { return (fz_off(d) + 2L * symv::nblk(d) + 31) / 32 * 32; }
__device__ __host__ __forceinline__ long rstride(int d) { return part_off(d) + symv::part_doubles(d); }

// y[row] = sum_j M[row][j] x[j] for RPW consecutive rows per wave; returns sums on lane 0.
__device__ __forceinline__ void wave_rows_dot(const double* __restrict__ M, const double* __restrict__ x, int d,
                                              int row0, double (&out)[RPW]) {
  const int lane = threadIdx.x & 63;
  double acc[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) acc[r] = 0.0;
  if ((d & 1) == 0) {
    const double2* x2 = reinterpret_cast<const double2*>(x);
    const int d2 = d >> 1;
    for (int j = lane; j < d2; j += 64) {
      const double2 xv = x2[j];
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        if (row0 + r < d) {
          const double2 mv = reinterpret_cast<const double2*>(M + (long)(row0 + r) * d)[j];
          acc[r] = fma(mv.x, xv.x, fma(mv.y, xv.y, acc[r]));
        }
      }
    }
  } else {
    for (int j = lane; j < d; j += 64) {
      const double xv = x[j];
#pragma unroll
      for (int r = 0; r < RPW; ++r)
        if (row0 + r < d) acc[r] = fma(M[(long)(row0 + r) * d + j], xv, acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) out[r] = wave_sum_f64(acc[r]);
}

}  // namespace biggemv
