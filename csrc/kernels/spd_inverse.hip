// Batched SPD inverse (A_n + s_{n,v} I)^{-1} for small d (<= 128), one workgroup per matrix.
//
// Kernel K2 of SURVEY.md §2.5, option "factor once, apply every iteration": the reference solves
// (H^T H + c rho I) x = r from scratch with LAPACK `\` in every local update
// (group_ADMM_closedForm.m:43,45,82,84; standared_ADMM.m:42,73). The shifted Gram is
// loop-invariant, so the framework inverts it once per (worker, degree c) and each iteration is one
// symmetric GEMV (gadmm_phase kernel). Several shifts per worker (`nvar`) cover the two chain
// degrees (end / middle) that D-GADMM re-chaining switches between, and the (N-1) rho hub of the
// star ADMM.
//
// Algorithm: in-LDS Gauss-Jordan without pivoting (backward stable for SPD matrices, same growth
// bound as Cholesky), 3 barriers per pivot, then symmetrised write-out so that consumers may read
// columns as rows (the coalesced symmetric-GEMV trick).
#include "gadmm_common.h"

namespace {

__global__ void __launch_bounds__(1024)
spd_inverse_gj_kernel(const double* __restrict__ A, const double* __restrict__ shift, int d,
                      int nvar, double* __restrict__ out, int* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) double M[];  // d x d (row stride d)
  __shared__ double piv_s;
  const int n = blockIdx.x, v = blockIdx.y;
  const double s = shift[n * nvar + v];
  const double* An = A + (long)n * d * d;
  const int dd = d * d;
  for (int e = threadIdx.x; e < dd; e += blockDim.x) {
    const int i = e / d, j = e % d;
    M[e] = An[e] + (i == j ? s : 0.0);
  }
  __syncthreads();
  for (int k = 0; k < d; ++k) {
    if (threadIdx.x == 0) {
      const double pk = M[k * d + k];
      if (!(pk > 0.0) && status) atomicExch(status, 1);  // not SPD (or NaN)
      piv_s = 1.0 / pk;
    }
    __syncthreads();
    const double p = piv_s;
    for (int j = threadIdx.x; j < d; j += blockDim.x)
      if (j != k) M[k * d + j] *= p;
    __syncthreads();
    for (int e = threadIdx.x; e < dd; e += blockDim.x) {
      const int i = e / d, j = e % d;
      if (i != k && j != k) M[e] -= M[i * d + k] * M[k * d + j];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < d; i += blockDim.x) M[i * d + k] = (i == k) ? p : -M[i * d + k] * p;
    __syncthreads();
  }
  double* o = out + ((long)n * nvar + v) * dd;
  for (int e = threadIdx.x; e < dd; e += blockDim.x) {
    const int i = e / d, j = e % d;
    o[e] = 0.5 * (M[e] + M[j * d + i]);
  }
}

}  // namespace

extern "C" int gadmm_spd_inverse_small_f64(const double* A, const double* shift, int N, int d, int nvar,
                                           double* out, int* status, hipStream_t st) {
  if (d > 128) {
    gadmm_set_error("spd_inverse_small: d=%d > 128 (use the blocked path)", d);
    return -1;
  }
  if (N <= 0) return 0;
  const size_t lds = (size_t)d * d * sizeof(double);
  const int threads = d <= 32 ? 256 : 1024;
  if (lds > 65536)
    GADMM_CHECK(hipFuncSetAttribute((const void*)spd_inverse_gj_kernel,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(spd_inverse_gj_kernel, dim3(N, nvar), dim3(threads), lds, st, A, shift, d, nvar, out,
                     status);
  GADMM_CHECK(hipGetLastError());
  return 0;
}
