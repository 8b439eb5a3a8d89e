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
#include <stdlib.h>

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

// d <= 64: 4 waves, thread (rb, j) owns column j of the rows i = rb (mod 4); no integer division and
// two barriers per pivot (pivot row scaled by wave 0 | rank-1 update + pivot column, each wave on
// its own rows, reading M[i][k] before any write). Same per-element arithmetic as
// spd_inverse_gj_kernel (fma(-a_ik, m_kj, m_ij), the same 1/p scalings), hence bit-identical, at
// ~1/5 of the time (profiles/r01b_e1q: 57 us for the 24 E1 inverses in the general kernel).
__global__ void __launch_bounds__(256)
spd_inverse_gj64_kernel(const double* __restrict__ A, const double* __restrict__ shift, int d, int nvar,
                        double* __restrict__ out, int* __restrict__ status) {
  __shared__ double M[64 * 64];
  __shared__ double piv_s;
  const int n = blockIdx.x, v = blockIdx.y;
  const double s = shift[n * nvar + v];
  const double* An = A + (long)n * d * d;
  const int j = threadIdx.x & 63, rb = threadIdx.x >> 6;
  const bool inj = j < d;
  for (int i = rb; i < d; i += 4)
    if (inj) M[i * d + j] = An[i * d + j] + (i == j ? s : 0.0);
  __syncthreads();
  for (int k = 0; k < d; ++k) {
    if (rb == 0) {  // pivot row k scaled by 1/M[k][k] (wave 0)
      const double pk = M[k * d + k];
      const double p = 1.0 / pk;
      if (j == 0) {
        if (!(pk > 0.0) && status) atomicExch(status, 1);  // not SPD (or NaN)
        piv_s = p;
      }
      if (inj && j != k) M[k * d + j] *= p;
    }
    __syncthreads();
    const double p = piv_s;
    const double mkj = inj ? M[k * d + j] : 0.0;
    // this wave's rows: read the pivot-column entries first (lane k rewrites them below)
    double aik[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = rb + 4 * q;
      aik[q] = i < d ? M[i * d + k] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int i = rb + 4 * q;
      if (i < d && inj) {
        if (j == k) M[i * d + k] = (i == k) ? p : -aik[q] * p;
        else if (i != k) M[i * d + j] -= aik[q] * mkj;
      }
    }
    __syncthreads();
  }
  double* o = out + ((long)n * nvar + v) * d * d;
  for (int i = rb; i < d; i += 4)
    if (inj) o[i * d + j] = 0.5 * (M[i * d + j] + M[j * d + i]);
}

// d <= 64, register rows: lane i of wave w keeps M[i][j] for j = w + 4c (c < 16) in VGPRs. Per
// pivot k the owner wave of column k publishes it to LDS (one barrier); every lane reads M[i][k] and
// M[k][k], takes row k of its own wave's columns from lane k by v_readlane, and updates its 16
// entries in registers. The per-element arithmetic is exactly spd_inverse_gj_kernel's (p = 1/m_kk,
// m_kj p, fma(-a_ik, m_kj p, m_ij), -a_ik p), so the result is bit-identical, with no LDS matrix
// traffic and one barrier per pivot instead of two plus 32 LDS accesses per lane.
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int NW>  // waves; lane i of wave w keeps columns j = w + NW c (c < 64 / NW)
__global__ void __launch_bounds__(64 * NW)
spd_inverse_reg64_kernel(const double* __restrict__ A, const double* __restrict__ shift, int d, int nvar,
                         double* __restrict__ out, int* __restrict__ status) {
  constexpr int NC = 64 / NW;
  __shared__ double Ms[64 * 65];    // the result, for the symmetrised write-out
  __shared__ double colv[2][65];    // the pivot column + [64] its reciprocal pivot, double-buffered
  const int n = blockIdx.x, v = blockIdx.y;
  const double s = shift[n * nvar + v];
  const double* An = A + (long)n * d * d;
  const int i = threadIdx.x & 63, w = threadIdx.x >> 6;
  double h[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int j = w + NW * c;
    h[c] = (i < d && j < d) ? An[i * d + j] + (i == j ? s : 0.0) : 0.0;
  }
  if (w == 0) {
    colv[0][i] = h[0];
    const double p0 = 1.0 / readlane_f64(h[0], 0);
    if (i == 0) colv[0][64] = p0;
  }
  __syncthreads();
  bool bad = false;  // a non-positive (or NaN) pivot: reported once after the loop
  for (int k = 0; k < d; ++k) {
    const double* cb = colv[k & 1];
    // the reciprocal pivot comes with the column: the owner wave divided while the others updated
    const double pk = cb[k], aik = cb[i], p = cb[64];
    bad |= !(pk > 0.0);  // not SPD (or NaN)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int j = w + NW * c;
      const double mkj = readlane_f64(h[c], k) * p;  // row k, scaled (lane k of this wave)
      double val = h[c];
      if (j == k) val = (i == k) ? p : -aik * p;
      else if (i == k) val = mkj;
      else val -= aik * mkj;
      h[c] = val;
    }
    const int kn = k + 1;
    if (kn < d && w == kn % NW) {  // owner of the next pivot column publishes it
      double nxt = 0.0;
#pragma unroll
      for (int c = 0; c < NC; ++c) nxt = (c == kn / NW) ? h[c] : nxt;
      colv[kn & 1][i] = nxt;
      const double pn = 1.0 / readlane_f64(nxt, kn);  // == every lane's old 1.0 / pk (bit-identical)
      if (i == 0) colv[kn & 1][64] = pn;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && bad && status) atomicExch(status, 1);
#pragma unroll
  for (int c = 0; c < NC; ++c) Ms[i * 65 + w + NW * c] = h[c];
  __syncthreads();
  double* o = out + ((long)n * nvar + v) * d * d;
  for (int r = w; r < d; r += NW)
    if (i < d) o[r * d + i] = 0.5 * (Ms[r * 65 + i] + Ms[i * 65 + r]);
}

}  // namespace

extern "C" int gadmm_spd_inverse_small_f64(const double* A, const double* shift, int N, int d, int nvar,
                                           double* out, int* status, hipStream_t st) {
  if (d > 128) {
    gadmm_set_error("spd_inverse_small: d=%d > 128 (use the blocked path)", d);
    return -1;
  }
  if (N <= 0) return 0;
  const char* gje = getenv("GADMM_GJ64");  // A/B switch (read per call: set-up only)
  const bool gj64 = !(gje && gje[0] == '0');
  // GADMM_INV_REG=0: the LDS 64-wide kernel (the tests' bit-identity cross-check). 8 waves per matrix:
  // 4 and 16 measured 35.3 / 32.0 vs 29.3 us for the headline's 24 x 2 inverses (profiles/r06_final/inv_p2)
  const char* rge = getenv("GADMM_INV_REG");
  const bool reg = !(rge && rge[0] == '0');
  if (d <= 64 && gj64 && reg) {
    hipLaunchKernelGGL(spd_inverse_reg64_kernel<8>, dim3(N, nvar), dim3(512), 0, st, A, shift, d, nvar, out, status);
    GADMM_CHECK(hipGetLastError());
    return 0;
  }
  if (d <= 64 && gj64) {
    hipLaunchKernelGGL(spd_inverse_gj64_kernel, dim3(N, nvar), dim3(256), 0, st, A, shift, d, nvar, out, status);
    GADMM_CHECK(hipGetLastError());
    return 0;
  }
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

// ---- test entry: the split-column quad GEMV (quad_gemv.h) on a batch of matrices ----------------
// y[b] = M[b] x[b] for row-major M[b] (rows x cols, both <= 64), one wave per matrix: lets the test
// suite check the device function every persistent kernel uses against a torch reference.
#include "quad_gemv.h"

namespace {
template <int T>
__global__ void __launch_bounds__(64) quad_gemv_test_kernel(const double* M, const double* x, double* y, int rows,
                                                            int cols) {
  __shared__ __attribute__((aligned(16))) double st[QSTAGE];
  const int b = blockIdx.x, lane = threadIdx.x;
  const double* Mb = M + (long)b * rows * cols;
  double m[4][T];
  const int i = lane & 15, c = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int row = i + 16 * r, col = c + 4 * t;
      m[r][t] = (row < rows && col < cols) ? Mb[(long)row * cols + col] : 0.0;
    }
  const double xv = lane < cols ? x[(long)b * cols + lane] : 0.0;
  const double v = quad_gemv<T>(m, xv, st);
  if (lane < rows) y[(long)b * rows + lane] = v;
}
}  // namespace

extern "C" int gadmm_quad_gemv_test(const double* M, const double* x, double* y, int batch, int rows, int cols,
                                    hipStream_t st) {
  if (rows < 1 || rows > 64 || cols < 1 || cols > 64 || batch < 1) {
    gadmm_set_error("quad_gemv_test: rows/cols must be in [1, 64]");
    return -1;
  }
  if (cols <= 32) hipLaunchKernelGGL(quad_gemv_test_kernel<8>, dim3(batch), dim3(64), 0, st, M, x, y, rows, cols);
  else if (cols <= 52) hipLaunchKernelGGL(quad_gemv_test_kernel<13>, dim3(batch), dim3(64), 0, st, M, x, y, rows, cols);
  else hipLaunchKernelGGL(quad_gemv_test_kernel<16>, dim3(batch), dim3(64), 0, st, M, x, y, rows, cols);
  GADMM_CHECK(hipGetLastError());
  return 0;
}
