// Large-d SPD inverse (A + s I)^{-1} (kernel K2 of SURVEY.md §2.5 for d > 128, e.g. the 10k-feature
// real-shaped config): blocked in-place Gauss-Jordan on the LOWER triangle with NB x NB pivot blocks,
// the rank-NB updates on f64 MFMA. The reference solves (H^T H + c rho I) x = r with LAPACK `\` inside
// every local update (group_ADMM_closedForm.m:43,45); the shifted Gram is loop-invariant, so the
// framework inverts it once per (worker, degree) and every iteration is one GEMV (chain_big.hip).
//
// In-place Gauss-Jordan on a symmetric matrix keeps a fixed structure: with P = processed and
// U = unprocessed indices, W_PP and W_UU are symmetric and W_UP = -W_PU^T. So the lower triangle
// determines everything, and the column panel of pivot block K = [k0, k0 + nb) is
//   C_i = W_iK  (i > K: stored),   C_i = -W_Ki^T  (i < k0: stored in block row K),
// while the row panel is W_Kj = sgn_j C_j^T (sgn = -1 for processed j < k0, +1 for j > K). Step K:
//   1. C (d x nb) gathered from the lower triangle; P = W_KK; Pi = P^-1 (nb = 64: the in-register small
//      inverse of spd_inverse.hip; nb = 128: this routine recursively with 64-blocks)
//   2. Lc = C Pi                                                             [MFMA GEMM, d x nb x nb]
//   3. lower tiles I >= J off K:  W_IJ -= sgn_J Lc_I C_J^T                   [MFMA rank-nb update]
//   4. the K cross: W_iK = -Lc_i (i > K),  W_Kj = -Lc_j^T (j < k0),  W_KK = Pi
// then the lower triangle is mirrored. Half the tiles of the full-matrix form, and at nb = 128 the
// update does 16 flops per byte of W it streams.
//
// GEMM tile: 256 threads (4 waves, 2 x 2), a 64 x 64 output tile per workgroup, each wave 32 x 32 as
// 2 x 2 v_mfma_f64_16x16x4_f64 tiles; K staged through LDS in chunks of 16 (A as [k][i], B as [k][j],
// rows padded by 4 doubles), the next chunk fetched into registers while the current one issues.
#include "gadmm_common.h"
#include <stdlib.h>
#include <mutex>

extern "C" int gadmm_spd_inverse_small_f64(const double* A, const double* shift, int N, int d, int nvar,
                                           double* out, int* status, hipStream_t st);

namespace {

constexpr int GT = 64;        // output tile
constexpr int GK = 16;        // K chunk
constexpr int GLD = GT + 4;   // LDS row stride (doubles)
constexpr int GNT = 256;

// MODE 0: C (M x N) = A (M x K) B (K x N), row-major with leading dimensions.
// MODE 1 (the Gauss-Jordan update, square M = N = d): B is read TRANSPOSED (B[j][k], ldb), only tiles
// on or below the diagonal and off the pivot block [s0, s1) are touched: C -= sgn_J A B^T with
// sgn_J = -1 for column tiles left of s0.
template <int MODE>
__global__ void __launch_bounds__(GNT) gemm_f64_kernel(int M, int N, int K, const double* __restrict__ A, int lda,
                                                      const double* __restrict__ B, int ldb, double* C, int ldc,
                                                      int s0, int s1) {
  __shared__ __attribute__((aligned(16))) double As[2][GK * GLD];
  __shared__ __attribute__((aligned(16))) double Bs[2][GK * GLD];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int row0 = blockIdx.y * GT, col0 = blockIdx.x * GT;
  if (MODE == 1 && (col0 > row0 || (row0 >= s0 && row0 < s1) || (col0 >= s0 && col0 < s1))) return;
  // per-thread staging: A chunk (64 rows x 16 k) and B chunk (16 k x 64 cols), 4 elements each
  double ra[4], rb[4];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int e = tid + GNT * p;
      {  // A[row0 + i][k0 + k]: e -> (i = e / 16, k = e % 16)
        const int i = e >> 4, k = e & 15;
        const int r = row0 + i, kk = k0 + k;
        ra[p] = (r < M && kk < K) ? A[(long)r * lda + kk] : 0.0;
      }
      if (MODE == 0) {  // B[k0 + k][col0 + j]: e -> (k = e / 64, j = e % 64)
        const int k = e >> 6, j = e & 63;
        const int kk = k0 + k, c = col0 + j;
        rb[p] = (kk < K && c < N) ? B[(long)kk * ldb + c] : 0.0;
      } else {  // B^T: B[col0 + j][k0 + k], e -> (j = e / 16, k = e % 16)
        const int j = e >> 4, k = e & 15;
        const int c = col0 + j, kk = k0 + k;
        rb[p] = (c < N && kk < K) ? B[(long)c * ldb + kk] : 0.0;
      }
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int e = tid + GNT * p;
      As[buf][(e & 15) * GLD + (e >> 4)] = ra[p];
      if (MODE == 0) Bs[buf][(e >> 6) * GLD + (e & 63)] = rb[p];
      else Bs[buf][(e & 15) * GLD + (e >> 4)] = rb[p];
    }
  };
  f64x4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = f64x4{0.0, 0.0, 0.0, 0.0};
  fetch(0);
  stash(0);
  __syncthreads();
  int cur = 0;
  for (int k0 = 0; k0 < K; k0 += GK) {
    const bool more = k0 + GK < K;
    if (more) fetch(k0 + GK);
    const double* a_s = As[cur];
    const double* b_s = Bs[cur];
#pragma unroll
    for (int ks = 0; ks < GK / 4; ++ks) {
      const int kr = ks * 4 + (lane >> 4);
      double av[2], bv[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) av[x] = a_s[kr * GLD + wr * 32 + x * 16 + (lane & 15)];
#pragma unroll
      for (int y = 0; y < 2; ++y) bv[y] = b_s[kr * GLD + wc * 32 + y * 16 + (lane & 15)];
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[x], bv[y], acc[x][y], 0, 0, 0);
    }
    if (more) stash(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  const double sg = (MODE == 1 && col0 < s0) ? -1.0 : 1.0;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int r = row0 + wr * 32 + x * 16 + (lane >> 4) + 4 * reg;  // f64 MFMA D layout
        const int c = col0 + wc * 32 + y * 16 + (lane & 15);
        if (r >= M || c >= N) continue;
        double* cp = C + (long)r * ldc + c;
        *cp = MODE == 0 ? acc[x][y][reg] : fma(-sg, acc[x][y][reg], *cp);
      }
}

// W = A_n + s I (copy with shift)
__global__ void shift_copy_kernel(const double* __restrict__ A, double s, int d, double* __restrict__ W) {
  const long n = (long)d * d;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const long i = e / d, j = e - i * d;
    W[e] = A[e] + (i == j ? s : 0.0);
  }
}

// P = W_KK from the lower triangle (nb x nb, contiguous, symmetric); C = the column panel
__global__ void panel_kernel(const double* __restrict__ W, int d, int k0, int nb, double* __restrict__ P,
                             double* __restrict__ C) {
  const long n = (long)d * nb;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int i = (int)(e / nb), q = (int)(e - (long)i * nb);
    double v = 0.0;
    if (i < k0) v = -W[(long)(k0 + q) * d + i];
    else if (i >= k0 + nb) v = W[(long)i * d + k0 + q];
    else {
      const int r = i - k0, hi = r > q ? r : q, lo = r > q ? q : r;
      P[r * nb + q] = W[(long)(k0 + hi) * d + k0 + lo];
    }
    C[e] = v;
  }
}

// the K cross: W_iK = -Lc_i (i > K), W_Kj = -Lc_j^T (j < k0), W_KK = Pi
__global__ void cross_kernel(double* __restrict__ W, int d, int k0, int nb, const double* __restrict__ Lc,
                             const double* __restrict__ Pi) {
  const long n = (long)d * nb;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const int i = (int)(e / nb), q = (int)(e - (long)i * nb);
    if (i < k0) W[(long)(k0 + q) * d + i] = -Lc[e];
    else if (i >= k0 + nb) W[(long)i * d + k0 + q] = -Lc[e];
    else W[(long)i * d + k0 + q] = Pi[(i - k0) * nb + q];
  }
}

// upper triangle = lower triangle
__global__ void mirror_kernel(double* W, int d) {
  const long n = (long)d * d;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    const long i = e / d, j = e - i * d;
    if (j > i) W[e] = W[j * d + i];
  }
}

int gemm_launch(int mode, int M, int N, int K, const double* A, int lda, const double* B, int ldb, double* C, int ldc,
                int s0, int s1, hipStream_t st) {
  const dim3 grid((N + GT - 1) / GT, (M + GT - 1) / GT);
  if (mode == 0) hipLaunchKernelGGL(gemm_f64_kernel<0>, grid, dim3(GNT), 0, st, M, N, K, A, lda, B, ldb, C, ldc, s0, s1);
  else hipLaunchKernelGGL(gemm_f64_kernel<1>, grid, dim3(GNT), 0, st, M, N, K, A, lda, B, ldb, C, ldc, s0, s1);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

inline int grid_for(long n) { return (int)((n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536); }

long ws_doubles(int d, int nb) {
  const long own = 2L * nb * nb + 2L * d * nb + 8;
  return nb > 64 ? own + ws_doubles(nb, 64) : own;
}

// In place: W (d x d, full) -> W^-1 (full, symmetric). ws: ws_doubles(d, nb), ws[zero] = 0.
int blocked_inplace(double* W, int d, int nb, double* ws, int* status, hipStream_t st) {
  // layout: [zero(8) | P | Pi | C | Lc | inner level]; the zero slot (the small inverse's shift) sits at
  // a fixed offset no call ever writes: C / Lc extents depend on the (recursive) call's d
  double* zero = ws;
  double* P = zero + 8;
  double* Pi = P + (long)nb * nb;
  double* C = Pi + (long)nb * nb;
  double* Lc = C + (long)d * nb;
  double* inner = Lc + (long)d * nb;
  for (int k0 = 0; k0 < d; k0 += nb) {
    const int b = d - k0 < nb ? d - k0 : nb;
    hipLaunchKernelGGL(panel_kernel, dim3(grid_for((long)d * b)), dim3(256), 0, st, W, d, k0, b, P, C);
    GADMM_CHECK(hipGetLastError());
    int rc;
    if (b <= 64) {
      if ((rc = gadmm_spd_inverse_small_f64(P, zero, 1, b, 1, Pi, status, st))) return rc;
    } else {
      GADMM_CHECK(hipMemcpyAsync(Pi, P, sizeof(double) * b * b, hipMemcpyDeviceToDevice, st));
      if ((rc = blocked_inplace(Pi, b, 64, inner, status, st))) return rc;
    }
    if ((rc = gemm_launch(0, d, b, b, C, b, Pi, b, Lc, b, 0, 0, st))) return rc;            // Lc = C Pi
    if ((rc = gemm_launch(1, d, d, b, Lc, b, C, b, W, d, k0, k0 + b, st))) return rc;       // lower update
    hipLaunchKernelGGL(cross_kernel, dim3(grid_for((long)d * b)), dim3(256), 0, st, W, d, k0, b, Lc, Pi);
    GADMM_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(mirror_kernel, dim3(grid_for((long)d * d)), dim3(256), 0, st, W, d);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // namespace

extern "C" {

// Workspace doubles (zeroed by the caller) for block size nb: one region per concurrent matrix stream.
long gadmm_spd_inverse_blocked_workspace(int d, int nb) { return 2 * ws_doubles(d, nb <= 0 ? 128 : nb); }

// out[n][v] = (A_n + shift[n][v] I)^-1, d x d each; shift_host: host array [N][nvar]. status: int
// (1 = a pivot was not positive). nb: 64 or 128 (0: 128).
int gadmm_spd_inverse_blocked_f64(const double* A, const double* shift_host, int N, int d, int nvar, double* out,
                                  double* ws, int* status, int nb, hipStream_t st) {
  if (nb <= 0) nb = 128;
  if ((nb != 64 && nb != 128) || d < 1 || N < 0 || nvar < 1) {
    gadmm_set_error("spd_inverse_blocked: bad arguments (d=%d nb=%d)", d, nb);
    return -1;
  }
  const long dd = (long)d * d;
  // Two matrices in flight: odd ones run on a second stream with their own workspace, so one matrix's
  // latency-bound pivot-block chain (panel, 128-block inverse, cross: ~15 launches per pivot block)
  // overlaps the other's MFMA rank-nb update (the real-shaped config inverts two 10k matrices per
  // engine). Each matrix's arithmetic is unchanged: bit-identical. The second stream waits for
  // everything enqueued on `st` before, and `st` waits for it at the end.
  const int total = N * nvar;
  if (total > 1) {
    // The side stream and its fork / join events are per device and process-wide: one caller at a
    // time enqueues through them (the lock covers the whole fork ... join, so two threads' matrices
    // never interleave on the shared side stream or overwrite each other's events).
    static std::mutex mu;
    std::lock_guard<std::mutex> lock(mu);
    int dev = 0;
    GADMM_CHECK(hipGetDevice(&dev));
    static hipStream_t side[64] = {};
    static hipEvent_t ev_in[64] = {}, ev_out[64] = {};
    if (dev < 0 || dev >= 64) {
      gadmm_set_error("spd_inverse_blocked: device %d", dev);
      return -1;
    }
    if (!side[dev]) {
      GADMM_CHECK(hipStreamCreateWithFlags(&side[dev], hipStreamNonBlocking));
      GADMM_CHECK(hipEventCreateWithFlags(&ev_in[dev], hipEventDisableTiming));
      GADMM_CHECK(hipEventCreateWithFlags(&ev_out[dev], hipEventDisableTiming));
    }
    hipStream_t st2 = side[dev];
    GADMM_CHECK(hipEventRecord(ev_in[dev], st));
    GADMM_CHECK(hipStreamWaitEvent(st2, ev_in[dev], 0));
    int rc = 0;
    for (int m = 0; m < total && rc == 0; ++m) {
      const int n = m / nvar, v = m % nvar;
      hipStream_t sm = (m & 1) ? st2 : st;
      double* W = out + (long)m * dd;
      hipLaunchKernelGGL(shift_copy_kernel, dim3(grid_for(dd)), dim3(256), 0, sm, A + (long)n * dd,
                         shift_host[n * nvar + v], d, W);
      const hipError_t le = hipGetLastError();
      if (le != hipSuccess) {
        gadmm_set_error("spd_inverse_blocked: shift_copy launch: %s", hipGetErrorString(le));
        rc = (int)le;
        break;
      }
      rc = blocked_inplace(W, d, nb, ws + ((m & 1) ? ws_doubles(d, nb) : 0), status, sm);
    }
    // Join the side stream on EVERY path (an error included): the caller frees `ws` / `out` once `st`
    // is done, so `st` must not finish before work already queued on st2; a capture's fork is joined too.
    const hipError_t e1 = hipEventRecord(ev_out[dev], st2);
    const hipError_t e2 = e1 == hipSuccess ? hipStreamWaitEvent(st, ev_out[dev], 0) : e1;
    if (rc) return rc;
    GADMM_CHECK(e2);
    return 0;
  }
  for (int n = 0; n < N; ++n)
    for (int v = 0; v < nvar; ++v) {
      double* W = out + ((long)n * nvar + v) * dd;
      hipLaunchKernelGGL(shift_copy_kernel, dim3(grid_for(dd)), dim3(256), 0, st, A + (long)n * dd,
                         shift_host[n * nvar + v], d, W);
      GADMM_CHECK(hipGetLastError());
      const int rc = blocked_inplace(W, d, nb, ws, status, st);
      if (rc) return rc;
    }
  return 0;
}

// Test entry: C = A B (row-major) with the MFMA tile kernel.
int gadmm_gemm_f64_test(int M, int N, int K, const double* A, const double* B, double* C, hipStream_t st) {
  return gemm_launch(0, M, N, K, A, K, B, N, C, N, 0, 0, st);
}

}  // extern "C"
