// Augmented Gram (K1) on the INT8 matrix cores: the Ozaki scheme (error-free slicing of the f64
// operands into int8 digits, exact int32 MFMA products, f64 recombination).
//
// gfx950's f64 MFMA peaks at 78.6 TF/s; its int8 MFMA (v_mfma_i32_32x32x32_i8) runs 2x the bf16 rate,
// ~64x the f64 one. A Gram A = X^T X of a tall shard (X: m x D, the real-shaped config: 625k x 10001
// per worker) is therefore computed here as
//   x_ij = 2^{e_j} sum_{p=1..S} d_p(i, j) 2^{-7 p},     d_p in [-127, 127]  (digits of x / 2^{e_j})
//   A_ab = 2^{e_a + e_b} sum_{L=2}^{S+1} 2^{-7 L} sum_{p+q=L} sum_i d_p(i, a) d_q(i, b)
// where e_j is the column's exponent (|x_ij| <= (127/128) 2^{e_j}), the digits are the round-to-nearest
// base-128 expansion (first digit within +-127, the others +-64; the residual after S digits is at most
// half a unit of the last one and unbiased -- truncated digits left a one-signed residual whose sum over
// the m samples biased the diagonal by ~1e-13 relative), and the pairs with p + q > S + 1 are dropped (each below
// 2^{-7(S+2)} of the column scales: far under f64 rounding). Every inner sum is an EXACT int32 MFMA
// accumulation (|d_p d_q| < 2^14; a chunk of K samples with at most S pairs per level stays below
// 2^31 for K * S * 127^2 < 2^31, K = 8192 here), so the only roundings are the f64 recombination and
// the chunk sums -- the result is as accurate as the f64-MFMA Gram (whose K-sum rounds at every
// step) or better; the S-digit residual of the inputs is <= 2^{-7S-1} of the column scale (S = 7: 2^-50).
//
// Kernels (host driver gadmm_gram_ozaki_f64 below, one chunk of KC samples at a time):
//   oz_colexp   column exponents of the augmented [X | y] over the whole shard (one pass)
//   oz_slice    digits of a chunk: S[p][kb][j][32] int8 -- slice p, 32-sample block kb, feature j,
//               the block's 32 samples contiguous, so one MFMA operand fragment is one 1 KB run
//   oz_gemm     lower-triangle tiles of 32 x 32 features per wave, all S(S+1)/2 digit pairs as int8
//               MFMAs into S level accumulators, flushed once per chunk into the f64 Gram
//   oz_finish   the f64 Gram -> A (full symmetric), b, y'y
#include <stdlib.h>
#include <string.h>
#include "gadmm_common.h"

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

namespace {

// One v_mfma_i32_32x32x32_i8 on raw per-lane fragments (layout probe for the tests: the lane maps of
// the A / B operands are established from exact integer data, tests/test_gpu.py).
__global__ void __launch_bounds__(64) mfma_i8_probe_kernel(const v4i* a, const v4i* b, int* d) {
  const int l = threadIdx.x;
  v16i c = {};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[l], b[l], c, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 16; ++r) d[l * 16 + r] = c[r];
}

constexpr int SL = 7;          // digits per value (7 bits each: 2^-49 of the column scale)
constexpr int KC = 8192;       // samples per chunk: SL * 127^2 * KC < 2^31 (exact int32 levels)
constexpr int KBC = KC / 32;   // 32-sample blocks per chunk
constexpr int OT = 128;        // output tile (features) per workgroup: 4 x 4 waves of 32 x 32
constexpr int GEMM_NT = 1024;  // 16 waves
constexpr int CE_NT = 256;     // column-exponent threads per workgroup (one column each)
constexpr int CE_R = 128;      // row splits of the column-exponent pass

__device__ __forceinline__ double aug_at(const double* X, const double* y, long i, int j, int m, int d) {
  if (i >= m) return 0.0;
  if (j < d) return X[i * d + j];
  if (j == d) return y[i];
  return 0.0;  // padding columns
}

// partial column max |x| of the augmented [X | y] over the rows of split blockIdx.y
__global__ void __launch_bounds__(CE_NT) oz_colmax_part(const double* X, const double* y, int m, int d, int Dp,
                                                        double* part) {
  const int j = blockIdx.x * CE_NT + threadIdx.x;
  if (j >= Dp) return;
  const long per = ((long)m + CE_R - 1) / CE_R;
  const long i0 = per * blockIdx.y, i1 = (i0 + per < m) ? i0 + per : m;
  double mx = 0.0;
  for (long i = i0; i < i1; ++i) mx = fmax(mx, fabs(aug_at(X, y, i, j, m, d)));
  part[(long)blockIdx.y * Dp + j] = mx;
}

// e_j with max |x_ij| <= (127/128) 2^{e_j}, 0 for an all-zero column: the first round-to-nearest digit
// then stays within [-127, 127]
__global__ void __launch_bounds__(CE_NT) oz_colexp(const double* part, int Dp, int* e) {
  const int j = blockIdx.x * CE_NT + threadIdx.x;
  if (j >= Dp) return;
  double mx = 0.0;
  for (int r = 0; r < CE_R; ++r) mx = fmax(mx, part[(long)r * Dp + j]);
  int E = 0;
  if (mx > 0.0) {
    const double f = frexp(mx, &E);  // mx = f 2^E, f in [0.5, 1)
    if (f > 127.0 / 128.0) ++E;
  }
  e[j] = E;
}

// Digits of samples [i0, i0 + KC) into S[p][kb][j][32] (int8): a workgroup takes 32 samples x 256
// features -- coalesced f64 row reads, digits through LDS, 32-byte sample runs written per feature.
constexpr int SLICE_NT = 256;
__global__ void __launch_bounds__(SLICE_NT) oz_slice(const double* X, const double* y, long i0, int m, int d, int Dp,
                                                     const int* e, signed char* S) {
  __shared__ signed char dig[SL][SLICE_NT][33];  // [slice][feature][sample] (+1: bank spread)
  const int kb = blockIdx.y;                       // 32-sample block of the chunk
  const int j = blockIdx.x * SLICE_NT + threadIdx.x;
  const bool on = j < Dp;
  const int ej = on ? e[j] : 0;
  for (int t = 0; t < 32; ++t) {
    const long i = i0 + (long)kb * 32 + t;
    double v = on ? ldexp(aug_at(X, y, i, j, m, d), -ej) : 0.0;  // |v| <= 127/128
#pragma unroll
    for (int p = 0; p < SL; ++p) {
      v *= 128.0;                      // exact (power of two)
      const double q = rint(v);        // nearest: |q| <= 127 for the first digit, <= 64 after
      v -= q;                          // exact (|v - q| <= 1/2, representable)
      dig[p][threadIdx.x][t] = (signed char)(int)q;
    }
  }
  __syncthreads();
  // write: for each slice, 256 features x 32 bytes = 8 KB contiguous; thread = one 32-byte run
  for (int p = 0; p < SL; ++p) {
    if (!on) continue;
    signed char* dst = S + (((long)p * KBC + kb) * Dp + j) * 32;
    int w[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      w[q] = (int)(unsigned char)dig[p][threadIdx.x][4 * q] | ((int)(unsigned char)dig[p][threadIdx.x][4 * q + 1] << 8) |
             ((int)(unsigned char)dig[p][threadIdx.x][4 * q + 2] << 16) |
             ((int)(unsigned char)dig[p][threadIdx.x][4 * q + 3] << 24);
    }
    v4i* d4 = reinterpret_cast<v4i*>(dst);
    d4[0] = v4i{w[0], w[1], w[2], w[3]};
    d4[1] = v4i{w[4], w[5], w[6], w[7]};
  }
}

// Lower-triangle tile id -> (ti, tj), ti >= tj
__device__ __forceinline__ void oz_tri(int t, int& ti, int& tj) {
  ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
  while (ti * (ti + 1) / 2 > t) --ti;
  tj = t - ti * (ti + 1) / 2;
}

// One chunk: C[a][b] += 2^{e_a + e_b} sum_L 2^{-7L} sum_{p+q=L} S_p[:, a]^T S_q[:, b] for the tile's
// lower blocks. LDS per K step: the A and B panels, [slice][32-block][half][feature in block][16 B]
// (a wave's ds_read_b128 of 16 lanes covers 256 contiguous bytes: conflict-free), double-buffered;
// the next step's panels are fetched into registers while this step's MFMAs issue.
__global__ void __launch_bounds__(GEMM_NT) oz_gemm(const signed char* S, int Dp, int nt, const int* e, double* C) {
  extern __shared__ __attribute__((aligned(16))) v4i lds4[];  // 2 buffers x 2 panels x SL x 4 x 2 x 32
  constexpr int PANEL = SL * 4 * 2 * 32;                       // v4i per panel
  int ti, tj;
  oz_tri((int)blockIdx.x, ti, tj);
  const bool diag = ti == tj;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, bi = wv >> 2, bj = wv & 3;
  const int a0 = ti * OT + bi * 32, b0 = tj * OT + bj * 32;
  const bool work = a0 < Dp && b0 < Dp && (!diag || bi >= bj);
  const int r = lane & 31, h = lane >> 5;
  // cooperative copy: element idx -> (panel, slice, block, feature r, half) ; 2 * SL * 4 * 32 * 2 v4i
  constexpr int NEL = 2 * PANEL;
  const int npanel = diag ? 1 : 2;
  v4i pre[4];
  auto fetch = [&](int kb) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = threadIdx.x + u * GEMM_NT;
      v4i v = {0, 0, 0, 0};
      if (idx < npanel * PANEL) {
        const int pn = idx / PANEL, rem = idx % PANEL;
        const int hh = rem & 1, rr = (rem >> 1) & 31, blk = (rem >> 6) & 3, p = rem >> 8;
        const int j = (pn == 0 ? ti : tj) * OT + blk * 32 + rr;
        if (j < Dp) v = *reinterpret_cast<const v4i*>(S + (((long)p * KBC + kb) * Dp + j) * 32 + 16 * hh);
      }
      pre[u] = v;
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = threadIdx.x + u * GEMM_NT;
      if (idx < npanel * PANEL) {
        const int pn = idx / PANEL, rem = idx % PANEL;
        const int hh = rem & 1, rr = (rem >> 1) & 31, blk = (rem >> 6) & 3, p = rem >> 8;
        lds4[buf * NEL + pn * PANEL + ((p * 4 + blk) * 2 + hh) * 32 + rr] = pre[u];
      }
    }
  };
  v16i acc[SL];
#pragma unroll
  for (int L = 0; L < SL; ++L) acc[L] = v16i{};
  fetch(0);
  stash(0);
  __syncthreads();
  for (int kb = 0; kb < KBC; ++kb) {
    const int buf = kb & 1;
    if (kb + 1 < KBC) fetch(kb + 1);
    if (work) {
      const v4i* PA = lds4 + buf * NEL;
      const v4i* PB = lds4 + buf * NEL + (diag ? 0 : PANEL);
      v4i fa[SL], fb[SL];
#pragma unroll
      for (int p = 0; p < SL; ++p) {
        fa[p] = PA[((p * 4 + bi) * 2 + h) * 32 + r];
        fb[p] = PB[((p * 4 + bj) * 2 + h) * 32 + r];
      }
#pragma unroll
      for (int p = 0; p < SL; ++p)
#pragma unroll
        for (int q = 0; q < SL - p; ++q)  // level p + q (digits p + 1, q + 1): sum <= SL + 1
          acc[p + q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[p], fb[q], acc[p + q], 0, 0, 0);
    }
    if (kb + 1 < KBC) {
      stash(buf ^ 1);
    }
    __syncthreads();
  }
  if (!work) return;
  // flush: level L (0-based) has scale 2^{-7 (L + 2)}; smallest first
  const int col = b0 + r;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const int row = a0 + (g & 3) + 8 * (g >> 2) + 4 * h;
    double v = 0.0;
#pragma unroll
    for (int L = SL - 1; L >= 0; --L) v = fma((double)acc[L][g], ldexp(1.0, -7 * (L + 2)), v);
    C[(long)row * Dp + col] += ldexp(v, e[row] + e[col]);
  }
}

// C (Dp x Dp, lower triangle) -> A (d x d, full symmetric), b (d), yy
__global__ void __launch_bounds__(256) oz_finish(const double* C, int Dp, int d, double* A, double* b, double* yy) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long dd = (long)d * d;
  if (idx < dd) {
    const int a = (int)(idx / d), c = (int)(idx % d);
    A[idx] = a >= c ? C[(long)a * Dp + c] : C[(long)c * Dp + a];
  } else if (idx < dd + d) {
    const int a = (int)(idx - dd);
    b[a] = C[(long)d * Dp + a];
  } else if (idx == dd + d) {
    yy[0] = C[(long)d * Dp + d];
  }
}

}  // namespace

extern "C" {

// Workspace bytes of gadmm_gram_ozaki_f64 for a shard of m x d (plus y): the f64 Gram of the padded
// augmented matrix, one chunk of digits, the column-max partials and exponents.
long gadmm_gram_ozaki_workspace(long m, int d) {
  (void)m;
  const long Dp = ((long)d + 1 + 31) / 32 * 32;
  return Dp * Dp * 8 + (long)SL * KC * Dp + (long)CE_R * Dp * 8 + Dp * 4 + 256;
}

// A_n = X_n^T X_n, b_n = X_n^T y_n, yy_n = y_n^T y_n for N shards X (N x m x d, row-major f64) on the
// int8 matrix cores (see the file comment). Deterministic (fixed chunk order, exact int32 sums).
int gadmm_gram_ozaki_f64(const double* X, const double* Y, int N, long m, int d, double* A, double* B, double* YY,
                         void* ws, long ws_bytes, hipStream_t st) {
  if (N <= 0 || m <= 0 || d <= 0) return 0;
  const int Dp = (d + 1 + 31) / 32 * 32;
  if (!X || !Y || !A || !B || !YY || !ws || ws_bytes < gadmm_gram_ozaki_workspace(m, d)) {
    gadmm_set_error("gram_ozaki: bad arguments or workspace (%ld < %ld bytes)", ws_bytes,
                    gadmm_gram_ozaki_workspace(m, d));
    return -1;
  }
  char* w = (char*)ws;
  double* C = (double*)w;
  signed char* S = (signed char*)(w + (long)Dp * Dp * 8);
  double* part = (double*)(w + (long)Dp * Dp * 8 + (long)SL * KC * Dp);
  int* e = (int*)((char*)part + (long)CE_R * Dp * 8);
  const int nt = (Dp + OT - 1) / OT;
  const int tiles = nt * (nt + 1) / 2;
  const size_t shm = (size_t)2 * 2 * SL * 4 * 2 * 32 * sizeof(v4i);  // 114,688 B
  static bool attr = false;
  if (!attr) {
    GADMM_CHECK(hipFuncSetAttribute((const void*)oz_gemm, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    attr = true;
  }
  for (int n = 0; n < N; ++n) {
    const double* Xn = X + (long)n * m * d;
    const double* Yn = Y + (long)n * m;
    hipLaunchKernelGGL(oz_colmax_part, dim3((Dp + CE_NT - 1) / CE_NT, CE_R), dim3(CE_NT), 0, st, Xn, Yn, (int)m, d,
                       Dp, part);
    hipLaunchKernelGGL(oz_colexp, dim3((Dp + CE_NT - 1) / CE_NT), dim3(CE_NT), 0, st, part, Dp, e);
    GADMM_CHECK(hipMemsetAsync(C, 0, (size_t)Dp * Dp * 8, st));
    for (long i0 = 0; i0 < m; i0 += KC) {
      hipLaunchKernelGGL(oz_slice, dim3((Dp + SLICE_NT - 1) / SLICE_NT, KBC), dim3(SLICE_NT), 0, st, Xn, Yn, i0,
                         (int)m, d, Dp, e, S);
      hipLaunchKernelGGL(oz_gemm, dim3(tiles), dim3(GEMM_NT), shm, st, S, Dp, nt, e, C);
    }
    const long tot = (long)d * d + d + 1;
    hipLaunchKernelGGL(oz_finish, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, C, Dp, d,
                       A + (long)n * d * d, B + (long)n * d, YY + n);
    GADMM_CHECK(hipGetLastError());
  }
  return 0;
}

int gadmm_mfma_i8_probe(const void* a_frag, const void* b_frag, int* d_out, hipStream_t st) {
  if (!a_frag || !b_frag || !d_out) {
    gadmm_set_error("mfma_i8_probe: null argument");
    return -1;
  }
  hipLaunchKernelGGL(mfma_i8_probe_kernel, dim3(1), dim3(64), 0, st, (const v4i*)a_frag, (const v4i*)b_frag, d_out);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"
