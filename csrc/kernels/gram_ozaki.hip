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
#include <algorithm>
#include <map>
#include <mutex>
#include <vector>
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
constexpr int OT = 64;         // output tile (features) per workgroup: 2 x 2 waves of 32 x 32
constexpr int GEMM_NT = 256;   // 4 waves
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
__global__ void __launch_bounds__(CE_NT) oz_colexp(const double* part, int Dp, int* e, double* cm) {
  const int j = blockIdx.x * CE_NT + threadIdx.x;
  if (j >= Dp) return;
  double mx = 0.0;
  for (int r = 0; r < CE_R; ++r) mx = fmax(mx, part[(long)r * Dp + j]);
  cm[j] = mx;
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

// One chunk: C[a][b] += 2^{e_a + e_b} sum_L 2^{-7L} sum_{p+q=L} S_p[:, a]^T S_q[:, b] for the tile's
// lower blocks. A workgroup is 4 waves on a 64 x 64 tile (one 32 x 32 block per wave: 7 level
// accumulators = 112 registers + 14 operand fragments; two workgroups per CU = 2 waves per SIMD, 256
// registers each -- the first cut, 16 waves on a 128 tile at 128 registers, spilled 238 VGPRs per lane).
// LDS per K step: the A and B panels, [slice][32-block][half][feature in block][16 B] (a ds_read_b128
// of 32 lanes covers 512 contiguous bytes: conflict-free), double-buffered; the next step's panels are
// fetched into registers while this step's MFMAs issue. Tile order (host-built list, oz_tile_list):
// lower-triangle tiles grouped in 8 x 8 super-blocks and dealt XCD-major (workgroup i runs on XCD i % 8),
// so the 64 workgroups an XCD runs at once share 16 panels in its L2 instead of one row's 65.
__global__ void __launch_bounds__(GEMM_NT, 2) oz_gemm(const signed char* S, int Dp, int tiles, const int2* list,
                                                      int kbn, const int* e, double* C) {
  extern __shared__ __attribute__((aligned(16))) v4i lds4[];  // 2 buffers x 2 panels x PANEL
  constexpr int NB = OT / 32;                                  // 32-feature blocks per tile side
  constexpr int PANEL = SL * NB * 2 * 32;                      // v4i per panel
  constexpr int NEL = 2 * PANEL;
  constexpr int PER = NEL / GEMM_NT;
  const int per_xcd = (tiles + 7) / 8;
  const int t = (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3);
  if (t >= tiles) return;
  const int ti = list[t].x, tj = list[t].y;
  const bool diag = ti == tj;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, bi = wv / NB, bj = wv % NB;
  const int a0 = ti * OT + bi * 32, b0 = tj * OT + bj * 32;
  const bool work = !diag || bi >= bj;
  const int r = lane & 31, h = lane >> 5;
  // Staging: element idx = threadIdx + u * GEMM_NT of the 2 panels, LDS image lane-linear
  // ([panel][slice][block][half][feature]: idx itself), global offsets precomputed once (Dp is a
  // multiple of OT, so every feature of every tile exists: no per-element bounds test -- the first
  // version's per-step index arithmetic issued about as many VALU cycles as its MFMAs, r05_h2 PMC).
  // A diagonal tile stages its one panel twice (uniform code; 1 tile in nt).
  static_assert(NEL % GEMM_NT == 0, "staging elements must divide evenly");
  unsigned off[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int idx = threadIdx.x + u * GEMM_NT;
    const int pn = idx / PANEL, rem = idx % PANEL;
    const int rr = rem & 31, hh = (rem >> 5) & 1, blk = (rem >> 6) % NB, p = (rem >> 6) / NB;
    const int j = (pn == 0 ? ti : tj) * OT + blk * 32 + rr;
    off[u] = (unsigned)(((long)p * KBC * Dp + j) * 32 + 16 * hh);
  }
  v4i pre[PER];
  auto fetch = [&](int kb) {
    const signed char* base = S + (long)kb * Dp * 32;  // wave-uniform
#pragma unroll
    for (int u = 0; u < PER; ++u) pre[u] = *reinterpret_cast<const v4i*>(base + off[u]);
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int u = 0; u < PER; ++u) lds4[buf * NEL + threadIdx.x + u * GEMM_NT] = pre[u];
  };
  v16i acc[SL];
#pragma unroll
  for (int L = 0; L < SL; ++L) acc[L] = v16i{};
  fetch(0);
  stash(0);
  __syncthreads();
  for (int kb = 0; kb < kbn; ++kb) {  // kbn: the chunk's 32-sample blocks (the last chunk is partial)
    const int buf = kb & 1;
    if (kb + 1 < kbn) fetch(kb + 1);
    if (work) {
      const v4i* PA = lds4 + buf * NEL;
      const v4i* PB = lds4 + buf * NEL + (diag ? 0 : PANEL);
      v4i fa[SL], fb[SL];
#pragma unroll
      for (int p = 0; p < SL; ++p) {
        fa[p] = PA[((p * NB + bi) * 2 + h) * 32 + r];
        fb[p] = PB[((p * NB + bj) * 2 + h) * 32 + r];
      }
      // all 14 fragment reads in flight before the first MFMA (left alone, hipcc sinks each A read to
      // its first use and waits lgkmcnt(0) there: seven exposed LDS round trips per step)
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int p = 0; p < SL; ++p)
#pragma unroll
        for (int q = 0; q < SL - p; ++q)  // level p + q (digits p + 1, q + 1): sum <= SL + 1
          acc[p + q] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[p], fb[q], acc[p + q], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    if (kb + 1 < kbn) stash(buf ^ 1);
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

// The column-range statistic of the gate (linalg.gram): max_j colmax_j / rms_j over the augmented
// columns j <= d, rms_j = sqrt(C_jj / m) from the Gram's own diagonal. The digits keep 49 bits of every
// value relative to its column's scale 2^{e_j} >= colmax_j, so an entry at the column's rms level keeps
// about 49 - log2(range) bits; the caller recomputes with the f64-MFMA Gram past its threshold.
__global__ void __launch_bounds__(256) oz_range(const double* cm, const double* C, int Dp, int d, long m,
                                                double* out) {
  __shared__ double red[256];
  double r = 0.0;
  for (int j = threadIdx.x; j <= d; j += 256) {
    const double cjj = C[(long)j * Dp + j];
    if (cjj > 0.0) r = fmax(r, cm[j] / sqrt(cjj / (double)m));
  }
  red[threadIdx.x] = r;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

}  // namespace

constexpr int OZ_SUPER = 8;  // tiles per super-block side

// Device list of the nt (nt + 1) / 2 lower-triangle tiles in super-block order, built once per nt
// (static cache; the Gram is never captured into a graph).
const int2* oz_tile_list(int nt) {
  static std::mutex mu;
  static std::map<int, int2*> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(nt);
  if (it != cache.end()) return it->second;
  std::vector<int2> L;
  L.reserve((size_t)nt * (nt + 1) / 2);
  const int ns = (nt + OZ_SUPER - 1) / OZ_SUPER;
  for (int I = 0; I < ns; ++I)
    for (int J = 0; J <= I; ++J)
      for (int i = I * OZ_SUPER; i < std::min((I + 1) * OZ_SUPER, nt); ++i)
        for (int j = J * OZ_SUPER; j < std::min((J + 1) * OZ_SUPER, nt) && j <= i; ++j) L.push_back(int2{i, j});
  int2* d = nullptr;
  if (hipMalloc(&d, L.size() * sizeof(int2)) != hipSuccess) return nullptr;
  if (hipMemcpy(d, L.data(), L.size() * sizeof(int2), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(d);
    return nullptr;
  }
  cache[nt] = d;
  return d;
}

extern "C" {

// Workspace bytes of gadmm_gram_ozaki_f64 for a shard of m x d (plus y): the f64 Gram of the padded
// augmented matrix, two chunk buffers of digits, the column-max partials and exponents.
long gadmm_gram_ozaki_workspace(long m, int d) {
  (void)m;
  const long Dp = ((long)d + 1 + OT - 1) / OT * OT;
  return Dp * Dp * 8 + 2L * SL * KC * Dp + (long)CE_R * Dp * 8 + Dp * 4 + Dp * 8 + 256;
}

// A_n = X_n^T X_n, b_n = X_n^T y_n, yy_n = y_n^T y_n for N shards X (N x m x d, row-major f64) on the
// int8 matrix cores (see the file comment). Deterministic (fixed chunk order, exact int32 sums).
// ``range_out`` (optional, N doubles): each shard's column-range statistic (oz_range) for the caller's
// accuracy gate.
// The memory-bound digit slicing of chunk c + 1 runs on a side stream into the other digit buffer
// while the MFMA-bound oz_gemm of chunk c runs on `st` (r05_h3: slicing was 11 % of the serial time).
int gadmm_gram_ozaki_f64(const double* X, const double* Y, int N, long m, int d, double* A, double* B, double* YY,
                         void* ws, long ws_bytes, double* range_out, hipStream_t st) {
  if (N <= 0 || m <= 0 || d <= 0) return 0;
  const int Dp = (d + 1 + OT - 1) / OT * OT;  // a multiple of the tile
  if (!X || !Y || !A || !B || !YY || !ws || ws_bytes < gadmm_gram_ozaki_workspace(m, d)) {
    gadmm_set_error("gram_ozaki: bad arguments or workspace (%ld < %ld bytes)", ws_bytes,
                    gadmm_gram_ozaki_workspace(m, d));
    return -1;
  }
  if ((long)SL * KBC * Dp * 32 >= (1L << 32)) {
    gadmm_set_error("gram_ozaki: d = %d exceeds the 32-bit staging offsets", d);
    return -1;
  }
  char* w = (char*)ws;
  double* C = (double*)w;
  signed char* Sbuf[2] = {(signed char*)(w + (long)Dp * Dp * 8),
                          (signed char*)(w + (long)Dp * Dp * 8 + (long)SL * KC * Dp)};
  double* part = (double*)(w + (long)Dp * Dp * 8 + 2L * SL * KC * Dp);
  int* e = (int*)((char*)part + (long)CE_R * Dp * 8);
  double* cm = (double*)((char*)e + ((long)Dp * 4 + 255) / 256 * 256);  // column maxima (the range gate)
  const int nt = Dp / OT;
  const int tiles = nt * (nt + 1) / 2;
  const int2* list = oz_tile_list(nt);
  if (!list) {
    gadmm_set_error("gram_ozaki: tile list allocation failed");
    return -1;
  }
  const size_t shm = (size_t)2 * 2 * SL * (OT / 32) * 2 * 32 * sizeof(v4i);  // 57,344 B: two per CU
  // side stream + events, per device and process-wide: one caller at a time (the lock spans fork ... join)
  static std::mutex mu;
  std::lock_guard<std::mutex> lock(mu);
  int dev = 0;
  GADMM_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) {
    gadmm_set_error("gram_ozaki: device %d", dev);
    return -1;
  }
  static hipStream_t side[64] = {};
  static hipEvent_t ev[64][6] = {};  // fork, join, sliced[2], multiplied[2]
  static bool attr[64] = {};
  if (!side[dev]) {
    GADMM_CHECK(hipStreamCreateWithFlags(&side[dev], hipStreamNonBlocking));
    for (int k = 0; k < 6; ++k) GADMM_CHECK(hipEventCreateWithFlags(&ev[dev][k], hipEventDisableTiming));
  }
  if (!attr[dev]) {
    GADMM_CHECK(hipFuncSetAttribute((const void*)oz_gemm, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    attr[dev] = true;
  }
  hipStream_t s2 = side[dev];
  hipEvent_t ev_fork = ev[dev][0], ev_join = ev[dev][1], *ev_s = &ev[dev][2], *ev_g = &ev[dev][4];
  const int nc = (int)((m + KC - 1) / KC);
  for (int n = 0; n < N; ++n) {
    const double* Xn = X + (long)n * m * d;
    const double* Yn = Y + (long)n * m;
    hipLaunchKernelGGL(oz_colmax_part, dim3((Dp + CE_NT - 1) / CE_NT, CE_R), dim3(CE_NT), 0, st, Xn, Yn, (int)m, d,
                       Dp, part);
    hipLaunchKernelGGL(oz_colexp, dim3((Dp + CE_NT - 1) / CE_NT), dim3(CE_NT), 0, st, part, Dp, e, cm);
    GADMM_CHECK(hipMemsetAsync(C, 0, (size_t)Dp * Dp * 8, st));
    GADMM_CHECK(hipEventRecord(ev_fork, st));
    hipError_t rc = hipStreamWaitEvent(s2, ev_fork, 0);
    for (int c = -1; c < nc && rc == hipSuccess; ++c) {
      if (c >= 0) {  // multiply chunk c (sliced on s2) on st
        rc = hipStreamWaitEvent(st, ev_s[c & 1], 0);
        if (rc != hipSuccess) break;
        const int kbn = (int)((std::min<long>(KC, m - (long)c * KC) + 31) / 32);
        hipLaunchKernelGGL(oz_gemm, dim3(8 * ((tiles + 7) / 8)), dim3(GEMM_NT), shm, st, Sbuf[c & 1], Dp, tiles,
                           list, kbn, e, C);
        rc = hipGetLastError();
        if (rc == hipSuccess) rc = hipEventRecord(ev_g[c & 1], st);
        if (rc != hipSuccess) break;
      }
      if (c + 1 < nc) {  // slice chunk c + 1 on s2 once chunk c - 1 (same buffer) is multiplied
        const int b = (c + 1) & 1;
        if (c >= 1) rc = hipStreamWaitEvent(s2, ev_g[b], 0);
        if (rc != hipSuccess) break;
        hipLaunchKernelGGL(oz_slice, dim3((Dp + SLICE_NT - 1) / SLICE_NT, KBC), dim3(SLICE_NT), 0, s2, Xn, Yn,
                           (long)(c + 1) * KC, (int)m, d, Dp, e, Sbuf[b]);
        rc = hipGetLastError();
        if (rc == hipSuccess) rc = hipEventRecord(ev_s[b], s2);
      }
    }
    // join on every path: the caller frees the workspace once `st` is done
    const hipError_t j1 = hipEventRecord(ev_join, s2);
    const hipError_t j2 = j1 == hipSuccess ? hipStreamWaitEvent(st, ev_join, 0) : j1;
    if (rc != hipSuccess) {
      gadmm_set_error("gram_ozaki: %s", hipGetErrorString(rc));
      return (int)rc;
    }
    GADMM_CHECK(j2);
    const long tot = (long)d * d + d + 1;
    hipLaunchKernelGGL(oz_finish, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, C, Dp, d,
                       A + (long)n * d * d, B + (long)n * d, YY + n);
    GADMM_CHECK(hipGetLastError());
    if (range_out) {
      hipLaunchKernelGGL(oz_range, dim3(1), dim3(256), 0, st, cm, C, Dp, d, m, range_out + n);
      GADMM_CHECK(hipGetLastError());
    }
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
