// Augmented Gram (K1) on the INT8 matrix cores by CRT slicing: one int8 GEMM per modulus, ONE int32
// accumulator per output element.
//
// The digit scheme of gram_ozaki.hip needs seven int32 level accumulators per output element, which caps
// its tile at 64 x 64 per workgroup (two per CU) and puts ~13 B/cycle/CU of panel traffic on each MFMA
// (about half of the int8 peak, profiles/r05_h). Here every augmented value x_ij (X | y, column j scaled
// by its power-of-two exponent e_j, |x_ij| <= (127/128) 2^{e_j}) becomes the integer
//   N_ij = rint(x_ij 2^{KB - e_j}),   |N_ij| < 2^KB,  KB = 49   (the digit scheme keeps the same 49 bits)
// and the integer Gram  G_ab = sum_i N_ia N_ib  (|G| < m 2^98 <= 2^119 for m <= 2^21) is computed modulo
// 19 pairwise coprime moduli p <= 127 (product ~2^121.8): for each p, the symmetric residues
// R_p = N mod p in [-63, 63] are int8, and  G mod p = R_p^T R_p mod p  is ONE int8 GEMM with exact int32
// accumulation (a chunk of KC samples: KC * 63^2 < 2^31), reduced mod p after every chunk. Garner's
// mixed-radix reconstruction then gives G_ab exactly, and
//   A_ab = 2^{e_a + e_b - 2 KB} G_ab
// with one rounding (the final double). So the result is exact for the 49-bit images of the inputs -- the
// digit scheme's accuracy, with 19 GEMMs instead of 28 digit-pair products, and a 256 x 256 tile per
// workgroup (8 waves of 128 x 64, 128 accumulator registers each): half the panel bytes per MFMA of the
// digit kernel's 64 x 64 tile.
//
// Kernels (host driver gadmm_gram_crt_f64 below, per shard, one chunk of KC samples at a time):
//   crt_colmax / crt_colexp   column exponents e_j of the augmented [X | y] (one pass)
//   crt_slice     residues of a chunk: R[p][kb][j][32] int8 -- modulus p, 32-sample block kb, feature j,
//                 the block's 32 samples contiguous (one MFMA operand half-fragment = 16 contiguous bytes)
//   crt_gemm      one workgroup per (lower-triangle 256 x 256 tile, modulus): LDS-DMA double-buffered
//                 panels (64 samples per stage), 16 v_mfma_i32_32x32x32_i8 per wave per stage; the chunk's
//                 sums go into the int16 residue matrices C_p (reduced mod p)
//   crt_finish    Garner per lower-triangle element -> A (full symmetric), b, y'y
//   crt_range     the column-range statistic of linalg.gram's accuracy gate
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

constexpr int NMOD = 19;
constexpr int kMod[NMOD] = {127, 125, 121, 113, 109, 107, 103, 101, 97, 89, 83, 79, 73, 71, 67, 61, 59, 53, 47};
// kInv[i][j] = (kMod[j] mod kMod[i])^{-1} mod kMod[i], j < i (Garner); generated and checked by
// tests/test_gram_crt_math.py
constexpr int kInv[NMOD][NMOD] = {
    {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {63, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {101, 91, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {105, 66, 99, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {103, 75, 100, 82, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {91, 6, 23, 18, 54, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {73, 89, 63, 31, 86, 26, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {35, 80, 96, 59, 38, 17, 51, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {55, 52, 93, 91, 89, 68, 81, 73, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {82, 47, 64, 26, 49, 5, 70, 52, 78, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {17, 2, 59, 36, 16, 45, 54, 60, 6, 14, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {28, 67, 32, 7, 29, 48, 56, 18, 22, 8, 20, 0, 0, 0, 0, 0, 0, 0, 0},
    {23, 66, 35, 42, 71, 58, 56, 60, 70, 32, 22, 61, 0, 0, 0, 0, 0, 0, 0},
    {52, 25, 27, 22, 43, 2, 20, 45, 41, 4, 6, 9, 36, 0, 0, 0, 0, 0, 0},
    {19, 52, 36, 51, 8, 62, 54, 2, 38, 64, 21, 28, 56, 17, 0, 0, 0, 0, 0},
    {49, 41, 60, 27, 14, 4, 16, 29, 39, 24, 25, 17, 56, 55, 51, 0, 0, 0, 0},
    {46, 17, 20, 47, 13, 16, 55, 52, 14, 2, 32, 3, 38, 5, 37, 30, 0, 0, 0},
    {48, 14, 46, 38, 18, 1, 35, 21, 47, 28, 23, 51, 8, 3, 19, 20, 9, 0, 0},
    {10, 44, 7, 5, 22, 29, 21, 27, 16, 28, 17, 25, 38, 2, 40, 37, 4, 8, 0}};
__constant__ int kModDev[NMOD] = {127, 125, 121, 113, 109, 107, 103, 101, 97, 89, 83, 79, 73, 71, 67, 61, 59, 53, 47};

constexpr int KB = 49;            // bits of every value's integer image (|N| < 2^KB)
constexpr long MAX_ROWS = 1L << 21;  // m 2^{2 KB} < M / 2 (the product of the moduli): exact reconstruction
constexpr int KC = 32768;         // samples per chunk: KC * 63^2 < 2^31 (exact int32 sums)
constexpr int KBC = KC / 32;      // 32-sample blocks per chunk
constexpr int TT = 256;           // output tile (features) per workgroup
constexpr int GNT = 512;          // 8 waves: 2 (rows of 128) x 4 (columns of 64)
constexpr int BKS = 2;            // 32-sample blocks per pipeline stage (64 samples)
constexpr int PANEL = BKS * TT * 32;           // bytes of one operand panel per stage (16 KB)
constexpr int STAGE = 2 * PANEL;               // A + B (32 KB)
constexpr int CE_NT = 256;        // column-exponent threads per workgroup
constexpr int CE_R = 128;         // row splits of the column-exponent pass
constexpr int SLT = 128;          // features per slicing workgroup

__device__ __forceinline__ double aug_at(const double* X, const double* y, long i, int j, long m, int d) {
  if (i >= m) return 0.0;
  if (j < d) return X[i * d + j];
  if (j == d) return y[i];
  return 0.0;  // padding columns
}

// partial column max |x| of the augmented [X | y] over the rows of split blockIdx.y
__global__ void __launch_bounds__(CE_NT) crt_colmax(const double* X, const double* y, long m, int d, int Dp,
                                                    double* part) {
  const int j = blockIdx.x * CE_NT + threadIdx.x;
  if (j >= Dp) return;
  const long per = (m + CE_R - 1) / CE_R;
  const long i0 = per * blockIdx.y, i1 = (i0 + per < m) ? i0 + per : m;
  double mx = 0.0;
  for (long i = i0; i < i1; ++i) mx = fmax(mx, fabs(aug_at(X, y, i, j, m, d)));
  part[(long)blockIdx.y * Dp + j] = mx;
}

// e_j with max |x_ij| <= (127/128) 2^{e_j} (0 for an all-zero column); cm_j = the column maximum
__global__ void __launch_bounds__(CE_NT) crt_colexp(const double* part, int Dp, int* e, double* cm) {
  const int j = blockIdx.x * CE_NT + threadIdx.x;
  if (j >= Dp) return;
  double mx = 0.0;
  for (int r = 0; r < CE_R; ++r) mx = fmax(mx, part[(long)r * Dp + j]);
  cm[j] = mx;
  int E = 0;
  if (mx > 0.0) {
    const double f = frexp(mx, &E);
    if (f > 127.0 / 128.0) ++E;
  }
  e[j] = E;
}

// Residues of samples [i0, i0 + 32 kbn) into R[p][kb][j][32]: a workgroup takes 32 samples x SLT
// features; the integer images go through LDS (each thread reads back only its own column), then per
// modulus every thread writes its feature's 32-byte run.
__global__ void __launch_bounds__(SLT) crt_slice(const double* X, const double* y, long i0, long m, int d, int Dp,
                                                 const int* e, signed char* R) {
  __shared__ double xs[32][SLT];
  const int kb = blockIdx.y;
  const int j = blockIdx.x * SLT + threadIdx.x;
  const bool on = j < Dp;
  const int ej = on ? e[j] : 0;
  for (int t = 0; t < 32; ++t) {
    const long i = i0 + (long)kb * 32 + t;
    xs[t][threadIdx.x] = on ? rint(ldexp(aug_at(X, y, i, j, m, d), KB - ej)) : 0.0;  // exact: |N| < 2^49
  }
  if (!on) return;
  for (int p = 0; p < NMOD; ++p) {
    const double mp = (double)kModDev[p], ip = 1.0 / mp, half = 0.5 * (mp - 1.0);
    int w[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      unsigned word = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const double nv = xs[4 * q + b][threadIdx.x];
        const double qq = floor(nv * ip);  // within one of floor(nv / p): |nv ip| < 2^43, error < 2^-9
        double r = fma(-qq, mp, nv);        // exact integer in [-p, 2p)
        if (r < 0.0) r += mp;
        if (r >= mp) r -= mp;
        if (r > half) r -= mp;              // symmetric residue in [-63, 63]
        word |= ((unsigned)(int)r & 0xffu) << (8 * b);
      }
      w[q] = (int)word;
    }
    v4i* d4 = reinterpret_cast<v4i*>(R + (((long)p * KBC + kb) * Dp + j) * 32);
    d4[0] = v4i{w[0], w[1], w[2], w[3]};
    d4[1] = v4i{w[4], w[5], w[6], w[7]};
  }
}

// One chunk of one modulus on one 256 x 256 lower-triangle tile: C_p[a][b] = (C_p + sum_k R_p[k][a]
// R_p[k][b]) mod p for the tile's features a (rows) and b (columns). 8 waves: wave (wr, wc) owns rows
// 128 wr .. +127 (4 blocks of 32) and columns 64 wc .. +63 (2 blocks). Per stage (64 samples = 2 MFMA
// K-steps) the A and B panels (each 2 x 256 features x 32 samples, 16 KB, contiguous in global memory
// and in LDS) come in by LDS-DMA (global_load_lds_dwordx4: a wave instruction moves 1 KB; 32 per stage,
// 4 per wave), double-buffered: stage s + 1's DMAs fly while stage s's 16 MFMAs per wave issue. A
// fragment read (ds_read_b128 of 64 lanes: 32 consecutive features x 2 halves) covers 1 KB contiguous:
// conflict-free.
__global__ void __launch_bounds__(GNT, 1) crt_gemm(const signed char* R, int Dp, int total, const int4* list,
                                                   int kbn, short* C, int first) {
  extern __shared__ __attribute__((aligned(16))) signed char lds[];  // 2 stages x STAGE bytes
  const int per_xcd = (total + 7) / 8;
  const int t = (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3);
  if (t >= total) return;
  const int4 job = list[t];
  const int ti = job.x, tj = job.y, p = job.z;
  const int mp = kModDev[p];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wr = wv >> 2, wc = wv & 3;
  const int r = lane & 31, h = lane >> 5;
  const signed char* gA = R + ((long)p * KBC * Dp + (long)ti * TT) * 32;  // + kb * Dp * 32
  const signed char* gB = R + ((long)p * KBC * Dp + (long)tj * TT) * 32;
  const long kbstride = (long)Dp * 32;
  // this wave's 4 DMA pieces per stage: piece c = 4 wv + u (0..31): panel c >> 4 (A / B), block
  // (c >> 3) & 1 of the stage, 1 KB part c & 7 of the 8 KB (256 features x 32 B) run
  auto issue = [&](int kb0, int buf) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = 4 * wv + u;
      const int pn = c >> 4, blk = (c >> 3) & 1, part = c & 7;
      const signed char* src = (pn ? gB : gA) + (long)(kb0 + blk) * kbstride + part * 1024 + lane * 16;
      signed char* dst = lds + buf * STAGE + pn * PANEL + blk * (TT * 32) + part * 1024;
      __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
    }
  };
  v16i acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = v16i{};
  const int nst = kbn / BKS;  // kbn is even (the slicer zero-fills to a stage boundary)
  issue(0, 0);
  for (int s = 0; s < nst; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // stage s landed (every wave's DMAs); every wave is done reading stage s - 1
    if (s + 1 < nst) issue((s + 1) * BKS, (s + 1) & 1);
    const signed char* SA = lds + (s & 1) * STAGE;
    const signed char* SB = SA + PANEL;
    v4i fa[BKS][4], fb[BKS][2];
#pragma unroll
    for (int k = 0; k < BKS; ++k) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
        fa[k][a] = *reinterpret_cast<const v4i*>(SA + k * (TT * 32) + (wr * 128 + 32 * a + r) * 32 + 16 * h);
#pragma unroll
      for (int b = 0; b < 2; ++b)
        fb[k][b] = *reinterpret_cast<const v4i*>(SB + k * (TT * 32) + (wc * 64 + 32 * b + r) * 32 + 16 * h);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int k = 0; k < BKS; ++k)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[k][a], fb[k][b], acc[a][b], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }
  // epilogue: C_p = (C_p + chunk sum) mod p, symmetric, as int16
  short* Cp = C + (long)p * Dp * Dp;
  const int hm = mp >> 1;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int col = tj * TT + wc * 64 + 32 * b + r;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int row = ti * TT + wr * 128 + 32 * a + (g & 3) + 8 * (g >> 2) + 4 * h;
        const long idx = (long)row * Dp + col;
        int v = acc[a][b][g] % mp;
        if (!first) v += Cp[idx];
        v %= mp;
        if (v > hm) v -= mp;
        if (v < -hm) v += mp;
        Cp[idx] = (short)v;
      }
    }
}

// Garner: the balanced mixed-radix digits of the integer whose residues are r (|G| < M / 2), evaluated
// as a double (Horner from the top: exact while below 2^53, one relative rounding per step above)
__device__ __forceinline__ double garner(const int (&res)[NMOD]) {
  int v[NMOD];
#pragma unroll
  for (int i = 0; i < NMOD; ++i) {
    int u = res[i];
#pragma unroll
    for (int j = 0; j < i; ++j) u = ((u - v[j]) * kInv[i][j]) % kMod[i];
    const int hm = kMod[i] >> 1;
    if (u > hm) u -= kMod[i];
    if (u < -hm) u += kMod[i];
    v[i] = u;
  }
  double val = (double)v[NMOD - 1];
#pragma unroll
  for (int i = NMOD - 2; i >= 0; --i) val = fma(val, (double)kMod[i], (double)v[i]);
  return val;
}

// C_p (lower triangle, row >= col) -> A (d x d full symmetric), b, yy; row = blockIdx.y
__global__ void __launch_bounds__(256) crt_finish(const short* C, int Dp, int d, const int* e, double* A, double* b,
                                                  double* yy) {
  const int a = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c > a || a > d) return;
  int res[NMOD];
#pragma unroll
  for (int i = 0; i < NMOD; ++i) res[i] = C[((long)i * Dp + a) * Dp + c];
  const double v = ldexp(garner(res), e[a] + e[c] - 2 * KB);
  if (a < d) {
    A[(long)a * d + c] = v;
    A[(long)c * d + a] = v;
  } else if (c < d) {
    b[c] = v;
  } else {
    yy[0] = v;
  }
}

// max_j colmax_j / rms_j over the augmented columns j <= d (rms_j from the Gram's own diagonal):
// linalg.gram's accuracy gate (the digit kernel's oz_range, here from A's diagonal and y'y)
__global__ void __launch_bounds__(256) crt_range(const double* cm, const double* A, const double* yy, int d, long m,
                                                 double* out) {
  __shared__ double red[256];
  double rr = 0.0;
  for (int j = threadIdx.x; j <= d; j += 256) {
    const double cjj = j < d ? A[(long)j * d + j] : yy[0];
    if (cjj > 0.0) rr = fmax(rr, cm[j] / sqrt(cjj / (double)m));
  }
  red[threadIdx.x] = rr;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

constexpr int SUPER = 8;  // tiles per super-block side

// Device list of (ti, tj, p) jobs: for each modulus, the lower-triangle tiles in 8 x 8 super-block order;
// workgroup i takes entry (i % 8) * per_xcd + i / 8, so each XCD walks a contiguous run of one modulus'
// super-blocks and its resident workgroups share panels in its L2. Built once per nt (static cache).
const int4* crt_job_list(int nt, int* count) {
  static std::mutex mu;
  static std::map<int, std::pair<int4*, int>> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(nt);
  if (it != cache.end()) {
    *count = it->second.second;
    return it->second.first;
  }
  std::vector<int4> L;
  const int ns = (nt + SUPER - 1) / SUPER;
  for (int p = 0; p < NMOD; ++p)
    for (int I = 0; I < ns; ++I)
      for (int J = 0; J <= I; ++J)
        for (int i = I * SUPER; i < std::min((I + 1) * SUPER, nt); ++i)
          for (int j = J * SUPER; j < std::min((J + 1) * SUPER, nt) && j <= i; ++j) L.push_back(int4{i, j, p, 0});
  int4* dptr = nullptr;
  if (hipMalloc(&dptr, L.size() * sizeof(int4)) != hipSuccess) return nullptr;
  if (hipMemcpy(dptr, L.data(), L.size() * sizeof(int4), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(dptr);
    return nullptr;
  }
  cache[nt] = {dptr, (int)L.size()};
  *count = (int)L.size();
  return dptr;
}

}  // namespace

extern "C" {

// Padded feature count (a multiple of the tile) of an augmented shard of d features.
static long crt_dp(int d) { return ((long)d + 1 + TT - 1) / TT * TT; }

// Workspace bytes of gadmm_gram_crt_f64: the int16 residue Grams (NMOD x Dp x Dp), two chunk buffers of
// residues (NMOD x KC x Dp int8 each), the column-max partials, exponents and maxima.
long gadmm_gram_crt_workspace(long m, int d) {
  (void)m;
  const long Dp = crt_dp(d);
  return (long)NMOD * Dp * Dp * 2 + 2L * NMOD * KC * Dp + (long)CE_R * Dp * 8 + Dp * 4 + Dp * 8 + 1024;
}

long gadmm_gram_crt_max_rows() { return MAX_ROWS; }

// A_n = X_n^T X_n, b_n = X_n^T y_n, yy_n = y_n^T y_n for N shards X (N x m x d, row-major f64) on the
// int8 matrix cores by CRT slicing (see the file comment). Deterministic (exact integer sums, one final
// rounding). ``range_out`` (optional, N doubles): each shard's column-range statistic. The slicing of
// chunk c + 1 runs on a side stream into the other residue buffer while chunk c's GEMM runs on `st`.
int gadmm_gram_crt_f64(const double* X, const double* Y, int N, long m, int d, double* A, double* B, double* YY,
                       void* ws, long ws_bytes, double* range_out, hipStream_t st) {
  if (N <= 0 || m <= 0 || d <= 0) return 0;
  const long Dp = crt_dp(d);
  if (!X || !Y || !A || !B || !YY || !ws || ws_bytes < gadmm_gram_crt_workspace(m, d)) {
    gadmm_set_error("gram_crt: bad arguments or workspace (%ld < %ld bytes)", ws_bytes, gadmm_gram_crt_workspace(m, d));
    return -1;
  }
  if (m > MAX_ROWS) {
    gadmm_set_error("gram_crt: %ld rows exceed the exact-reconstruction bound %ld", m, MAX_ROWS);
    return -1;
  }
  char* w = (char*)ws;
  short* C = (short*)w;
  signed char* Rbuf[2] = {(signed char*)(w + (long)NMOD * Dp * Dp * 2),
                          (signed char*)(w + (long)NMOD * Dp * Dp * 2 + (long)NMOD * KC * Dp)};
  double* part = (double*)(w + (long)NMOD * Dp * Dp * 2 + 2L * NMOD * KC * Dp);
  int* e = (int*)((char*)part + (long)CE_R * Dp * 8);
  double* cm = (double*)((char*)e + ((long)Dp * 4 + 255) / 256 * 256);
  const int nt = (int)(Dp / TT);
  int total = 0;
  const int4* list = crt_job_list(nt, &total);
  if (!list) {
    gadmm_set_error("gram_crt: job list allocation failed");
    return -1;
  }
  const size_t shm = (size_t)2 * STAGE;  // 64 KB
  static std::mutex mu;                  // the side stream and events: one caller at a time
  std::lock_guard<std::mutex> lock(mu);
  int dev = 0;
  GADMM_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) {
    gadmm_set_error("gram_crt: device %d", dev);
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
    GADMM_CHECK(hipFuncSetAttribute((const void*)crt_gemm, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    attr[dev] = true;
  }
  hipStream_t s2 = side[dev];
  hipEvent_t ev_fork = ev[dev][0], ev_join = ev[dev][1], *ev_s = &ev[dev][2], *ev_g = &ev[dev][4];
  const int nc = (int)((m + KC - 1) / KC);
  for (int n = 0; n < N; ++n) {
    const double* Xn = X + (long)n * m * d;
    const double* Yn = Y + (long)n * m;
    hipLaunchKernelGGL(crt_colmax, dim3((unsigned)((Dp + CE_NT - 1) / CE_NT), CE_R), dim3(CE_NT), 0, st, Xn, Yn, m, d,
                       (int)Dp, part);
    hipLaunchKernelGGL(crt_colexp, dim3((unsigned)((Dp + CE_NT - 1) / CE_NT)), dim3(CE_NT), 0, st, part, (int)Dp, e, cm);
    GADMM_CHECK(hipEventRecord(ev_fork, st));
    hipError_t rc = hipStreamWaitEvent(s2, ev_fork, 0);
    for (int c = -1; c < nc && rc == hipSuccess; ++c) {
      if (c >= 0) {  // multiply chunk c (sliced on s2) on st
        rc = hipStreamWaitEvent(st, ev_s[c & 1], 0);
        if (rc != hipSuccess) break;
        long rows = std::min<long>(KC, m - (long)c * KC);
        int kbn = (int)((rows + 31) / 32);
        kbn += kbn & 1;  // whole stages (the slicer zero-fills the extra block)
        hipLaunchKernelGGL(crt_gemm, dim3((unsigned)(8 * ((total + 7) / 8))), dim3(GNT), shm, st, Rbuf[c & 1],
                           (int)Dp, total, list, kbn, C, c == 0 ? 1 : 0);
        rc = hipGetLastError();
        if (rc == hipSuccess) rc = hipEventRecord(ev_g[c & 1], st);
        if (rc != hipSuccess) break;
      }
      if (c + 1 < nc) {  // slice chunk c + 1 on s2 once chunk c - 1 (same buffer) is multiplied
        const int bsel = (c + 1) & 1;
        if (c >= 1) rc = hipStreamWaitEvent(s2, ev_g[bsel], 0);
        if (rc != hipSuccess) break;
        long rows = std::min<long>(KC, m - (long)(c + 1) * KC);
        int kbn = (int)((rows + 31) / 32);
        kbn += kbn & 1;
        hipLaunchKernelGGL(crt_slice, dim3((unsigned)((Dp + SLT - 1) / SLT), (unsigned)kbn), dim3(SLT), 0, s2, Xn, Yn,
                           (long)(c + 1) * KC, m, d, (int)Dp, e, Rbuf[bsel]);
        rc = hipGetLastError();
        if (rc == hipSuccess) rc = hipEventRecord(ev_s[bsel], s2);
      }
    }
    // join on every path: the caller frees the workspace once `st` is done
    const hipError_t j1 = hipEventRecord(ev_join, s2);
    const hipError_t j2 = j1 == hipSuccess ? hipStreamWaitEvent(st, ev_join, 0) : j1;
    if (rc != hipSuccess) {
      gadmm_set_error("gram_crt: %s", hipGetErrorString(rc));
      return (int)rc;
    }
    GADMM_CHECK(j2);
    hipLaunchKernelGGL(crt_finish, dim3((unsigned)((d + 1 + 255) / 256), (unsigned)(d + 1)), dim3(256), 0, st, C,
                       (int)Dp, d, e, A + (long)n * d * d, B + (long)n * d, YY + n);
    GADMM_CHECK(hipGetLastError());
    if (range_out) {
      hipLaunchKernelGGL(crt_range, dim3(1), dim3(256), 0, st, cm, A + (long)n * d * d, YY + n, d, m, range_out + n);
      GADMM_CHECK(hipGetLastError());
    }
  }
  return 0;
}

}  // extern "C"
