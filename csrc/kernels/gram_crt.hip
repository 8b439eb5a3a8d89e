// Augmented Gram (K1) on the INT8 matrix cores by CRT slicing: one int8 GEMM per modulus, ONE int32
// accumulator per output element.
//
// The digit scheme of gram_ozaki.hip needs seven int32 level accumulators per output element, which caps
// its tile at 64 x 64 per workgroup (two per CU) and puts ~13 B/cycle/CU of panel traffic on each MFMA
// (about half of the int8 peak, profiles/r05_h). Here every augmented value x_ij (X | y, column j scaled
// by its power-of-two exponent e_j, |x_ij| <= (127/128) 2^{e_j}) becomes the integer
//   N_ij = rint(x_ij 2^{KB - e_j}),   |N_ij| < 2^KB,  KB = 49   (the digit scheme keeps the same 49 bits)
// and the integer Gram  G_ab = sum_i N_ia N_ib  (|G| < m 2^98 <= 2^119 for m <= 2^21) is computed modulo
// 16 pairwise coprime moduli p <= 234 (product ~2^123.0): for each p, residues R_p == N mod p with
// |R_p| <= 120 are int8, and  G mod p = R_p^T R_p mod p  is ONE int8 GEMM with exact int32 accumulation
// (a chunk of KC samples: KC * 120^2 < 2^31), reduced mod p after every chunk. Garner's
// mixed-radix reconstruction then gives G_ab exactly, and
//   A_ab = 2^{e_a + e_b - 2 KB} G_ab
// with one rounding (the final double). So the result is exact for the 49-bit images of the inputs -- the
// digit scheme's accuracy, with 16 GEMMs instead of 28 digit-pair products, and a 256 x 256 tile per
// workgroup (8 waves of 128 x 64, 128 accumulator registers each): half the panel bytes per MAC of the
// digit kernel's 64 x 64 tile.
//
// Kernels (host driver gadmm_gram_crt_f64 below, per shard, one chunk of KC samples at a time):
//   crt_colmax / crt_colexp   column exponents e_j of the augmented [X | y] (one pass)
//   crt_slice     residues of a chunk: R[p][kb][h][j][16] int8 -- modulus p, 32-sample block kb, half h of
//                 the block (samples 16 h ..), feature j: one MFMA operand fragment row = 16 contiguous
//                 bytes, and the 64 features of one LDS-DMA piece 1 KB contiguous
//   crt_gemm      one workgroup per (lower-triangle 256 x 256 tile, modulus): a 4-stage LDS-DMA ring of
//                 panels (64 samples per stage), 32 v_mfma_i32_16x16x64_i8 per wave per stage with the next
//                 stage's fragment reads and DMA pieces interleaved between them; the chunk's sums go into
//                 the int16 residue matrices C_p (reduced mod p). 74 % MFMA busy (profiles/r06_crt)
//   crt_finish    Garner per lower-triangle element -> A (full symmetric), b, y'y
//   crt_range     the column-range statistic of linalg.gram's accuracy gate
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <utility>
#include <map>
#include <mutex>
#include <vector>
#include "gadmm_common.h"

typedef int v4i __attribute__((ext_vector_type(4)));

namespace {

constexpr int NMOD = 16;
// pairwise coprime, each <= 234 so that the slicer's representatives |r| <= 0.511 p <= 120 fit int8 (below), product
// 2^123.0 > 2 * 2^21 * 2^98 (greedy from 234 down: 16 moduli instead of the 19 moduli <= 127 of the first cut,
// ~16 % fewer int8 GEMMs, profiles/r06_crt)
constexpr int kMod[NMOD] = {234, 233, 229, 227, 223, 217, 215, 211, 209, 199, 197, 193, 191, 181, 179, 173};
// kInv[i][j] = (kMod[j] mod kMod[i])^{-1} mod kMod[i], j < i (Garner); generated and checked by
// tests/test_gram_crt_math.py
constexpr int kInv[NMOD][NMOD] = {
    {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {46, 172, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {65, 38, 114, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {142, 67, 186, 56, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {166, 95, 199, 152, 181, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {34, 12, 169, 18, 27, 108, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {156, 48, 129, 66, 88, 176, 53, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {92, 61, 115, 151, 15, 183, 35, 105, 0, 0, 0, 0, 0, 0, 0, 0},
    {91, 41, 73, 64, 141, 188, 112, 83, 20, 0, 0, 0, 0, 0, 0, 0},
    {16, 104, 117, 46, 144, 69, 11, 183, 115, 99, 0, 0, 0, 0, 0, 0},
    {113, 111, 59, 176, 148, 185, 79, 118, 181, 161, 145, 0, 0, 0, 0, 0},
    {40, 141, 186, 69, 6, 169, 8, 86, 138, 24, 32, 96, 0, 0, 0, 0},
    {41, 94, 132, 122, 125, 176, 16, 175, 97, 171, 34, 166, 163, 0, 0, 0},
    {166, 63, 111, 138, 118, 33, 5, 28, 6, 9, 10, 64, 15, 90, 0, 0},
    {156, 124, 34, 157, 45, 59, 103, 41, 149, 20, 137, 26, 125, 65, 29, 0}};
__constant__ int kModDev[NMOD] = {234, 233, 229, 227, 223, 217, 215, 211, 209, 199, 197, 193, 191, 181, 179, 173};

constexpr int KB = 49;            // bits of every value's integer image (|N| < 2^KB)
constexpr long MAX_ROWS = 1L << 21;  // m 2^{2 KB} < M / 2 (the product of the moduli): exact reconstruction
constexpr int KC = 32768;         // samples per chunk: KC * 120^2 < 2^31 (exact int32 sums)
constexpr int KBC = KC / 32;      // 32-sample blocks per chunk
constexpr int KBCP = KBC + 4;     // residue-buffer slots per modulus: a chunk zero-filled to whole stages
constexpr int TT = 256;           // output tile (features) per workgroup
constexpr int GNT = 512;          // 8 waves: 2 (rows of 128) x 4 (columns of 64)
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

// Residues of samples [i0, i0 + 32 kbn) (zero from iend on) into R[p][kb][h][j][16]: a thread takes one
// feature and 16 samples (one half h) at a time, so a wave's store per modulus is 1 KB contiguous (with
// [j][32] rows, each store covered half of a 2 KB span: the slicer ran at ~2.4 TB/s). Each integer image N is split
// once into 13-bit digits, N = d3 2^39 + d2 2^26 + d1 2^13 + d0 (d3 in [-2^10, 2^10), the others in
// [0, 2^13); exact double floor / fma), held as floats with d0 offset by MAGIC = 1.5 2^23. Then per modulus,
// in f32 only (exact: every intermediate is an integer below 2^24; |S' - MAGIC| < 2^13 + 2^13 (233 + 233) +
// 2^10 233 < 2^22 for every p <= 234):
//   S' = MAGIC + d0 + d1 (2^13 mod p) + d2 (2^26 mod p) + d3 (2^39 mod p)   in [2^23, 2^24), S' - MAGIC == N mod p
//   q  = rint(S' / p - MAGIC / p)         (one fma with rounded constants: within 0.011 of (S' - MAGIC) / p)
//   t  = S' - q p = MAGIC + r,  |r| <= 120 (|(S' - MAGIC) / p - q| <= 0.511 for 173 <= p <= 234)
// and the low byte of t's bit pattern IS r as int8 (the exponent is fixed at 2^23 over the whole range).
// r is a valid int8 representative of N mod p (not always the balanced one, which nothing needs: the GEMM
// epilogue reduces mod p, and the chunk sums stay exact, KC 120^2 < 2^31). Six f32 instructions per residue;
// round 6's first version (a per-modulus f64 divide-and-correct) made the slicer 12 % of the Gram, and
// plain int products compile to quarter-rate v_mul_lo_u32 / v_mad_u64_u32 (profiles/r06_crt).
constexpr float MAGIC = 12582912.0f;  // 1.5 2^23
constexpr int p2mod(int k, int p) {
  int r = 1 % p;
  for (int i = 0; i < k; ++i) r = (r * 2) % p;
  return r;
}
template <int P>
__device__ __forceinline__ unsigned crt_res(float D0, float d1, float d2, float d3) {
  constexpr int mp = kMod[P];
  constexpr float w1 = (float)p2mod(13, mp), w2 = (float)p2mod(26, mp), w3 = (float)p2mod(39, mp);
  constexpr float fp = (float)mp, ip = 1.0f / (float)mp, nm = -MAGIC / (float)mp;
  const float S = __builtin_fmaf(d3, w3, __builtin_fmaf(d2, w2, __builtin_fmaf(d1, w1, D0)));
  const float q = __builtin_rintf(__builtin_fmaf(S, ip, nm));
  return __float_as_uint(__builtin_fmaf(-q, fp, S));  // low byte = r
}
template <int P>
__device__ __forceinline__ void crt_res_store(const float (&D)[4][16], signed char* dst) {
  int w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned u[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) u[b] = crt_res<P>(D[0][4 * q + b], D[1][4 * q + b], D[2][4 * q + b], D[3][4 * q + b]);
    // v_perm_b32 (selector bytes 0-3: src1's bytes, 4-7: src0's, 0x0c: zero): the four low bytes in order
    const unsigned lo = __builtin_amdgcn_perm(u[1], u[0], 0x0c0c0400u);
    const unsigned hi = __builtin_amdgcn_perm(u[3], u[2], 0x0c0c0400u);
    w[q] = (int)__builtin_amdgcn_perm(hi, lo, 0x05040100u);
  }
  *reinterpret_cast<v4i*>(dst) = v4i{w[0], w[1], w[2], w[3]};
}
template <int... Ps>
__device__ __forceinline__ void crt_res_all(const float (&D)[4][16], signed char* dst, long pstride,
                                            std::integer_sequence<int, Ps...>) {
  (crt_res_store<Ps>(D, dst + Ps * pstride), ...);
}
__global__ void __launch_bounds__(SLT) crt_slice(const double* X, const double* y, long i0, long iend, int d, int Dp,
                                                 const int* e, signed char* R) {
  // iend: the chunk's end (min(m, i0 + KC)); the blocks padded up to a whole stage beyond it are zeros
  const int kb = blockIdx.y;
  const int j = blockIdx.x * SLT + threadIdx.x;
  if (j >= Dp) return;
  const int ej = e[j];
#pragma unroll 1
  for (int hh = 0; hh < 2; ++hh) {
    float D[4][16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const long i = i0 + (long)kb * 32 + hh * 16 + t;
      const double n = rint(ldexp(aug_at(X, y, i, j, iend, d), KB - ej));  // exact: |N| < 2^49
      const double a3 = floor(n * 0x1p-39);
      const double r3 = fma(-a3, 0x1p39, n);
      const double a2 = floor(r3 * 0x1p-26);
      const double r2 = fma(-a2, 0x1p26, r3);
      const double a1 = floor(r2 * 0x1p-13);
      D[3][t] = (float)a3;
      D[2][t] = (float)a2;
      D[1][t] = (float)a1;
      D[0][t] = (float)fma(-a1, 0x1p13, r2) + MAGIC;
    }
    crt_res_all(D, R + (long)kb * Dp * 32 + (long)hh * Dp * 16 + (long)j * 16, (long)KBCP * Dp * 32,
                std::make_integer_sequence<int, NMOD>{});
  }
}

// One chunk of one modulus on one 256 x 256 lower-triangle tile: C_p[a][b] = (C_p + sum_k R_p[k][a]
// R_p[k][b]) mod p for the tile's features a (rows) and b (columns). 8 waves: wave (wr, wc) owns rows
// 128 wr .. +127 (4 blocks of 32) and columns 64 wc .. +63 (2 blocks). Per stage (64 samples = 2 MFMA
// K-steps) the A and B panels (each 2 x 256 features x 32 samples, 16 KB, contiguous in global memory
// and in LDS) come in by LDS-DMA (global_load_lds_dwordx4: a wave instruction moves 1 KB; 32 per stage,
// 4 per wave) through a 4-buffer ring, three stages ahead of the 16 MFMAs per wave of the current one. A
// fragment read (ds_read_b128 of 64 lanes: 32 consecutive features x 2 halves) covers 1 KB contiguous:
// conflict-free.
// s_waitcnt through the builtin (not inline asm: the compiler's wait-count pass treats an asm statement
// as unknown LDS / memory traffic and then drains every later use to lgkmcnt(0), which would put the
// stage's fragment reads back in front of the MFMAs they are meant to overlap). gfx9 encoding: vmcnt
// bits [3:0] and [15:14], expcnt [6:4], lgkmcnt [11:8]; unnamed counters at their maxima.
template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt((0xF) | (0x3 << 14) | (0x7 << 4)); }

// BKS: 32-sample blocks per pipeline stage (even); NSTG: LDS ring of stage buffers (NSTG - 1 stages in
// flight). The MFMA is v_mfma_i32_16x16x64_i8: per 64-sample K step a wave reads FA = 8 A and FB = 4 B
// fragments (16 contiguous bytes per lane of the LDS image below) and runs 32 MFMAs into 32 accumulators
// of 16 x 16 (128 registers). Against v_mfma_i32_32x32x32_i8 with the same reads and accumulator
// registers per stage (4 + 2 fragments and 8 MFMAs per 32-sample step): 0.94 vs 1.12 s at
// 2 x 625k x 10k, same box (profiles/r06_crt/mf) -- the MI355X_MICROARCH.md observation that the
// 16 x 16 shapes deliver ~1.15x the 32 x 32 ones' rate, here for int8.
template <int BKS, int NSTG>
__global__ void __launch_bounds__(GNT, 1) crt_gemm(const signed char* R, int Dp, int per, const int4* list,
                                                   int kbn, short* C, int first) {
  constexpr int MF = 16, FA = 8, FB = 4, FR = FA + FB, NACC = 4;
  constexpr int KS = BKS / 2;  // MFMA K steps (64 samples) per stage
  static_assert(KS * 2 == BKS, "whole K steps per stage");
  constexpr int PANEL = BKS * TT * 32;  // bytes of one operand panel per stage
  constexpr int STAGE = 2 * PANEL;      // A + B
  constexpr int P = 2 * BKS;            // DMA pieces (1 KB) per wave per stage
  extern __shared__ __attribute__((aligned(16))) signed char lds[];  // NSTG stages x STAGE bytes
  const int4 job = list[(int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3)];  // crt_job_list
  if (job.x < 0) return;
  const int ti = job.x, tj = job.y, p = job.z;
  const int mp = kModDev[p];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wr = wv >> 2, wc = wv & 3;
  const signed char* gA = R + (long)p * KBCP * Dp * 32 + (long)ti * TT * 16;  // + kb * Dp * 32 + h * Dp * 16
  const signed char* gB = R + (long)p * KBCP * Dp * 32 + (long)tj * TT * 16;
  const long kbstride = (long)Dp * 32;
  // LDS image of a stage: [panel A / B][32-sample block][half of the block: samples 16 h ..][feature][16 B]
  // -- the global layout's order, so every DMA piece is 1 KB contiguous on both sides, and a fragment
  // read is conflict-free in ds_read_b128's lane groups: lanes 16 q .. 16 q + 15 read 16 consecutive
  // features of the (block q / 2, half q % 2) plane, the planes 4 KB apart (with [feature][32 B] rows the
  // 32-B stride used only half of the banks: 2-way conflicts). This wave's P pieces per stage: piece c = P wv + u: panel c / (8 BKS), block
  // (c / 8) % BKS, half (c / 4) % 2, features 64 (c % 4) .. + 63 (1 KB of LDS).
  // a fragment's lane offset inside a K step of a panel: lane l holds samples 16 (l / 16) .. + 15 of row l % 16
  const int lane_off = (lane >> 5) * (TT * 32) + ((lane >> 4) & 1) * (TT * 16) + (lane & 15) * 16;
  v4i acc[FA * FB];
#pragma unroll
  for (int i = 0; i < FA * FB; ++i) acc[i] = v4i{};
  const int nst = kbn / BKS;  // kbn is a multiple of BKS (the slicer zero-fills to a stage boundary)
  // Software pipeline over stages, two levels deep:
  //  * LDS-DMA: a ring of NSTG stage buffers, NSTG - 1 stages in flight (stage s + NSTG - 1 is issued during
  //    stage s into stage s - 1's buffer). Every step issues its P pieces -- past the last stage they
  //    re-load stage nst - 1 into the free buffer -- so the count of this wave's pieces still flying at the
  //    top of a step is always (NSTG - 2) P and the wait is one counted vmcnt. A raw s_barrier -- not
  //    __syncthreads(), whose fence would drain them (cdna_hip_programming.md §5, "Pipelining across
  //    barriers") -- then makes every wave's stage s visible and every wave's fragment reads of stage s - 1
  //    complete;
  //  * fragments: stage s's NR ds_read_b128 go into one register set while the NM MFMAs of stage s - 1 run
  //    from the other;
  //  * one interleaved stream per step: MFMA, fragment read, MFMA, ..., with a DMA piece after every
  //    NM / P MFMAs (pinned by sched_group_barrier). An LDS-DMA piece costs its wave 60-185 issue cycles
  //    (MI355X_MICROARCH.md, per-instruction constants): issued as a block at the top of the step, behind
  //    the barrier that lines both waves of a SIMD up, they idled the matrix pipe (51 % MFMA busy); between
  //    MFMAs they overlap the matrix pipe's work.
  constexpr int NM = KS * FA * FB, NR = KS * FR, EVERY = NM / P;
  static_assert(NR <= NM && NM % P == 0, "interleave shape");
  v4i fr0[NR], fr1[NR];
  auto read_frag = [&](const signed char* SA, int i, v4i (&fr)[NR]) {
    const int ks = i / FR, f = i % FR;
    const int step_off = ks * 2 * (TT * 32);
    const signed char* q = f < FA ? SA + step_off + (wr * 128 + MF * f) * 16
                                  : SA + PANEL + step_off + (wc * 64 + MF * (f - FA)) * 16;
    fr[i] = *reinterpret_cast<const v4i*>(q + lane_off);
  };
  auto mma = [&](int m, const v4i (&fr)[NR]) {
    const int ks = m / (FA * FB), a = (m / FB) % FA, b = m % FB;
    acc[a * FB + b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fr[ks * FR + a], fr[ks * FR + FA + b], acc[a * FB + b], 0, 0, 0);
  };
  auto issue_piece = [&](int st, int u) {  // piece u of this wave for stage st (clamped to the last stage)
    const int sc = st < nst ? st : nst - 1;
    const int c = P * wv + u;
    const int pn = c / (8 * BKS), blk = (c >> 3) % BKS, hh = (c >> 2) & 1, q = c & 3;
    const signed char* src = (pn ? gB : gA) + (long)(sc * BKS + blk) * kbstride + (long)hh * (kbstride / 2) + (q * 64 + lane) * 16;
    signed char* dst = lds + (st % NSTG) * STAGE + pn * PANEL + blk * (TT * 32) + hh * (TT * 16) + q * 1024;
    __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
  };
  auto top = [&]() {
    wait_vm<(NSTG - 2) * P>();
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
  };
  // stage s: read its fragments into fr while the MFMAs of stage s - 1 run from fu
  auto step = [&](int s, v4i (&fr)[NR], const v4i (&fu)[NR]) {
    top();
    const signed char* SA = lds + (s % NSTG) * STAGE;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      mma(m, fu);
      if (m < NR) read_frag(SA, m, fr);
      if (m % EVERY == EVERY - 1) issue_piece(s + NSTG - 1, m / EVERY);
    }
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                  // MFMA
      if (m < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);      // DS read
      if (m % EVERY == EVERY - 1) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (LDS-DMA)
    }
    __builtin_amdgcn_s_setprio(0);
  };
  if (nst > 0) {
    for (int s0 = 0; s0 < NSTG - 1; ++s0)
#pragma unroll
      for (int u = 0; u < P; ++u) issue_piece(s0, u);
    top();
#pragma unroll
    for (int u = 0; u < P; ++u) issue_piece(NSTG - 1, u);
#pragma unroll
    for (int i = 0; i < NR; ++i) read_frag(lds, i, fr0);
    int s = 1;
    for (; s + 1 < nst; s += 2) {
      step(s, fr1, fr0);
      step(s + 1, fr0, fr1);
    }
    wait_lgkm0();
    if (s < nst) {  // nst even: stage nst - 1 still to read
      step(s, fr1, fr0);
      wait_lgkm0();
#pragma unroll
      for (int m = 0; m < NM; ++m) mma(m, fr1);
    } else {  // nst odd: stage nst - 1 is in fr0
#pragma unroll
      for (int m = 0; m < NM; ++m) mma(m, fr0);
    }
    wait_vm<0>();  // the clamped re-loads past the last stage land before the workgroup's LDS is released
  }
  // epilogue: C_p = (C_p + chunk sum) mod p, symmetric, as int16. The previous chunks' residues of one
  // accumulator are read before any is used: a per-element load behind the `first` test would make hipcc
  // branch around each load and wait for it alone (cdna_hip_programming.md §5, trap (c)).
  // Output element g of accumulator (a, b): row 16 a + 4 (lane / 16) + g, column 16 b + lane % 16.
  short* Cp = C + (long)p * Dp * Dp;
  const int hm = mp >> 1;
#pragma unroll
  for (int a = 0; a < FA; ++a)
#pragma unroll
    for (int b = 0; b < FB; ++b) {
      const int col = tj * TT + wc * 64 + MF * b + (lane & (MF - 1));
      const long base = (long)(ti * TT + wr * 128 + MF * a + 4 * (lane / MF)) * Dp + col;
      auto roff = [&](int g) -> long { return (long)g * Dp; };
      int old[NACC];
      if (first) {
#pragma unroll
        for (int g = 0; g < NACC; ++g) old[g] = 0;
      } else {
#pragma unroll
        for (int g = 0; g < NACC; ++g) old[g] = Cp[base + roff(g)];
      }
#pragma unroll
      for (int g = 0; g < NACC; ++g) {
        int v = acc[a * FB + b][g] % mp + old[g];
        v %= mp;
        if (v > hm) v -= mp;
        if (v < -hm) v += mp;
        Cp[base + roff(g)] = (short)v;
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

// Device job lists, one run per XCD: workgroup i takes entry (i % 8) * per + i / 8 of a list of 8 runs of
// `per` entries ({-1} pads a short run), i.e. XCD i % 8 walks its own run (the round-robin dispatch of
// consecutive workgroups to the 8 XCDs). Jobs are (ti, tj, p) lower-triangle tiles of one modulus after
// another, in 16 x 16 super-blocks, each cut into eight 4 x 8 sub-blocks dealt to the 8 XCDs (least-loaded
// first): the XCDs work on ONE super-block at a time, so an XCD's ~32 resident workgroups share 12 panels in
// its L2 and the super-block's 32 panels are shared across XCDs in the Infinity Cache. Measured against each
// XCD taking a contiguous eighth of the jobs (8 unrelated regions streamed from HBM): L2 hit 58 -> 68 %,
// 1.36 -> 1.32 s at 2 x 625k x 10k (profiles/r06_crt). Built once per nt (static cache).
struct JobList {
  int4* dev;
  int per;
};
JobList crt_job_list(int nt) {
  static std::mutex mu;
  static std::map<int, JobList> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(nt);
  if (it != cache.end()) return it->second;
  std::vector<std::vector<int4>> run(8);
  {
    constexpr int S = 16;
    const int ns = (nt + S - 1) / S;
    for (int p = 0; p < NMOD; ++p)
      for (int I = 0; I < ns; ++I)
        for (int J = 0; J <= I; ++J) {
          std::vector<std::vector<int4>> sub;
          for (int sb = 0; sb < 8; ++sb) {
            const int i0 = I * S + 4 * (sb >> 1), j0 = J * S + 8 * (sb & 1);
            std::vector<int4> t;
            for (int i = i0; i < std::min(i0 + 4, nt); ++i)
              for (int j = j0; j < std::min(j0 + 8, nt) && j <= i; ++j) t.push_back(int4{i, j, p, 0});
            if (!t.empty()) sub.push_back(std::move(t));
          }
          // largest sub-block first, each to the least-loaded XCD: the runs stay within a few jobs of
          // each other (max / mean 1.006 at d = 10k), so the XCDs stay on the same super-block
          std::stable_sort(sub.begin(), sub.end(), [](const std::vector<int4>& a, const std::vector<int4>& b) {
            return a.size() > b.size();
          });
          for (auto& t : sub) {
            int x = 0;
            for (int k = 1; k < 8; ++k)
              if (run[k].size() < run[x].size()) x = k;
            run[x].insert(run[x].end(), t.begin(), t.end());
          }
        }
  }
  size_t per = 0;
  for (auto& r : run) per = std::max(per, r.size());
  std::vector<int4> flat(8 * per, int4{-1, -1, -1, 0});
  for (int x = 0; x < 8; ++x) std::copy(run[x].begin(), run[x].end(), flat.begin() + x * per);
  JobList jl{nullptr, (int)per};
  if (hipMalloc(&jl.dev, flat.size() * sizeof(int4)) != hipSuccess) return JobList{nullptr, 0};
  if (hipMemcpy(jl.dev, flat.data(), flat.size() * sizeof(int4), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(jl.dev);
    return JobList{nullptr, 0};
  }
  cache[nt] = jl;
  return jl;
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
  return (long)NMOD * Dp * Dp * 2 + 2L * NMOD * KBCP * 32 * Dp + (long)CE_R * Dp * 8 + Dp * 4 + Dp * 8 + 1024;
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
  const long rbytes = (long)NMOD * KBCP * 32 * Dp;
  signed char* Rbuf[2] = {(signed char*)(w + (long)NMOD * Dp * Dp * 2),
                          (signed char*)(w + (long)NMOD * Dp * Dp * 2 + rbytes)};
  double* part = (double*)(w + (long)NMOD * Dp * Dp * 2 + 2L * rbytes);
  int* e = (int*)((char*)part + (long)CE_R * Dp * 8);
  double* cm = (double*)((char*)e + ((long)Dp * 4 + 255) / 256 * 256);
  const int nt = (int)(Dp / TT);
  const JobList jl = crt_job_list(nt);
  const int4* list = jl.dev;
  if (!list) {
    gadmm_set_error("gram_crt: job list allocation failed");
    return -1;
  }
  // pipeline: 2 blocks (64 samples) per stage, a ring of 4 stage buffers (128 KB of LDS). Measured against
  // 4x2, 3x3, 2x3 and 1x4 (BKS x NSTG) at 625k x 10k: 0.742 s vs 0.818 / 0.853 / 0.776 / 0.780 (profiles/r06_crt)
  constexpr int bks = 2, nstg = 4;
  const void* kfn = (const void*)crt_gemm<bks, nstg>;
  const size_t shm = (size_t)nstg * 2 * bks * TT * 32;
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
    GADMM_CHECK(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    attr[dev] = true;
  }
  hipStream_t s2 = side[dev];
  hipEvent_t ev_fork = ev[dev][0], ev_join = ev[dev][1], *ev_s = &ev[dev][2], *ev_g = &ev[dev][4];
  const int nc = (int)((m + KC - 1) / KC);
  int Dp32 = (int)Dp;
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
        kbn = (kbn + bks - 1) / bks * bks;  // whole stages (the slicer zero-fills the extra blocks)
        const signed char* Rc = Rbuf[c & 1];
        int per_ = jl.per, first_ = c == 0 ? 1 : 0;
        void* kargs[] = {(void*)&Rc, (void*)&Dp32, (void*)&per_, (void*)&list, (void*)&kbn, (void*)&C,
                         (void*)&first_};
        rc = hipLaunchKernel(kfn, dim3((unsigned)(8 * jl.per)), dim3(GNT), kargs, shm, st);
        if (rc == hipSuccess) rc = hipGetLastError();
        if (rc == hipSuccess) rc = hipEventRecord(ev_g[c & 1], st);
        if (rc != hipSuccess) break;
      }
      if (c + 1 < nc) {  // slice chunk c + 1 on s2 once chunk c - 1 (same buffer) is multiplied
        const int bsel = (c + 1) & 1;
        if (c >= 1) rc = hipStreamWaitEvent(s2, ev_g[bsel], 0);
        if (rc != hipSuccess) break;
        long rows = std::min<long>(KC, m - (long)(c + 1) * KC);
        int kbn = (int)((rows + 31) / 32);
        kbn = (kbn + bks - 1) / bks * bks;
        hipLaunchKernelGGL(crt_slice, dim3((unsigned)((Dp + SLT - 1) / SLT), (unsigned)kbn), dim3(SLT), 0, s2, Xn, Yn,
                           (long)(c + 1) * KC, std::min<long>(m, (long)(c + 2) * KC), d, (int)Dp, e, Rbuf[bsel]);
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
