// Split-column ("quad") register GEMV for matrices with <= 64 rows, shared by the persistent
// linear kernels (chain_blocked.hip) and the logistic inner-GD phase (chain_small.hip).
#pragma once
#include <hip/hip_runtime.h>

// Split-column register GEMV for d <= 64 ("quad" layout). Lane l = i + 16c (i < 16, c < 4) holds
// the rows i, i+16, i+32, i+48 of M restricted to the columns j = c + 4t (t < T), so each lane
// needs only T broadcast x values instead of 4T: the LDS data return of a GEMV drops from 4T
// ds_read_b128 per wave (reg_gemv, the phase bottleneck at several GEMV waves per CU,
// profiles/r01_persistent_timeline) to T/2 + 4 reads. Lane (i, c) accumulates exactly reg_gemv's
// accumulator a_c (columns j = c mod 4, ascending) for its four rows; the four partials of row l
// meet in lane l through wave-private LDS and are added ((a0 + a1) + a2) + a3, so the result is
// bit-identical to reg_gemv / symv_lds / symv_cols. x: this lane's element x_l (zero beyond d).
// st: QSTAGE doubles of LDS private to the calling wave. Returns y_l in lane l.
constexpr int QX = 18;  // permuted-x class stride: 2*18 mod 32 banks = 4 -> disjoint 4-bank windows
constexpr int QR = 68;  // partial class stride: 2*68 mod 32 = 8
constexpr int QSTAGE = 4 * QX + 4 * QR;

template <int T>
__device__ __forceinline__ void quad_load(double (&m)[4][T], const double* M, int d, bool on) {
  const int lane = threadIdx.x & 63, i = lane & 15, c = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int row = i + 16 * r, col = c + 4 * t;
      m[r][t] = (on && row < d && col < d) ? M[(long)row * d + col] : 0.0;
    }
}

// Transpose-reduce of the four per-class partials of a quad GEMV without LDS: lane i + 16c holds
// p[r] = class c's partial of row i + 16r. Two v_permlane32_swap exchanges (class pairs {0,1} <->
// {2,3}) then two v_permlane16_swap exchanges (0 <-> 1, 2 <-> 3) leave lane l = i + 16g holding
// class c's partial of row l in p[c], which are summed ((p0 + p1) + p2) + p3: the same order as
// the LDS reduction, so the result is bit-identical, with 8 cross-lane VALU moves instead of two
// dependent LDS round trips.
__device__ __forceinline__ void swap32_f64(double& a, double& b) {  // lanes 32-63 of a <-> lanes 0-31 of b
  const long long ua = __double_as_longlong(a), ub = __double_as_longlong(b);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
  a = __longlong_as_double(((long long)hi[0] << 32) | lo[0]);
  b = __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ void swap16_f64(double& a, double& b) {  // lanes 16-31 (48-63) of a <-> 0-15 (32-47) of b
  const long long ua = __double_as_longlong(a), ub = __double_as_longlong(b);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ua, (unsigned)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
  a = __longlong_as_double(((long long)hi[0] << 32) | lo[0]);
  b = __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ double quad_reduce(double (&p)[4]) {
  swap32_f64(p[0], p[2]);
  swap32_f64(p[1], p[3]);
  swap16_f64(p[0], p[1]);
  swap16_f64(p[2], p[3]);
  return ((p[0] + p[1]) + p[2]) + p[3];
}

template <int T>
__device__ __forceinline__ double quad_gemv(const double (&m)[4][T], double x, double* st) {
  static_assert(T >= 1 && T <= 16, "quad layout covers d <= 64");
  const int lane = threadIdx.x & 63, c = lane >> 4;
  st[(lane & 3) * QX + (lane >> 2)] = x;
  asm volatile("" ::: "memory");  // LDS is in order within a wave; keep the compiler from hoisting
  const double* xs = st + c * QX;
  double p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int t = 0; t < T; t += 2) {  // x pairs consumed as they arrive (VGPR budget at 3 waves/SIMD)
    const double2 xp = *reinterpret_cast<const double2*>(xs + t);
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = fma(m[r][t], xp.x, p[r]);
    if (t + 1 < T) {
#pragma unroll
      for (int r = 0; r < 4; ++r) p[r] = fma(m[r][t + 1], xp.y, p[r]);
    }
  }
#ifdef GADMM_QUAD_LDS_REDUCE  // the LDS transpose-reduce (A/B reference build)
  double* red = st + 4 * QX;
#pragma unroll
  for (int r = 0; r < 4; ++r) red[c * QR + (lane & 15) + 16 * r] = p[r];
  asm volatile("" ::: "memory");
  const double q0 = red[lane], q1 = red[QR + lane], q2 = red[2 * QR + lane], q3 = red[3 * QR + lane];
  asm volatile("" ::: "memory");  // the next call's writes stay behind these reads
  return ((q0 + q1) + q2) + q3;
#else
  asm volatile("" ::: "memory");  // the next call's x store stays behind this call's x reads
  return quad_reduce(p);
#endif
}

// quad_gemv with the broadcast vector already staged by another wave in quad_gemv's x layout
// (xs0[(l & 3) * QX + (l >> 2)] = x_l): the same FMAs and reduction, without this wave's staging write.
template <int T>
__device__ __forceinline__ double quad_gemv_staged(const double (&m)[4][T], const double* xs0) {
  static_assert(T >= 1 && T <= 16, "quad layout covers d <= 64");
  const int lane = threadIdx.x & 63, c = lane >> 4;
  const double* xs = xs0 + c * QX;
  double p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int t = 0; t < T; t += 2) {
    const double2 xp = *reinterpret_cast<const double2*>(xs + t);
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = fma(m[r][t], xp.x, p[r]);
    if (t + 1 < T) {
#pragma unroll
      for (int r = 0; r < 4; ++r) p[r] = fma(m[r][t + 1], xp.y, p[r]);
    }
  }
  asm volatile("" ::: "memory");
  return quad_reduce(p);
}

// Quad layout kept in LDS instead of VGPRs (a matrix used off the critical path, e.g. the exact
// objective's Gram): element m[r][t] of lane l at Ml[((t >> 1) * 4 + r) * 128 + 2 l + (t & 1)], so a
// lane reads its (t, t + 1) pair with one 16-byte load. quad_gemv_lds performs quad_gemv's FMAs in
// the same order (bit-identical). Ml: 4 * 64 * (T + (T & 1)) doubles of LDS private to the wave.
template <int T>
__device__ __forceinline__ void quad_store_lds(double* Ml, const double* M, int d, bool on) {
  const int lane = threadIdx.x & 63, i = lane & 15, c = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int t = 0; t < T + (T & 1); ++t) {
      const int row = i + 16 * r, col = c + 4 * t;
      Ml[((t >> 1) * 4 + r) * 128 + 2 * lane + (t & 1)] =
          (on && t < T && row < d && col < d) ? M[(long)row * d + col] : 0.0;
    }
}

template <int T>
__device__ __forceinline__ double quad_gemv_lds(const double* Ml, double x, double* st) {
  static_assert(T >= 1 && T <= 16, "quad layout covers d <= 64");
  const int lane = threadIdx.x & 63, c = lane >> 4;
  st[(lane & 3) * QX + (lane >> 2)] = x;
  asm volatile("" ::: "memory");
  const double* xs = st + c * QX;
  double p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int t = 0; t < T; t += 2) {
    const double2 xp = *reinterpret_cast<const double2*>(xs + t);
    double2 mv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mv[r] = *reinterpret_cast<const double2*>(Ml + ((t >> 1) * 4 + r) * 128 + 2 * lane);
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = fma(mv[r].x, xp.x, p[r]);
    if (t + 1 < T) {
#pragma unroll
      for (int r = 0; r < 4; ++r) p[r] = fma(mv[r].y, xp.y, p[r]);
    }
  }
  asm volatile("" ::: "memory");
  return quad_reduce(p);
}

// One row group r of quad_gemv_lds (rows i + 16 r): lane (i, c)'s partial p[r] -- the accumulator
// quad_gemv keeps for that group, same FMAs in the same order. Four waves running r = 0..3 and a
// quad_reduce of their four partials (in lane order) give quad_gemv's result bit for bit; each wave
// reads a quarter of the image (chain_blocked.hip: the hosted halo head).
template <int T>
__device__ __forceinline__ double quad_rowgroup_lds(const double* Ml, int r, double x, double* st) {
  static_assert(T >= 1 && T <= 16, "quad layout covers d <= 64");
  const int lane = threadIdx.x & 63, c = lane >> 4;
  st[(lane & 3) * QX + (lane >> 2)] = x;
  asm volatile("" ::: "memory");
  const double* xs = st + c * QX;
  double p = 0.0;
#pragma unroll
  for (int t = 0; t < T; t += 2) {
    const double2 xp = *reinterpret_cast<const double2*>(xs + t);
    const double2 mv = *reinterpret_cast<const double2*>(Ml + ((t >> 1) * 4 + r) * 128 + 2 * lane);
    p = fma(mv.x, xp.x, p);
    if (t + 1 < T) p = fma(mv.y, xp.y, p);
  }
  asm volatile("" ::: "memory");  // the next call's x store stays behind this call's x reads
  return p;
}

// Paired layout for two matrices with <= 52 rows held by one wave (chain_blocked_pair_kernel):
// each keeps its row groups r = 0..2 (rows i + 16r) as in quad_load, and the two share ONE register
// block for rows 48..51: lanes with i < 4 hold matrix 0's row 48 + i, lanes with 4 <= i < 8 hold
// matrix 1's row 48 + (i - 4). 3T + 3T + T doubles per lane instead of 8T (T = 13: 182 VGPRs, so
// two waves per SIMD fit in the 256-register budget). Same per-row accumulation order as quad_gemv.
template <int T>
__device__ __forceinline__ void quad_load_pair(double (&m0)[3][T], double (&m1)[3][T], double (&s3)[T],
                                               const double* M0, const double* M1, int d, bool on0, bool on1) {
  const int lane = threadIdx.x & 63, i = lane & 15, c = lane >> 4;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int row = i + 16 * r, col = c + 4 * t;
      m0[r][t] = (on0 && row < d && col < d) ? M0[(long)row * d + col] : 0.0;
      m1[r][t] = (on1 && row < d && col < d) ? M1[(long)row * d + col] : 0.0;
    }
  const int q = i & 3, which = i >> 2;  // which = 0: matrix 0, 1: matrix 1, else unused
  const double* Ms = which == 0 ? M0 : M1;
  const bool ons = (which == 0 && on0) || (which == 1 && on1);
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int row = 48 + q, col = c + 4 * t;
    s3[t] = (ons && row < d && col < d) ? Ms[(long)row * d + col] : 0.0;
  }
}

// y_l = (M_sel x)_l for the paired layout (sel = 0 / 1, wave-uniform), lane l in, lane l out.
template <int T>
__device__ __forceinline__ double quad_gemv_pair(const double (&m)[3][T], const double (&s3)[T], int sel, double x,
                                                 double* st) {
  static_assert(T >= 1 && T <= 13, "paired layout covers d <= 52");
  const int lane = threadIdx.x & 63, i = lane & 15, c = lane >> 4;
  st[(lane & 3) * QX + (lane >> 2)] = x;
  asm volatile("" ::: "memory");
  const double* xs = st + c * QX;
  double p[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int t = 0; t < T; t += 2) {
    const double2 xp = *reinterpret_cast<const double2*>(xs + t);
#pragma unroll
    for (int r = 0; r < 3; ++r) p[r] = fma(m[r][t], xp.x, p[r]);
    p[3] = fma(s3[t], xp.x, p[3]);
    if (t + 1 < T) {
#pragma unroll
      for (int r = 0; r < 3; ++r) p[r] = fma(m[r][t + 1], xp.y, p[r]);
      p[3] = fma(s3[t + 1], xp.y, p[3]);
    }
  }
  double* red = st + 4 * QX;
#pragma unroll
  for (int r = 0; r < 3; ++r) red[c * QR + i + 16 * r] = p[r];
  if ((i >> 2) == sel) red[c * QR + 48 + (i & 3)] = p[3];
  asm volatile("" ::: "memory");
  const double q0 = red[lane], q1 = red[QR + lane], q2 = red[2 * QR + lane], q3 = red[3 * QR + lane];
  asm volatile("" ::: "memory");
  return ((q0 + q1) + q2) + q3;
}
