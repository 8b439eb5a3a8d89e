// Exact local solve for logistic GADMM: one phase (all heads or all tails of this rank), each
// updating worker minimises its augmented Lagrangian exactly by Newton's method instead of the
// reference's inexact inner GD (logReg_GD.m). This is the semantics of the dead CVX variant
// group_ADMM_logistic.m:26-49: true proximal terms rho/2 ||x - theta_nbr||^2, not
// gradients frozen at the pre-update iterate. It is what reaches a 1e-8 objective gap on logistic
// problems (the linearised inner GD stalls near 4e-5 at rho = 3e-4).
//
// Worker n solves   min_x  f_n(x) + mu_n^T x + rho/2 sum_{nbr} ||x - theta_nbr||^2,
//   f_n(x) = lam/2 ||x||^2 + sum_i log(1 + exp(-y_i x_i^T x))
// with steps  dx = H^-1 g,  x <- x - dx  until max|dx| < 1e-13 max(1, max|x|) (<= 50 steps),
//   g = -X^T (y . sigma(-y . Xx)) + (lam + deg rho) x + mu - rho (theta_l + theta_r)
//   H = X^T diag(w) X + (lam + deg rho) I,   w = sigma (1 - sigma)
// (the same stopping rule and iteration cap as models/logistic.py:newton_prox, the torch path).
// Chord-Newton (PhaseArgs.step = contraction threshold c > 0): H^-1 is refreshed only when a step
// contracts by less than c (|dx_k| > c |dx_{k-1}|) or none is cached; otherwise the last inverse of
// this worker -- kept in global memory across ADMM iterations, keyed by its shift -- is reused. The
// fixed point (g = 0) and the stopping rule are those of exact Newton; step = 0 refreshes every step.
//
// One 512-thread workgroup per worker (d, m <= 64), everything in LDS:
//   margins / gradient: 4 threads per row (column) with two xor shuffles;
//   Hessian: v_mfma_f64_16x16x4_f64, a 4 x 4 grid of 16 x 16 tiles, two per wave, K = samples;
//   inverse: in-place block Gauss-Jordan with 4 x 4 pivot blocks (SPD, no pivoting); lane i of wave
//     w keeps row i's columns j = w (mod 8) in registers, each block's 4 columns go through LDS, one
//     barrier per 4 pivots; the inverse stays in registers, so H^-1 g is 8 FMAs per lane + one
//     cross-wave sum.
#include "gadmm_common.h"
#include "gadmm_chain.h"
#include "chain_device.h"

namespace {

constexpr int NTN = 512;           // 8 waves: each keeps 8 of a row's 64 columns in the solve
constexpr int NWV = NTN / 64;
constexpr int NCW = 64 / NWV;      // columns per lane
constexpr int NEWTON_MAX = 50;
constexpr double NEWTON_TOL = 1e-13;
constexpr long NEWTON_HSTRIDE = 64 * 64 + 8;  // per-worker inverse store: register image + valid flag + shift

__device__ __forceinline__ double readlane_f64(double v, int l) {  // l wave-uniform
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double wave_max_f64(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

}  // namespace

// TL: instrumented instantiation (GADMM_NEWTON_TL=1): s_memrealtime stamps of every Newton step of
// every worker into PhaseArgs.rbuf as long long [n_local][NEWTON_MAX][5]: step start, sigma terms,
// gradient (+ Hessian), inversion (= the previous stamp on chord steps), update + test. The low bit
// of the last stamp is set on steps that refreshed the inverse.
template <bool TL>
__global__ void __launch_bounds__(NTN) chain_phase_logistic_newton(PhaseArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int flag_lds, conv_lds, refresh_lds;
  ChainCtl* ctl = a.ctl;
  if (ctl->done) return;
  const int it = ctl->iter;
  const int pending = ctl->pending;
  const PhaseSlot sl = a.slots[blockIdx.x];
  const int d = a.d, m = a.m;
  const int DP = (d + 3) & ~3;  // X row stride: 4-column blocks are 16-B aligned, padding is zero
  const int DH = d | 1;         // H row stride (odd: a column walk spreads over the banks)
  double* Xs = lds;             // [m][DP]
  double* Hs = Xs + m * DP;     // [d][DH] Hessian (full, symmetric)
  double* xv = Hs + d * DH;     // [64] current iterate
  double* gv = xv + 64;         // [64] gradient
  double* sv = gv + 64;         // [64] y_i sigma(-y_i z_i); at the end the per-sample losses
  double* wv = sv + 64;         // [64] sigma (1 - sigma)
  double* cv = wv + 64;         // [64] mu - rho (theta_l + theta_r): the x-independent gradient part
  double* yv = cv + 64;         // [64] labels
  double* colv = yv + 64;       // [2][4][64] pivot-block columns of the inversion (double-buffered)
  double* pv = colv + 512;      // [NWV][64] per-wave partial sums of H^-1 g
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const double rho = a.rho, lam = a.lam;
  double* th = a.theta;
  const double* thw = th + (long)sl.gid * d;
  const double* thl = sl.left >= 0 ? th + (long)sl.left * d : nullptr;
  const double* thr = sl.right >= 0 ? th + (long)sl.right * d : nullptr;
  double* mu = a.mu + (long)sl.li * d;
  const double* Xg = a.X + (long)sl.li * m * d;
  const double* Yg = a.Y + (long)sl.li * m;
  const double shift = lam + rho * (double)((thl ? 1 : 0) + (thr ? 1 : 0));  // lam + deg rho
  // the worker's inverse Hessian of its last refresh, in register-image layout [c][wave][lane]
  // (+ [4096] valid flag, [4097] the shift it was built with); chord threshold 0: exact Newton
  const double chord = a.step;
  double* hg = a.Minv ? const_cast<double*>(a.Minv) + (long)sl.li * NEWTON_HSTRIDE : nullptr;

  for (int idx = t; idx < m * DP; idx += NTN) {
    const int r = idx / DP, c = idx - r * DP;
    Xs[idx] = c < d ? Xg[(long)r * d + c] : 0.0;
  }
  if (t < d) {
    double mm = mu[t];
    if ((a.flags & PH_PRE_DUAL) && pending) {  // lazy end-of-iteration dual (reference order)
      if (thl) mm = mm - rho * (thl[t] - thw[t]);
      if (thr) mm = mm + rho * (thw[t] - thr[t]);
      mu[t] = mm;
    }
    double c = mm;
    if (thl) c = c - rho * thl[t];
    if (thr) c = c - rho * thr[t];
    cv[t] = c;
    xv[t] = thw[t];
  } else if (t < 64) {
    // padding slots d..63 are read by the 64-wide loops below (H^-1 g multiplies them by the
    // identity padding's exact zeros): they must hold finite values, not a previous kernel's LDS
    cv[t] = 0.0;
    xv[t] = 0.0;
    gv[t] = 0.0;
  }
  if (t < m) yv[t] = Yg[t];
  else if (t < 64) {
    yv[t] = 0.0;
    sv[t] = 0.0;
    wv[t] = 0.0;
  }
  double h[NCW];  // lane i of wave w: row i of the inverse, columns j = w + NWV c
  bool refresh = true;
  if (hg && chord > 0.0 && hg[4096] == 1.0 && hg[4097] == shift) {
#pragma unroll
    for (int c = 0; c < NCW; ++c) h[c] = hg[(c * NWV + wid) * 64 + lane];
    refresh = false;
  }
  lds_barrier();

  int used = 0, refreshed = 0;
  double nd_prev = 0.0;
  long long* tl = TL ? reinterpret_cast<long long*>(a.rbuf) + (long)sl.li * NEWTON_MAX * 5 : nullptr;
  for (int k = 0; k < NEWTON_MAX; ++k) {
    if (TL && t == 0) tl[k * 5] = (long long)__builtin_amdgcn_s_memrealtime();
    {  // margins z_i = X[i,:] x -> sigma terms; thread (i, q) sums columns j = q (mod 4)
      const int i = t >> 2, q = t & 3;
      double z = 0.0;
      if (i < m)
#pragma unroll 4
        for (int j = q; j < d; j += 4) z = fma(Xs[i * DP + j], xv[j], z);
      z += __shfl_xor(z, 1, 64);
      z += __shfl_xor(z, 2, 64);
      if (q == 0 && i < m) {
        const double y = yv[i];
        const double p = 1.0 / (1.0 + exp(y * z));  // sigma(-y z)
        sv[i] = y * p;
        wv[i] = p * (1.0 - p);
      }
    }
    lds_barrier();
    if (TL && t == 0) tl[k * 5 + 1] = (long long)__builtin_amdgcn_s_memrealtime();
    {  // gradient; thread (j, q) sums samples i = q (mod 4)
      const int j = t >> 2, q = t & 3;
      double s = 0.0;
      if (j < d)
#pragma unroll 4
        for (int i = q; i < m; i += 4) s = fma(Xs[i * DP + j], sv[i], s);
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      if (q == 0 && j < d) gv[j] = -s + shift * xv[j] + cv[j];
    }
    if (refresh) {
      // Hessian X^T diag(w) X + shift I on f64 MFMA: the 4 x 4 grid of 16 x 16 tiles (d <= 64), two
      // per wave, K = samples in chunks of 4. v_mfma_f64_16x16x4_f64: A[i][k] = lane (k = l >> 4,
      // i = l & 15), B[k][j] likewise, D row (l >> 4) + 4 reg, column l & 15.
      const int k4 = lane >> 4, c16 = lane & 15;
      const int R0 = wid >> 2, C0 = wid & 3, R1 = R0 + 2;  // tiles (R0, C0) and (R0 + 2, C0)
      f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
      const int ca = 16 * R0 + c16, cb = 16 * R1 + c16, cc = 16 * C0 + c16;
      for (int k0 = 0; k0 < m; k0 += 4) {
        const int kk = k0 + k4;
        const bool kin = kk < m;
        const double w = kin ? wv[kk] : 0.0;
        const double* xr = Xs + (kin ? kk : 0) * DP;
        const double a0 = ca < DP ? w * xr[ca] : 0.0;
        const double a1 = cb < DP ? w * xr[cb] : 0.0;
        const double bv = (kin && cc < DP) ? xr[cc] : 0.0;
        acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bv, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bv, acc1, 0, 0, 0);
      }
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int col = 16 * C0 + c16, r0 = 16 * R0 + k4 + 4 * reg, r1 = 16 * R1 + k4 + 4 * reg;
        if (col < d && r0 < d) Hs[r0 * DH + col] = acc0[reg] + (r0 == col ? shift : 0.0);
        if (col < d && r1 < d) Hs[r1 * DH + col] = acc1[reg] + (r1 == col ? shift : 0.0);
      }
    }
    lds_barrier();
    if (TL && t == 0) tl[k * 5 + 2] = (long long)__builtin_amdgcn_s_memrealtime();
    if (refresh) {
      // In-place block Gauss-Jordan INVERSION of the SPD Hessian with 4 x 4 pivot blocks, no
      // pivoting. Lane i of wave w keeps row i's columns j = w + 8c in registers. Block K = p..p+3:
      //   P = A_KK, Pi = P^-1;  non-pivot rows: L_i = A_iK Pi,  A_ij -= L_i A_Kj (j not in K),
      //   A_iK = -L_i;  pivot rows: A_Kj = Pi A_Kj (j not in K),  A_KK = Pi.
      // Only column K is published (slab[q][j] = A_{j, p+q}); the pivot ROWS follow from the
      // structure of in-place Gauss-Jordan on a symmetric matrix: the processed / unprocessed cross
      // blocks are antisymmetric (A_UP = -A_PU^T), the rest symmetric, so A_{p+q, j} = -slab[q][j] for
      // already processed columns j < p and +slab[q][j] otherwise. Indices >= d: identity padding.
      const int i = lane;
#pragma unroll
      for (int c = 0; c < NCW; ++c) {
        const int j = wid + NWV * c;
        h[c] = (i < d && j < d) ? Hs[i * DH + j] : (i == j ? 1.0 : 0.0);
      }
      const int nb = (d + 3) >> 2;
      for (int bb = 0; bb < nb; ++bb) {
        const int p = 4 * bb;
        double* slab = colv + (bb & 1) * 256;  // [4][64]: column p + q of the current matrix
        {  // the block's 4 columns belong to waves (p mod NWV) .. +3, register p / NWV
          const int q = wid - (p % NWV);
          if (q >= 0 && q < 4) {
            double hv = 0.0;
#pragma unroll
            for (int c = 0; c < NCW; ++c) hv = (c == p / NWV) ? h[c] : hv;
            slab[q * 64 + i] = hv;
          }
        }
        lds_barrier();
        double P[4][4], R[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          R[q] = slab[q * 64 + i];  // A[i][p + q]
#pragma unroll
          for (int r = 0; r < 4; ++r) P[q][r] = slab[q * 64 + p + r];  // A[p + r][p + q] (symmetric block)
        }
        const bool pivrow = (i >> 2) == bb;
        if (pivrow) {  // solve with e_(i - p): the lane's row of Pi
#pragma unroll
          for (int q = 0; q < 4; ++q) R[q] = (q == (i & 3)) ? 1.0 : 0.0;
        }
        // l = Pi R by 2 x 2 blocks P = [A B; B^T D] (the same on every lane): A^-1 and the Schur
        // complement S = D - B^T A^-1 B inverted by their determinants (a short dependent chain on
        // the critical path of every block, between the barrier and the row updates)
        auto rcp = [](double v) {  // v_rcp_f64 (~2^-29) + one Newton-Raphson step (~2^-58)
          const double r = __builtin_amdgcn_rcp(v);
          return fma(r, fma(-v, r, 1.0), r);
        };
        const double a00 = P[0][0], a01 = P[1][0], a11 = P[1][1];
        const double ia = rcp(fma(a00, a11, -a01 * a01));
        const double A00 = a11 * ia, A01 = -a01 * ia, A11 = a00 * ia;  // A^-1
        const double b00 = P[2][0], b01 = P[3][0], b10 = P[2][1], b11 = P[3][1];  // B[i][j] = P[j + 2][i]
        const double w00 = fma(A00, b00, A01 * b10), w01 = fma(A00, b01, A01 * b11);  // W = A^-1 B
        const double w10 = fma(A01, b00, A11 * b10), w11 = fma(A01, b01, A11 * b11);
        const double s00 = P[2][2] - fma(b00, w00, b10 * w10);  // S = D - B^T W
        const double s01 = P[3][2] - fma(b00, w01, b10 * w11);
        const double s11 = P[3][3] - fma(b01, w01, b11 * w11);
        const double is = rcp(fma(s00, s11, -s01 * s01));
        const double y0 = fma(A00, R[0], A01 * R[1]), y1 = fma(A01, R[0], A11 * R[1]);  // A^-1 r_top
        const double z2 = R[2] - fma(b00, y0, b10 * y1), z3 = R[3] - fma(b01, y0, b11 * y1);
        const double l2 = fma(s11, z2, -s01 * z3) * is, l3 = fma(s00, z3, -s01 * z2) * is;  // S^-1 z
        const double l0 = y0 - fma(w00, l2, w01 * l3), l1 = y1 - fma(w10, l2, w11 * l3);
        // the block's columns j = p .. p+3 sit in register c = p / NWV of waves p % NWV .. +3, so "j in K"
        // and the sign of A_{p+q, j} are wave-uniform; only the pivot-row case varies by lane
        const int cK = p / NWV, wK = wid - p % NWV;
        const double lw = wK == 0 ? l0 : (wK == 1 ? l1 : (wK == 2 ? l2 : l3));  // l[j - p] for j in K
#pragma unroll
        for (int c = 0; c < NCW; ++c) {
          const int j = wid + NWV * c;
          const double tq = fma(l0, slab[j], fma(l1, slab[64 + j], fma(l2, slab[128 + j], l3 * slab[192 + j])));
          const bool inK = c == cK && wK >= 0 && wK < 4;
          const double sg = j < p ? -1.0 : 1.0;  // A_{p+q, j} = sg * slab[q][j]
          double v;
          if (inK) v = pivrow ? lw : -lw;                  // Pi[i-p][j-p], or -L_i
          else v = pivrow ? sg * tq : fma(-sg, tq, h[c]);  // (Pi A_Kj)_i, or A_ij - L_i A_Kj
          h[c] = v;
        }
      }
      ++refreshed;
    }
    if (TL && t == 0) tl[k * 5 + 3] = (long long)__builtin_amdgcn_s_memrealtime();
    {  // dx = H^-1 g: per-wave partials over the wave's 8 columns, summed in wave order by wave 0
      double s = 0.0;
#pragma unroll
      for (int c = 0; c < NCW; ++c) s = fma(h[c], gv[wid + NWV * c], s);
      pv[wid * 64 + lane] = s;
    }
    lds_barrier();
    if (wid == 0) {
      const bool in = lane < d;
      double r = 0.0;
#pragma unroll
      for (int w = 0; w < NWV; ++w) r += pv[w * 64 + lane];
      const double xo = in ? xv[lane] : 0.0;
      const double xn = xo - (in ? r : 0.0);
      if (in) xv[lane] = xn;
      const double mdx = wave_max_f64(in ? fabs(r) : 0.0), mx = wave_max_f64(in ? fabs(xn) : 0.0);
      if (lane == 0) {
        conv_lds = (mdx < NEWTON_TOL * fmax(1.0, mx)) ? 1 : 0;
        // chord steps reuse the inverse while they contract by at least `chord` per step
        refresh_lds = (chord <= 0.0 || (!refresh && k > 0 && mdx > chord * nd_prev)) ? 1 : 0;
      }
      nd_prev = mdx;
    }
    lds_barrier();
    if (TL && t == 0) tl[k * 5 + 4] = ((long long)__builtin_amdgcn_s_memrealtime() & ~1LL) | (refresh ? 1 : 0);
    used = k + 1;
    if (conv_lds) break;
    refresh = refresh_lds != 0;
  }
  if (t == 0 && !conv_lds) atomicAdd(&ctl->inner_fail, 1);  // the step cap ended the solve unconverged
  if (hg && refreshed && chord > 0.0) {  // keep the newest inverse for this worker's next solve
#pragma unroll
    for (int c = 0; c < NCW; ++c) hg[(c * NWV + wid) * 64 + lane] = h[c];
    if (t == 0) {  // read by the next phase launch (kernel boundary: no fence needed)
      hg[4097] = shift;
      hg[4096] = 1.0;
    }
  }

  {  // local objective lam/2 |x|^2 + sum_i softplus(-y_i z_i) at the new iterate
    const int i = t >> 2, q = t & 3;
    double z = 0.0;
    if (i < m)
      for (int j = q; j < d; j += 4) z = fma(Xs[i * DP + j], xv[j], z);
    z += __shfl_xor(z, 1, 64);
    z += __shfl_xor(z, 2, 64);
    if (q == 0 && i < m) sv[i] = softplus(-yv[i] * z);
  }
  lds_barrier();
  if (wid == 0) {
    const bool in = lane < d;
    const double x = in ? xv[lane] : 0.0;
    const double part = wave_sum_f64(lane < m ? sv[lane] : 0.0);
    const double xx = wave_sum_f64(x * x);
    double* thw_out = th + (long)sl.gid * d;
    double rp = 0.0;
    if (in) {
      thw_out[lane] = x;
      if (a.flags & PH_POST_DUAL) {  // tails: both neighbours are fresh heads
        double mm = mu[lane];
        if (thl) mm = mm - rho * (thl[lane] - x);
        if (thr) mm = mm + rho * (x - thr[lane]);
        mu[lane] = mm;
        if (thl) rp = fma(thl[lane] - x, thl[lane] - x, rp);  // K4 primal residual of the tail's edges
        if (thr) rp = fma(x - thr[lane], x - thr[lane], rp);
      }
    }
    if (a.rres && (a.flags & PH_POST_DUAL)) {
      const double rs = wave_sum_f64(rp);
      if (lane == 0 && it - 1 < a.max_iter) a.rres[(long)(it - 1) * a.n_total + sl.gid] = rs;
    }
    if (lane == 0) {
      a.objw[sl.li] = lam * 0.5 * xx + part;
      if (a.inner_iters) a.inner_iters[sl.li] = used;
    }
  }
  if (a.flags & PH_FINISH) {
    if (phase_arrive(ctl, a.n_slots, &flag_lds)) finish_iteration(a, it);
  }
}

extern "C" {

size_t gadmm_chain_newton_lds(int d, int m) {
  const int DP = (d + 3) & ~3, DH = d | 1;
  return (size_t)(m * DP + d * DH + 14 * 64 + NWV * 64) * sizeof(double);
}

// Launch one Newton phase (PhaseArgs.solver == 1, logistic model). d, m <= 64.
int gadmm_chain_phase_newton(const PhaseArgs* args, hipStream_t st) {
  const PhaseArgs& a = *args;
  if (a.n_slots <= 0) return 0;
  if (a.d < 1 || a.d > 64 || a.m < 1 || a.m > 64) {
    gadmm_set_error("chain_phase newton: needs 1 <= d, m <= 64 (got d=%d, m=%d)", a.d, a.m);
    return -1;
  }
  static const bool attr = [] {  // once, outside any stream capture of the caller's later phases
    return hipFuncSetAttribute((const void*)chain_phase_logistic_newton<false>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) == hipSuccess &&
           hipFuncSetAttribute((const void*)chain_phase_logistic_newton<true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) == hipSuccess;
  }();
  const size_t lds = gadmm_chain_newton_lds(a.d, a.m);
  if (!attr && lds > 65536) {
    gadmm_set_error("chain_phase newton: %zu B of LDS needs the dynamic-LDS attribute", lds);
    return -1;
  }
  if (a.rbuf) hipLaunchKernelGGL(chain_phase_logistic_newton<true>, dim3(a.n_slots), dim3(NTN), lds, st, a);
  else hipLaunchKernelGGL(chain_phase_logistic_newton<false>, dim3(a.n_slots), dim3(NTN), lds, st, a);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"
