// Exact local solve for logistic GADMM: one phase (all heads or all tails of this rank), each
// updating worker minimises its augmented Lagrangian exactly by Newton's method instead of the
// reference's inexact inner GD (logReg_GD.m). This is the semantics of the dead CVX variant
// group_ADMM_logistic.m:26-49: true proximal terms rho/2 ||x - theta_nbr||^2, not
// gradients frozen at the pre-update iterate. It is what reaches a 1e-8 objective gap on logistic
// problems (the linearised inner GD stalls near 4e-5 at rho = 3e-4).
//
// Worker n solves   min_x  f_n(x) + mu_n^T x + rho/2 sum_{nbr} ||x - theta_nbr||^2,
//   f_n(x) = lam/2 ||x||^2 + sum_i log(1 + exp(-y_i x_i^T x))
// with Newton steps  H dx = g,  x <- x - dx  until max|dx| < 1e-13 max(1, max|x|) (<= 50 steps),
//   g = -X^T (y . sigma(-y . Xx)) + (lam + deg rho) x + mu - rho (theta_l + theta_r)
//   H = X^T diag(w) X + (lam + deg rho) I,   w = sigma (1 - sigma)
// (the same stopping rule and iteration cap as models/logistic.py:newton_prox, the torch path).
//
// One 256-thread workgroup per worker (d, m <= 64), everything in LDS:
//   margins / gradient: 4 threads per row (column) with two xor shuffles;
//   Hessian: lower-triangular 4x4 register blocks (two 16-B LDS reads per operand per sample);
//   factorisation: symmetric Gaussian elimination H = L D L^T in place (SPD, no pivoting), wave w
//     updates the columns j = w (mod 4), lane i row i, one LDS barrier per pivot;
//   substitution: wave 0, column-oriented, the pivot value broadcast by a lane shuffle.
#include "gadmm_common.h"
#include "gadmm_chain.h"
#include "chain_device.h"

namespace {

constexpr int NTN = 256;
constexpr int NEWTON_MAX = 50;
constexpr double NEWTON_TOL = 1e-13;

__device__ __forceinline__ double wave_max_f64(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

}  // namespace

__global__ void __launch_bounds__(NTN) chain_phase_logistic_newton(PhaseArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int flag_lds, conv_lds;
  ChainCtl* ctl = a.ctl;
  if (ctl->done) return;
  const int it = ctl->iter;
  const int pending = ctl->pending;
  const PhaseSlot sl = a.slots[blockIdx.x];
  const int d = a.d, m = a.m;
  const int DP = (d + 3) & ~3;  // X row stride: 4-column blocks are 16-B aligned, padding is zero
  const int DH = d | 1;         // H row stride (odd: a column walk spreads over the banks)
  double* Xs = lds;             // [m][DP]
  double* Hs = Xs + m * DP;     // [d][DH] lower triangle, factorised in place
  double* xv = Hs + d * DH;     // [64] current iterate
  double* gv = xv + 64;         // [64] Newton right-hand side (gradient)
  double* sv = gv + 64;         // [64] y_i sigma(-y_i z_i); at the end the per-sample losses
  double* wv = sv + 64;         // [64] sigma (1 - sigma)
  double* cv = wv + 64;         // [64] mu - rho (theta_l + theta_r): the x-independent gradient part
  double* yv = cv + 64;         // [64] labels
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
  }
  if (t < m) yv[t] = Yg[t];
  lds_barrier();

  int used = 0;
  for (int k = 0; k < NEWTON_MAX; ++k) {
    {  // margins z_i = X[i,:] x -> sigma terms; thread (i, q) sums columns j = q (mod 4)
      const int i = t >> 2, q = t & 3;
      double z = 0.0;
      if (i < m)
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
    {  // gradient; thread (j, q) sums samples i = q (mod 4)
      const int j = t >> 2, q = t & 3;
      double s = 0.0;
      if (j < d)
        for (int i = q; i < m; i += 4) s = fma(Xs[i * DP + j], sv[i], s);
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      if (q == 0 && j < d) gv[j] = -s + shift * xv[j] + cv[j];
    }
    {  // Hessian, lower 4x4 blocks (bj >= bk)
      const int bj = t >> 4, bk = t & 15;
      if (bj >= bk && 4 * bj < d) {
        double acc[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int v = 0; v < 4; ++v) acc[u][v] = 0.0;
        for (int i = 0; i < m; ++i) {
          const double w = wv[i];
          const double2 a01 = *reinterpret_cast<const double2*>(Xs + i * DP + 4 * bj);
          const double2 a23 = *reinterpret_cast<const double2*>(Xs + i * DP + 4 * bj + 2);
          const double2 b01 = *reinterpret_cast<const double2*>(Xs + i * DP + 4 * bk);
          const double2 b23 = *reinterpret_cast<const double2*>(Xs + i * DP + 4 * bk + 2);
          const double wa[4] = {w * a01.x, w * a01.y, w * a23.x, w * a23.y};
          const double bb[4] = {b01.x, b01.y, b23.x, b23.y};
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int v = 0; v < 4; ++v) acc[u][v] = fma(wa[u], bb[v], acc[u][v]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int r = 4 * bj + u, c = 4 * bk + v;
            if (r < d && c <= r) Hs[r * DH + c] = acc[u][v] + (r == c ? shift : 0.0);
          }
      }
    }
    lds_barrier();
    // H = L D L^T in place: after pivot p, Hs[i][p] / Hs[p][p] = L[i][p] and Hs[p][p] = D[p]
    for (int p = 0; p < d - 1; ++p) {
      const int i = lane;
      if (i > p && i < d) {
        const double lip = Hs[i * DH + p] / Hs[p * DH + p];
        for (int j = p + 1 + ((wid - p - 1) & 3); j <= i; j += 4) Hs[i * DH + j] = fma(-lip, Hs[j * DH + p], Hs[i * DH + j]);
      }
      lds_barrier();
    }
    if (wid == 0) {
      const bool in = lane < d;
      const double dinv = in ? 1.0 / Hs[lane * DH + lane] : 0.0;
      double r = in ? gv[lane] : 0.0;
      for (int p = 0; p < d - 1; ++p) {  // L y = g (unit lower, column by column)
        const double rp = __shfl(r, p, 64), dp = __shfl(dinv, p, 64);
        if (lane > p && in) r = fma(-Hs[lane * DH + p] * dp, rp, r);
      }
      r *= dinv;                          // D^{-1}
      for (int p = d - 1; p > 0; --p) {   // L^T dx = y (row p of L read across the lanes)
        const double xp = __shfl(r, p, 64);
        if (lane < p) r = fma(-Hs[p * DH + lane] * dinv, xp, r);
      }
      const double xo = in ? xv[lane] : 0.0;
      const double xn = xo - (in ? r : 0.0);
      if (in) xv[lane] = xn;
      const double mdx = wave_max_f64(in ? fabs(r) : 0.0), mx = wave_max_f64(in ? fabs(xn) : 0.0);
      if (lane == 0) conv_lds = (mdx < NEWTON_TOL * fmax(1.0, mx)) ? 1 : 0;
    }
    lds_barrier();
    used = k + 1;
    if (conv_lds) break;
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
    if (in) {
      thw_out[lane] = x;
      if (a.flags & PH_POST_DUAL) {  // tails: both neighbours are fresh heads
        double mm = mu[lane];
        if (thl) mm = mm - rho * (thl[lane] - x);
        if (thr) mm = mm + rho * (x - thr[lane]);
        mu[lane] = mm;
      }
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
  return (size_t)(m * DP + d * DH + 6 * 64) * sizeof(double);
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
    return hipFuncSetAttribute((const void*)chain_phase_logistic_newton, hipFuncAttributeMaxDynamicSharedMemorySize,
                               96 * 1024) == hipSuccess;
  }();
  const size_t lds = gadmm_chain_newton_lds(a.d, a.m);
  if (!attr && lds > 65536) {
    gadmm_set_error("chain_phase newton: %zu B of LDS needs the dynamic-LDS attribute", lds);
    return -1;
  }
  hipLaunchKernelGGL(chain_phase_logistic_newton, dim3(a.n_slots), dim3(NTN), lds, st, a);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"
