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
// One 512-thread workgroup per worker (d, m <= 64), everything in LDS:
//   margins / gradient: 4 threads per row (column) with two xor shuffles;
//   Hessian: lower-triangular 4x4 register blocks (two 16-B LDS reads per operand per sample), the
//     samples split over a lane pair;
//   solve: block Gauss-Jordan on [H | g] with 4 x 4 pivot blocks (SPD, no pivoting); lane i of wave
//     w keeps row i's columns j = w (mod 8) in registers, each block's 4 columns go through LDS,
//     one barrier per 4 pivots, no back substitution.
#include "gadmm_common.h"
#include "gadmm_chain.h"
#include "chain_device.h"

namespace {

constexpr int NTN = 512;           // 8 waves: each keeps 8 of a row's 64 columns in the solve
constexpr int NWV = NTN / 64;
constexpr int NCW = 64 / NWV;      // columns per lane
constexpr int NEWTON_MAX = 50;
constexpr double NEWTON_TOL = 1e-13;

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
// gradient + Hessian, Gauss-Jordan, update + test.
template <bool TL>
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
  double* colv = yv + 64;       // [2][4][64] pivot-block columns of the solve (double-buffered)
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
    {  // Hessian, lower 4x4 blocks (bj >= bk); the four lanes of a quad split the samples
      const int nbr = (d + 3) >> 2, nb = nbr * (nbr + 1) / 2, half = t & 3;
      for (int b = t >> 2; b < nb; b += NTN / 4) {
        int bj = 0, bk = b;
        while (bk > bj) {  // block-row bj holds bj + 1 blocks
          bk -= bj + 1;
          ++bj;
        }
        double acc[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int v = 0; v < 4; ++v) acc[u][v] = 0.0;
#pragma unroll 4
        for (int i = half; i < m; i += 4) {
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
            const double t2 = acc[u][v] + __shfl_xor(acc[u][v], 1, 64);
            const double tot = t2 + __shfl_xor(t2, 2, 64);
            const int r = 4 * bj + u, c = 4 * bk + v;
            if (half == 0 && r < d && c <= r) Hs[r * DH + c] = tot + (r == c ? shift : 0.0);
          }
      }
    }
    lds_barrier();
    if (TL && t == 0) tl[k * 5 + 2] = (long long)__builtin_amdgcn_s_memrealtime();
    {  // Block Gauss-Jordan on [H | g] with 4 x 4 pivot blocks (SPD, no pivoting). Lane i of wave w
       // keeps row i's columns j = w + 8c (c < 8) in registers; wave 0 also carries g_i. Block b
       // (pivots p = 4b .. 4b + 3) has one column in each of four waves: they publish them into a
       // double-buffered LDS slab, one barrier, then every lane eliminates the
       // block from its row (rows above the block too, so no back substitution is left):
       //   l_i = H[i][p:p+4] P^-1,  H[i][:] -= l_i H[p:p+4][:],  g_i -= l_i g[p:p+4]
       // (P = the 4 x 4 pivot block, solved redundantly per lane by 2 x 2 blocks). Indices >= d are
       // identity padding. A pivot row keeps row (i - p) of P^-1 for the final block solve.
      const int i = lane;
      double h[NCW];
#pragma unroll
      for (int c = 0; c < NCW; ++c) {
        const int j = wid + NWV * c;
        h[c] = (i < d && j < d) ? (j <= i ? Hs[i * DH + j] : Hs[j * DH + i]) : (i == j ? 1.0 : 0.0);
      }
      double gi = (wid == 0 && i < d) ? gv[i] : 0.0;
      double pr0 = 0.0, pr1 = 0.0, pr2 = 0.0, pr3 = 0.0;  // row (i mod 4) of this lane's pivot-block inverse
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
          R[q] = slab[q * 64 + i];  // H[i][p + q]
#pragma unroll
          for (int r = 0; r < 4; ++r) P[q][r] = slab[q * 64 + p + r];  // H[p + r][p + q] (symmetric)
        }
        const bool pivrow = (i >> 2) == bb;
        if (pivrow) {  // solve with e_(i - p): the lane's row of P^-1
#pragma unroll
          for (int q = 0; q < 4; ++q) R[q] = (q == (i & 3)) ? 1.0 : 0.0;
        }
        // l = P^-1 R by 2 x 2 blocks P = [A B; B^T D] (the same on every lane): A^-1 and the Schur
        // complement S = D - B^T A^-1 B inverted by their determinants. The dependent chain is ~20
        // f64 operations instead of ~35 for a 4 x 4 L D L^T: this solve sits on the critical path
        // of every block, between the barrier and the row updates.
        auto rcp = [](double v) {  // v_rcp_f64 (~2^-29) + one Newton-Raphson step (~2^-58)
          const double r = __builtin_amdgcn_rcp(v);
          return fma(r, fma(-v, r, 1.0), r);
        };
        const double a00 = P[0][0], a01 = P[1][0], a11 = P[1][1];  // lower entries, as published
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
        double f0 = l0, f1 = l1, f2 = l2, f3 = l3;
        if (pivrow) {
          pr0 = l0;
          pr1 = l1;
          pr2 = l2;
          pr3 = l3;
          f0 = f1 = f2 = f3 = 0.0;  // pivot rows are not eliminated by their own block
        }
#pragma unroll
        for (int c = 0; c < NCW; ++c) {
          const int j = wid + NWV * c;  // H[p + q][j] = H[j][p + q] for the trailing columns j >= p + 4
          double v = h[c];
          v = fma(-f0, slab[0 * 64 + j], v);
          v = fma(-f1, slab[1 * 64 + j], v);
          v = fma(-f2, slab[2 * 64 + j], v);
          v = fma(-f3, slab[3 * 64 + j], v);
          h[c] = v;  // columns j < p + 4 are done: updating them too is harmless and branch-free
        }
        if (wid == 0) {
          const double g0 = readlane_f64(gi, p), g1 = readlane_f64(gi, p + 1), g2 = readlane_f64(gi, p + 2),
                       g3 = readlane_f64(gi, p + 3);
          gi = fma(-f0, g0, fma(-f1, g1, fma(-f2, g2, fma(-f3, g3, gi))));
        }
      }
      lds_barrier();
      if (TL && t == 0) tl[k * 5 + 3] = (long long)__builtin_amdgcn_s_memrealtime();
      if (wid == 0) {
        const bool in = lane < d;
        const int q0 = lane & ~3;  // the lane's pivot block: dx = P^-1 g over the block
        const double g0 = __shfl(gi, q0, 64), g1 = __shfl(gi, q0 + 1, 64), g2 = __shfl(gi, q0 + 2, 64),
                     g3 = __shfl(gi, q0 + 3, 64);
        const double r = in ? fma(pr0, g0, fma(pr1, g1, fma(pr2, g2, pr3 * g3))) : 0.0;  // dx
        const double xo = in ? xv[lane] : 0.0;
        const double xn = xo - (in ? r : 0.0);
        if (in) xv[lane] = xn;
        const double mdx = wave_max_f64(in ? fabs(r) : 0.0), mx = wave_max_f64(in ? fabs(xn) : 0.0);
        if (lane == 0) conv_lds = (mdx < NEWTON_TOL * fmax(1.0, mx)) ? 1 : 0;
      }
    }
    lds_barrier();
    if (TL && t == 0) tl[k * 5 + 4] = (long long)__builtin_amdgcn_s_memrealtime();
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
  return (size_t)(m * DP + d * DH + 14 * 64) * sizeof(double);
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
