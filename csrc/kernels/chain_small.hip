// Fused per-phase kernels of the chain engine for small/medium d (<= 256): one workgroup per
// updating worker. Kernels K3+K2-apply+K4+K5 (linear) and K8+K6 (logistic) of SURVEY.md §2.5.
//
// One launch = one GADMM phase (all heads, or all tails, of this rank):
//   [lazy dual]  mu_n += rho (th_n - th_r) - rho (th_l - th_n)        (heads: pending from last iter)
//   rhs          r_n = b_n - mu_n + rho th_l + rho th_r               (dynamic_group_ADMM_closedForm.m:84-86)
//   solve        th_n = (A_n + deg rho I)^{-1} r_n                    (one symmetric GEMV, inverse cached)
//   [post dual]  tails update mu right after their solve (both neighbours are fresh heads)
//   objective    f_n = 1/2 th^T A th - b^T th + 1/2 y^T y              (group_ADMM_closedForm.m:96-101)
//   [finish]     last arriving workgroup sums f_n in a fixed order, records the trace, decides
//                convergence (|obj - obj0| < tol, :105-108) and advances the device iteration
//                counter; every later launch sees `done` and returns at once.
// The per-worker dual mu_n (= lambda_n - lambda_{n-1} in edge form) is the D-GADMM
// parameterisation (dynamic_group_ADMM_closedForm.m:153-168); it equals the edge-dual GADMM of
// group_ADMM_closedForm.m:93-95 for the identity chain.
//
// "Lazy dual": the reference updates every dual after the tail phase. A head's update needs the
// tails' fresh theta, so it is deferred to the start of the next head phase, where the head reads
// exactly the same values (nothing changes in between). When the chain changes (D-GADMM) the
// engine first runs chain_dual_flush_kernel with the OLD chain.
//
// GEMV: lanes own output rows i = lane + 64c and the 4 waves split the summation index; since the
// cached matrices are symmetric, row j of the matrix is read as column j (coalesced 8-B loads of a
// contiguous row per j). Partial sums combine in LDS in a fixed order -> bitwise reproducible.
//
// Inter-workgroup hand-off (finish): every storing wave drains (s_waitcnt vmcnt(0)), workgroup
// barrier, one lane releases at agent scope and takes a ticket; the last arriver acquires at agent
// scope before reading other workgroups' results (cdna_hip_programming.md §6 Guideline 16).
#include <stdlib.h>
#include "gadmm_common.h"
#include "gadmm_chain.h"
#include "chain_device.h"
#include "quad_gemv.h"


namespace {

constexpr int NT = 256;
constexpr int NW = NT / 64;

// out[i] = sum_j M[j*d + i] * x[j]  (M symmetric), for i < d. x, out in LDS; red: NW*64*NC.
template <int NC>
__device__ __forceinline__ void symv_cols(const double* __restrict__ M, const double* x, double* out,
                                          double* red, int d) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = 0.0;
  int j = w;
  // 2-way unrolled over j for memory-level parallelism
  for (; j + NW < d; j += 2 * NW) {
    const double x0 = x[j], x1 = x[j + NW];
    const double* r0 = M + (long)j * d;
    const double* r1 = M + (long)(j + NW) * d;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      if (i < d) acc[c] = fma(r1[i], x1, fma(r0[i], x0, acc[c]));
    }
  }
  for (; j < d; j += NW) {
    const double x0 = x[j];
    const double* r0 = M + (long)j * d;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      if (i < d) acc[c] = fma(r0[i], x0, acc[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) red[w * 64 * NC + c * 64 + lane] = acc[c];
  __syncthreads();
  for (int i = threadIdx.x; i < d; i += NT) {
    const int c = i >> 6, l = i & 63;
    double s = 0.0;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) s += red[ww * 64 * NC + c * 64 + l];
    out[i] = s;
  }
  __syncthreads();
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// Linear regression phase kernel.
template <int NC>
__global__ void __launch_bounds__(NT) chain_phase_linear(PhaseArgs a) {
  __shared__ __attribute__((aligned(16))) double sh_r[64 * NC];
  __shared__ __attribute__((aligned(16))) double sh_t[64 * NC];
  __shared__ __attribute__((aligned(16))) double sh_q[64 * NC];
  __shared__ __attribute__((aligned(16))) double red[NW * 64 * NC];
  __shared__ double scratch[NW];
  __shared__ int flag_lds;
  ChainCtl* ctl = a.ctl;
  if (ctl->done) return;
  const int it = ctl->iter;
  const int pending = ctl->pending;
  const PhaseSlot sl = a.slots[blockIdx.x];
  const int d = a.d;
  const double rho = a.rho;
  double* th = a.theta;
  const double* thw = th + (long)sl.gid * d;
  const double* thl = sl.left >= 0 ? th + (long)sl.left * d : nullptr;
  const double* thr = sl.right >= 0 ? th + (long)sl.right * d : nullptr;
  double* mu = a.mu + (long)sl.li * d;
  const double* b = a.b + (long)sl.li * d;
  const int deg = (thl != nullptr) + (thr != nullptr);

  for (int j = threadIdx.x; j < d; j += NT) {
    double m = mu[j];
    if ((a.flags & PH_PRE_DUAL) && pending) {
      if (thl) m = m - rho * (thl[j] - thw[j]);
      if (thr) m = m + rho * (thw[j] - thr[j]);
      mu[j] = m;
    }
    double r = b[j] - m;
    if (thl) r = r + rho * thl[j];
    if (thr) r = r + rho * thr[j];
    sh_r[j] = r;
  }
  __syncthreads();
  const double* Mi = a.Minv + ((long)sl.li * a.nvar + a.deg_to_var[deg]) * (long)d * d;
  symv_cols<NC>(Mi, sh_r, sh_t, red, d);
  double* thw_out = th + (long)sl.gid * d;
  double rpart = 0.0;
  for (int j = threadIdx.x; j < d; j += NT) {
    const double t = sh_t[j];
    thw_out[j] = t;
    if (a.flags & PH_POST_DUAL) {
      double m = mu[j];
      if (thl) m = m - rho * (thl[j] - t);
      if (thr) m = m + rho * (t - thr[j]);
      mu[j] = m;
      if (a.rres) {  // K4 primal residual of the tail's two edges
        if (thl) rpart = fma(thl[j] - t, thl[j] - t, rpart);
        if (thr) rpart = fma(t - thr[j], t - thr[j], rpart);
      }
    }
  }
  if (a.rres && (a.flags & PH_POST_DUAL)) {
    const double rs = block_sum_f64(rpart, scratch);
    if (threadIdx.x == 0 && it - 1 < a.max_iter) a.rres[(long)(it - 1) * a.n_total + sl.gid] = rs;
    __syncthreads();  // scratch is reused by the objective's block sum
  }
  if (a.flags & PH_OBJ) {
    symv_cols<NC>(a.A + (long)sl.li * d * d, sh_t, sh_q, red, d);
    double part = 0.0;
    for (int j = threadIdx.x; j < d; j += NT) part += (0.5 * sh_q[j] - b[j]) * sh_t[j];
    const double f = block_sum_f64(part, scratch) + 0.5 * a.yy[sl.li];
    if (threadIdx.x == 0) a.objw[sl.li] = f;
  }
  if (a.flags & PH_FINISH) {
    if (phase_arrive(ctl, a.n_slots, &flag_lds)) finish_iteration(a, it);
  }
}

// ------------------------------------------------------------------------------------------------
// Logistic regression phase kernel: inexact local solve by <= max_inner GD steps with the proximal
// terms frozen at the pre-update iterate (group_ADMM_logistic_GD.m:30,39,82,85; logReg_GD.m:3-23),
// the shard resident in LDS (row-major X and its transpose, so both GEMVs read contiguously).
template <int NC, int MC, bool LDSX>
__global__ void __launch_bounds__(NT) chain_phase_logistic(PhaseArgs a) {
  extern __shared__ __attribute__((aligned(16))) double dyn[];  // LDSX: X [m][d], XT [d][m]
  __shared__ __attribute__((aligned(16))) double sh_x[64 * NC];
  __shared__ __attribute__((aligned(16))) double sh_g[64 * NC];
  __shared__ __attribute__((aligned(16))) double sh_shift[64 * NC];
  __shared__ __attribute__((aligned(16))) double sh_z[64 * MC];
  __shared__ __attribute__((aligned(16))) double sh_y[64 * MC];
  __shared__ __attribute__((aligned(16))) double red[NW * 64 * (NC > MC ? NC : MC)];
  __shared__ double scratch[NW];
  __shared__ int flag_lds;
  __shared__ int conv_lds;
  ChainCtl* ctl = a.ctl;
  if (ctl->done) return;
  const int it = ctl->iter;
  const int pending = ctl->pending;
  const PhaseSlot sl = a.slots[blockIdx.x];
  const int d = a.d, m = a.m;
  const double rho = a.rho;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* th = a.theta;
  const double* thw = th + (long)sl.gid * d;
  const double* thl = sl.left >= 0 ? th + (long)sl.left * d : nullptr;
  const double* thr = sl.right >= 0 ? th + (long)sl.right * d : nullptr;
  double* mu = a.mu + (long)sl.li * d;
  const double* Xg = a.X + (long)sl.li * m * d;
  const double* Yg = a.Y + (long)sl.li * m;
  double* Xs = dyn;
  double* XTs = dyn + (long)m * d;

  if (LDSX) {
    for (int e = threadIdx.x; e < m * d; e += NT) {
      const double v = Xg[e];
      Xs[e] = v;
      XTs[(e % d) * m + e / d] = v;
    }
  }
  for (int i = threadIdx.x; i < m; i += NT) sh_y[i] = Yg[i];
  for (int j = threadIdx.x; j < d; j += NT) {
    double mm = mu[j];
    if ((a.flags & PH_PRE_DUAL) && pending) {
      if (thl) mm = mm - rho * (thl[j] - thw[j]);
      if (thr) mm = mm + rho * (thw[j] - thr[j]);
      mu[j] = mm;
    }
    const double x0 = thw[j];
    double s = mm;  // = -C1 + C2 in edge form
    if (thl) s = s + rho * (x0 - thl[j]);
    if (thr) s = s + rho * (x0 - thr[j]);
    sh_shift[j] = s;
    sh_x[j] = x0;
  }
  __syncthreads();

  auto compute_z = [&]() {  // z = X x  (m outputs)
    if (LDSX) {
      double acc[MC];
#pragma unroll
      for (int c = 0; c < MC; ++c) acc[c] = 0.0;
      for (int j = w; j < d; j += NW) {
        const double xj = sh_x[j];
        const double* row = XTs + (long)j * m;
#pragma unroll
        for (int c = 0; c < MC; ++c) {
          const int i = lane + 64 * c;
          if (i < m) acc[c] = fma(row[i], xj, acc[c]);
        }
      }
#pragma unroll
      for (int c = 0; c < MC; ++c) red[w * 64 * MC + c * 64 + lane] = acc[c];
      __syncthreads();
      for (int i = threadIdx.x; i < m; i += NT) {
        double s = 0.0;
#pragma unroll
        for (int ww = 0; ww < NW; ++ww) s += red[ww * 64 * MC + (i >> 6) * 64 + (i & 63)];
        sh_z[i] = s;
      }
      __syncthreads();
    } else {
      // wave per row, lanes over columns
      for (int i = w; i < m; i += NW) {
        const double* row = Xg + (long)i * d;
        double acc = 0.0;
        for (int j = lane; j < d; j += 64) acc = fma(row[j], sh_x[j], acc);
        acc = wave_sum_f64(acc);
        if (lane == 0) sh_z[i] = acc;
      }
      __syncthreads();
    }
  };

  int used = 0;
  for (int k = 0; k < a.max_inner; ++k) {
    compute_z();
    for (int i = threadIdx.x; i < m; i += NT) {
      const double yi = sh_y[i];
      sh_z[i] = yi / (1.0 + exp(yi * sh_z[i]));  // s_i
    }
    if (threadIdx.x == 0) conv_lds = 1;
    __syncthreads();
    // g = -X^T s + lam x + shift
    double acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.0;
    for (int i = w; i < m; i += NW) {
      const double si = sh_z[i];
      const double* row = LDSX ? (Xs + (long)i * d) : (Xg + (long)i * d);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int j = lane + 64 * c;
        if (j < d) acc[c] = fma(row[j], si, acc[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) red[w * 64 * NC + c * 64 + lane] = acc[c];
    __syncthreads();
    for (int j = threadIdx.x; j < d; j += NT) {
      double s = 0.0;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) s += red[ww * 64 * NC + (j >> 6) * 64 + (j & 63)];
      const double xj = sh_x[j];
      const double g = -s + a.lam * xj + sh_shift[j];
      const double xn = xj - a.step * g;
      if (!(fabs(xn - xj) < a.inner_tol)) conv_lds = 0;
      sh_x[j] = xn;
    }
    __syncthreads();
    used = k + 1;
    if (conv_lds) break;
  }
  // final local objective at the new iterate
  compute_z();
  double part = 0.0;
  for (int i = threadIdx.x; i < m; i += NT) part += softplus(-sh_y[i] * sh_z[i]);
  double xx = 0.0;
  for (int j = threadIdx.x; j < d; j += NT) xx += sh_x[j] * sh_x[j];
  const double lossv = block_sum_f64(part, scratch);
  const double xnorm = block_sum_f64(xx, scratch);
  double* thw_out = th + (long)sl.gid * d;
  double rp = 0.0;
  for (int j = threadIdx.x; j < d; j += NT) {
    const double t = sh_x[j];
    thw_out[j] = t;
    if (a.flags & PH_POST_DUAL) {
      double mm = mu[j];
      if (thl) mm = mm - rho * (thl[j] - t);
      if (thr) mm = mm + rho * (t - thr[j]);
      mu[j] = mm;
      if (thl) rp = fma(thl[j] - t, thl[j] - t, rp);  // K4 primal residual of the tail's edges
      if (thr) rp = fma(t - thr[j], t - thr[j], rp);
    }
  }
  if (a.rres && (a.flags & PH_POST_DUAL)) {
    const double rs = block_sum_f64(rp, scratch);
    if (threadIdx.x == 0 && it - 1 < a.max_iter) a.rres[(long)(it - 1) * a.n_total + sl.gid] = rs;
  }
  if (threadIdx.x == 0) {
    a.objw[sl.li] = a.lam * 0.5 * xnorm + lossv;
    if (a.inner_iters) a.inner_iters[sl.li] = used;
  }
  if (a.flags & PH_FINISH) {
    if (phase_arrive(ctl, a.n_slots, &flag_lds)) finish_iteration(a, it);
  }
}

// sum_k M[k * stride] * v[k], k < n: 8 independent LDS loads of each operand per batch (one wait per
// batch instead of one per element), 4 partial sums combined in a fixed order.
__device__ __forceinline__ double dot_strided8(const double* M, int stride, const double* v, int n) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int k = 0;
  for (; k + 8 <= n; k += 8) {
    double mv[8], vv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      mv[q] = M[(k + q) * stride];
      vv[q] = v[k + q];
    }
    a0 = fma(mv[0], vv[0], a0);
    a1 = fma(mv[1], vv[1], a1);
    a2 = fma(mv[2], vv[2], a2);
    a3 = fma(mv[3], vv[3], a3);
    a0 = fma(mv[4], vv[4], a0);
    a1 = fma(mv[5], vv[5], a1);
    a2 = fma(mv[6], vv[6], a2);
    a3 = fma(mv[7], vv[7], a3);
  }
  for (; k < n; ++k) a0 = fma(M[k * stride], v[k], a0);
  return (a0 + a1) + (a2 + a3);
}

// ------------------------------------------------------------------------------------------------
// Logistic phase, one WAVE per worker (the inner GD is latency-bound: ~100 dependent steps of two
// 50 x 50 GEMVs). Lane l owns margin row i = l + 64k and coordinate j = l + 64k; both GEMVs read
// LDS contiguously across lanes (X^T for the margins, X for the gradient) with the other operand
// broadcast from LDS; the all-coordinates stopping test of logReg_GD.m:21 is a wave vote. No
// workgroup barriers beyond the single wave's own LDS ordering.
template <int C>
__global__ void __launch_bounds__(64) chain_phase_logistic_wave(PhaseArgs a) {
  extern __shared__ __attribute__((aligned(16))) double dyn[];  // X [m][d] | XT [d][m] | x [64C] | s [64C]
  __shared__ double scratch[1];
  __shared__ int flag_lds;
  ChainCtl* ctl = a.ctl;
  if (ctl->done) return;
  const int it = ctl->iter;
  const int pending = ctl->pending;
  const PhaseSlot sl = a.slots[blockIdx.x];
  const int d = a.d, m = a.m;
  const double rho = a.rho, lam = a.lam, step = a.step;
  const int lane = threadIdx.x;
  double* th = a.theta;
  const double* thw = th + (long)sl.gid * d;
  const double* thl = sl.left >= 0 ? th + (long)sl.left * d : nullptr;
  const double* thr = sl.right >= 0 ? th + (long)sl.right * d : nullptr;
  double* mu = a.mu + (long)sl.li * d;
  const double* Xg = a.X + (long)sl.li * m * d;
  const double* Yg = a.Y + (long)sl.li * m;
  double* Xs = dyn;
  double* XTs = dyn + (long)m * d;
  double* xs = XTs + (long)m * d;
  double* ss = xs + 64 * C;
  for (int e = lane; e < m * d; e += 64) {
    const double v = Xg[e];
    Xs[e] = v;
    XTs[(e % d) * m + e / d] = v;
  }
  double x[C], sh[C], yv[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int j = lane + 64 * c;
    x[c] = 0.0;
    sh[c] = 0.0;
    yv[c] = 0.0;
    if (j < d) {
      double mm = mu[j];
      if ((a.flags & PH_PRE_DUAL) && pending) {
        if (thl) mm = mm - rho * (thl[j] - thw[j]);
        if (thr) mm = mm + rho * (thw[j] - thr[j]);
        mu[j] = mm;
      }
      const double x0 = thw[j];
      double s = mm;  // -C1 + C2 (edge form) == mu
      if (thl) s = s + rho * (x0 - thl[j]);
      if (thr) s = s + rho * (x0 - thr[j]);
      sh[c] = s;
      x[c] = x0;
      xs[j] = x0;
    }
    if (j < m) yv[c] = Yg[j];
  }
  __syncthreads();
  int used = 0;
  for (int k = 0; k < a.max_inner; ++k) {
    // margins z_i = X[i,:] x  -> s_i = y_i / (1 + exp(y_i z_i))
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int i = lane + 64 * c;
      if (i < m) {
        const double z = dot_strided8(XTs + i, m, xs, d);
        ss[i] = yv[c] / (1.0 + exp(yv[c] * z));
      }
    }
    __syncthreads();
    bool conv = true;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int j = lane + 64 * c;
      if (j < d) {
        const double g = -dot_strided8(Xs + j, d, ss, m) + lam * x[c] + sh[c];
        const double xn = x[c] - step * g;
        conv &= fabs(xn - x[c]) < a.inner_tol;
        x[c] = xn;
      }
    }
    __syncthreads();  // every lane has read ss / xs of this step
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int j = lane + 64 * c;
      if (j < d) xs[j] = x[c];
    }
    __syncthreads();
    used = k + 1;
    if (__all(conv)) break;
  }
  // local objective lam/2 |x|^2 + sum softplus(-y z) at the new iterate
  double part = 0.0, xx = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int i = lane + 64 * c;
    if (i < m) {
      const double z = dot_strided8(XTs + i, m, xs, d);
      part += softplus(-yv[c] * z);
    }
    const int j = lane + 64 * c;
    if (j < d) xx += x[c] * x[c];
  }
  part = wave_sum_f64(part);
  xx = wave_sum_f64(xx);
  double* thw_out = th + (long)sl.gid * d;
  double rp = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int j = lane + 64 * c;
    if (j < d) {
      const double t = x[c];
      thw_out[j] = t;
      if (a.flags & PH_POST_DUAL) {
        double mm = mu[j];
        if (thl) mm = mm - rho * (thl[j] - t);
        if (thr) mm = mm + rho * (t - thr[j]);
        mu[j] = mm;
        if (thl) rp = fma(thl[j] - t, thl[j] - t, rp);  // K4 primal residual of the tail's edges
        if (thr) rp = fma(t - thr[j], t - thr[j], rp);
      }
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
  (void)scratch;
  if (a.flags & PH_FINISH) {
    if (phase_arrive(ctl, a.n_slots, &flag_lds)) finish_iteration(a, it);
  }
}

// ------------------------------------------------------------------------------------------------
// Logistic phase, one wave per worker, shard in REGISTERS (d, m <= 4T <= 64; default for E3/E4).
// Both inner-GD GEMVs run in the split-column quad layout (quad_gemv.h): lane (i, c) holds
// X[i + 16r][c + 4t] (margins z = X x) and X[c + 4t][i + 16r] (gradient X^T s), so a step is two
// register GEMVs with 7 LDS broadcast reads each plus the elementwise sigmoid, instead of ~150 LDS
// reads through the staged shard (chain_phase_logistic_wave, 1.8 us per inner step). Same
// semantics as logReg_GD.m:3-25 (frozen proximal shift, all-coordinate |dx| < tol break).
template <int T>
__global__ void __launch_bounds__(64) chain_phase_logistic_quad(PhaseArgs a) {
  __shared__ __attribute__((aligned(16))) double st[QSTAGE];
  __shared__ int flag_lds;
  ChainCtl* ctl = a.ctl;
  if (ctl->done) return;
  const int it = ctl->iter;
  const int pending = ctl->pending;
  const PhaseSlot sl = a.slots[blockIdx.x];
  const int d = a.d, m = a.m;
  const double rho = a.rho, lam = a.lam, step = a.step;
  const int lane = threadIdx.x, qi = lane & 15, qc = lane >> 4;
  double* th = a.theta;
  const double* thw = th + (long)sl.gid * d;
  const double* thl = sl.left >= 0 ? th + (long)sl.left * d : nullptr;
  const double* thr = sl.right >= 0 ? th + (long)sl.right * d : nullptr;
  double* mu = a.mu + (long)sl.li * d;
  const double* Xg = a.X + (long)sl.li * m * d;
  const double* Yg = a.Y + (long)sl.li * m;
  double Xq[4][T], XTq[4][T];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int row = qi + 16 * r, col = qc + 4 * t;
      Xq[r][t] = (row < m && col < d) ? Xg[(long)row * d + col] : 0.0;   // X[row][col]
      XTq[r][t] = (col < m && row < d) ? Xg[(long)col * d + row] : 0.0;  // X^T[row][col]
    }
  const bool inj = lane < d, ini = lane < m;
  double x = 0.0, sh = 0.0, yv = 0.0;
  if (inj) {
    double mm = mu[lane];
    if ((a.flags & PH_PRE_DUAL) && pending) {
      if (thl) mm = mm - rho * (thl[lane] - thw[lane]);
      if (thr) mm = mm + rho * (thw[lane] - thr[lane]);
      mu[lane] = mm;
    }
    const double x0 = thw[lane];
    double s = mm;  // -C1 + C2 (edge form) == mu
    if (thl) s = s + rho * (x0 - thl[lane]);
    if (thr) s = s + rho * (x0 - thr[lane]);
    sh = s;
    x = x0;
  }
  if (ini) yv = Yg[lane];
  int used = 0;
  for (int k = 0; k < a.max_inner; ++k) {
    const double z = quad_gemv<T>(Xq, x, st);                   // margins z_i = X[i,:] x
    const double sv = ini ? yv / (1.0 + exp(yv * z)) : 0.0;    // y_i / (1 + e^{y_i z_i})
    const double gx = quad_gemv<T>(XTq, sv, st);               // (X^T s)_j
    bool conv = true;
    if (inj) {
      const double g = -gx + lam * x + sh;
      const double xn = x - step * g;
      conv = fabs(xn - x) < a.inner_tol;
      x = xn;
    }
    used = k + 1;
    if (__all(conv)) break;
  }
  // local objective lam/2 |x|^2 + sum softplus(-y z) at the new iterate
  const double z = quad_gemv<T>(Xq, x, st);
  const double part = wave_sum_f64(ini ? softplus(-yv * z) : 0.0);
  const double xx = wave_sum_f64(inj ? x * x : 0.0);
  double* thw_out = th + (long)sl.gid * d;
  double rp = 0.0;
  if (inj) {
    thw_out[lane] = x;
    if (a.flags & PH_POST_DUAL) {
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
  if (a.flags & PH_FINISH) {
    if (phase_arrive(ctl, a.n_slots, &flag_lds)) finish_iteration(a, it);
  }
}

// ------------------------------------------------------------------------------------------------
// Apply the pending heads' dual updates with the chain they were computed on (used before a
// re-chain and before checkpointing). One workgroup per slot of the OLD head plan.
__global__ void __launch_bounds__(NT) chain_dual_flush_kernel(const PhaseSlot* slots, int n_slots, int d,
                                                              double rho, const double* theta, double* mu_all,
                                                              ChainCtl* ctl, int clear_pending) {
  if (!ctl->pending) return;
  const PhaseSlot sl = slots[blockIdx.x];
  const double* thw = theta + (long)sl.gid * d;
  const double* thl = sl.left >= 0 ? theta + (long)sl.left * d : nullptr;
  const double* thr = sl.right >= 0 ? theta + (long)sl.right * d : nullptr;
  double* mu = mu_all + (long)sl.li * d;
  for (int j = threadIdx.x; j < d; j += NT) {
    double m = mu[j];
    if (thl) m = m - rho * (thl[j] - thw[j]);
    if (thr) m = m + rho * (thw[j] - thr[j]);
    mu[j] = m;
  }
  (void)n_slots;
  (void)clear_pending;
}

__global__ void chain_clear_pending_kernel(ChainCtl* ctl) {
  if (threadIdx.x == 0) ctl->pending = 0;
}

// Multi-rank monitor: `reduced` holds the all-reduced per-iteration objective ring. Checks every
// iteration finished since the last monitor call, in order, exactly like the reference stop rule.
__global__ void chain_monitor_kernel(ChainCtl* ctl, const double* reduced, int ring, int n_total, double* trace,
                                     int max_iter, double obj0, double tol) {
  if (threadIdx.x != 0) return;
  if (ctl->done) return;
  const int last = ctl->iter - 1;
  for (int j = ctl->monitored + 1; j <= last; ++j) {
    const double* row = reduced + (long)((j - 1) % ring) * n_total;
    double s = 0.0;
    for (int g = 0; g < n_total; ++g) s += row[g];  // worker order == the single-rank finish
    if (j - 1 < max_iter) trace[j - 1] = s;
    ctl->monitored = j;
    if (!(s == s) || isinf(s)) {
      ctl->done = 3;
      ctl->conv_iter = j;
      return;
    }
    if (fabs(s - obj0) < tol) {
      ctl->done = 1;
      ctl->conv_iter = j;
      return;
    }
    if (j >= max_iter) {
      ctl->done = 2;
      ctl->conv_iter = j;
      return;
    }
  }
}

__global__ void chain_reset_kernel(ChainCtl* ctl, int start_iter, int pending) {
  if (threadIdx.x != 0) return;
  ctl->iter = start_iter;
  ctl->done = 0;
  ctl->conv_iter = 0;
  ctl->pending = pending;
  ctl->ticket = 0u;
  ctl->monitored = start_iter - 1;
  ctl->inner_fail = 0;
}

// ------------------------------------------------------------------------------------------------
extern "C" {

int gadmm_chain_phase_big(const PhaseArgs* args, hipStream_t st);
int gadmm_chain_phase_newton(const PhaseArgs* args, hipStream_t st);

int gadmm_chain_phase(const PhaseArgs* args, hipStream_t st) {
  const PhaseArgs& a = *args;
  if (a.n_slots <= 0) return 0;
  if (a.model == MODEL_LOGISTIC && a.solver == 1) return gadmm_chain_phase_newton(args, st);
  if (a.d > 256) {
    if (a.model != MODEL_LINEAR) {
      gadmm_set_error("chain_phase: logistic with d=%d > 256 is not supported by the fused kernels", a.d);
      return -1;
    }
    return gadmm_chain_phase_big(args, st);
  }
  const int nc = (a.d + 63) / 64;
  if (a.model == MODEL_LINEAR) {
    switch (nc) {
      case 1: hipLaunchKernelGGL(chain_phase_linear<1>, dim3(a.n_slots), dim3(NT), 0, st, a); break;
      case 2: hipLaunchKernelGGL(chain_phase_linear<2>, dim3(a.n_slots), dim3(NT), 0, st, a); break;
      default: hipLaunchKernelGGL(chain_phase_linear<4>, dim3(a.n_slots), dim3(NT), 0, st, a); break;
    }
  } else {
    const bool ldsx = (long)a.m * a.d <= 8192 && a.m <= 256;
    const size_t lds = ldsx ? (size_t)2 * a.m * a.d * sizeof(double) : 0;
    const int mc = (a.m + 63) / 64;
#define GADMM_LOG_LAUNCH(NCv, MCv, L)                                                                  \
  do {                                                                                               \
    auto kfn = chain_phase_logistic<NCv, MCv, L>;                                                    \
    if (lds > 65536) GADMM_CHECK(hipFuncSetAttribute((const void*)kfn,                               \
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    hipLaunchKernelGGL(kfn, dim3(a.n_slots), dim3(NT), lds, st, a);                                  \
  } while (0)
    if (ldsx) {
      // one wave per worker (default); GADMM_LOGISTIC_BLOCK=1 selects the 4-wave variant
      static const bool block4 = getenv("GADMM_LOGISTIC_BLOCK") != nullptr;
      // GADMM_LOGISTIC_QUAD=0: the LDS-staged one-wave kernel (A/B measurements)
      static const bool quad = !(getenv("GADMM_LOGISTIC_QUAD") && getenv("GADMM_LOGISTIC_QUAD")[0] == '0');
      const int dm = a.d > a.m ? a.d : a.m;
      // (the four-wave quad variant, GADMM_LOGISTIC_QUAD4=1, measured 7.20 vs 6.96 ms per solve -- its two
      // barriers per inner step cost more than the 3T FMAs they save per lane -- was removed in round 6)
      if (!block4 && quad && dm <= 64) {
        if (dm <= 32) hipLaunchKernelGGL(chain_phase_logistic_quad<8>, dim3(a.n_slots), dim3(64), 0, st, a);
        else if (dm <= 52) hipLaunchKernelGGL(chain_phase_logistic_quad<13>, dim3(a.n_slots), dim3(64), 0, st, a);
        else hipLaunchKernelGGL(chain_phase_logistic_quad<16>, dim3(a.n_slots), dim3(64), 0, st, a);
      } else if (!block4) {
        const int cmax = nc > mc ? nc : mc;
        const size_t lw = lds + (size_t)2 * 64 * cmax * sizeof(double);
#define GADMM_LOGW_LAUNCH(CV)                                                                           \
  do {                                                                                                  \
    auto kfn = chain_phase_logistic_wave<CV>;                                                           \
    if (lw > 65536) GADMM_CHECK(hipFuncSetAttribute((const void*)kfn,                                   \
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lw)); \
    hipLaunchKernelGGL(kfn, dim3(a.n_slots), dim3(64), lw, st, a);                                      \
  } while (0)
        if (cmax == 1) GADMM_LOGW_LAUNCH(1);
        else if (cmax == 2) GADMM_LOGW_LAUNCH(2);
        else GADMM_LOGW_LAUNCH(4);
#undef GADMM_LOGW_LAUNCH
      } else if (nc == 1 && mc == 1) GADMM_LOG_LAUNCH(1, 1, true);
      else if (nc <= 2 && mc <= 2) GADMM_LOG_LAUNCH(2, 2, true);
      else GADMM_LOG_LAUNCH(4, 4, true);
    } else {
      if (a.m > 256) {
        // sh_z / sh_y hold the whole shard's margins; larger shards use the row-blocked path.
        gadmm_set_error("chain_phase logistic: m=%d > 256 needs the row-blocked engine path", a.m);
        return -1;
      }
      if (nc == 1) GADMM_LOG_LAUNCH(1, 4, false);
      else GADMM_LOG_LAUNCH(4, 4, false);
    }
#undef GADMM_LOG_LAUNCH
  }
  GADMM_CHECK(hipGetLastError());
  return 0;
}

int gadmm_chain_dual_flush(const PhaseSlot* slots, int n_slots, int d, double rho, const double* theta, double* mu,
                           ChainCtl* ctl, hipStream_t st) {
  if (n_slots > 0)
    hipLaunchKernelGGL(chain_dual_flush_kernel, dim3(n_slots), dim3(NT), 0, st, slots, n_slots, d, rho, theta, mu,
                       ctl, 1);
  hipLaunchKernelGGL(chain_clear_pending_kernel, dim3(1), dim3(64), 0, st, ctl);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

int gadmm_chain_monitor(ChainCtl* ctl, const double* reduced, int ring, int n_total, double* trace, int max_iter,
                        double obj0, double tol, hipStream_t st) {
  hipLaunchKernelGGL(chain_monitor_kernel, dim3(1), dim3(64), 0, st, ctl, reduced, ring, n_total, trace, max_iter,
                     obj0, tol);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// Fresh-solve reset in ONE launch (was four torch fills + the control reset): theta, mu, part = 0,
// trace = NaN, control block as chain_reset_kernel.
__global__ void chain_reset_state_kernel(ChainCtl* ctl, int start_iter, int pending, double* theta, long n_theta,
                                         double* mu, long n_mu, double* trace, long n_trace, double* part,
                                         long n_part, long long* stamp) {
  const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x, step = (long)gridDim.x * blockDim.x;
  if (stamp && i0 == 0) *stamp = (long long)__builtin_amdgcn_s_memrealtime();  // the solve's real-clock start
  for (long i = i0; i < n_theta; i += step) theta[i] = 0.0;
  for (long i = i0; i < n_mu; i += step) mu[i] = 0.0;
  for (long i = i0; i < n_part; i += step) part[i] = 0.0;
  const double qnan = __longlong_as_double(0x7ff8000000000000ll);
  for (long i = i0; i < n_trace; i += step) trace[i] = qnan;
  if (i0 == 0) {
    ctl->iter = start_iter;
    ctl->done = 0;
    ctl->conv_iter = 0;
    ctl->pending = pending;
    ctl->ticket = 0u;
    ctl->monitored = start_iter - 1;
    ctl->inner_fail = 0;
  }
}

// stamp (nullable): also record the real-clock start (gadmm_write_stamp) in the same launch
int gadmm_chain_reset_state_stamp(ChainCtl* ctl, int start_iter, int pending, double* theta, long n_theta, double* mu,
                                  long n_mu, double* trace, long n_trace, double* part, long n_part, long long* stamp,
                                  hipStream_t st) {
  long mx = n_theta > n_mu ? n_theta : n_mu;
  mx = mx > n_trace ? mx : n_trace;
  int blocks = (int)((mx + 255) / 256);
  blocks = blocks < 1 ? 1 : (blocks > 64 ? 64 : blocks);
  hipLaunchKernelGGL(chain_reset_state_kernel, dim3(blocks), dim3(256), 0, st, ctl, start_iter, pending, theta,
                     n_theta, mu, n_mu, trace, n_trace, part, n_part, stamp);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

int gadmm_chain_reset_state(ChainCtl* ctl, int start_iter, int pending, double* theta, long n_theta, double* mu,
                            long n_mu, double* trace, long n_trace, double* part, long n_part, hipStream_t st) {
  return gadmm_chain_reset_state_stamp(ctl, start_iter, pending, theta, n_theta, mu, n_mu, trace, n_trace, part,
                                       n_part, nullptr, st);
}

int gadmm_chain_reset(ChainCtl* ctl, int start_iter, int pending, hipStream_t st) {
  hipLaunchKernelGGL(chain_reset_kernel, dim3(1), dim3(64), 0, st, ctl, start_iter, pending);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"

// Real-clock reference: s_memrealtime (100 MHz, the clock every monitor stamps decisions with) at the
// point of the stream where a solve starts.
__global__ void stamp_kernel(long long* p) {
  if (threadIdx.x == 0) *p = (long long)__builtin_amdgcn_s_memrealtime();
}

extern "C" int gadmm_write_stamp(long long* p, hipStream_t st) {
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, st, p);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// Close an iteration on a rank that owns no tail worker (multi-rank chains can leave a rank with
// heads only): sums the local objectives and advances the counter exactly like the tail's FINISH.
__global__ void chain_close_kernel(PhaseArgs a) {
  if (a.ctl->done) return;
  finish_iteration(a, a.ctl->iter);
}

extern "C" int gadmm_chain_close(const PhaseArgs* args, hipStream_t st) {
  hipLaunchKernelGGL(chain_close_kernel, dim3(1), dim3(64), 0, st, *args);
  GADMM_CHECK(hipGetLastError());
  return 0;
}
