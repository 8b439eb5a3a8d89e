// Large-d first-order comparators (d > 128; the real-shaped 10k config): GD, DGD, LAG-PS / LAG-WK,
// cyclic / randomized IAG and dual averaging of GD_DGD_LAG.m / dual_averaging.m,
// as stream-ordered kernels with the stop rule on the device (engine/first_order_big.py enqueues
// blocks of iterations and looks at the control word once per block, like star_big.hip).
//
// An iteration is HBM-bound on the d x d Grams: every A_n (and the local sum A_sum for the server's
// objective) is stored as its block-packed lower triangle (sym_gemv.h: 400 MB instead of 800 MB at
// d = 10k) and multiplied by the symmetric GEMV of sym_gemv.h. Everything else is O(N d) and fused
// into one or two elementwise kernels per iteration:
//   GD     q = A_sum th                 obj(th), th -= a g with g = q - b_sum (ones at it = 1)
//   DGD    q_n = A_n th_n               G[n] = q_n - b_n, obj; th_n -= a/100 * (neighbour average of G)
//   IAG    q = A_w th (refreshing w), q' = A_sum th: T[w] = q - b_w; obj; th -= a/N sum_n T[n]
//   LAG    q_n = A_n th (every worker)  triggers from the 10-deep history of |th^k - th^{k-1}|^2,
//                                       conditional uploads into T, th -= a sum_n T[n]
//   DualAv q_n = A_n th_n               obj of the previous iterate; the Gauss-Seidel (or Jacobi)
//                                       sweep Z_n = mix(Z_nbr) + g_n, th_n = -a Z_n, per element
// Vectors are zero padded to symv::padded(d) (the GEMV reads whole 128-blocks); the padding is never
// written. Objective partials are per (worker, 128-element block) and summed in a fixed order.
#include "gadmm_common.h"
#include "gadmm_chain.h"
#include "sym_gemv.h"

namespace {

constexpr int EB = 128;  // elementwise block = one symv block row
constexpr int TRIG = 10;  // LAG trigger slot (GD_DGD_LAG.m:18)

// y_s = M_s x_s (count slots; padded vectors, M_s block-packed); work: count x part_doubles
__global__ void __launch_bounds__(symv::NT) fob_symv_part(const double* Mp, long mstride, const double* x,
                                                          long xstride, double* work, int d, const ChainCtl* ctl) {
  __shared__ symv::dv2 tl[symv::NT / 64][64];
  if (ctl && ctl->done) return;
  const int s = blockIdx.y;
  symv::part_block(Mp + s * mstride, x + s * xstride, work + s * symv::part_doubles(d), symv::nblk(d), blockIdx.x, tl);
}

__global__ void __launch_bounds__(symv::RNT) fob_symv_reduce(const double* work, double* y, long ystride, int d,
                                                             const ChainCtl* ctl) {
  __shared__ double red[symv::RG][symv::B];
  if (ctl && ctl->done) return;
  const int s = blockIdx.y, t = blockIdx.x, k = threadIdx.x, j = t * symv::B + k;
  const double v = symv::reduce_row(work + s * symv::part_doubles(d), symv::nblk(d), t, red);
  if (k < symv::B && j < d) y[s * ystride + j] = v;
}

__device__ __forceinline__ double block_sum(double v, double* sh) {
  v = wave_sum_f64(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int q = 0; q < (int)(blockDim.x >> 6); ++q) t += sh[q];
  __syncthreads();
  return t;  // valid on thread 0
}

// ---- GD (server step with the stacked gradient, GD_DGD_LAG.m:88-118): obj partials at th, th -= a g
__global__ void __launch_bounds__(EB) fob_gd(const double* q, const double* bsum, double* th, double* part, int d,
                                             double step, int faithful, const ChainCtl* ctl) {
  __shared__ double sh[2];
  if (ctl->done) return;
  const int j = blockIdx.x * EB + threadIdx.x;
  double p = 0.0;
  if (j < d) {
    const double t = th[j];
    p = (0.5 * q[j] - bsum[j]) * t;
    const double g = (faithful && ctl->iter == 1) ? 1.0 : q[j] - bsum[j];
    th[j] = t - step * g;
  }
  const double s = block_sum(p, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// ---- DGD: G[gid] = q_n - b_n (ones at it = 1) + obj partials of th_n
__global__ void __launch_bounds__(EB) fob_dgd_grad(const double* q, long dp, const double* b, const double* th,
                                                   double* G, double* part, int d, int w_lo, int faithful,
                                                   const ChainCtl* ctl) {
  __shared__ double sh[2];
  if (ctl->done) return;
  const int n = blockIdx.y, j = blockIdx.x * EB + threadIdx.x;
  double p = 0.0;
  if (j < d) {
    const double qq = q[n * dp + j], bb = b[(long)n * d + j];
    p = (0.5 * qq - bb) * th[n * dp + j];
    G[(long)(w_lo + n) * d + j] = (faithful && ctl->iter == 1) ? 1.0 : qq - bb;
  }
  const double s = block_sum(p, sh);
  if (threadIdx.x == 0) part[(long)n * gridDim.x + blockIdx.x] = s;
}

// th_n -= a/100 * neighbour average of G (GD_DGD_LAG.m:155-171; the torch path's operation order)
__global__ void __launch_bounds__(EB) fob_dgd_update(double* th, long dp, const double* G, int d, int w_lo,
                                                     int n_total, double step, const ChainCtl* ctl) {
  if (ctl->done) return;
  const int n = blockIdx.y, j = blockIdx.x * EB + threadIdx.x;
  if (j >= d) return;
  const int w = w_lo + n;
  const double t = th[n * dp + j], gw = G[(long)w * d + j];
  double v;
  if (n_total == 1) v = t - step * gw;
  else if (w == 0) v = t - 0.5 * step * (gw + G[(long)(w + 1) * d + j]);
  else if (w == n_total - 1) v = t - 0.5 * step * (gw + G[(long)(w - 1) * d + j]);
  else v = t - (1.0 / 3.0) * step * (gw + G[(long)(w + 1) * d + j] + G[(long)(w - 1) * d + j]);
  th[n * dp + j] = v;
}

// ---- server tables (IAG, LAG): obj partials of the replicated th from q = A_sum th (IAG) and the
// server step th -= a * sum_n T[n] (worker order); dth: |th_new - th|^2 partials (LAG triggers)
__global__ void __launch_bounds__(EB) fob_server(const double* q, const double* bsum, double* th, const double* T,
                                                 double* part, double* dpart, int d, int n_total, double step,
                                                 const ChainCtl* ctl) {
  __shared__ double sh[2];
  if (ctl->done) return;
  const int j = blockIdx.x * EB + threadIdx.x;
  double p = 0.0, dd = 0.0;
  if (j < d) {
    const double t = th[j];
    if (q) p = (0.5 * q[j] - bsum[j]) * t;
    double s = 0.0;
    for (int n = 0; n < n_total; ++n) s += T[(long)n * d + j];
    const double tn = t - step * s;
    th[j] = tn;
    dd = (tn - t) * (tn - t);
  }
  const double s1 = block_sum(p, sh);
  if (threadIdx.x == 0 && part) part[blockIdx.x] = s1;
  const double s2 = block_sum(dd, sh);
  if (threadIdx.x == 0 && dpart) dpart[blockIdx.x] = s2;
}

// IAG refresh of worker w (local index li): T[w] = q - b_li
__global__ void __launch_bounds__(EB) fob_iag_refresh(const double* q, const double* b, double* T, int d, int li,
                                                      int w, const ChainCtl* ctl) {
  if (ctl->done || ctl->iter <= 1) return;
  const int j = blockIdx.x * EB + threadIdx.x;
  if (j < d) T[(long)w * d + j] = q[j] - b[(long)li * d + j];
}

// ---- LAG: grads at th for every worker (q_n - b_n), obj partials, trigger distances per block
__global__ void __launch_bounds__(EB) fob_lag_grad(const double* q, long dp, const double* b, const double* th,
                                                   double* GN, const double* Gl, const double* thhat, double* part,
                                                   double* ddpart, int d, int ps, const ChainCtl* ctl) {
  __shared__ double sh[2];
  if (ctl->done) return;
  const int n = blockIdx.y, j = blockIdx.x * EB + threadIdx.x;
  double p = 0.0, dd = 0.0;
  if (j < d) {
    const double qq = q[n * dp + j], bb = b[(long)n * d + j], t = th[j];
    const double g = qq - bb;
    GN[(long)n * d + j] = g;
    p = (0.5 * qq - bb) * t;
    const double df = ps ? thhat[(long)n * d + j] - t : g - Gl[(long)n * d + j];
    dd = df * df;
  }
  const double s1 = block_sum(p, sh);
  if (threadIdx.x == 0) part[(long)n * gridDim.x + blockIdx.x] = s1;
  const double s2 = block_sum(dd, sh);
  if (threadIdx.x == 0) ddpart[(long)n * gridDim.x + blockIdx.x] = s2;
}

// LAG decisions (one thread per local worker): mask_n from the trigger of GD_DGD_LAG.m:211-227 /
// :287-300 (nothing before iter > 10), the upload count into cnt[it - 1]; ring[TRIG + 2] holds
// |th^k - th^{k-1}|^2 of the last iterations (slot k % (TRIG + 1))
__global__ void fob_lag_decide(const double* ddpart, int nblk, const double* hsq, const double* ring, int* mask,
                               double* cnt, int n_local, int w_lo, int ps, double thrd, int faithful,
                               const ChainCtl* ctl) {
  if (ctl->done || threadIdx.x != 0) return;
  const int it = ctl->iter;
  double trig = 0.0;
  if (it > TRIG)
    for (int k = 1; k <= TRIG; ++k) trig += ring[(it - k) % (TRIG + 1)];  // the torch path's order: n = 1..10
  int c = 0;
  for (int n = 0; n < n_local; ++n) {
    int m = 0;
    if (it > TRIG) {
      double dd = 0.0;
      for (int k = 0; k < nblk; ++k) dd += ddpart[(long)n * nblk + k];
      m = ps ? (hsq[w_lo + n] * dd > thrd * trig) : (dd > thrd * trig);
    }
    c += m;
    // forced refresh of worker 1 every iteration > 1 (LAG-PS quirk 4), not counted: mask 2
    mask[n] = m ? 1 : ((ps && faithful && it > 1 && w_lo + n == 0) ? 2 : 0);
  }
  if (it - 1 >= 0) cnt[it - 1] = (double)c;
}

// rows[it - 1] = how many of this rank's table rows travel this iteration (mask != 0: the triggered
// uploads plus LAG-PS's forced worker-1 refresh): the conditional exchange's payload (multi-rank LAG)
__global__ void fob_lag_rows(const int* mask, int n_local, double* rows, const ChainCtl* ctl) {
  if (ctl->done || threadIdx.x != 0) return;
  int r = 0;
  for (int n = 0; n < n_local; ++n) r += mask[n] != 0;
  if (ctl->iter >= 1) rows[ctl->iter - 1] = (double)r;
}

// LAG uploads: masked workers take their new gradient (and PS its th-hat) into G_loc and the table
__global__ void __launch_bounds__(EB) fob_lag_apply(const double* GN, double* Gl, double* thhat, const double* th,
                                                    double* T, const int* mask, int d, int w_lo, int ps,
                                                    const ChainCtl* ctl) {
  if (ctl->done) return;
  const int n = blockIdx.y, j = blockIdx.x * EB + threadIdx.x;
  const int m = mask[n];
  if (j >= d || m == 0) return;
  const double g = GN[(long)n * d + j];
  Gl[(long)n * d + j] = g;
  if (ps && m == 1) thhat[(long)n * d + j] = th[j];
  T[(long)(w_lo + n) * d + j] = g;
}

// ---- dual averaging: obj partials of th_n^{it-1} (the previous iterate) and the sweep
__global__ void __launch_bounds__(EB) fob_da_obj(const double* q, long dp, const double* b, const double* th,
                                                 double* part, int d, const ChainCtl* ctl) {
  __shared__ double sh[2];
  if (ctl->done) return;
  const int n = blockIdx.y, j = blockIdx.x * EB + threadIdx.x;
  double p = 0.0;
  if (j < d) p = (0.5 * q[n * dp + j] - b[(long)n * d + j]) * th[n * dp + j];
  const double s = block_sum(p, sh);
  if (threadIdx.x == 0) part[(long)n * gridDim.x + blockIdx.x] = s;
}

// one thread per element: the workers in chain order (Z overwritten in place: Gauss-Seidel, or
// the previous sweep's Z for both neighbours in Jacobi mode), th_n = -a Z_n (dual_averaging.m:34-44).
// Z is the chain-wide table (n_total x d, global worker rows); this rank sweeps its rows w_lo ..
// w_lo + n - 1 (one rank: all of them). Across ranks the rows next to the segment are ghosts filled by
// the exchanges around the sweep (engine/first_order_big.py): row w_lo - 1 holds the left neighbour
// rank's Z of THIS sweep (Gauss-Seidel; Jacobi: of the previous one), row w_lo + n its right neighbour's
// of the previous sweep -- exactly the values the one-rank sweep reads there. Zp: (n x d) local copy.
__global__ void __launch_bounds__(EB) fob_da_sweep(const double* q, long dp, const double* b, double* th, double* Z,
                                                   double* Zp, int d, int n, int w_lo, int n_total, double alpha,
                                                   int jacobi, const ChainCtl* ctl) {
  if (ctl->done) return;
  const int j = blockIdx.x * EB + threadIdx.x;
  if (j >= d) return;
  for (int k = 0; k < n; ++k) Zp[(long)k * d + j] = Z[(long)(w_lo + k) * d + j];
  for (int k = 0; k < n; ++k) {
    const int w = w_lo + k;
    const double g = q[k * dp + j] - b[(long)k * d + j];
    const bool hl = w > 0, hr = w < n_total - 1;
    // the left ghost (k = 0) and right ghost (k = n - 1) rows already carry the right semantics
    const double left = hl ? ((jacobi && k > 0) ? Zp[(long)(k - 1) * d + j] : Z[(long)(w - 1) * d + j]) : 0.0;
    const double right = hr ? (k < n - 1 ? Zp[(long)(k + 1) * d + j] : Z[(long)(w + 1) * d + j]) : 0.0;
    double zn;
    if (!hl && !hr) zn = g;
    else if (!hl) zn = right + g;
    else if (!hr) zn = left + g;
    else zn = 0.5 * right + 0.5 * left + g;
    Z[(long)w * d + j] = zn;
    th[k * dp + j] = -alpha * zn;
  }
}

__global__ void fob_objw(const double* part, int nblk, const double* yy, double* objw, int n_local, int w_lo,
                         int n_total, const ChainCtl* ctl) {
  if (ctl->done) return;
  for (int g = threadIdx.x; g < n_total; g += blockDim.x) objw[g] = 0.0;
  __syncthreads();
  for (int n = threadIdx.x; n < n_local; n += blockDim.x) {
    double f = 0.0;
    for (int k = 0; k < nblk; ++k) f += part[(long)n * nblk + k];
    objw[w_lo + n] = f + 0.5 * yy[n];
  }
}

// ---- finish: per-worker objectives (partials in block order + 1/2 y'y) -> trace, stop rule, iter.
// nw objective rows of nblk partials each (nw = 1: the replicated-theta algorithms, yy = y'y sum).
// `shift` = 1: the objective belongs to the previous iteration (dual averaging evaluates th^{it-1}
// with the GEMV of iteration it); ring / dpart: LAG's |dth|^2 history.
__global__ void fob_finish(const double* part, int nw, int nblk, const double* yy, double* trace, long long* tstamp,
                           int max_iter, double obj0, double tol, int shift, const double* dpart, int dnblk,
                           double* ring, ChainCtl* ctl) {
  if (threadIdx.x != 0 || ctl->done) return;
  const int it = ctl->iter;
  if (dpart) {  // LAG: |th^{it} - th^{it-1}|^2 into the ring slot it % 11 (read from iteration it + 1 on)
    // dpart has one partial per 128-element block of theta (dnblk of them), independent of the
    // objective rows' `nblk` (LAG's objective comes as one entry per worker: nblk = 1). Summing only
    // `nblk` partials here kept the first 128 coordinates of the step at d > 128 -- an underestimated
    // trigger threshold, extra uploads (tools/lag_diverge.py, profiles/r05_a).
    double s = 0.0;
    for (int k = 0; k < dnblk; ++k) s += dpart[k];
    ring[it % (TRIG + 1)] = s;
  }
  const int rec = it - shift;  // the iteration this objective belongs to
  if (rec >= 1) {
    double obj = 0.0;
    for (int w = 0; w < nw; ++w) {
      double f = 0.0;
      for (int k = 0; k < nblk; ++k) f += part[(long)w * nblk + k];
      obj += f + 0.5 * yy[w];
    }
    if (rec - 1 < max_iter) {
      trace[rec - 1] = obj;
      tstamp[rec - 1] = (long long)__builtin_amdgcn_s_memrealtime();
    }
    int code = 0;
    if (!(obj == obj) || isinf(obj)) code = 3;
    else if (tol >= 0.0 && fabs(obj - obj0) < tol) code = 1;
    else if (rec >= max_iter) code = 2;
    if (code) {
      ctl->done = code;
      ctl->conv_iter = rec;
    }
  }
  ctl->iter = it + 1;
}

// ---- Jacobi-preconditioned CG for the large-d optimum oracle (models/linear.py:_cg_solve) -----------
// One workgroup of CG_NT threads runs every vector step of an iteration (d = 10k: ten elements per
// thread); the products are the block-packed symmetric GEMV above (gadmm_symv_batch). Dot products are
// block sums in a fixed order, broadcast to every thread: deterministic. sc = [r.z, scratch, bad].
constexpr int CG_NT = 1024;

__device__ __forceinline__ double cg_allsum(double v, double* sh) {
  v = wave_sum_f64(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();  // sh is reused by the next call
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int q = 0; q < CG_NT / 64; ++q) t += sh[q];  // the same order on every thread
  return t;
}

// dinv = 1 / diag(M), x = dinv * b, sc[1] = |b|^2, sc[2] = number of non-positive pivots. The diagonal
// is read with stride `ds`: d + 1 for a full d x d M, 1 for a diagonal vector (the distributed CG,
// whose M = sum over ranks of the local Grams exists only as its all-reduced diagonal)
__global__ void __launch_bounds__(CG_NT) cg_begin(const double* M, long ds, const double* b, double* dinv,
                                                   double* x, double* sc, int d) {
  __shared__ double sh[CG_NT / 64];
  double bb = 0.0, bad = 0.0;
  for (int j = threadIdx.x; j < d; j += CG_NT) {
    const double m = M[(long)j * ds];
    const double di = 1.0 / m;
    bad += (m > 0.0) ? 0.0 : 1.0;
    dinv[j] = di;
    x[j] = di * b[j];
    bb = fma(b[j], b[j], bb);
  }
  bb = cg_allsum(bb, sh);
  bad = cg_allsum(bad, sh);
  if (threadIdx.x == 0) {
    sc[1] = bb;
    sc[2] = bad;
  }
}

// q = M x0: res = b - q, z = dinv res, p = z, sc[0] = res . z
__global__ void __launch_bounds__(CG_NT) cg_begin2(const double* b, const double* dinv, const double* q, double* res,
                                                    double* z, double* p, double* sc, int d) {
  __shared__ double sh[CG_NT / 64];
  double rz = 0.0;
  for (int j = threadIdx.x; j < d; j += CG_NT) {
    const double r = b[j] - q[j], zz = dinv[j] * r;
    res[j] = r;
    z[j] = zz;
    p[j] = zz;
    rz = fma(r, zz, rz);
  }
  rz = cg_allsum(rz, sh);
  if (threadIdx.x == 0) sc[0] = rz;
}

// q = M p: one CG iteration's vector work
__global__ void __launch_bounds__(CG_NT) cg_step(const double* q, const double* dinv, double* x, double* res, double* z,
                                                  double* p, double* sc, int d) {
  __shared__ double sh[CG_NT / 64];
  const double rz = sc[0];
  double pq = 0.0;
  for (int j = threadIdx.x; j < d; j += CG_NT) pq = fma(p[j], q[j], pq);
  pq = cg_allsum(pq, sh);
  const double alpha = rz / pq;
  double rzn = 0.0;
  for (int j = threadIdx.x; j < d; j += CG_NT) {
    x[j] = fma(alpha, p[j], x[j]);
    const double r = fma(-alpha, q[j], res[j]), zz = dinv[j] * r;
    res[j] = r;
    z[j] = zz;
    rzn = fma(r, zz, rzn);
  }
  rzn = cg_allsum(rzn, sh);
  const double beta = rzn / rz;
  for (int j = threadIdx.x; j < d; j += CG_NT) p[j] = fma(beta, p[j], z[j]);
  if (threadIdx.x == 0) sc[0] = rzn;  // every thread read sc[0] before cg_allsum's barriers
}

// q = M x: sc[1] = |b - q|^2 (the true residual)
__global__ void __launch_bounds__(CG_NT) cg_resid(const double* b, const double* q, double* sc, int d) {
  __shared__ double sh[CG_NT / 64];
  double e2 = 0.0;
  for (int j = threadIdx.x; j < d; j += CG_NT) {
    const double e = b[j] - q[j];
    e2 = fma(e, e, e2);
  }
  e2 = cg_allsum(e2, sh);
  if (threadIdx.x == 0) sc[1] = e2;
}

// ---- residual of the optimum oracle: sum_r (X_r . x - y_r)^2 over a tall (rows x d) shard -----------
// One wave per row at a time (16-byte loads, eight in flight per lane), rows dealt round-robin over the
// grid's waves; per-workgroup partials, then one workgroup sums them in a fixed order (deterministic).
// The shard is read once at HBM speed (rocBLAS gemv took 22 ms for 100 GB at d = 10k).
constexpr int RS_NT = 256;

__global__ void __launch_bounds__(RS_NT) resid_sq_part(const double* __restrict__ X, const double* __restrict__ y,
                                                       const double* __restrict__ x, long rows, int d,
                                                       double* __restrict__ part) {
  __shared__ double sh[RS_NT / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long nw = (long)gridDim.x * (RS_NT / 64);
  double acc = 0.0;
  for (long r = (long)blockIdx.x * (RS_NT / 64) + w; r < rows; r += nw) {
    const double* row = X + r * d;
    double s0 = 0.0, s1 = 0.0;
    if ((d & 1) == 0) {
      const int d2 = d >> 1;
      const symv::dv2* r2 = reinterpret_cast<const symv::dv2*>(row);
      const symv::dv2* x2 = reinterpret_cast<const symv::dv2*>(x);
      for (int j = lane; j < d2; j += 64) {
        const symv::dv2 a = __builtin_nontemporal_load(r2 + j), b = x2[j];
        s0 = fma(a.x, b.x, s0);
        s1 = fma(a.y, b.y, s1);
      }
    } else {
      for (int j = lane; j < d; j += 64) s0 = fma(row[j], x[j], s0);
    }
    const double dot = wave_sum_f64(s0 + s1);
    const double e = dot - y[r];
    acc = fma(e, e, acc);  // identical on every lane of the wave
  }
  if (lane == 0) sh[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int q = 0; q < RS_NT / 64; ++q) t += sh[q];
    part[blockIdx.x] = t;
  }
}

__global__ void __launch_bounds__(1024) resid_sq_final(const double* __restrict__ part, int n, double* out) {
  __shared__ double sh[16];
  double t = 0.0;
  for (int k = threadIdx.x; k < n; k += 1024) t += part[k];
  t = wave_sum_f64(t);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int q = 0; q < 16; ++q) s += sh[q];
    out[0] = s;
  }
}

}  // namespace

extern "C" {

// y_s = M_s x_s for `count` slots: M block-packed (stride mstride doubles), x zero padded (xstride),
// y (ystride); work: count * part_doubles(d). ctl: optional skip word (done != 0: no-op).
int gadmm_symv_batch(const double* Mp, long mstride, const double* x, long xstride, double* y, long ystride,
                     double* work, int count, int d, const ChainCtl* ctl, hipStream_t st) {
  if (!Mp || !x || !y || !work || count < 1 || d < 1) {
    gadmm_set_error("symv_batch: bad arguments");
    return -1;
  }
  hipLaunchKernelGGL(fob_symv_part, dim3((unsigned)symv::nstored(d), count), dim3(symv::NT), 0, st, Mp, mstride, x,
                     xstride, work, d, ctl);
  hipLaunchKernelGGL(fob_symv_reduce, dim3(symv::nblk(d), count), dim3(symv::RNT), 0, st, work, y, ystride, d, ctl);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

long gadmm_symv_work_doubles(int d) { return symv::part_doubles(d); }
long gadmm_sym_padded(int d) { return symv::padded(d); }

int gadmm_fob_gd(const double* q, const double* bsum, double* th, double* part, int d, double step, int faithful,
                 const ChainCtl* ctl, hipStream_t st) {
  hipLaunchKernelGGL(fob_gd, dim3((d + EB - 1) / EB), dim3(EB), 0, st, q, bsum, th, part, d, step, faithful, ctl);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

int gadmm_fob_dgd_grad(const double* q, long dp, const double* b, const double* th, double* G, double* part, int d,
                       int n_local, int w_lo, int faithful, const ChainCtl* ctl, hipStream_t st) {
  hipLaunchKernelGGL(fob_dgd_grad, dim3((d + EB - 1) / EB, n_local), dim3(EB), 0, st, q, dp, b, th, G, part, d, w_lo,
                     faithful, ctl);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

int gadmm_fob_dgd_update(double* th, long dp, const double* G, int d, int n_local, int w_lo, int n_total, double step,
                         const ChainCtl* ctl, hipStream_t st) {
  hipLaunchKernelGGL(fob_dgd_update, dim3((d + EB - 1) / EB, n_local), dim3(EB), 0, st, th, dp, G, d, w_lo, n_total,
                     step, ctl);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

int gadmm_fob_server(const double* q, const double* bsum, double* th, const double* T, double* part, double* dpart,
                     int d, int n_total, double step, const ChainCtl* ctl, hipStream_t st) {
  hipLaunchKernelGGL(fob_server, dim3((d + EB - 1) / EB), dim3(EB), 0, st, q, bsum, th, T, part, dpart, d, n_total,
                     step, ctl);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

int gadmm_fob_iag_refresh(const double* q, const double* b, double* T, int d, int li, int w, const ChainCtl* ctl,
                          hipStream_t st) {
  hipLaunchKernelGGL(fob_iag_refresh, dim3((d + EB - 1) / EB), dim3(EB), 0, st, q, b, T, d, li, w, ctl);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

int gadmm_fob_lag(const double* q, long dp, const double* b, const double* th, double* GN, double* Gl, double* thhat,
                  double* T, double* part, double* ddpart, const double* hsq, const double* ring, int* mask,
                  double* cnt, int d, int n_local, int w_lo, int ps, double thrd, int faithful, const ChainCtl* ctl,
                  hipStream_t st) {
  const int nblk = (d + EB - 1) / EB;
  hipLaunchKernelGGL(fob_lag_grad, dim3(nblk, n_local), dim3(EB), 0, st, q, dp, b, th, GN, Gl, thhat, part, ddpart, d,
                     ps, ctl);
  hipLaunchKernelGGL(fob_lag_decide, dim3(1), dim3(64), 0, st, ddpart, nblk, hsq, ring, mask, cnt, n_local, w_lo, ps,
                     thrd, faithful, ctl);
  hipLaunchKernelGGL(fob_lag_apply, dim3(nblk, n_local), dim3(EB), 0, st, GN, Gl, thhat, th, T, mask, d, w_lo, ps, ctl);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

int gadmm_fob_lag_rows(const int* mask, int n_local, double* rows, const ChainCtl* ctl, hipStream_t st) {
  hipLaunchKernelGGL(fob_lag_rows, dim3(1), dim3(64), 0, st, mask, n_local, rows, ctl);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// per-worker objective partials of th_n (rows of q / th with stride dp), e.g. dual averaging's
// previous iterate
int gadmm_fob_worker_obj(const double* q, long dp, const double* b, const double* th, double* part, int d, int n,
                         const ChainCtl* ctl, hipStream_t st) {
  const int nblk = (d + EB - 1) / EB;
  hipLaunchKernelGGL(fob_da_obj, dim3(nblk, n), dim3(EB), 0, st, q, dp, b, th, part, d, ctl);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// per-worker objectives into global slots: objw[w_lo + n] = sum_k part[n][k] + 1/2 yy_n (block order),
// every other slot 0 (so an all-reduce of objw over the ranks is exact)
int gadmm_fob_objw(const double* part, int nblk, const double* yy, double* objw, int n_local, int w_lo, int n_total,
                   const ChainCtl* ctl, hipStream_t st) {
  hipLaunchKernelGGL(fob_objw, dim3(1), dim3(64), 0, st, part, nblk, yy, objw, n_local, w_lo, n_total, ctl);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

int gadmm_fob_da_sweep(const double* q, long dp, const double* b, double* th, double* Z, double* Zp, int d, int n,
                       int w_lo, int n_total, double alpha, int jacobi, const ChainCtl* ctl, hipStream_t st) {
  if (n < 1 || w_lo < 0 || w_lo + n > n_total) {
    gadmm_set_error("fob_da_sweep: rows %d + %d of %d", w_lo, n, n_total);
    return -1;
  }
  hipLaunchKernelGGL(fob_da_sweep, dim3((d + EB - 1) / EB), dim3(EB), 0, st, q, dp, b, th, Z, Zp, d, n, w_lo, n_total,
                     alpha, jacobi, ctl);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

int gadmm_fob_finish(const double* part, int nw, int nblk, const double* yy, double* trace, long long* tstamp,
                     int max_iter, double obj0, double tol, int shift, const double* dpart, int dnblk, double* ring,
                     ChainCtl* ctl, hipStream_t st) {
  if (dpart && (dnblk < 1 || !ring)) {
    gadmm_set_error("fob_finish: the step partials need their block count and the ring");
    return -1;
  }
  hipLaunchKernelGGL(fob_finish, dim3(1), dim3(64), 0, st, part, nw, nblk, yy, trace, tstamp, max_iter, obj0, tol,
                     shift, dpart, dnblk, ring, ctl);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// CG steps of the large-d optimum oracle (see cg_begin ...): single-workgroup launches on `st`
int gadmm_cg_begin(const double* M, const double* b, double* dinv, double* x, double* sc, int d, hipStream_t st) {
  if (!M || !b || !dinv || !x || !sc || d < 1) {
    gadmm_set_error("cg_begin: bad arguments (d=%d)", d);
    return -1;
  }
  hipLaunchKernelGGL(cg_begin, dim3(1), dim3(CG_NT), 0, st, M, (long)d + 1, b, dinv, x, sc, d);
  GADMM_CHECK(hipGetLastError());
  return 0;
}
// the same from diag(M) alone (distributed CG: the all-reduced diagonal of the rank-summed Gram)
int gadmm_cg_begin_diag(const double* diag, const double* b, double* dinv, double* x, double* sc, int d,
                        hipStream_t st) {
  if (!diag || !b || !dinv || !x || !sc || d < 1) {
    gadmm_set_error("cg_begin_diag: bad arguments (d=%d)", d);
    return -1;
  }
  hipLaunchKernelGGL(cg_begin, dim3(1), dim3(CG_NT), 0, st, diag, 1L, b, dinv, x, sc, d);
  GADMM_CHECK(hipGetLastError());
  return 0;
}
int gadmm_cg_begin2(const double* b, const double* dinv, const double* q, double* res, double* z, double* p, double* sc,
                    int d, hipStream_t st) {
  if (!b || !dinv || !q || !res || !z || !p || !sc || d < 1) {
    gadmm_set_error("cg_begin2: bad arguments (d=%d)", d);
    return -1;
  }
  hipLaunchKernelGGL(cg_begin2, dim3(1), dim3(CG_NT), 0, st, b, dinv, q, res, z, p, sc, d);
  GADMM_CHECK(hipGetLastError());
  return 0;
}
int gadmm_cg_step(const double* q, const double* dinv, double* x, double* res, double* z, double* p, double* sc, int d,
                  hipStream_t st) {
  if (!q || !dinv || !x || !res || !z || !p || !sc || d < 1) {
    gadmm_set_error("cg_step: bad arguments (d=%d)", d);
    return -1;
  }
  hipLaunchKernelGGL(cg_step, dim3(1), dim3(CG_NT), 0, st, q, dinv, x, res, z, p, sc, d);
  GADMM_CHECK(hipGetLastError());
  return 0;
}
int gadmm_cg_resid(const double* b, const double* q, double* sc, int d, hipStream_t st) {
  if (!b || !q || !sc || d < 1) {
    gadmm_set_error("cg_resid: bad arguments (d=%d)", d);
    return -1;
  }
  hipLaunchKernelGGL(cg_resid, dim3(1), dim3(CG_NT), 0, st, b, q, sc, d);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// out[0] = sum_r (X_r . x - y_r)^2 for X (rows x d, row-major), y (rows); part: >= 4096 doubles of scratch
int gadmm_resid_sq(const double* X, const double* y, const double* x, long rows, int d, double* part, double* out,
                   hipStream_t st) {
  if (!X || !y || !x || !part || !out || rows < 1 || d < 1) {
    gadmm_set_error("resid_sq: bad arguments (rows=%ld d=%d)", rows, d);
    return -1;
  }
  const long want = (rows + 3) / 4;
  const int grid = (int)(want < 4096 ? want : 4096);
  hipLaunchKernelGGL(resid_sq_part, dim3(grid), dim3(RS_NT), 0, st, X, y, x, rows, d, part);
  hipLaunchKernelGGL(resid_sq_final, dim3(1), dim3(1024), 0, st, part, grid, out);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"
