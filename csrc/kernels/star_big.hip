// Star (parameter-server) ADMM for large d -- standared_ADMM.m:17-88, the
// comparator of BASELINE configs[4] ("10M x 10k sharded across 8 GPUs vs standard-ADMM baseline").
//
// The persistent star kernel (star_persistent.hip) keeps every worker's inverse in registers, d <= 64.
// At d = 10k an inverse is 800 MB, so an iteration is three HBM-streaming GEMV passes and a handful
// of collectives; the host enqueues blocks of iterations without synchronising and every kernel
// leaves at once after the device-side stop rule fired (ctl->done), so a solve costs one host
// round trip per block, not per iteration. Per iteration (N workers, the hub = worker N - 1 also
// owns a shard):
//   sb_rhs    (non-hub local workers)  r_i = b_i - lam_i + rho th_hub                        (:42)
//   sb_sym_*  th_i = (A_i + rho I)^{-1} r_i           [packed lower triangle, sym_gemv.h]
//   sb_sum    agg = [sum_i lam_i, sum_i th_i] over this rank's non-hub workers (worker order)
//   -- reduce(agg) to the hub rank (RCCL ncclReduce; nothing on one rank)                  (:66-71)
//   sb_hubrhs r_h = b_h + agg_lam + rho agg_th                                            (:73)
//   sb_sym_*  th_hub = (A_h + (N-1) rho I)^{-1} r_h   (hub rank)
//   -- broadcast(th_hub) from the hub rank (RCCL ncclBroadcast)
//   sb_post   lam_i += rho (th_i - th_hub), f_i(th_i), f_h(th_hub)                        (:84-88)
//   -- allreduce(objp) (RCCL or the IPC device collective; nothing on one rank): objp holds one
//      slot per GLOBAL worker, non-zero only on its owner, so the sum is exact and sb_finish adds
//      the N objectives in worker order -- the same bits as one rank, on every rank
//   sb_finish trace[it] = obj, |obj - obj0| < tol -> done                                  (:95-107)
// Objective: identity mode f = (1/2 (r - c rho th) - b)^T th + 1/2 y^T y, from (A + c rho I) th = r
// (no extra pass over the inverse); exact mode (obj_mode 0) adds one GEMV with A per worker.
#include "gadmm_common.h"
#include "gadmm_chain.h"
#include "big_gemv.h"

using namespace biggemv;

struct StarBigArgs {
  int d, n_total, n_local, hub_li;  // hub_li: local index of the hub (-1: the hub is on another rank)
  int max_iter, obj_mode, pad0, pad1;
  double rho, obj0, tol;
  const double* Minv;  // [n_local][packed_doubles(d)]: block-packed lower triangles (sym_gemv.h) of
                       // (A_i + rho I)^-1, the hub's (A_h + (N-1) rho I)^-1
  const double* A;     // [n_local][d][d] (exact objective mode)
  const double* b;     // [n_local][d]
  const double* yy;    // [n_local]
  double* theta;       // [n_local][d]
  double* lam;         // [n_local][d] (the hub's row unused)
  double* th_hub;      // [d] the broadcast buffer (theta of the hub, previous iteration on entry)
  double* agg;         // [2 d] reduce buffer
  double* rbuf;        // [n_local][rstride(d)] right-hand sides + objective partials
  double* objw;        // [n_local] per-worker objective
  double* objp;        // [n_total] per-worker objectives, this rank's slots only (allreduce buffer)
  double* trace;       // [max_iter]
  ChainCtl* ctl;       // iter (next iteration), done, conv_iter
  long long* tstamp;   // [max_iter] s_memrealtime (100 MHz) when each iteration's stop rule ran
  const int* gid;      // [n_local] global worker id of each local worker
};

namespace {

__global__ void __launch_bounds__(NT) sb_rhs(StarBigArgs a) {
  if (a.ctl->done) return;
  const int s = blockIdx.y;
  if (s == a.hub_li) return;
  const int j = blockIdx.x * NT + threadIdx.x;
  if (j >= a.d) return;
  const long d = a.d;
  a.rbuf[s * rstride(a.d) + j] = a.b[s * d + j] - a.lam[s * d + j] + a.rho * a.th_hub[j];
}

// theta_s = Minv_s r_s for the local workers s with (s == hub_li) == hub: Minv_s block-packed lower
// triangles (sym_gemv.h), partials of every stored block, then the fixed-order reduction
__global__ void __launch_bounds__(symv::NT) sb_sym_part(StarBigArgs a, int hub) {
  __shared__ symv::dv2 tl[symv::NT / 64][64];
  if (a.ctl->done) return;
  const int s = blockIdx.y;
  if ((s == a.hub_li) != (hub != 0)) return;
  const int d = a.d;
  double* rb = a.rbuf + s * rstride(d);
  symv::part_block(a.Minv + (long)s * symv::packed_doubles(d), rb, rb + part_off(d), symv::nblk(d), blockIdx.x, tl);
}

__global__ void __launch_bounds__(symv::RNT) sb_sym_reduce(StarBigArgs a, int hub) {
  __shared__ double red[symv::RG][symv::B];
  if (a.ctl->done) return;
  const int s = blockIdx.y;
  if ((s == a.hub_li) != (hub != 0)) return;
  const int d = a.d, t = blockIdx.x, k = threadIdx.x, j = t * symv::B + k;
  const double y = symv::reduce_row(a.rbuf + s * rstride(d) + part_off(d), symv::nblk(d), t, red);
  if (k < symv::B && j < d) {
    a.theta[(long)s * d + j] = y;
    if (hub) a.th_hub[j] = y;
  }
}

__global__ void __launch_bounds__(NT) sb_sum(StarBigArgs a) {
  if (a.ctl->done) return;
  const int j = blockIdx.x * NT + threadIdx.x;
  if (j >= a.d) return;
  const long d = a.d;
  double sl = 0.0, st = 0.0;
  for (int s = 0; s < a.n_local; ++s) {  // worker order
    if (s == a.hub_li) continue;
    sl += a.lam[s * d + j];
    st += a.theta[s * d + j];
  }
  a.agg[j] = sl;
  a.agg[d + j] = st;
}

__global__ void __launch_bounds__(NT) sb_hubrhs(StarBigArgs a) {
  if (a.ctl->done || a.hub_li < 0) return;
  const int j = blockIdx.x * NT + threadIdx.x;
  if (j >= a.d) return;
  const long d = a.d;
  const int h = a.hub_li;
  a.rbuf[h * rstride(a.d) + j] = a.b[h * d + j] + a.agg[j] + a.rho * a.agg[d + j];
}

// exact objective mode: per-workgroup partials of sum_i (1/2 (A th)_i - b_i) th_i (as chain_big_obj)
__global__ void __launch_bounds__(NT) sb_obj(StarBigArgs a) {
  __shared__ double wsum[NT / 64];
  if (a.ctl->done) return;
  const int s = blockIdx.y;
  const int d = a.d;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row0 = blockIdx.x * ROWS_PER_WG + w * RPW;
  const double* th = a.theta + (long)s * d;
  double part = 0.0;
  if (row0 < d) {
    double q[RPW];
    wave_rows_dot(a.A + (long)s * d * d, th, d, row0, q);
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < RPW; ++k)
        if (row0 + k < d) part += (0.5 * q[k] - a.b[(long)s * d + row0 + k]) * th[row0 + k];
  }
  if (lane == 0) wsum[w] = part;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < NT / 64; ++k) t += wsum[k];
    a.rbuf[s * rstride(d) + obj_off(d) + blockIdx.x] = t;
  }
}

// dual update (non-hub workers) and the objective term of every element, one block row of B elements
// per workgroup; per-row partials into the worker's r-buffer (sb_local_obj sums them in row order)
__global__ void __launch_bounds__(symv::B) sb_post(StarBigArgs a) {
  __shared__ double wpart[symv::B / 64];
  if (a.ctl->done) return;
  const int s = blockIdx.y, t = blockIdx.x, k = threadIdx.x, j = t * symv::B + k;
  const long d = a.d;
  const bool hub = s == a.hub_li;
  const double c = hub ? (double)(a.n_total - 1) * a.rho : a.rho;
  double* r = a.rbuf + s * rstride(a.d);
  double part = 0.0;
  if (j < d) {
    const double th = a.theta[s * d + j];
    if (!hub) a.lam[s * d + j] += a.rho * (th - a.th_hub[j]);
    if (a.obj_mode != 0) part = (0.5 * (r[j] - c * th) - a.b[s * d + j]) * th;
  }
  part = wave_sum_f64(part);
  if ((k & 63) == 0) wpart[k >> 6] = part;
  __syncthreads();
  if (k == 0) r[fz_off(a.d) + t] = wpart[0] + wpart[1];
}

// the local objectives (fixed order: strided per thread, then the block reduction) and this rank's
// per-global-worker objective slots
__global__ void __launch_bounds__(256) sb_local_obj(StarBigArgs a) {
  __shared__ double scratch[16];
  if (a.ctl->done) return;
  const int nbr = symv::nblk(a.d), nblk = (a.d + ROWS_PER_WG - 1) / ROWS_PER_WG;
  for (int s = 0; s < a.n_local; ++s) {
    const double* r = a.rbuf + s * rstride(a.d);
    double t = 0.0;
    if (a.obj_mode != 0) {
      for (int k = threadIdx.x; k < nbr; k += blockDim.x) t += r[fz_off(a.d) + k];
    } else {  // sb_obj's per-workgroup partials
      for (int k = threadIdx.x; k < nblk; k += blockDim.x) t += r[obj_off(a.d) + k];
    }
    const double f = block_sum_f64(t, scratch);
    if (threadIdx.x == 0) a.objw[s] = f + 0.5 * a.yy[s];
    __syncthreads();  // scratch is reused by the next worker
  }
  for (int g = threadIdx.x; g < a.n_total; g += blockDim.x) a.objp[g] = 0.0;
  __syncthreads();
  for (int s = threadIdx.x; s < a.n_local; s += blockDim.x) a.objp[a.gid[s]] = a.objw[s];
}

__global__ void sb_finish(StarBigArgs a) {
  if (threadIdx.x != 0) return;
  ChainCtl* ctl = a.ctl;
  if (ctl->done) return;
  const int it = ctl->iter;
  double obj = 0.0;
  for (int g = 0; g < a.n_total; ++g) obj += a.objp[g];  // worker order
  if (it - 1 < a.max_iter) {
    a.trace[it - 1] = obj;
    a.tstamp[it - 1] = (long long)__builtin_amdgcn_s_memrealtime();
  }
  int code = 0;
  if (!(obj == obj) || isinf(obj)) code = 3;
  else if (fabs(obj - a.obj0) < a.tol) code = 1;
  else if (it >= a.max_iter) code = 2;
  if (code) {
    ctl->done = code;
    ctl->conv_iter = it;
  }
  ctl->iter = it + 1;
}

}  // namespace

extern "C" {

int gadmm_star_big_abi_layout(long long* out, int n) {
  long long v[] = {(long long)sizeof(StarBigArgs), (long long)offsetof(StarBigArgs, rho),
                   (long long)offsetof(StarBigArgs, Minv), (long long)offsetof(StarBigArgs, ctl),
                   (long long)offsetof(StarBigArgs, tstamp), (long long)offsetof(StarBigArgs, gid)};
  const int k = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < n && i < k; ++i) out[i] = v[i];
  return k;
}

long gadmm_star_big_rstride(int d) { return rstride(d); }

static bool sb_ok(const StarBigArgs& a) {
  return a.d >= 1 && a.n_local >= 1 && a.n_total >= a.n_local && a.hub_li < a.n_local && a.Minv && a.b && a.yy &&
         a.theta && a.lam && a.th_hub && a.agg && a.rbuf && a.objw && a.objp && a.trace && a.ctl && a.tstamp && a.gid &&
         (a.obj_mode != 0 || a.A) && a.max_iter >= 1;
}

// Stage 1 of an iteration: the non-hub workers' solves and this rank's [sum lam, sum theta].
int gadmm_star_big_workers(const StarBigArgs* args, hipStream_t st) {
  const StarBigArgs& a = *args;
  if (!sb_ok(a)) {
    gadmm_set_error("star_big: bad arguments");
    return -1;
  }
  const int d = a.d, nb = (d + NT - 1) / NT, nblk = (d + ROWS_PER_WG - 1) / ROWS_PER_WG;
  (void)nblk;
  hipLaunchKernelGGL(sb_rhs, dim3(nb, a.n_local), dim3(NT), 0, st, a);
  hipLaunchKernelGGL(sb_sym_part, dim3((unsigned)symv::nstored(d), a.n_local), dim3(symv::NT), 0, st, a, 0);
  hipLaunchKernelGGL(sb_sym_reduce, dim3(symv::nblk(d), a.n_local), dim3(symv::RNT), 0, st, a, 0);
  hipLaunchKernelGGL(sb_sum, dim3(nb), dim3(NT), 0, st, a);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// Stage 2 (after the reduce of agg to the hub rank): the hub's solve (no-op off the hub rank).
int gadmm_star_big_hub(const StarBigArgs* args, hipStream_t st) {
  const StarBigArgs& a = *args;
  if (a.hub_li < 0) return 0;
  const int d = a.d, nb = (d + NT - 1) / NT, nblk = (d + ROWS_PER_WG - 1) / ROWS_PER_WG;
  (void)nblk;
  hipLaunchKernelGGL(sb_hubrhs, dim3(nb), dim3(NT), 0, st, a);
  hipLaunchKernelGGL(sb_sym_part, dim3((unsigned)symv::nstored(d), a.n_local), dim3(symv::NT), 0, st, a, 1);
  hipLaunchKernelGGL(sb_sym_reduce, dim3(symv::nblk(d), a.n_local), dim3(symv::RNT), 0, st, a, 1);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// Stage 3 (after the broadcast of th_hub): duals, objectives, this rank's objective into objp.
int gadmm_star_big_post(const StarBigArgs* args, hipStream_t st) {
  const StarBigArgs& a = *args;
  const int d = a.d, nblk = (d + ROWS_PER_WG - 1) / ROWS_PER_WG;
  if (a.obj_mode == 0) hipLaunchKernelGGL(sb_obj, dim3(nblk, a.n_local), dim3(NT), 0, st, a);
  hipLaunchKernelGGL(sb_post, dim3(symv::nblk(d), a.n_local), dim3(symv::B), 0, st, a);
  hipLaunchKernelGGL(sb_local_obj, dim3(1), dim3(256), 0, st, a);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// Stage 4 (after the allreduce of objp): trace, stop rule, iteration counter.
int gadmm_star_big_finish(const StarBigArgs* args, hipStream_t st) {
  hipLaunchKernelGGL(sb_finish, dim3(1), dim3(64), 0, st, *args);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"
