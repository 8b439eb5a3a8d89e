// Large-d (d > 256) phase of the chain engine: the 10M x 10k "LinearRegression_Real-shaped" config
// (BASELINE.json configs[4]). Per worker the cached inverse is 10k x 10k f64 = 800 MB, so one
// phase is an HBM-streaming GEMV over the whole chip, split into three launches:
//   chain_big_rhs   r_n = b_n - mu_n + rho th_l + rho th_r      (+ lazy head dual), one thread/elem
//   chain_big_sym_* th_n = (A_n + deg rho I)^{-1} r_n            the inverse stored as its block-packed
//                   lower triangle (sym_gemv.h: half the bytes of the full matrix), partials + reduce
//   [chain_big_obj] (A_n th_n)_i -> per-workgroup objective partials   (exact objective mode)
//                   (the reduce also applies the tail dual update and emits per-row objective /
//                   residual partials)
//   chain_big_post  per-worker sums of those partials, local objective, last-arriver iteration close
// Every load of the matrix is a contiguous 1-KiB wave access, every reduction has a fixed order
// (deterministic). r (80 KB) is re-read from L2 by every workgroup.
// Objective, exact mode: f = sum_i (1/2 (A th)_i - b_i) th_i + 1/2 y^T y with partials per workgroup
// summed in a fixed order; identity mode uses A th = r - deg rho th (no second 800 MB pass).
#include "gadmm_common.h"
#include "gadmm_chain.h"
#include "chain_device.h"
#include "big_gemv.h"

namespace {

using namespace biggemv;

struct SlotView {
  int li, gid, left, right, deg;
};

__device__ __forceinline__ SlotView slot_view(const PhaseArgs& a, int s) {
  const PhaseSlot sl = a.slots[s];
  SlotView v{sl.li, sl.gid, sl.left, sl.right, (sl.left >= 0) + (sl.right >= 0)};
  return v;
}

}  // namespace

__global__ void __launch_bounds__(NT) chain_big_rhs(PhaseArgs a) {
  if (a.ctl->done) return;
  const int pending = a.ctl->pending;
  const SlotView s = slot_view(a, blockIdx.y);
  const int j = blockIdx.x * NT + threadIdx.x;
  if (j >= a.d) return;
  const long d = a.d;
  const double* th = a.theta;
  const double tw = th[s.gid * d + j];
  const double tl = s.left >= 0 ? th[s.left * d + j] : 0.0;
  const double tr = s.right >= 0 ? th[s.right * d + j] : 0.0;
  double m = a.mu[s.li * d + j];
  if ((a.flags & PH_PRE_DUAL) && pending) {
    if (s.left >= 0) m = m - a.rho * (tl - tw);
    if (s.right >= 0) m = m + a.rho * (tw - tr);
    a.mu[s.li * d + j] = m;
  }
  double r = a.b[s.li * d + j] - m;
  if (s.left >= 0) r = r + a.rho * tl;
  if (s.right >= 0) r = r + a.rho * tr;
  a.rbuf[s.li * rstride(a.d) + j] = r;
}

// th_n = M r_n with M the block-packed lower triangle of (A_n + deg rho I)^{-1} (sym_gemv.h): partials
// of every stored block, then their fixed-order reduction straight into the theta table
__global__ void __launch_bounds__(symv::NT) chain_big_sym_part(PhaseArgs a) {
  __shared__ symv::dv2 tl[symv::NT / 64][64];
  if (a.ctl->done) return;
  const SlotView s = slot_view(a, blockIdx.y);
  const int d = a.d;
  const double* Mp = a.Minv + ((long)s.li * a.nvar + a.deg_to_var[s.deg]) * symv::packed_doubles(d);
  double* rb = a.rbuf + s.li * rstride(d);
  symv::part_block(Mp, rb, rb + part_off(d), symv::nblk(d), blockIdx.x, tl);
}

// th_n: the fixed-order reduction of the block partials straight into the theta table, fused with the
// elementwise tail of the phase -- the tails' dual update, the K4 primal residual and the identity-mode
// objective term of every element -- whose per-block-row partials chain_big_post sums in row order
__global__ void __launch_bounds__(symv::RNT) chain_big_sym_reduce(PhaseArgs a) {
  __shared__ double red[symv::RG][symv::B];
  __shared__ double wpart[2][2];
  if (a.ctl->done) return;
  const SlotView s = slot_view(a, blockIdx.y);
  const int d = a.d, t = blockIdx.x, k = threadIdx.x, j = t * symv::B + k;
  const int lane = k & 63, w = k >> 6;
  double* rb = a.rbuf + s.li * rstride(d);
  const double y = symv::reduce_row(rb + part_off(d), symv::nblk(d), t, red);
  double po = 0.0, pr = 0.0;
  if (k < symv::B && j < d) {
    const long dl = d;
    const double* th = a.theta;
    a.theta[s.gid * dl + j] = y;
    if (a.flags & PH_POST_DUAL) {
      const double tl = s.left >= 0 ? th[s.left * dl + j] : 0.0;
      const double tr = s.right >= 0 ? th[s.right * dl + j] : 0.0;
      double m = a.mu[s.li * dl + j];
      if (s.left >= 0) m = m - a.rho * (tl - y);
      if (s.right >= 0) m = m + a.rho * (y - tr);
      a.mu[s.li * dl + j] = m;
      if (s.left >= 0) pr = fma(tl - y, tl - y, pr);
      if (s.right >= 0) pr = fma(y - tr, y - tr, pr);
    }
    if (a.obj_mode != 0) po = (0.5 * (rb[j] - s.deg * a.rho * y) - a.b[s.li * dl + j]) * y;
  }
  if (w < 2) {  // the B = 2 waves that own elements (wave-uniform)
    po = wave_sum_f64(po);
    pr = wave_sum_f64(pr);
    if (lane == 0) {
      wpart[w][0] = po;
      wpart[w][1] = pr;
    }
  }
  __syncthreads();
  if (k == 0) {
    rb[fz_off(d) + t] = wpart[0][0] + wpart[1][0];
    rb[fz_off(d) + symv::nblk(d) + t] = wpart[0][1] + wpart[1][1];
  }
}

// exact objective: per-workgroup partial of sum_i (1/2 (A th)_i - b_i) th_i
__global__ void __launch_bounds__(NT) chain_big_obj(PhaseArgs a) {
  __shared__ double wsum[NT / 64];
  if (a.ctl->done) return;
  const SlotView s = slot_view(a, blockIdx.y);
  const int d = a.d;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row0 = blockIdx.x * ROWS_PER_WG + w * RPW;
  const double* th = a.theta + (long)s.gid * d;
  double part = 0.0;
  if (row0 < d) {
    double q[RPW];
    wave_rows_dot(a.A + (long)s.li * d * d, th, d, row0, q);
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < RPW; ++k)
        if (row0 + k < d) part += (0.5 * q[k] - a.b[(long)s.li * d + row0 + k]) * th[row0 + k];
  }
  if (lane == 0) wsum[w] = part;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int k = 0; k < NT / 64; ++k) t += wsum[k];
    a.rbuf[s.li * rstride(d) + obj_off(d) + blockIdx.x] = t;
  }
}

// the phase's per-worker sums (fixed order: strided per thread, then the block reduction), the local
// objective, and the last arriver's iteration close
__global__ void __launch_bounds__(256) chain_big_post(PhaseArgs a) {
  __shared__ double scratch[16];
  __shared__ int flag_lds;
  if (a.ctl->done) return;
  const int it = a.ctl->iter;
  const SlotView s = slot_view(a, blockIdx.x);
  const double* r = a.rbuf + s.li * rstride(a.d);
  const int nbr = symv::nblk(a.d);
  if (a.rres && (a.flags & PH_POST_DUAL)) {  // K4 primal residual of the tail's two edges
    double t = 0.0;
    for (int k = threadIdx.x; k < nbr; k += blockDim.x) t += r[fz_off(a.d) + nbr + k];
    const double rs = block_sum_f64(t, scratch);
    if (threadIdx.x == 0 && it - 1 < a.max_iter) a.rres[(long)(it - 1) * a.n_total + s.gid] = rs;
    __syncthreads();  // scratch is reused below
  }
  double t = 0.0;
  if (a.obj_mode != 0) {
    for (int k = threadIdx.x; k < nbr; k += blockDim.x) t += r[fz_off(a.d) + k];
  } else {  // chain_big_obj's per-workgroup partials
    const int nblk = (a.d + ROWS_PER_WG - 1) / ROWS_PER_WG;
    for (int k = threadIdx.x; k < nblk; k += blockDim.x) t += r[obj_off(a.d) + k];
  }
  const double f = block_sum_f64(t, scratch);
  if (threadIdx.x == 0) a.objw[s.li] = f + 0.5 * a.yy[s.li];
  if (a.flags & PH_FINISH) {
    if (phase_arrive(a.ctl, a.n_slots, &flag_lds)) finish_iteration(a, it);
  }
}

// full [count][d][d] -> block-packed lower triangles [count][packed_doubles(d)]; the diagonal blocks'
// upper halves are mirrored from their lower halves (the stored matrix is exactly symmetric), padding 0
__global__ void __launch_bounds__(256) sym_pack_kernel(const double* __restrict__ full, double* __restrict__ packed,
                                                       int d) {
  int I, J;
  symv::block_ij(blockIdx.x, I, J);
  const long m = blockIdx.y;
  const double* F = full + m * (long)d * d;
  double* out = packed + m * symv::packed_doubles(d) + (long)blockIdx.x * symv::B * symv::B;
  for (int e = threadIdx.x; e < symv::B * symv::B; e += blockDim.x) {
    const int rr = e / symv::B, cc = e % symv::B;
    int row = I * symv::B + rr, col = J * symv::B + cc;
    if (I == J && cc > rr) {  // upper half of a diagonal block: its mirror
      const int t = row;
      row = col;
      col = t;
    }
    out[e] = (row < d && col < d) ? F[(long)row * d + col] : 0.0;
  }
}

extern "C" {

// Pack `count` full symmetric d x d matrices into the block-packed lower-triangle layout of sym_gemv.h.
int gadmm_sym_pack_f64(const double* full, double* packed, int count, int d, hipStream_t st) {
  if (!full || !packed || count < 1 || d < 1) {
    gadmm_set_error("sym_pack: bad arguments");
    return -1;
  }
  hipLaunchKernelGGL(sym_pack_kernel, dim3((unsigned)symv::nstored(d), count), dim3(256), 0, st, full, packed, d);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

long gadmm_chain_big_rbuf_stride(int d) { return rstride(d); }

// doubles of one block-packed lower-triangle matrix (sym_gemv.h)
long gadmm_sym_packed_doubles(int d) { return symv::packed_doubles(d); }

int gadmm_chain_phase_big(const PhaseArgs* args, hipStream_t st) {
  const PhaseArgs& a = *args;
  if (a.n_slots <= 0) return 0;
  if (a.rbuf == nullptr) {
    gadmm_set_error("chain_phase_big: rbuf workspace missing");
    return -1;
  }
  const int d = a.d;
  hipLaunchKernelGGL(chain_big_rhs, dim3((d + NT - 1) / NT, a.n_slots), dim3(NT), 0, st, a);
  const int nblk = (d + ROWS_PER_WG - 1) / ROWS_PER_WG;
  hipLaunchKernelGGL(chain_big_sym_part, dim3((unsigned)symv::nstored(d), a.n_slots), dim3(symv::NT), 0, st, a);
  hipLaunchKernelGGL(chain_big_sym_reduce, dim3(symv::nblk(d), a.n_slots), dim3(symv::RNT), 0, st, a);
  if (a.obj_mode == 0 && (a.flags & PH_OBJ))
    hipLaunchKernelGGL(chain_big_obj, dim3(nblk, a.n_slots), dim3(NT), 0, st, a);
  hipLaunchKernelGGL(chain_big_post, dim3(a.n_slots), dim3(256), 0, st, a);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"
