// Persistent single-launch logistic GADMM with the reference's inexact local solver (inner GD,
// logReg_GD.m; group_ADMM_logistic_GD.m): the whole solve in ONE kernel per GPU, BASELINE configs[2].
//
// The graph engine runs a logistic iteration as two phase kernels (heads, tails), each one wave per
// worker that loads its shard into VGPRs, runs <= max_inner GD steps and exits (chain_small.hip:
// chain_phase_logistic_quad). Here every worker is ONE resident wave for the entire solve: the shard
// X (margins) and X^T (gradient) stay in VGPRs in the split-column quad layout (quad_gemv.h), and
// the per-phase costs of the graph path -- a kernel boundary, the shard reload, the phase ticket --
// become a neighbour wait on tagged theta granules. The hand-off / stop protocol is the linear
// per-worker kernel's (chain_persistent.hip): data-is-flag 16-byte granules, the monitor workgroup
// sums f_n in worker order and posts the decision of iteration i; a worker starts iteration i only
// after the decision of i - lag, so every worker (on every GPU) leaves at the same boundary.
//
// Per iteration i (group_ADMM_logistic_GD.m:15-103, logReg_GD.m:3-25), worker n with chain
// neighbours l, r:
//   head:  wait tails' theta^{i-1}; lazy dual mu -= rho (th_l - th), mu += rho (th - th_r) (the
//          reference's end-of-iteration dual, applied once the tails are known); GD from th^{i-1}
//   tail:  wait heads' theta^i; GD; dual update with the fresh heads
//   GD:    shift s = mu + rho (x0 - th_l) + rho (x0 - th_r) frozen; x <- x - step (-X^T (y / (1 +
//          e^{y X x})) + lam x + s) until every |dx| < inner_tol or max_inner steps
//   f_n = lam/2 |x|^2 + sum_i log(1 + e^{-y_i x_i^T x}) -> monitor
// Arithmetic identical to chain_phase_logistic_quad (same GEMVs, same order), so the objective trace
// is bit-identical to the graph engine's.
// Single GPU: agent-scope granules; several GPUs (xGMI fabric): system scope, boundary theta also
// pushed into the neighbour GPU's table. Every spin has a deadline (done = 4).
#include "gadmm_common.h"
#include "gadmm_chain.h"
#include "persist_device.h"
#include "chain_device.h"
#include "fast_sigm.h"
#include <cstddef>
#include <stdlib.h>

struct LogiArgs {
  const double* X;  // [n_local][m][d]
  const double* Y;  // [n_local][m]
  int m, max_inner;
  double lam, step, inner_tol;
  int* inner_iters;  // [n_local] optional: GD steps of the worker's last local solve
  double* scratch;   // Newton pipeline only (chain_persistent_newton.hip): per-worker refresh images
};

template <int T, bool SYS>
__global__ void __launch_bounds__(64) chain_persistent_logistic_kernel(PersistArgs a, LogiArgs g) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int d = a.d, n = a.n, m = g.m;
  const int lane = threadIdx.x, qi = lane & 15, qc = lane >> 4;
  const __amdgpu_buffer_rsrc_t rth = rsrc_of(a.thg);
  const __amdgpu_buffer_rsrc_t rob = rsrc_of(a.objg);
  const unsigned long long deadline = now_ticks() + (unsigned long long)a.timeout_ticks;
  __shared__ int xcd_lds;
  const bool packed = !SYS && a.xcd > 0;   // XCD packing (PersistArgs::xcd)
  if (packed && (blockIdx.x & 7u)) return;  // a spacer block: only b % 8 == 0 work (one XCD)
  const int bid = packed ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  bool local = false;  // publish with plain stores (every block verified on this XCD)
  if (!SYS && a.xcd > 1) local = xcd_verdict(a.xchk, bid, a.n_local + (a.has_monitor ? 1 : 0), deadline, &xcd_lds, (unsigned)a.xtag);
  if (!SYS && bid == 0 && threadIdx.x == 0) a.ctl->placed = a.xcd > 0 ? (local ? 2 : 1) : 0;

  if (a.has_monitor && bid == a.n_local) {
    // ---------------------------------------------------------------- monitor (one wave)
    double* vals = lds;  // [n]
    for (int it = a.start_iter;; ++it) {
      const unsigned tag = make_tag(a.epoch, it);
      const int slot = it % a.ring;
      bool okall = true;
      for (int w = lane; w < n; w += 64) {
        double v = 0.0;
        for (int spin = 0;; ++spin) {
          if (load_granule<SYS>(rob, (slot * n + w) * 16, tag, &v)) break;
          if ((spin & 7) == 7 && now_ticks() > deadline) {
            okall = false;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        vals[w] = v;
      }
      const bool ok = __all(okall);
      unsigned code = 0;
      if (lane == 0) {
        if (!ok) {
          code = 4;
        } else {
          double s = 0.0;
          for (int w = 0; w < n; ++w) s += vals[w];  // worker order, == the graph engine's finish
          if (it - 1 < a.max_iter) a.trace[it - 1] = s;
          if (!(s == s) || isinf(s)) code = 3;
          else if (fabs(s - a.obj0) < a.tol) code = 1;
          else if (it >= a.max_iter) code = 2;
          if (a.tstamp && it - 1 < a.max_iter) a.tstamp[it - 1] = (long long)now_ticks();
        }
        const unsigned long long dv = ((unsigned long long)tag << 32) | code;
        for (int r = 0; r < a.nranks; ++r) store_dec<SYS>(a.dec_push[r] + slot, dv);
      }
      if (__shfl((int)code, 0, 64)) return;
    }
  }

  // ------------------------------------------------------------------ worker (one wave)
  const PhaseSlot sl = a.slots[bid];
  const int li = sl.li, w = sl.gid, left = sl.left, right = sl.right;
  const bool head = (a.pos[bid] % 2) == 0;
  const double rho = a.rho, lam = g.lam, step = g.step;
  double* st = lds;  // QSTAGE doubles: quad GEMV staging
  u32x4* const p0 = a.push ? a.push[2 * bid] : nullptr;
  u32x4* const p1 = a.push ? a.push[2 * bid + 1] : nullptr;
  const __amdgpu_buffer_rsrc_t rp0 = rsrc_of(p0 ? (const void*)p0 : (const void*)a.thg);
  const __amdgpu_buffer_rsrc_t rp1 = rsrc_of(p1 ? (const void*)p1 : (const void*)a.thg);
  const double* Xg = g.X + (long)li * m * d;
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
  const double yv = ini ? g.Y[(long)li * m + lane] : 0.0;
  double th = inj ? a.theta[(long)w * d + lane] : 0.0;  // theta_n^{i-1}
  double mu = inj ? a.mu[(long)li * d + lane] : 0.0;
  double tl = (inj && left >= 0) ? a.theta[(long)left * d + lane] : 0.0;
  double tr = (inj && right >= 0) ? a.theta[(long)right * d + lane] : 0.0;
  int pending = a.pending_in;
  int stop_code = 0, stop_iter = 0, abort = 0, used = 0;

  int it = a.start_iter;
  for (;; ++it) {
    if (it > a.max_iter + a.lag) break;
    // -- neighbours' theta (heads: tails' theta^{it-1}; tails: heads' theta^it) and the decision of
    // it - lag, polled in one loop
    const bool check = it - a.start_iter >= a.lag;
    const int jdec = it - a.lag;
    const bool need_nb = head ? it > a.start_iter : true;
    const int jnb = head ? it - 1 : it;
    const unsigned tnb = make_tag(a.epoch, jnb), tj = make_tag(a.epoch, jdec);
    const int ra = need_nb ? left : -1, rb = need_nb ? right : -1;
    bool decided = !check;
    unsigned long long dv = 0;
    int outcome = 0;  // 1 go, 2 stop, 3 timeout
    for (int spin = 0;; ++spin) {
      bool nb = true;
      if (inj) {
        if (ra >= 0) nb &= load_granule<SYS>(rth, (ra * d + lane) * 16, tnb, &tl);
        if (rb >= 0) nb &= load_granule<SYS>(rth, (rb * d + lane) * 16, tnb, &tr);
      }
      if (!decided) {
        dv = __shfl(load_dec<SYS>(&a.decg[jdec % a.ring]), 0, 64);
        decided = (unsigned)(dv >> 32) == tj;
      }
      if (decided && (unsigned)(dv & 0xffffffffu) != 0u) { outcome = 2; break; }
      if (decided && __all(nb)) { outcome = 1; break; }
      if ((spin & 7) == 7 && now_ticks() > deadline) { outcome = 3; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (outcome != 1) {
      if (outcome == 2) {
        stop_code = (int)(unsigned)(dv & 0xffffffffu);
        stop_iter = jdec;
      } else {
        abort = 1;
      }
      break;
    }
    // -- lazy dual (heads), frozen proximal shift, inner GD (logReg_GD.m)
    double sh = 0.0, x = 0.0;
    if (inj) {
      double mm = mu;
      if (head && pending) {
        if (left >= 0) mm = mm - rho * (tl - th);
        if (right >= 0) mm = mm + rho * (th - tr);
        mu = mm;
      }
      double s = mm;  // -C1 + C2 (edge form) == mu
      if (left >= 0) s = s + rho * (th - tl);
      if (right >= 0) s = s + rho * (th - tr);
      sh = s;
      x = th;
    }
    used = 0;
    for (int k = 0; k < g.max_inner; ++k) {
      const double z = quad_gemv<T>(Xq, x, st);                 // margins z_i = X[i,:] x
      const double sv = ini ? yv / (1.0 + exp(yv * z)) : 0.0;  // y_i / (1 + e^{y_i z_i})
      const double gx = quad_gemv<T>(XTq, sv, st);             // (X^T s)_j
      bool conv = true;
      if (inj) {
        const double gr = -gx + lam * x + sh;
        const double xn = x - step * gr;
        conv = fabs(xn - x) < g.inner_tol;
        x = xn;
      }
      used = k + 1;
      if (__all(conv)) break;
    }
    // -- publish theta^it: own table + the remote neighbours' tables
    const unsigned tag = make_tag(a.epoch, it);
    if (inj) {
      put_granule<SYS>(local, rth, (w * d + lane) * 16, tag, x);
      if (p0) store_granule<SYS>(rp0, (w * d + lane) * 16, tag, x);
      if (p1) store_granule<SYS>(rp1, (w * d + lane) * 16, tag, x);
    }
    if (!head) {  // tails: both neighbours are this iteration's heads -> dual update now
      double rp = 0.0;
      if (inj) {
        double mm = mu;
        if (left >= 0) mm = mm - rho * (tl - x);
        if (right >= 0) mm = mm + rho * (x - tr);
        mu = mm;
        if (left >= 0) rp = fma(tl - x, tl - x, rp);  // K4 primal residual of the two edges
        if (right >= 0) rp = fma(x - tr, x - tr, rp);
      }
      if (a.rres) {
        const double rs = wave_sum_f64(rp);
        if (lane == 0 && it - 1 < a.max_iter) a.rres[(long)(it - 1) * n + w] = rs;
      }
    } else {
      pending = 1;
    }
    th = x;
    // -- f_n(theta^it) = lam/2 |x|^2 + sum softplus(-y z) at the new iterate -> monitor
    const double z = quad_gemv<T>(Xq, x, st);
    const double part = wave_sum_f64(ini ? softplus(-yv * z) : 0.0);
    const double xx = wave_sum_f64(inj ? x * x : 0.0);
    if (lane == 0) put_granule<SYS>(local, rob, ((it % a.ring) * n + w) * 16, tag, lam * 0.5 * xx + part);
  }
  // final state (plain stores; visible to the host after the kernel)
  if (inj) {
    a.theta[(long)w * d + lane] = th;
    a.mu[(long)li * d + lane] = mu;
  }
  if (lane == 0) {
    if (g.inner_iters) g.inner_iters[li] = used;
    if (abort) {
      a.ctl->done = 4;
    } else if (bid == 0 && stop_code) {
      a.ctl->done = stop_code;
      a.ctl->conv_iter = stop_iter;
      a.ctl->iter = it;
      a.ctl->pending = 1;
      a.ctl->monitored = stop_iter;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// GADMM_LOGISTIC_ZREC=1: the inner GD with the margins carried by a recursion on a SECOND wave. A step
//   z = X x,  s = y / (1 + e^{y z}),  x' = x - step (-X^T s + lam x + sh)
// has two dependent GEMVs. Since z' = X x' = z - step (-K s + lam z + c) with K = X X^T (m x m, built
// once per launch by GEMVs of the register X) and c = X sh (per local solve), the next margins need
// only s: wave 1 ("margins") runs s_k -> K s_k -> z_{k+1} -> s_{k+1} while wave 0 ("iterate") takes
// s_k -> X^T s_k -> x_{k+1} and the break test, so each step's dependent chain holds ONE GEMV. s_k
// goes wave 1 -> wave 0 through a 4-slot LDS ring with release / acquire flags (solve id * 1024 + k);
// wave 1 runs ahead and stops when wave 0 posts the solve's end; every solve restarts the recursion
// from z_0 = X x_0 exactly (no drift across solves). The iterate update, break rule, objective and
// hand-offs are the one-wave kernel's; only s_k differs in rounding (z from the recursion), so traces
// match the other engines to ~1e-13 instead of bit for bit.
constexpr int ZR_NT = 128;
constexpr int ZR_SLOTS = 64;  // s ring depth; the margins wave checks it every ZR_CHK steps
// (same-box A/B, E3 bench: 8/4 5.34, 16/4 5.34, 16/8 5.17, 32/8 5.11, 64/8 4.93 ms; 128/8 with an early-end
// check every 8 steps 5.41, 32/16 with one every step 5.43: profiles/r06_logistic)
constexpr int ZR_CHK = 8;

__device__ __forceinline__ int zr_load_acq(const int* p) {
  const int v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  return v;
}
__device__ __forceinline__ void zr_store_rel(int* p, int v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The per-step ring posts (s produced, s consumed) without the release fence: a wave's LDS operations
// are performed in order, so the flag cannot become visible before the slot data written (or read)
// before it; the fence only held the flag back by one LDS round trip on the margins wave's chain.
// GADMM_LOGISTIC_POSTFENCE=1 (PersistArgs::dbg bit 17) restores the fenced posts (A/B).
__device__ __forceinline__ void zr_post(int* p, int v, bool fenced) {
  if (fenced || !GADMM_LDS_IN_ORDER) {  // fence-free only where in-order LDS is documented
    zr_store_rel(p, v);
    return;
  }
  asm volatile("" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// s = y / (1 + e^{y z}) on the margins wave's critical path: inv1pexp_fast (fast_sigm.h). Measured 5.64 ->
// 5.21 ms on E3, one box (profiles/r05_j/r5jf); the default (GADMM_LOGISTIC_FASTSIGM=0: libm exp and
// the IEEE quotient). The traces stay within 1e-12 of torch.
__device__ __forceinline__ double zr_sigm(double yv, double z) { return yv * inv1pexp_fast(yv * z); }

template <int T, bool SYS>
__global__ void __launch_bounds__(ZR_NT) chain_persistent_logistic_zrec_kernel(PersistArgs a, LogiArgs g) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int d = a.d, n = a.n, m = g.m;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, qi = lane & 15, qc = lane >> 4;
  // worker LDS: [2][QSTAGE] per-wave GEMV staging | zc [2][64] (z_0, c) | s ring [8][4 QX] (each slot
  // in quad_gemv's x layout, read by the iterate wave's GEMV in place) | K [64][64] (row-major, built
  // once) | control ints
  double* st = lds + wv * QSTAGE;
  double* zc = lds + 2 * QSTAGE;
  double* sring = zc + 128;
  double* Kb = sring + ZR_SLOTS * 4 * QX;
  int* ctl = (int*)(Kb + 64 * 64);  // [0] start (solve id), [1] s produced, [2] s consumed, [3] solve end, [4] quit,
                                    // [5] c posted (solve id)
  const __amdgpu_buffer_rsrc_t rth = rsrc_of(a.thg);
  const __amdgpu_buffer_rsrc_t rob = rsrc_of(a.objg);
  const unsigned long long deadline = now_ticks() + (unsigned long long)a.timeout_ticks;
  __shared__ int xcd_lds;
  const bool packed = !SYS && a.xcd > 0;
  if (packed && (blockIdx.x & 7u)) return;
  const int bid = packed ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  bool local = false;
  if (!SYS && a.xcd > 1) local = xcd_verdict(a.xchk, bid, a.n_local + (a.has_monitor ? 1 : 0), deadline, &xcd_lds, (unsigned)a.xtag);
  if (!SYS && bid == 0 && threadIdx.x == 0) a.ctl->placed = a.xcd > 0 ? (local ? 2 : 1) : 0;

  if (a.has_monitor && bid == a.n_local) {
    if (wv != 0) return;  // the monitor is one wave (the one-wave kernel's code)
    double* vals = lds;
    for (int it = a.start_iter;; ++it) {
      const unsigned tag = make_tag(a.epoch, it);
      const int slot = it % a.ring;
      bool okall = true;
      for (int w = lane; w < n; w += 64) {
        double v = 0.0;
        for (int spin = 0;; ++spin) {
          if (load_granule<SYS>(rob, (slot * n + w) * 16, tag, &v)) break;
          if ((spin & 7) == 7 && now_ticks() > deadline) {
            okall = false;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        vals[w] = v;
      }
      const bool ok = __all(okall);
      unsigned code = 0;
      if (lane == 0) {
        if (!ok) {
          code = 4;
        } else {
          double sum = 0.0;
          for (int w = 0; w < n; ++w) sum += vals[w];
          if (it - 1 < a.max_iter) a.trace[it - 1] = sum;
          if (!(sum == sum) || isinf(sum)) code = 3;
          else if (fabs(sum - a.obj0) < a.tol) code = 1;
          else if (it >= a.max_iter) code = 2;
          if (a.tstamp && it - 1 < a.max_iter) a.tstamp[it - 1] = (long long)now_ticks();
        }
        const unsigned long long dv = ((unsigned long long)tag << 32) | code;
        for (int r = 0; r < a.nranks; ++r) store_dec<SYS>(a.dec_push[r] + slot, dv);
      }
      if (__shfl((int)code, 0, 64)) return;
    }
  }

  const PhaseSlot sl = a.slots[bid];
  const int li = sl.li, w = sl.gid, left = sl.left, right = sl.right;
  const bool head = (a.pos[bid] % 2) == 0;
  const double rho = a.rho, lam = g.lam, step = g.step;
  const double* Xg = g.X + (long)li * m * d;
  const bool inj = lane < d, ini = lane < m;
  const double yv = ini ? g.Y[(long)li * m + lane] : 0.0;
  const bool post_fence = (a.dbg & (1 << 17)) != 0;
  if (threadIdx.x < 8) ctl[threadIdx.x] = 0;
  __syncthreads();

  if (wv == 1) {
    // ---------------------------------------------------------------- margins wave
    const bool zr_fast = (a.dbg & 32) == 0;  // GADMM_LOGISTIC_FASTSIGM=0: libm exp and IEEE divide (A/B)
    int sid = 0;
    for (;;) {  // one local solve per start
      int s0 = 0;
      for (int spin = 0;; ++spin) {
        s0 = zr_load_acq(&ctl[0]);
        if (s0 > sid || zr_load_acq(&ctl[4])) break;
        if ((spin & 63) == 63 && now_ticks() > deadline) return;
        __builtin_amdgcn_s_sleep(1);
      }
      if (s0 <= sid) return;  // quit
      sid = s0;
      static_assert(T <= 16, "quad layout");
      double Kq[4][T];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < T; ++t) Kq[r][t] = Kb[(qi + 16 * r) * 64 + qc + 4 * t];  // built by wave 0 before start 1
      double z = zc[lane];
      double cc = 0.0;
      const double decay = 1.0 - step * lam;
      bool ended = false;
      for (int k = 0; k < g.max_inner && !ended; ++k) {
        const double sv = ini ? (zr_fast ? zr_sigm(yv, z) : yv / (1.0 + exp(yv * z))) : 0.0;
        // z' = (1 - step lam) z - step c + step (K s): the part without K s is formed while the GEMV runs
        double zpart = fma(decay, z, -step * cc);
        if (k >= ZR_SLOTS - ZR_CHK && k % ZR_CHK == 0) {
          // slots of steps k .. k + ZR_CHK - 1 are free once steps <= k + ZR_CHK - 1 - ZR_SLOTS were read;
          // the iterate wave's end of the solve also ends this run-ahead
          for (int spin = 0;; ++spin) {
            if (zr_load_acq(&ctl[3]) == sid) { ended = true; break; }
            if (zr_load_acq(&ctl[2]) >= sid * 1024 + k + ZR_CHK - ZR_SLOTS) break;
            if ((spin & 63) == 63 && now_ticks() > deadline) return;
          }
          if (ended) break;
        }
        double* slot = sring + (k % ZR_SLOTS) * 4 * QX;
        slot[(lane & 3) * QX + (lane >> 2)] = sv;  // quad_gemv's x layout: both waves' GEMVs read it in place
        zr_post(&ctl[1], sid * 1024 + k + 1, post_fence);
        const double u = quad_gemv_staged<T>(Kq, slot);  // (K s)_i
        if (k == 0) {  // c = X sh arrives after z_0 (the iterate wave posts z_0 first)
          for (int spin = 0;; ++spin) {
            if (zr_load_acq(&ctl[5]) == sid) break;
            if ((spin & 63) == 63 && now_ticks() > deadline) return;
          }
          cc = zc[64 + lane];
          zpart = fma(decay, z, -step * cc);
        }
        z = ini ? fma(step, u, zpart) : 0.0;
      }
    }
  }

  // ------------------------------------------------------------------ iterate wave (wave 0)
  u32x4* const p0 = a.push ? a.push[2 * bid] : nullptr;
  u32x4* const p1 = a.push ? a.push[2 * bid + 1] : nullptr;
  const __amdgpu_buffer_rsrc_t rp0 = rsrc_of(p0 ? (const void*)p0 : (const void*)a.thg);
  const __amdgpu_buffer_rsrc_t rp1 = rsrc_of(p1 ? (const void*)p1 : (const void*)a.thg);
  double Xq[4][T], XTq[4][T];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int row = qi + 16 * r, col = qc + 4 * t;
      Xq[r][t] = (row < m && col < d) ? Xg[(long)row * d + col] : 0.0;
      XTq[r][t] = (col < m && row < d) ? Xg[(long)col * d + row] : 0.0;
    }
  // K = X X^T, column j = X (row j of X): m GEMVs into the row-major LDS image the margins wave loads
  for (int j = 0; j < m; ++j) {
    const double xr = inj ? Xg[(long)j * d + lane] : 0.0;
    const double kc = quad_gemv<T>(Xq, xr, st);
    Kb[lane * 64 + j] = ini ? kc : 0.0;
  }
  for (int j = m; j < 64; ++j) Kb[lane * 64 + j] = 0.0;
  double th = inj ? a.theta[(long)w * d + lane] : 0.0;
  double mu = inj ? a.mu[(long)li * d + lane] : 0.0;
  double tl = (inj && left >= 0) ? a.theta[(long)left * d + lane] : 0.0;
  double tr = (inj && right >= 0) ? a.theta[(long)right * d + lane] : 0.0;
  int pending = a.pending_in;
  int stop_code = 0, stop_iter = 0, abort = 0, used = 0, sid = 0;

  int it = a.start_iter;
  for (;; ++it) {
    if (it > a.max_iter + a.lag) break;
    const bool check = it - a.start_iter >= a.lag;
    const int jdec = it - a.lag;
    const bool need_nb = head ? it > a.start_iter : true;
    const int jnb = head ? it - 1 : it;
    const unsigned tnb = make_tag(a.epoch, jnb), tj = make_tag(a.epoch, jdec);
    const int ra = need_nb ? left : -1, rb = need_nb ? right : -1;
    bool decided = !check;
    unsigned long long dv = 0;
    int outcome = 0;
    for (int spin = 0;; ++spin) {
      bool nb = true;
      if (inj) {
        if (ra >= 0) nb &= load_granule<SYS>(rth, (ra * d + lane) * 16, tnb, &tl);
        if (rb >= 0) nb &= load_granule<SYS>(rth, (rb * d + lane) * 16, tnb, &tr);
      }
      if (!decided) {
        dv = __shfl(load_dec<SYS>(&a.decg[jdec % a.ring]), 0, 64);
        decided = (unsigned)(dv >> 32) == tj;
      }
      if (decided && (unsigned)(dv & 0xffffffffu) != 0u) { outcome = 2; break; }
      if (decided && __all(nb)) { outcome = 1; break; }
      if ((spin & 7) == 7 && now_ticks() > deadline) { outcome = 3; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (outcome != 1) {
      if (outcome == 2) {
        stop_code = (int)(unsigned)(dv & 0xffffffffu);
        stop_iter = jdec;
      } else {
        abort = 1;
      }
      break;
    }
    double sh = 0.0, x = 0.0;
    if (inj) {
      double mm = mu;
      if (head && pending) {
        if (left >= 0) mm = mm - rho * (tl - th);
        if (right >= 0) mm = mm + rho * (th - tr);
        mu = mm;
      }
      double s = mm;
      if (left >= 0) s = s + rho * (th - tl);
      if (right >= 0) s = s + rho * (th - tr);
      sh = s;
      x = th;
    }
    // margins wave: z_0 = X x_0 and c = X sh, then go
    const double z0 = quad_gemv<T>(Xq, x, st);
    zc[lane] = ini ? z0 : 0.0;
    ++sid;
    zr_store_rel(&ctl[0], sid);  // the margins wave starts from z_0 ...
    const double c0 = quad_gemv<T>(Xq, sh, st);
    zc[64 + lane] = ini ? c0 : 0.0;
    zr_store_rel(&ctl[5], sid);  // ... and needs c only after its first K s
    used = 0;
    for (int k = 0; k < g.max_inner; ++k) {
      const int want = sid * 1024 + k + 1;
      bool got = false;
      for (int spin = 0;; ++spin) {
        if (zr_load_acq(&ctl[1]) >= want) { got = true; break; }
        if ((spin & 63) == 63 && now_ticks() > deadline) break;
      }
      if (!got) { abort = 1; break; }
      const double gx = quad_gemv_staged<T>(XTq, sring + (k % ZR_SLOTS) * 4 * QX);
      zr_post(&ctl[2], want, post_fence);  // (after this GEMV's reads of the slot, LDS in order)
      bool conv = true;
      if (inj) {
        const double gr = -gx + lam * x + sh;
        const double xn = x - step * gr;
        conv = fabs(xn - x) < g.inner_tol;
        x = xn;
      }
      used = k + 1;
      if (__all(conv)) break;
    }
    zr_store_rel(&ctl[3], sid);  // this solve is over: the margins wave stops its run-ahead
    if (abort) break;
    const unsigned tag = make_tag(a.epoch, it);
    if (inj) {
      put_granule<SYS>(local, rth, (w * d + lane) * 16, tag, x);
      if (p0) store_granule<SYS>(rp0, (w * d + lane) * 16, tag, x);
      if (p1) store_granule<SYS>(rp1, (w * d + lane) * 16, tag, x);
    }
    if (!head) {
      double rp = 0.0;
      if (inj) {
        double mm = mu;
        if (left >= 0) mm = mm - rho * (tl - x);
        if (right >= 0) mm = mm + rho * (x - tr);
        mu = mm;
        if (left >= 0) rp = fma(tl - x, tl - x, rp);
        if (right >= 0) rp = fma(x - tr, x - tr, rp);
      }
      if (a.rres) {
        const double rs = wave_sum_f64(rp);
        if (lane == 0 && it - 1 < a.max_iter) a.rres[(long)(it - 1) * n + w] = rs;
      }
    } else {
      pending = 1;
    }
    th = x;
    const double z = quad_gemv<T>(Xq, x, st);
    const double part = wave_sum_f64(ini ? softplus(-yv * z) : 0.0);
    const double xx = wave_sum_f64(inj ? x * x : 0.0);
    if (lane == 0) put_granule<SYS>(local, rob, ((it % a.ring) * n + w) * 16, tag, lam * 0.5 * xx + part);
  }
  zr_store_rel(&ctl[4], 1);  // the margins wave leaves
  if (inj) {
    a.theta[(long)w * d + lane] = th;
    a.mu[(long)li * d + lane] = mu;
  }
  if (lane == 0) {
    if (g.inner_iters) g.inner_iters[li] = used;
    if (abort) {
      a.ctl->done = 4;
    } else if (bid == 0 && stop_code) {
      a.ctl->done = stop_code;
      a.ctl->conv_iter = stop_iter;
      a.ctl->iter = it;
      a.ctl->pending = 1;
      a.ctl->monitored = stop_iter;
    }
  }
}

extern "C" long gadmm_resident_capacity(const void* fn, int threads, size_t shm);
extern "C" int gadmm_xcd_mode(const PersistArgs* a, int blocks, long cap_total);  // chain_persistent.hip
extern "C" unsigned gadmm_next_xtag();  // chain_persistent.hip

// (Round 5's four-wave sample-class split kernel, GADMM_LOGISTIC_SPLIT=1, was bit-identical but slower --
// 6.60 / 6.71 vs 6.37 / 6.39 ms, profiles/r05_c: the inner step is bound by its dependent chain, not FMA
// issue -- and was removed in round 6.)
// The margins recursion (two waves per worker) is the default: 6.3 -> 5.0-5.3 ms on E3 at the reference's
// 53 iterations (profiles/r05_j), 4.93 ms with the 64-slot ring (profiles/r06_logistic);
// GADMM_LOGISTIC_ZREC=0 selects the one-wave kernel, bit-identical to the graph engine.
static bool logi_zrec() {
  const char* e = getenv("GADMM_LOGISTIC_ZREC");
  return !(e && e[0] == '0');
}

static const void* logi_variant(const PersistArgs& a, const LogiArgs& g) {
  const int mx = a.d > g.m ? a.d : g.m;
  if (mx > 64 || a.n_epochs > 0) return nullptr;
  if (logi_zrec()) {
    if (a.sys_scope) {
      if (mx <= 52) return (const void*)chain_persistent_logistic_zrec_kernel<13, true>;
      return (const void*)chain_persistent_logistic_zrec_kernel<16, true>;
    }
    if (mx <= 52) return (const void*)chain_persistent_logistic_zrec_kernel<13, false>;
    return (const void*)chain_persistent_logistic_zrec_kernel<16, false>;
  }
  if (a.sys_scope) {
    if (mx <= 52) return (const void*)chain_persistent_logistic_kernel<13, true>;
    return (const void*)chain_persistent_logistic_kernel<16, true>;
  }
  if (mx <= 52) return (const void*)chain_persistent_logistic_kernel<13, false>;
  return (const void*)chain_persistent_logistic_kernel<16, false>;
}

static int logi_threads() { return logi_zrec() ? ZR_NT : 64; }

static size_t logi_shm(const PersistArgs& a) {
  const size_t mon = (size_t)a.n * 8;
  const size_t wk = logi_zrec() ? (size_t)(2 * QSTAGE + 128 + ZR_SLOTS * 4 * QX + 64 * 64) * 8 + 32
                                 : (size_t)QSTAGE * 8;
  return mon > wk ? mon : wk;
}

extern "C" {

int gadmm_logi_abi_layout(long long* out, int n) {
  long long v[] = {(long long)sizeof(LogiArgs), (long long)offsetof(LogiArgs, lam),
                   (long long)offsetof(LogiArgs, inner_iters)};
  const int k = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < n && i < k; ++i) out[i] = v[i];
  return k;
}

// Workgroups the logistic persistent kernel can keep resident (0: shape not eligible).
long gadmm_chain_persistent_logistic_capacity(const PersistArgs* args, const LogiArgs* g) {
  const void* fn = logi_variant(*args, *g);
  return fn ? gadmm_resident_capacity(fn, logi_threads(), logi_shm(*args)) : 0;
}

int gadmm_chain_persistent_logistic_launch(const PersistArgs* args, const LogiArgs* gargs, hipStream_t st) {
  const PersistArgs& a = *args;
  const LogiArgs& g = *gargs;
  const void* fn = logi_variant(a, g);
  if (!fn || !g.X || !g.Y || g.max_inner < 1 || a.ring <= a.lag + 1 || a.start_iter + a.max_iter + a.lag >= (1 << 20) ||
      (a.has_monitor && !a.dec_push)) {
    gadmm_set_error("persistent logistic kernel: unsupported configuration (d=%d m=%d)", a.d, g.m);
    return -1;
  }
  const size_t shm = logi_shm(a);
  const int blocks = a.n_local + (a.has_monitor ? 1 : 0);
  const long cap = gadmm_resident_capacity(fn, logi_threads(), shm);
  if (blocks > cap) {
    gadmm_set_error("persistent logistic kernel: %d workgroups but only %ld can be resident", blocks, cap);
    return -2;
  }
  if (shm > 65536) GADMM_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  PersistArgs ka = a;
  ka.xcd = gadmm_xcd_mode(&a, blocks, cap);
  ka.xtag = (int)gadmm_next_xtag();  // fresh placement-check tag: no memset of xchk
  const char* fs = getenv("GADMM_LOGISTIC_FASTSIGM");
  if (fs && fs[0] == '0') ka.dbg |= 32;
  const char* pf = getenv("GADMM_LOGISTIC_POSTFENCE");
  if (pf && pf[0] == '1') ka.dbg |= 1 << 17;
  void* kargs[] = {&ka, const_cast<LogiArgs*>(&g)};
  GADMM_CHECK(hipLaunchKernel(fn, dim3(ka.xcd > 0 ? 8 * blocks : blocks), dim3(logi_threads()), kargs, shm, st));
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"
