// Persistent single-launch GADMM (linear, closed form): the whole solve in ONE kernel per GPU.
//
// Why: at the reference shapes (N = 24..50 workers, d = 50) an iteration is two dependent phases of
// ~1 us of arithmetic each; as separate launches every phase pays a kernel boundary and re-reads
// the worker's cached inverse and Gram from L2/MALL (profiles/r01_baseline_multikernel: 7.7 us per
// phase). Here each worker is one resident workgroup that keeps (A + c rho I)^{-1} and A in LDS for
// the entire solve; the only traffic per phase is the neighbours' theta (<= 2 x 400 B).
//
// Schedule == group_ADMM_closedForm.m / dynamic_group_ADMM_closedForm.m with a static chain:
//   head (even chain position) at iteration i: wait tails' theta^{i-1}; lazy dual update (the
//   reference's end-of-iteration dual, applied when both tails are known); solve; publish theta^i.
//   tail at iteration i: wait heads' theta^i; solve; publish theta^i; dual update.
//   every worker then publishes f_n(theta_n^i); the monitor workgroup sums them in worker order,
//   records the trace and posts the stop decision for iteration i (|obj - obj0| < tol).
//   A worker starts iteration i only after the decision of iteration i - LAG is known, so all
//   workers (on every GPU) leave at the same iteration boundary; the reported count is exact.
//
// Hand-offs use the data-is-flag granule form of cdna_hip_programming.md §6 Guideline 16 (R2): each
// double travels as one 16-byte {tag, lo, tag, hi} write-through store; the consumer re-reads its
// 16-byte granule until both tags equal the expected tag (a torn 16-B store is two 8-B halves, each
// carrying its own tag, so tearing is always detected). No flags, no fences, no counters.
// Single GPU: sc1 (agent) granules in hipMalloc memory. Multi-GPU (xgmi fabric): sc0|sc1 (system)
// granules in fine-grained uncached memory shared by IPC; remote stores travel over xGMI.
// Tags are salted with a per-solve epoch, so buffers need no re-zeroing between solves.
// Every spin is bounded by a wall-clock deadline (s_memrealtime); on timeout the kernel records
// done = 4 and every workgroup exits.
// One wave per worker, one hand-off wait per phase on the critical path: poll back to back (same-box
// A/B, profiles/r02_pollab: per-worker E1 3.065 -> 3.016 ms, D-GADMM 1.51 -> 1.48 ms; the blocked and
// star kernels keep the default pause, where polling back to back measured no gain)
#define GADMM_POLL_SLEEP 0
#include "gadmm_common.h"
#include "gadmm_chain.h"
#include "persist_device.h"
#include <stdlib.h>
#include <string.h>
#include <atomic>
#include <mutex>

namespace {

constexpr int NT = 256;
constexpr int NW = 4;

}  // namespace

// REG = true: d <= 64, ONE wave per worker that keeps its rows of (A + deg rho I)^{-1} and A in
// VGPRs (lane i holds row i): a phase's GEMV is 64 FMAs per lane with x broadcast from LDS, and no
// cross-wave reduction or barrier sits on the critical path (tools/persist_timeline.py measured
// ~0.9 us of LDS-GEMV + barriers per phase in the 4-wave LDS variant at d = 50).
// The register GEMV uses the split-column quad layout (quad_gemv.h, QT columns per lane, 7 LDS
// broadcasts per GEMV instead of 26), bit-identical to the LDS variants. NV = 2: D-GADMM in one
// launch with both degree variants of the inverse in registers (the degree changes on re-chain).
// REG = false: 4 waves, matrices in LDS (64 < d <= 128, or D-GADMM with three degree variants).
// TL: instrumented instantiation (s_memrealtime timeline); production instantiations have no stamps.
template <int NC, bool SYS, bool REG, int QT = 1, int NV = 1, bool TL = false>
__global__ void __launch_bounds__(REG ? 64 : NT) chain_persistent_kernel(PersistArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int abort_lds;
  __shared__ int stop_lds;
  const int d = a.d, n = a.n;
  const int lane = threadIdx.x & 63;
  const bool w0 = threadIdx.x < 64;  // wave 0 owns the worker state; waves 1..3 help in the GEMVs
  const __amdgpu_buffer_rsrc_t rth = rsrc_of(a.thg);
  // theta table rows (row_it / row_prev in the loop). D-GADMM: a ring of `ring` iteration slots, because at a
  // re-chain a head still reads its OLD tails' theta^{it-1} while those tails, no longer its
  // neighbours, may already run ahead (up to lag iterations: the stop rule bounds the skew) and
  // would overwrite a single slot. Static chains: one slot (a producer needs the consumer's next
  // theta before it can overwrite).
  const bool ring_tab = a.n_epochs > 0;
  const __amdgpu_buffer_rsrc_t rob = rsrc_of(a.objg);
  const unsigned long long deadline = now_ticks() + (unsigned long long)a.timeout_ticks;
  __shared__ int xcd_lds;
  const bool packed = !SYS && a.xcd > 0;   // XCD packing (PersistArgs::xcd)
  if (packed && (blockIdx.x & 7u)) return;  // a spacer block: only b % 8 == 0 work (one XCD)
  const int bid = packed ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  if (threadIdx.x == 0) {
    abort_lds = 0;
    stop_lds = 0;
  }
  lds_barrier();
  bool local = false;  // publish with plain stores (every block verified on this XCD)
  if (!SYS && a.xcd > 1) local = xcd_verdict(a.xchk, bid, a.n_local + (a.has_monitor ? 1 : 0), deadline, &xcd_lds, (unsigned)a.xtag);
  if (!SYS && bid == 0 && threadIdx.x == 0) a.ctl->placed = a.xcd > 0 ? (local ? 2 : 1) : 0;

  if (a.has_monitor && bid == a.n_local) {
    // ---------------------------------------------------------------- monitor workgroup
    double* vals = lds;  // [n]
    for (int it = a.start_iter;; ++it) {
      if (a.hard_stop > 0 && it > a.hard_stop) {  // chunk exhausted without a stop decision
        if (threadIdx.x == 0) a.ctl->done = 5;
        return;
      }
      const unsigned tag = make_tag(a.epoch, it);
      const int slot = it % a.ring;
      if (w0) {
        for (int w = lane; w < n; w += 64) {
          double v = 0.0;
          for (;;) {
            if (load_granule<SYS>(rob, (slot * n + w) * 16, tag, &v)) break;
            if (now_ticks() > deadline) {
              abort_lds = 1;
              break;
            }
            GADMM_POLL_PAUSE();
          }
          vals[w] = v;
        }
      }
      lds_barrier();
      if (threadIdx.x == 0) {
        unsigned code = 0;
        if (abort_lds) {
          code = 4;
        } else {
          double s = 0.0;
          for (int w = 0; w < n; ++w) s += vals[w];  // fixed order: deterministic, == multi-kernel path
          if (it - 1 < a.max_iter) a.trace[it - 1] = s;
          if (!(s == s) || isinf(s)) code = 3;
          else if (fabs(s - a.obj0) < a.tol) code = 1;
          else if (it >= a.max_iter) code = 2;
          if (a.tstamp && it - 1 < a.max_iter) a.tstamp[it - 1] = (long long)now_ticks();
        }
        const unsigned long long dv = ((unsigned long long)tag << 32) | code;
        for (int r = 0; r < a.nranks; ++r) store_dec<SYS>(a.dec_push[r] + slot, dv);
        if (code) {
          stop_lds = 1;
          if (a.hard_stop > 0) {  // chunked: the workers may stop at hard_stop before seeing this decision
            a.ctl->done = (int)code;
            a.ctl->conv_iter = it;
          }
        }
        const int k = it - a.start_iter;
        if (TL && k < a.timeline_iters) a.timeline[((long)bid * a.timeline_iters + k) * 8] = (long long)now_ticks();
      }
      lds_barrier();
      if (stop_lds) return;
    }
  }

  // ------------------------------------------------------------------ worker workgroup
  // Static chain: workgroup b runs slot b of the position-sorted plan. D-GADMM (n_epochs > 0, LDS
  // variant only): workgroup b is local worker b for the whole launch and takes its slot / position
  // of each epoch from ep_slots / ep_pos (chains pre-drawn by the seeded schedule on the host).
  const bool dyn = a.n_epochs > 0;
  PhaseSlot sl = dyn ? a.ep_slots[bid] : a.slots[bid];
  int pos = dyn ? a.ep_pos[bid] : a.pos[bid];
  const int li = sl.li, w = sl.gid;
  int left = sl.left, right = sl.right;
  bool head = (pos % 2) == 0;
  int deg = (left >= 0) + (right >= 0);
  const double rho = a.rho;
  double crho = deg * rho;
  int ep = 0;
  int next_start = (dyn && a.n_epochs > 1) ? a.epoch_start[1] : 0x7fffffff;
  // the next epoch's slot / position / start, loaded one epoch ahead: at coherence 1 a re-chain every
  // iteration would otherwise put three dependent global loads on the critical path
  PhaseSlot nsl = sl;
  int npos = pos, nnext = 0x7fffffff;
  if (dyn && a.n_epochs > 1) {
    nsl = a.ep_slots[(long)a.n_local + bid];
    npos = a.ep_pos[(long)a.n_local + bid];
    nnext = a.n_epochs > 2 ? a.epoch_start[2] : 0x7fffffff;
  }
  u32x4* const p0 = a.push ? a.push[2 * bid] : nullptr;
  u32x4* const p1 = a.push ? a.push[2 * bid + 1] : nullptr;
  const __amdgpu_buffer_rsrc_t rp0 = rsrc_of(p0 ? (const void*)p0 : (const void*)a.thg);
  const __amdgpu_buffer_rsrc_t rp1 = rsrc_of(p1 ? (const void*)p1 : (const void*)a.thg);

  const long msz = REG ? 0 : (long)d * d;
  const int nM = (dyn && !REG) ? a.nvar : 1;                   // inverses kept in LDS
  double* Mall = lds;                                          // [nM][d*d]
  double* Al = lds + nM * msz;                                 // d*d (obj_mode 0)
  double* xv = Al + (a.obj_mode == 0 ? msz : 0);               // [64*NC] rhs / theta staging
  double* red = xv + 64 * NC;                                  // [NW*NC*64]
  double* Ml = Mall + ((dyn && !REG) ? (long)a.deg_to_var[deg] * msz : 0);
  double* st = lds;                                            // REG: quad GEMV staging (QSTAGE doubles)
  int vsel = (dyn && REG) ? a.deg_to_var[deg] : 0;             // REG + D-GADMM: register variant in use

  const double* Mg = a.Minv + ((long)li * a.nvar + a.deg_to_var[deg]) * (long)d * d;
  const double* Ag = a.A + (long)li * d * d;
  // REG + D-GADMM (NV = 2): the objective's Gram in LDS (quad order, after the GEMV staging): it is
  // used off the critical path, and next to the two inverses in VGPRs it pushed them into AGPR moves
  // (coherence 1: 0.880 -> 0.840 ms; with one inverse, NV = 1, registers stay faster: 3.07 vs 3.14 ms)
  constexpr bool AQ_LDS = REG && NV > 1;
  double Mq[REG ? NV : 1][REG ? 4 : 1][REG ? QT : 1], Aq[REG && !AQ_LDS ? 4 : 1][REG && !AQ_LDS ? QT : 1];
  double* Aql = lds + QSTAGE;
  if constexpr (REG) {
    if (dyn) {
#pragma unroll
      for (int v = 0; v < NV; ++v)
        quad_load<QT>(Mq[v], a.Minv + ((long)li * a.nvar + (v < a.nvar ? v : 0)) * d * d, d, v < a.nvar);
    } else {
      quad_load<QT>(Mq[0], Mg, d, true);
    }
    if constexpr (AQ_LDS) quad_store_lds<QT>(Aql, Ag, d, a.obj_mode == 0);
    else quad_load<QT>(Aq, Ag, d, a.obj_mode == 0);
  } else {
    if (dyn) {
      const double* Mw = a.Minv + (long)li * a.nvar * d * d;
      for (long e = threadIdx.x; e < (long)a.nvar * d * d; e += NT) Mall[e] = Mw[e];
    } else {
      for (int e = threadIdx.x; e < d * d; e += NT) Ml[e] = Mg[e];
    }
    if (a.obj_mode == 0)
      for (int e = threadIdx.x; e < d * d; e += NT) Al[e] = Ag[e];
  }
  // worker state, meaningful in wave 0 (lane owns elements i = lane + 64c)
  double th[NC], mu[NC], bb[NC], tl[NC], tr[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = lane + 64 * c;
    const bool in = w0 && i < d;
    th[c] = in ? a.theta[(long)w * d + i] : 0.0;
    mu[c] = in ? a.mu[(long)li * d + i] : 0.0;
    bb[c] = in ? a.b[(long)li * d + i] : 0.0;
    tl[c] = (in && left >= 0) ? a.theta[(long)left * d + i] : 0.0;
    tr[c] = (in && right >= 0) ? a.theta[(long)right * d + i] : 0.0;
  }
  const double half_yy = 0.5 * a.yy[li];
  // a pending (lazy) dual is owed only by a worker that was a head in the last iteration run: in a
  // D-GADMM continuation epoch 0 is that iteration's chain, and a tail must not flush twice
  int pending = (a.pending_in && head) ? 1 : 0;
  int stop_code = 0, stop_iter = 0;
  lds_barrier();

  int it = a.start_iter;
  bool hard_stopped = false;
  // ring slots as counters (no integer division in the loop): rs = it % ring; the theta-table row of
  // worker x's theta^it is rs * n + x (D-GADMM ring) or x (static chains), theta^{it-1} uses rs_prev
  int rs = a.start_iter % a.ring;
  for (;; ++it, rs = rs + 1 == a.ring ? 0 : rs + 1) {
    const int rs_prev = rs == 0 ? a.ring - 1 : rs - 1;
    const int row_it = ring_tab ? rs * n : 0, row_prev = ring_tab ? rs_prev * n : 0;
    if (a.hard_stop > 0 && it > a.hard_stop) {  // end of this chunk's epochs: state = after hard_stop
      hard_stopped = true;
      break;
    }
    if (it > a.max_iter + a.lag) break;
    const long long t_start = TL ? (long long)now_ticks() : 0;
    if (dyn && it == next_start) {
      // re-chain (dynamic_group_ADMM_closedForm.m:18-21): a worker that was a head still owes the
      // previous iteration's dual, computed with its OLD neighbours' theta^{it-1} (every worker that
      // reached this iteration has published theta^{it-1}); then it takes its new slot.
      if (w0 && pending && (it > a.start_iter || a.cont)) {
        const unsigned tp = make_tag(a.epoch, it - 1);
        const int ok = wait_pair<NC, SYS>(rth, d, left >= 0 ? row_prev + left : -1, tp, tl,
                                          right >= 0 ? row_prev + right : -1, tp, tr, deadline);
        if (ok != 1 && lane == 0) abort_lds = 1;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          double m = mu[c];
          if (left >= 0) m = m - rho * (tl[c] - th[c]);
          if (right >= 0) m = m + rho * (th[c] - tr[c]);
          mu[c] = m;
        }
      }
      pending = 0;
      ++ep;
      sl = nsl;
      pos = npos;
      left = sl.left;
      right = sl.right;
      head = (pos % 2) == 0;
      deg = (left >= 0) + (right >= 0);
      crho = deg * rho;
      if constexpr (REG) vsel = a.deg_to_var[deg];
      else Ml = Mall + (long)a.deg_to_var[deg] * msz;
      next_start = nnext;
      if (ep + 1 < a.n_epochs) {  // prefetch the epoch after (consumed at the next re-chain)
        nsl = a.ep_slots[(long)(ep + 1) * a.n_local + bid];
        npos = a.ep_pos[(long)(ep + 1) * a.n_local + bid];
        nnext = ep + 2 < a.n_epochs ? a.epoch_start[ep + 2] : 0x7fffffff;
      }
    }
    long long t_ready = 0, t_pub = 0, t_bar = 0, t_gemv = 0;
    // -- stop rule: decision of iteration it - lag (all workers leave at the same boundary). Its
    // load is issued here and resolved after the neighbour wait, so its latency overlaps the wait;
    // nothing is committed before the barrier that publishes the decision.
    const bool check = it - a.start_iter >= a.lag;
    const int jdec = it - a.lag;

    // -- neighbours' theta, the stop decision, and the rhs (wave 0). The decision of iteration
    // it - lag is polled in the same loop as the neighbours' granules (one round trip for both);
    // a stop decision abandons the wait, since a neighbour that already saw it publishes no more.
    // Nothing is committed before the barrier that publishes the outcome.
    double mun[NC];
    double rv = 0.0;  // REG: this lane's rhs element (the quad GEMV's input)
    if (w0) {
      const bool need_nb = head ? (it > a.start_iter || a.cont) : true;
      const int jnb = head ? it - 1 : it;
      const unsigned tnb = make_tag(a.epoch, jnb);
      const int ra = need_nb ? left : -1, rb = need_nb ? right : -1;
      const int row_nb = head ? row_prev : row_it;  // table rows of theta^jnb
      int dslot = rs - a.lag;  // == jdec % ring
      if (dslot < 0) dslot += a.ring;
      const unsigned tj = make_tag(a.epoch, jdec);
      bool decided = !check;
      unsigned long long dv = 0;
      int outcome = 0;  // 1 go, 2 stop, 3 timeout
      for (int spin = 0;; ++spin) {
        bool nb = true;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int i = lane + 64 * c;
          if (i < d) {
            if (ra >= 0) nb &= load_granule<SYS>(rth, ((row_nb + ra) * d + i) * 16, tnb, &tl[c]);
            if (rb >= 0) nb &= load_granule<SYS>(rth, ((row_nb + rb) * d + i) * 16, tnb, &tr[c]);
          }
        }
        if (!decided) {
          dv = __shfl(load_dec<SYS>(&a.decg[dslot]), 0, 64);
          decided = (unsigned)(dv >> 32) == tj;
        }
        if (decided && (unsigned)(dv & 0xffffffffu) != 0u) { outcome = 2; break; }
        if (decided && __all(nb)) { outcome = 1; break; }
        if ((spin & 7) == 7 && now_ticks() > deadline) { outcome = 3; break; }
        GADMM_POLL_PAUSE();
      }
      if (lane == 0) {
        if (TL) t_ready = (long long)now_ticks();
        if (outcome == 3) abort_lds = 1;
        if (outcome == 2) {
          stop_lds = 1;
          stop_code = (int)(unsigned)(dv & 0xffffffffu);
          stop_iter = jdec;
        }
      }
      if (head) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {  // lazy end-of-iteration dual (reference order: -rho(th_l - th) then +rho(th - th_r))
          double m = mu[c];
          if (pending) {
            if (left >= 0) m = m - rho * (tl[c] - th[c]);
            if (right >= 0) m = m + rho * (th[c] - tr[c]);
          }
          mun[c] = m;
        }
      } else {
#pragma unroll
        for (int c = 0; c < NC; ++c) mun[c] = mu[c];
      }
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int i = lane + 64 * c;
        double r = bb[c] - mun[c];
        if (left >= 0) r = r + rho * tl[c];
        if (right >= 0) r = r + rho * tr[c];
        if constexpr (REG) rv = i < d ? r : 0.0;
        else if (i < d) xv[i] = r;
      }
    }
    lds_barrier();
    if (abort_lds || stop_lds) break;
    if (TL) t_bar = (long long)now_ticks();
    if (w0) {
#pragma unroll
      for (int c = 0; c < NC; ++c) mu[c] = mun[c];
    }

    // -- solve theta = (A + deg rho I)^{-1} r
    double tn[NC];
    if constexpr (REG) {
      if (NV > 1 && vsel == 1) tn[0] = quad_gemv<QT>(Mq[NV > 1 ? 1 : 0], rv, st);
      else tn[0] = quad_gemv<QT>(Mq[0], rv, st);
    } else {
      symv_lds<NC>(Ml, xv, tn, red, d);
    }
    if (TL) t_gemv = (long long)now_ticks();
    double part = 0.0;
    if (w0) {
      const unsigned tag = make_tag(a.epoch, it);
#pragma unroll
      for (int c = 0; c < NC; ++c) {  // publish theta^it: local table + remote neighbours' tables
        const int i = lane + 64 * c;
        if (i < d) {
          put_granule<SYS>(local, rth, ((row_it + w) * d + i) * 16, tag, tn[c]);
          if (p0) store_granule<SYS>(rp0, (w * d + i) * 16, tag, tn[c]);
          if (p1) store_granule<SYS>(rp1, (w * d + i) * 16, tag, tn[c]);
        }
      }
      if (SYS && dyn && a.ep_push) {
        // D-GADMM across GPUs: to the ranks of this epoch's neighbours, and of the next epoch's when
        // it starts at it + 1 (a new neighbour's head reads theta^it as its previous iterate)
        unsigned mask = a.ep_push[(long)ep * a.n_local + bid];
        if (it + 1 == next_start) mask |= a.ep_push[(long)(ep + 1) * a.n_local + bid];
        while (mask) {
          const int r = __builtin_ctz(mask);
          mask &= mask - 1u;
          const __amdgpu_buffer_rsrc_t rr = rsrc_of(a.peer_thg[r]);
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            const int i = lane + 64 * c;
            if (i < d) store_granule<SYS>(rr, ((row_it + w) * d + i) * 16, tag, tn[c]);
          }
        }
      }
      if (TL) t_pub = (long long)now_ticks();
      if (!head) {  // tails: both neighbours are this iteration's heads -> dual update now
        double rp = 0.0;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          double m = mu[c];
          if (left >= 0) m = m - rho * (tl[c] - tn[c]);
          if (right >= 0) m = m + rho * (tn[c] - tr[c]);
          mu[c] = m;
          if (a.rres && lane + 64 * c < d) {  // K4 primal residual of the tail's two edges
            if (left >= 0) rp = fma(tl[c] - tn[c], tl[c] - tn[c], rp);
            if (right >= 0) rp = fma(tn[c] - tr[c], tn[c] - tr[c], rp);
          }
        }
        if (a.rres) {
          const double rs = wave_sum_f64(rp);
          if (lane == 0 && it - 1 < a.max_iter) a.rres[(long)(it - 1) * n + w] = rs;
        }
      } else {
        pending = 1;
      }
      if (a.obj_mode != 0) {  // A th = r - deg rho th  (xv still holds r)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int i = lane + 64 * c;
          if (i < d) part += (0.5 * ((REG ? rv : xv[i]) - crho * tn[c]) - bb[c]) * tn[c];
        }
      }
    }
    if (a.obj_mode == 0) {  // exact: 1/2 th^T A th - b^T th + 1/2 y^T y
      lds_barrier();
      if (w0) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int i = lane + 64 * c;
          if (i < d) xv[i] = tn[c];
        }
      }
      lds_barrier();
      double q[NC];
      if constexpr (AQ_LDS) q[0] = quad_gemv_lds<QT>(Aql, lane < d ? tn[0] : 0.0, st);
      else if constexpr (REG) q[0] = quad_gemv<QT>(Aq, lane < d ? tn[0] : 0.0, st);
      else symv_lds<NC>(Al, xv, q, red, d);
      if (w0) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int i = lane + 64 * c;
          if (i < d) part += (0.5 * q[c] - bb[c]) * tn[c];
        }
      }
    }
    if (w0) {
      const double f = wave_sum_f64(part) + half_yy;
      if (lane == 0) put_granule<SYS>(local, rob, (rs * n + w) * 16, make_tag(a.epoch, it), f);
#pragma unroll
      for (int c = 0; c < NC; ++c) th[c] = tn[c];
      const int k = it - a.start_iter;
      if (TL && lane == 0 && k < a.timeline_iters) {
        long long* tl = a.timeline + ((long)bid * a.timeline_iters + k) * 8;
        tl[0] = t_start;
        tl[1] = t_ready;
        tl[2] = t_pub;
        tl[3] = (long long)now_ticks();
        tl[4] = t_bar;
        tl[5] = t_gemv;
      }
    }
    lds_barrier();
  }

  // write back the final state (plain stores; visible to the host after the kernel)
  if (w0) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      if (i < d) {
        a.theta[(long)w * d + i] = th[c];
        a.mu[(long)li * d + i] = mu[c];
      }
    }
  }
  if (threadIdx.x == 0) {
    if (abort_lds) {
      a.ctl->done = 4;
    } else if (bid == 0 && stop_code) {
      a.ctl->done = stop_code;
      a.ctl->conv_iter = stop_iter;
      a.ctl->iter = it;
      a.ctl->pending = 1;
      a.ctl->monitored = stop_iter;
    } else if (bid == 0 && hard_stopped) {  // done / conv_iter come from the monitor (rank 0)
      a.ctl->iter = it;
      a.ctl->pending = 1;
    }
  }
}

extern "C" {

// LDS bytes the persistent kernel needs; 0 if the shape is not eligible.
long gadmm_chain_persistent_lds_dyn(int d, int obj_mode, int n_inv) {
  if (d > 128) return 0;
  const int nc = (d + 63) / 64;
  long doubles = (long)(n_inv + (obj_mode == 0 ? 1 : 0)) * d * d + 64 * nc + NW * nc * 64 + NW + 16;
  long bytes = doubles * 8;
  if (bytes > 160 * 1024 - 64) return 0;
  return bytes;
}

long gadmm_chain_persistent_lds(int d, int obj_mode) {
  if (d > 128) return 0;
  const int nc = (d + 63) / 64;
  long doubles = (long)(obj_mode == 0 ? 2 : 1) * d * d + 64 * nc + NW * nc * 64 + NW + 16;
  long bytes = doubles * 8;
  if (bytes > 160 * 1024 - 64) return 0;
  return bytes;
}

}  // extern "C"

// The kernel variant the launcher runs for these arguments, its block size and dynamic LDS bytes.
struct PVariant {
  const void* fn = nullptr;
  int threads = 0;
  size_t shm = 0;
};

static PVariant pick_variant(const PersistArgs& a) {
  PVariant v;
  const bool dyn = a.n_epochs > 0;
  const long lds = dyn ? gadmm_chain_persistent_lds_dyn(a.d, a.obj_mode, a.nvar)
                       : gadmm_chain_persistent_lds(a.d, a.obj_mode);
  if (lds == 0) return v;
  const long monitor_lds = (long)a.n * 8;
  const long reg_lds = (long)(QSTAGE + 4 * 64 * 16) * 8;  // REG: GEMV staging + the Gram in quad order (T <= 16)
  const size_t shm = (size_t)(lds > monitor_lds ? lds : monitor_lds);
#define GADMM_P_PICK(NCv, SYSv, REGv, ...)                                                         \
  do {                                                                                             \
    v.fn = (const void*)chain_persistent_kernel<NCv, SYSv, REGv, ##__VA_ARGS__>;                   \
    v.shm = REGv ? (size_t)(monitor_lds > reg_lds ? monitor_lds : reg_lds) : shm;                    \
    v.threads = REGv ? 64 : NT;                                                                    \
  } while (0)
  static const bool force_lds = getenv("GADMM_PERSIST_LDS") != nullptr;  // A/B switch
  const bool tl = a.timeline != nullptr;  // instrumented instantiations (one GPU, register kernel, LDS d <= 64)
  if (a.d <= DREG && !force_lds && (!dyn || a.nvar <= 2)) {
    // register kernel: QT = 13 covers d <= 52 (E1/E5), 16 covers d <= 64
    if (tl && !a.sys_scope && a.d <= 52) {
      if (dyn) GADMM_P_PICK(1, false, true, 13, 2, true);
      else GADMM_P_PICK(1, false, true, 13, 1, true);
    } else if (dyn) {
      if (a.sys_scope) {
        if (a.d <= 52) GADMM_P_PICK(1, true, true, 13, 2);
        else GADMM_P_PICK(1, true, true, 16, 2);
      } else {
        if (a.d <= 52) GADMM_P_PICK(1, false, true, 13, 2);
        else GADMM_P_PICK(1, false, true, 16, 2);
      }
    } else if (a.sys_scope) {
      if (a.d <= 52) GADMM_P_PICK(1, true, true, 13, 1);
      else GADMM_P_PICK(1, true, true, 16, 1);
    } else {
      if (a.d <= 52) GADMM_P_PICK(1, false, true, 13, 1);
      else GADMM_P_PICK(1, false, true, 16, 1);
    }
  } else if (a.d <= 64) {
    if (a.sys_scope) GADMM_P_PICK(1, true, false);
    else if (tl) GADMM_P_PICK(1, false, false, 1, 1, true);
    else GADMM_P_PICK(1, false, false);
  } else {
    if (a.sys_scope) GADMM_P_PICK(2, true, false);
    else GADMM_P_PICK(2, false, false);
  }
#undef GADMM_P_PICK
  return v;
}

// Workgroups of `fn` (block size, dynamic LDS) that the device can hold resident at once:
// occupancy per CU x CUs. GADMM_CU_BUDGET=<n> replaces the CU count (tests of a partitioned or
// shared device). A persistent launch needs every one of its workgroups resident together: the
// workers spin on each other, so a workgroup that waits for a CU would stall the rest until the
// deadline. 0 on error.
// Occupancy of (kernel, threads, LDS, device), queried once: eligibility checks and launches ask for
// it several times per solve
namespace {
struct OccEntry {
  const void* fn;
  int threads, dev, per_cu;
  size_t shm;
};
std::mutex g_occ_mu;
OccEntry g_occ[128];
int g_occ_n = 0;
}  // namespace

extern "C" long gadmm_resident_capacity(const void* fn, int threads, size_t shm) {
  int dev = 0, per_cu = -1;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  {
    std::lock_guard<std::mutex> lk(g_occ_mu);
    for (int i = 0; i < g_occ_n; ++i)
      if (g_occ[i].fn == fn && g_occ[i].threads == threads && g_occ[i].shm == shm && g_occ[i].dev == dev) {
        per_cu = g_occ[i].per_cu;
        break;
      }
  }
  if (per_cu < 0) {
    per_cu = 0;
    if (shm > 65536 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess)
      return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, shm) != hipSuccess) return 0;
    std::lock_guard<std::mutex> lk(g_occ_mu);
    if (g_occ_n < 128) g_occ[g_occ_n++] = OccEntry{fn, threads, dev, per_cu, shm};
  }
  long cus = gadmm_cu_count();
  if (cus <= 0) return 0;
  if (const char* e = getenv("GADMM_CU_BUDGET")) {
    const long b = atol(e);
    if (b > 0 && b < cus) cus = b;
  }
  return (long)per_cu * cus;
}

// Effective XCD packing mode (PersistArgs::xcd / StarArgs::xcd `want`; env GADMM_XCD overrides it for
// A/B runs) of a launch of `blocks` working workgroups: one GPU only (`multi` = 0), and only when all
// of them fit on one XCD (cap_total / 8 of the `cap_total` resident slots), since packing deals every
// one of them there. Mode 2 needs the placement-check buffer.
extern "C" int gadmm_xcd_pick(int want, int multi, int blocks, long cap_total, const void* xchk) {
  int x = want;
  if (const char* e = getenv("GADMM_XCD")) x = atoi(e);
  if (x < 0) x = 0;
  if (x > 2) x = 2;
  if (multi || blocks > XCHK || (long)blocks > cap_total / 8) x = 0;
  if (x == 2 && !xchk) x = 1;
  return x;
}

extern "C" int gadmm_xcd_mode(const PersistArgs* a, int blocks, long cap_total) {
  return gadmm_xcd_pick(a->xcd, a->sys_scope || a->nranks > 1, blocks, cap_total, a->xchk);
}

// PersistArgs::xtag of a launch: fresh per launch in this process (high bit set, so never XTAG nor a
// zeroed granule), so the placement-check granules an earlier launch left in xchk never match.
extern "C" unsigned gadmm_next_xtag() {
  static std::atomic<unsigned> launches{0};
  return 0x80000000u | ((launches.fetch_add(1, std::memory_order_relaxed) + 1u) & 0x7fffffffu);
}

extern "C" {

// Workgroups the persistent kernel for `args` can keep resident (0: shape not eligible).
long gadmm_chain_persistent_capacity(const PersistArgs* args) {
  const PVariant v = pick_variant(*args);
  return v.fn ? gadmm_resident_capacity(v.fn, v.threads, v.shm) : 0;
}

int gadmm_chain_persistent_launch(const PersistArgs* args, hipStream_t st) {
  const PersistArgs& a = *args;
  const bool dyn = a.n_epochs > 0;
  if (dyn && (a.push || !a.epoch_start || !a.ep_slots || !a.ep_pos)) {
    gadmm_set_error("persistent chain kernel: dynamic epochs need epoch tables (epoch_start[0] == start_iter) "
                    "and per-epoch push masks instead of static push targets");
    return -1;
  }
  if (dyn && a.nranks > 1 && (!a.sys_scope || !a.ep_push || !a.peer_thg || a.nranks > 32)) {
    gadmm_set_error("persistent chain kernel: multi-rank D-GADMM needs the xGMI fabric (ep_push, peer_thg)");
    return -1;
  }
  const PVariant v = pick_variant(a);
  if (!v.fn) {
    gadmm_set_error("persistent chain kernel: d=%d not eligible", a.d);
    return -1;
  }
  if ((a.hard_stop > 0 || a.cont) && (!dyn || a.hard_stop < 0 || (a.hard_stop > 0 && a.hard_stop < a.start_iter))) {
    gadmm_set_error("persistent chain kernel: epoch chunks (hard_stop %d, cont %d) need the dynamic mode and "
                    "hard_stop >= start_iter", a.hard_stop, a.cont);
    return -1;
  }
  const int blocks = a.n_local + (a.has_monitor ? 1 : 0);
  const long cap = gadmm_resident_capacity(v.fn, v.threads, v.shm);
  if (blocks > cap) {
    gadmm_set_error("persistent chain kernel: %d workgroups but only %ld can be resident", blocks, cap);
    return -2;
  }
  if (a.ring <= a.lag + 1) {
    gadmm_set_error("persistent chain kernel: ring must exceed lag + 1");
    return -1;
  }
  if (a.start_iter + a.max_iter + a.lag >= (1 << 20)) {
    gadmm_set_error("persistent chain kernel: iteration tags limited to 2^20");
    return -1;
  }
  if (v.shm > 65536) GADMM_CHECK(hipFuncSetAttribute(v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)v.shm));
  PersistArgs ka = a;
  ka.xcd = gadmm_xcd_mode(&a, blocks, cap);
  ka.xtag = (int)gadmm_next_xtag();  // fresh placement-check tag: no memset of xchk
  void* kargs[] = {&ka};
  GADMM_CHECK(hipLaunchKernel(v.fn, dim3(ka.xcd > 0 ? 8 * blocks : blocks), dim3(v.threads), kargs, v.shm, st));
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// ---- xGMI fabric buffers: fine-grained (uncached) device memory exported by IPC -----------------
int gadmm_xgmi_alloc(size_t bytes, void** ptr, char* handle64) {
  GADMM_CHECK(hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached));
  GADMM_CHECK(hipMemset(*ptr, 0, bytes));
  hipIpcMemHandle_t h;
  GADMM_CHECK(hipIpcGetMemHandle(&h, *ptr));
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "unexpected IPC handle size");
  memcpy(handle64, &h, 64);
  GADMM_CHECK(hipDeviceSynchronize());
  return 0;
}

int gadmm_xgmi_open(const char* handle64, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle64, 64);
  GADMM_CHECK(hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess));
  return 0;
}

int gadmm_xgmi_close(void* ptr) {
  GADMM_CHECK(hipIpcCloseMemHandle(ptr));
  return 0;
}

int gadmm_xgmi_free(void* ptr) {
  GADMM_CHECK(hipFree(ptr));
  return 0;
}

int gadmm_device_can_access_peer(int dev, int peer) {
  int ok = 0;
  if (hipDeviceCanAccessPeer(&ok, dev, peer) != hipSuccess) return -1;
  return ok;
}

}  // extern "C"
