// Temporally blocked persistent GADMM (linear, closed form, one GPU, d <= 64).
//
// Why: in the one-workgroup-per-worker kernel (chain_persistent.hip) an iteration is two dependent
// cross-CU hand-offs of ~0.8 us each plus two phases of compute (profiles/r01_persistent_timeline).
// Here a workgroup owns a contiguous chain segment of L positions and ALSO computes a halo of
// H = 2k positions on each side, one wave per computed worker, with every worker's row of
// (A + deg rho I)^{-1} in VGPRs. Head -> tail -> head dependencies inside the computed range are
// LDS + workgroup-barrier hand-offs (tens of ns). Each phase invalidates one more position at each
// edge of the computed range (a worker needs both neighbours' fresh theta), so after k iterations
// exactly the owned segment is still exact. Then the workgroups exchange the (theta, mu) of their
// owned workers through data-is-flag granules and refresh their halos: ONE cross-CU hand-off per k
// iterations instead of 2k. The halo recomputation costs idle waves, not latency.
//
// Arithmetic is identical to the other engines (reg_gemv order == symv_lds == symv_cols, the exact
// objective 1/2 th^T A th - b^T th + 1/2 y^T y with A from LDS in the same order, the monitor sums
// f_n in worker order), so iterates and objective traces are bit-identical to the multi-kernel
// and per-worker persistent paths.
//
// Schedule per iteration it (reference semantics, group_ADMM_closedForm.m / A4 with a static chain):
//   [every k iterations] publish owned (theta, mu), refresh halo (theta, mu)      -- 1 hand-off
//   [stop rule] decision of iteration it - lag (prefetched one iteration ahead)
//   head phase: heads apply the lazy dual with the tails' theta^{it-1}, solve, write theta^it to LDS
//   barrier
//   tail phase: tails solve with the heads' theta^it, dual update
//   barrier
// Owned workers also post theta^it into a ring; OBJECTIVE workgroups (one wave per worker, A_n in
// VGPRs) evaluate f_n(theta^it) off the critical path and feed the monitor, which sums in worker
// order and posts the stop decision (monitor as in chain_persistent.hip). Grid: W worker
// workgroups, Wo objective workgroups, 1 monitor.
#include "gadmm_common.h"
#include "gadmm_chain.h"
#include "persist_device.h"
#include <stdlib.h>

namespace {

constexpr int MAXW = 12;  // computed workers (waves) per workgroup: 3 waves per SIMD -> <= 170 VGPRs
// one quad_store_lds image at DB = 52 (T = 13): the hosted halo head's inverse in LDS (HALO)
constexpr int HIMG52 = 4 * 64 * 14;
// DYN: epochs per launch whose tables are staged in LDS at the kernel start (epoch starts, and per
// computed / objective position its slot and flush pair), so a re-chain reads them in ~0.1 us
// instead of a cold HBM round trip; the host caps a launch at EPL epochs.
constexpr int EPL = 256;
// DYN LDS after the worker / objective layout, per wave (each wave stages and reads only its own
// rows: no barrier): [MAXW][EPL] slots (int4), [MAXW][EPL] flush pairs (int2), [MAXW][EPL] epoch starts
constexpr long DYN_LDS_BYTES = (long)MAXW * EPL * (16 + 8 + 4);
struct EpochLds {
  int4* sl;
  int2* fl;
  int* st;
};
__device__ __forceinline__ EpochLds epoch_lds(double* base, int v) {
  int4* sl = reinterpret_cast<int4*>(base);
  int2* fl = reinterpret_cast<int2*>(sl + MAXW * EPL);
  int* st = reinterpret_cast<int*>(fl + MAXW * EPL);
  return {sl + v * EPL, fl + v * EPL, st + v * EPL};
}

// Padded inverse image of PersistArgs::minv_pad, per (worker, variant): the quad register layout of
// quad_load<QT> stored lane-major in (t, t + 1) pairs -- element Mq[r][t] of lane l at
// ((t >> 1) * 4 + r) * 128 + 2 l + (t & 1) (quad_store_lds's layout), zero beyond d. A reload is then
// 4 * ceil(QT / 2) coalesced 16-byte loads per lane (1 KB contiguous per wave instruction) with no
// bounds masks.
template <int QT>
__device__ __forceinline__ void quad_load_image(double (&m)[4][QT], const double* img) {
  const int lane = threadIdx.x & 63;
  const double2* p = reinterpret_cast<const double2*>(img) + lane;
#pragma unroll
  for (int t = 0; t < QT; t += 2)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double2 v = p[((t >> 1) * 4 + r) * 64];
      m[r][t] = v.x;
      if (t + 1 < QT) m[r][t + 1] = v.y;
    }
}

// Stages a launch's epoch tables for chain position q into this wave's LDS rows (DYN); the wave's
// own later LDS reads are ordered after these stores (in-order LDS within a wave).
__device__ __forceinline__ void stage_epochs(const PersistArgs& a, int q, const EpochLds& el, bool flush) {
  const int lane = threadIdx.x & 63;
  for (int e = lane; e < a.n_epochs; e += 64) {
    el.sl[e] = reinterpret_cast<const int4*>(a.ep_slots)[(long)e * a.n + q];
    if (flush) el.fl[e] = reinterpret_cast<const int2*>(a.ep_flush)[(long)e * a.n + q];
    el.st[e] = a.epoch_start[e];
  }
}
}  // namespace



// ---- monitor workgroup (same protocol as chain_persistent): sums f_n in worker order, records the
// trace and posts the stop decision of every iteration to every rank's decision ring
template <bool SYS, bool TL>
__device__ __forceinline__ void blocked_monitor(const PersistArgs& a, double* lds, int v, int lane,
                                                unsigned long long deadline, __amdgpu_buffer_rsrc_t rob, int bid) {
  const int n = a.n;
  if (v != 0) return;
  double* vals = lds;  // [n]
  for (int it = a.start_iter;; ++it) {
    if (a.hard_stop > 0 && it > a.hard_stop) {  // D-GADMM chunk exhausted without a stop decision
      if (lane == 0) a.ctl->done = 5;
      return;
    }
    const unsigned tag = make_tag(a.epoch, it);
    const int slot = it % a.ring;
    bool okall = true;
    for (int w = lane; w < n; w += 64) {
      double val = 0.0;
      for (int spin = 0;; ++spin) {
        if (load_granule<SYS>(rob, (slot * n + w) * 16, tag, &val)) break;
        if ((spin & 7) == 7 && now_ticks() > deadline) {
          okall = false;
          break;
        }
        GADMM_POLL_PAUSE();
      }
      vals[w] = val;
    }
    const bool ok = __all(okall);
    unsigned code = 0;
    if (lane == 0) {
      if (!ok) {
        code = 4;
      } else {
        double s = 0.0;
        for (int w = 0; w < n; ++w) s += vals[w];  // worker order: == the other engines
        if (it - 1 < a.max_iter) a.trace[it - 1] = s;
        if (!(s == s) || isinf(s)) code = 3;
        else if (fabs(s - a.obj0) < a.tol) code = 1;
        else if (it >= a.max_iter) code = 2;
        if (a.tstamp && it - 1 < a.max_iter) a.tstamp[it - 1] = (long long)now_ticks();
      }
      const unsigned long long dv = ((unsigned long long)tag << 32) | code;
      for (int r = 0; r < a.nranks; ++r) store_dec<SYS>(a.dec_push[r] + slot, dv);
      if (code && a.hard_stop > 0) {  // chunked: the workers may reach the hard stop before seeing it
        a.ctl->done = (int)code;
        a.ctl->conv_iter = it;
      }
      const int kk = it - a.start_iter;
      if (TL && kk < a.timeline_iters) a.timeline[((long)bid * a.timeline_iters + kk) * 8] = (long long)now_ticks();
    }
    if (__shfl((int)code, 0, 64)) return;
  }
}

// ---- objective workgroup: wave v evaluates f_q(theta_q^it) of owned chain position q (A_q in VGPRs,
// quad layout) off the critical path and posts it to the monitor ring
template <int QT, bool SYS, bool DYN = false>
__device__ __forceinline__ void blocked_objective(const PersistArgs& a, double* lds, int v, int lane, int q,
                                                  unsigned long long deadline, __amdgpu_buffer_rsrc_t rob,
                                                  __amdgpu_buffer_rsrc_t rtab, bool local = false) {
  const int d = a.d, n = a.n;
  const long ring_base = 2L * n * 2 * d;  // theta ring [ring][n][d] after the exchange table
  // DYN (one GPU, li == worker id): the wave follows WORKER q instead of position q -- its Gram stays
  // resident and a re-chain only changes which ring row carries theta_q (ep_pos [E][n], staged in LDS
  // with the epoch starts), so no A / b / yy reload lands on the stop-rule pipeline at a re-chain
  const EpochLds el = epoch_lds(lds + MAXW * 64 + MAXW * QSTAGE, v);
  int* posl = reinterpret_cast<int*>(el.fl);  // [EPL] position of worker q per epoch (DYN)
  if constexpr (DYN) {
    for (int e = lane; e < a.n_epochs; e += 64) {
      posl[e] = a.ep_pos[(long)e * n + q];
      el.st[e] = a.epoch_start[e];
    }
  }
  const PhaseSlot so = a.slots[DYN ? 0 : q];
  const int li = DYN ? q : so.li, gid = DYN ? q : so.gid;
  int row = DYN ? posl[0] : q;  // the ring row carrying this wave's theta
  const bool in = lane < d;
  double Aq[4][QT];
  quad_load<QT>(Aq, a.A + (long)li * d * d, d, true);
  const double bo = in ? a.b[(long)li * d + lane] : 0.0;
  const double hy = 0.5 * a.yy[li];
  double* xo = lds + v * QSTAGE;
  int ep = 0, next_start = (DYN && a.n_epochs > 1) ? el.st[1] : 0x7fffffff;
  for (int it = a.start_iter;; ++it) {
    if (a.hard_stop > 0 && it > a.hard_stop) return;  // D-GADMM chunk end: no theta^it comes
    if constexpr (DYN) {
      if (it == next_start) {  // D-GADMM re-chain: worker q now sits at another position
        ++ep;
        next_start = ep + 1 < a.n_epochs ? el.st[ep + 1] : 0x7fffffff;
        row = posl[ep];
      }
    }
    const unsigned tag = make_tag(a.epoch, it);
    const long off = (ring_base + ((long)(it % a.ring) * n + row) * d + lane) * 16;
    double x = 0.0;
    for (int spin = 0;; ++spin) {
      const bool ok = !in || load_granule<SYS>(rtab, (int)off, tag, &x);
      if (__all(ok)) break;
      if ((spin & 7) == 7) {
        // the run ended: the workers stop at iteration j + lag after a stop decision for j, so
        // theta^it never comes once decision[it - lag] says stop (on every rank's own ring)
        if (it - a.start_iter >= a.lag) {
          const unsigned long long dv = load_dec<SYS>(&a.decg[(it - a.lag) % a.ring]);
          if ((unsigned)(dv >> 32) == make_tag(a.epoch, it - a.lag) && (unsigned)(dv & 0xffffffffu) != 0u) return;
        }
        if (now_ticks() > deadline) return;  // the monitor times out and reports it
      }
      GADMM_POLL_PAUSE();
    }
    const double qv = quad_gemv<QT>(Aq, in ? x : 0.0, xo);  // (A th)_i in the order of every other engine
    const double part = in ? (0.5 * qv - bo) * x : 0.0;
    const double f = wave_sum_f64(part) + hy;
    if (lane == 0) put_granule<SYS>(local, rob, ((it % a.ring) * n + gid) * 16, tag, f);
  }
}

// DB: register row length (multiple of 4, >= d); 52 keeps d = 50 within the 3-waves-per-SIMD budget.
// SYS: multi-GPU (xGMI fabric): system-scope granules in IPC fine-grained memory; this rank owns
// chain positions [seg_lo, seg_hi] and pushes owned (theta, mu) into its peers' exchange tables.
// Block layout: [0, W) worker workgroups, [W, W + Wo) objective workgroups, W + Wo the monitor
// (rank 0 only).
// TL: the instrumented instantiation (timeline stamps, experiment bits); the production one has no
// diagnostics code in its loop.
// DYN: D-GADMM in one launch (single GPU). Positions stay with their workgroups; at every epoch
// start (ep_slots [E][n] in chain-position order, ep_pos [E][n] worker -> position) the owned
// positions publish their worker's (theta, mu) by WORKER id into an epoch table, and every computed
// position loads the state of the worker that the new chain puts there, with its inverse, b and A.
// A worker that was a head owes its dual of the last iteration of the old chain: the loader applies
// it with the worker's OLD neighbours' theta, read from the same table (the reference order,
// dynamic_group_ADMM_closedForm.m:153-168). The regular halo schedule restarts after the switch.
// HALO (SYS only): the data-local halo mode (PersistArgs::dl_halo, one workgroup per segment: no
// intra-rank exchange is compiled in).
template <int DB, bool SYS, bool TL, bool DYN = false, bool HALO = false>
__global__ void __launch_bounds__(64 * MAXW) chain_blocked_kernel(PersistArgs a) {
  constexpr int QT = DB / 4;  // quad layout: columns per lane
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int abort_lds, stop_lds, stop_iter_lds;
  const int d = a.d, n = a.n;
  const int lane = threadIdx.x & 63;
  const int v = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: per-wave state in SGPRs
  const int k = a.blk_k, L = a.blk_len, H = 2 * a.blk_k;
  const bool multi = a.nranks > 1;
  const int seg_lo = multi ? a.seg_lo : 0, seg_hi = multi ? a.seg_hi : n - 1;
  const int nseg = seg_hi - seg_lo + 1;
  const int W = (nseg + L - 1) / L;
  const int Wo = (nseg + MAXW - 1) / MAXW;
  // data-local mode (PersistArgs::blk_dl): the computed ranges stop at this rank's segment edges, and
  // a segment-edge position gets its other-rank neighbour's theta every phase through the theta ring
  const bool dl = SYS && multi && a.blk_dl != 0;
  const unsigned long long deadline = now_ticks() + (unsigned long long)a.timeout_ticks;
  const __amdgpu_buffer_rsrc_t rob = rsrc_of(a.objg);
  const __amdgpu_buffer_rsrc_t rtab = rsrc_of(a.blk_tab);
  const bool packed = !SYS && a.xcd > 0;  // XCD packing (PersistArgs::xcd)
  if (packed && (blockIdx.x & 7u)) return;  // a spacer block: only b % 8 == 0 work (one XCD)
  const int bid = packed ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  if (threadIdx.x == 0) {
    abort_lds = 0;
    stop_lds = 0;
  }
  lds_barrier();
  const long ring_base = 2L * n * 2 * d;  // theta ring [ring][n][d] after the exchange table
  const long etab_base = 2L * n * 2 * d + (long)a.ring * n * d;
  bool local = false;  // publish with plain stores (every block verified on this XCD)
  if (!SYS && a.xcd > 1) local = xcd_verdict(a.xchk, bid, W + Wo + 1, deadline, &stop_iter_lds, (unsigned)a.xtag);
  if (!SYS && bid == 0 && threadIdx.x == 0) a.ctl->placed = a.xcd > 0 ? (local ? 2 : 1) : 0;

  if (bid == W + Wo) {
    blocked_monitor<SYS, TL>(a, lds, v, lane, deadline, rob, bid);
    return;
  }

  if (bid >= W) {
    const int q = seg_lo + (bid - W) * MAXW + v;  // an owned chain position
    if (q <= seg_hi) blocked_objective<QT, SYS, DYN>(a, lds, v, lane, q, deadline, rob, rtab, local);
    return;
  }

  // ---------------------------------------------------------------------- worker workgroup
  const int g = bid;
  const int s0 = seg_lo + g * L, e0 = min(seg_hi + 1, s0 + L) - 1;  // owned chain positions [s0, e0]
  // HALO: the range also takes the other rank's boundary head next to a boundary tail of this rank
  // (see dlh below): one more wave on that side
  const int hl = HALO && dl && seg_lo > 0 && (seg_lo % 2) == 1, hr = HALO && dl && seg_hi < n - 1 && (seg_hi % 2) == 1;
  // Hosted halo head: when the segment and its halo head exceed MAXW waves (2 ranks x 12 workers: 13),
  // the waves stay the segment's own and the halo head h is computed by the segment's TAIL waves in
  // the head phase, where tails idle: h's inverse sits in LDS as a quad image, four tail waves (one
  // per SIMD) each run one of its four row groups (13 FMAs after 7 + 7 LDS reads, in parallel), and
  // the boundary tail next to h folds the four partials with quad_reduce at the start of its tail
  // phase -- the register GEMV's FMA and reduction order, so h's theta is bit-identical to its
  // owner's. (Round 3's single-wave LDS GEMV put ~1 us on the head phase.) One hosted side per
  // segment (the launcher checks it).
  const bool hosted = HALO && dl && (seg_hi - seg_lo + 1 + hl + hr > MAXW);
  const int hd = hosted ? (hr ? 1 : -1) : 0;                   // side of the hosted head
  const int hp = hd > 0 ? seg_hi + 1 : (hd < 0 ? seg_lo - 1 : 0);  // its chain position
  const int ra = max(dl ? seg_lo - (hosted ? 0 : hl) : 0, s0 - H), rb = min(dl ? seg_hi + (hosted ? 0 : hr) : n - 1, e0 + H);
  const int nv = rb - ra + 1;
  // Wave v computes local position u. Waves are dealt to the 4 SIMDs round-robin (v mod 4), so
  // v < MAXW/2 take the heads and the rest the tails: each phase keeps every SIMD busy with
  // MAXW/8 GEMV waves instead of piling a phase's 6 GEMVs onto two SIMDs (identity map: heads
  // are every other wave -> SIMDs 0 and 2 only).
  const int h0 = ra & 1;  // parity offset: position ra + u is a head iff u has parity h0
  const int u = v < MAXW / 2 ? 2 * v + h0 : 2 * (v - MAXW / 2) + (1 - h0);
  const int p = ra + u;  // this wave's chain position
  const bool active = u < nv;
  const bool owned = active && p >= s0 && p <= e0;
  PhaseSlot sl = DYN ? a.ep_slots[active ? p : 0] : a.slots[active ? p : 0];  // sorted by chain position
  int li = sl.li, w = sl.gid;
  const bool has_l = active && sl.left >= 0, has_r = active && sl.right >= 0;
  const bool head = (p % 2) == 0;
  const int deg = (int)has_l + (int)has_r;
  const double rho = a.rho;
  const bool in = lane < d;
  // Decision wave: polls the stop decision during the tail phase, when heads are idle. A halo head
  // is preferred: it never stores to global memory, so its decision load does not queue behind
  // write-through granule stores (vmcnt counts stores on gfx9).
  // Next best: an idle wave (u >= nv: no position). A computed tail can never be it (it is busy in
  // exactly the phase the poll runs in) -- a workgroup whose only position is a tail (one worker per
  // rank, odd position) polls on an idle wave.
  // Invariant: every wave of the workgroup, inactive ones included, executes the same sequence of
  // lds_barrier()s (exchange, re-chain, stop) -- the decision wave may be an idle one, which is only
  // correct because idle waves follow the active waves' schedule exactly (DYN: from the same staged
  // epoch starts, see stage_epochs below).
  int vdec = -1;
  for (int u = 0; u < nv && vdec < 0; ++u)
    if (((ra + u) % 2) == 0 && (ra + u < s0 || ra + u > e0)) vdec = u;
  if (vdec < 0 && nv < MAXW) vdec = nv;
  if (vdec < 0) vdec = (ra % 2 == 0) ? 0 : 1;
  const bool dec_wave = u == vdec;

  double* thS = lds;                       // [MAXW][64] theta of every computed worker
  double* xs = thS + MAXW * 64;            // [MAXW][QSTAGE] per-wave quad GEMV staging
  double* myx = xs + v * QSTAGE;
  // the wave's neighbours inside the computed range (outside it the halo worker is already stale)
  const double* thL = thS + (u > 0 ? u - 1 : u) * 64;
  const double* thR = thS + (u + 1 < nv ? u + 1 : u) * 64;
  const bool nbl = has_l && u > 0, nbr = has_r && u + 1 < nv;
  // data-local segment edges: the neighbour beyond seg_lo / seg_hi is another rank's worker. It is
  // never stale: its theta^j arrives in THIS rank's theta ring (row seg_lo - 1 / seg_hi + 1, slot
  // j % ring, tag j), pushed there by its owner right after its solve; the owner of an edge position
  // pushes its own theta^j into the neighbour rank's ring the same way (no mu, no shard crosses).
  // (p == seg_lo implies u == 0 and p == seg_hi implies u == nv - 1, so nbl / nbr are false there.)
  // (the range edges: ra / rb; p == ra implies u == 0 and p == rb implies u == nv - 1)
  // hosted mode: hdir != 0 on the boundary tail next to the hosted head (h = p + hdir); hq = 0..3 on the
  // four tail waves (v = MAXW/2 .. MAXW/2 + 3: one per SIMD) that run h's row groups
  const int hdir = (hosted && active && p == hp - hd) ? hd : 0;
  const int hq = (hosted && v >= MAXW / 2 && v < MAXW / 2 + 4) ? v - MAXW / 2 : -1;
  const bool rl = dl && has_l && p == ra && hdir != -1, rr = dl && has_r && p == rb && hdir != 1;
  // Halo mode (HALO, PersistArgs::dl_halo; one workgroup per segment, every segment >= 2 positions,
  // segment + halo within MAXW waves): at a rank boundary whose near side is a TAIL t, this rank also
  // computes the other rank's boundary head h (one more wave, h's inverse from h's shard, which this
  // rank holds). h polls its far neighbour f = t -+ 2 (another rank's tail, pushed after f's tail
  // phase) in the head phase; t then reads h from LDS and needs no hand-off, and h's owner no longer
  // pushes h. Per boundary and iteration still two pushes (t's and f's), but both go tail phase ->
  // next head phase, so the two ranks pipeline one phase apart and the critical cycle carries one
  // cross-rank hop per iteration instead of two (head -> tail -> head).
  const bool dlh = HALO && dl;
  const bool lb_tail = hl != 0, rb_tail = hr != 0;
  // pushes of this wave's theta^j into the left / right neighbour rank's ring (row p, slot j % ring)
  // (without the halo: the edge positions themselves, rl / rr; push_remote runs only when rpush)
  const bool pl = dlh ? (owned && !head && ((p == seg_lo && has_l) || (p == seg_lo + 1 && seg_lo > 0 && !lb_tail)))
                      : rl;
  const bool pr = dlh ? (owned && !head && ((p == seg_hi && has_r) || (p == seg_hi - 1 && seg_hi < n - 1 && !rb_tail)))
                      : rr;
  const bool rpush = dlh ? (pl || pr) : owned && (rl || rr);

  // DYN: this wave's epoch rows in LDS (after thS and the staging area; see DYN_LDS_BYTES)
  const EpochLds el = epoch_lds(lds + MAXW * 64 + MAXW * QSTAGE, v);
  if constexpr (DYN) {
    // EVERY wave stages the epoch starts: inactive waves (u >= nv, e.g. an idle decision wave) run the
    // same per-iteration barrier schedule, re-chain barrier included, off `next_start`, so they must
    // read the same starts as the active ones; their slot rows (position 0) go unused
    stage_epochs(a, active ? p : 0, el, active);
  }
  // Positions that ever solve: in a block, phase phi solves the owned range widened by 2k - 1 - phi,
  // so heads up to 2k - 1 and tails up to 2k - 2 positions away from it; the outermost halo only
  // carries theta. DYN: only these reload an inverse at a re-chain.
  const int odist = u < s0 - ra ? (s0 - ra) - u : (u > e0 - ra ? u - (e0 - ra) : 0);
  const bool solver = active && odist <= (head ? 2 * k - 1 : 2 * k - 2);
  double Mq[4][QT];
  quad_load<QT>(Mq, a.Minv + ((long)li * a.nvar + a.deg_to_var[deg]) * (long)d * d, d, active);
  // y = (A + deg rho I)^{-1} r for this wave's worker (r: this lane's element)
  auto solve = [&](double r) -> double {
    const double y = quad_gemv<QT>(Mq, in ? r : 0.0, myx);
    return in ? y : 0.0;
  };
  double th = (active && in) ? a.theta[(long)w * d + lane] : 0.0;
  double mu = (active && in) ? a.mu[(long)li * d + lane] : 0.0;
  double bb = (active && in) ? a.b[(long)li * d + lane] : 0.0;
  thS[u * 64 + lane] = th;
  // hosted halo head (HALO): its inverse as a quad image in LDS (after thS and the staging area) and its
  // state in LDS: hst = [theta 64 | mu, two iteration-parity buffers 2 x 64 | b 64 | row-group partials
  // 4 x 64]; hsl / hsr: the head has a left / right neighbour (uniform)
  double* Mh = lds + MAXW * 64 + MAXW * QSTAGE;
  double* hst = Mh + HIMG52;
  bool hsl = false, hsr = false;
  if (HALO && hosted) {
    const PhaseSlot sh = a.slots[hp];
    hsl = sh.left >= 0;
    hsr = sh.right >= 0;
    if (hdir != 0) {  // the boundary tail stages h's inverse and state once
      const int deg_h = (int)hsl + (int)hsr;
      quad_store_lds<QT>(Mh, a.Minv + ((long)sh.li * a.nvar + a.deg_to_var[deg_h]) * (long)d * d, d, true);
      hst[lane] = in ? a.theta[(long)sh.gid * d + lane] : 0.0;
      hst[64 + (a.start_iter & 1) * 64 + lane] = in ? a.mu[(long)sh.li * d + lane] : 0.0;
      hst[192 + lane] = in ? a.b[(long)sh.li * d + lane] : 0.0;
    }
  }
  int pending = a.pending_in;
  // DYN: epoch cursor, regular exchange schedule (restarts after every re-chain) and its slot
  // counter, and the epoch exchange table [2][n][2][d] after the theta ring
  int ep = 0, next_start = (DYN && a.n_epochs > 1) ? el.st[1] : 0x7fffffff;
  int next_x = a.start_iter + k, xc = 0;
  // Only the positions whose result still reaches an owned one before the next exchange are solved:
  // in phase phi of a block (phi = 0, 1 the head / tail phase of its first iteration, ...) that is the
  // owned range widened by 2k - 1 - phi on each side; the rest of the halo is stale anyway. Fewer GEMV
  // waves then share the SIMDs (three of the four phases of a k = 2 block run <= 1 per SIMD).
  const int uo_lo = s0 - ra, uo_hi = e0 - ra;
  int blk0 = a.start_iter;  // first iteration of the current block (after an exchange / re-chain)
  if (threadIdx.x == 0) stop_iter_lds = 0;
  lds_barrier();

  // a stop decision for iteration j arrives before iteration j + lag runs: polled during the tail
  // phase of iteration j + lag - 1 and published by that phase's closing barrier
  // owned (theta, mu) after iteration j, for the exchange at the start of iteration j + 1: into
  // this GPU's table and into every peer GPU that computes position p too
  auto publish = [&](int j) {
    const unsigned tag = make_tag(a.epoch, j + 1);
    const int sel = xc & 1;  // exchange table slot: alternates per exchange (every rank counts alike)
    const int base = ((sel * n + p) * 2) * d;
    put_granule<SYS>(local, rtab, (base + lane) * 16, tag, th);
    put_granule<SYS>(local, rtab, (base + d + lane) * 16, tag, mu);
    for (int q = 0; q < a.blk_npeer; ++q)
      if (p >= a.blk_peer_lo[q] && p <= a.blk_peer_hi[q]) {
        const __amdgpu_buffer_rsrc_t rpe = rsrc_of(a.blk_peer_tab[q]);
        store_granule<SYS>(rpe, (base + lane) * 16, tag, th);
        store_granule<SYS>(rpe, (base + d + lane) * 16, tag, mu);
      }
  };
  unsigned long long dv_pref = 0;  // decision wave, lane 0: decision[it + 1 - lag] prefetched
  int it = a.start_iter;
  bool hard_stopped = false;
  long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // Objective-ring posts of owned workers go out in the phase their wave idles in: heads post
  // theta^it during the tail phase, tails post theta^{it-1} at the start of iteration it
  // (ring_defer), so neither sits on a phase's critical path. Ring and decision slots are counters
  // (no integer division in the loop).
  const int ring_p = (int)((ring_base + (long)(active ? p : 0) * d + lane) * 16);  // (slot 0, p, lane)
  const int ring_slot_bytes = n * d * 16;
  const bool ring_post = owned && in && !(TL && (a.dbg & 2));
  const int ring_l = (int)((ring_base + (long)(rl ? p - 1 : 0) * d + lane) * 16);  // slot 0, row p - 1
  const int ring_r = (int)((ring_base + (long)(rr ? p + 1 : 0) * d + lane) * 16);  // slot 0, row p + 1
  const __amdgpu_buffer_rsrc_t rdl0 = rsrc_of(pl && a.dl_tab[0] ? (const void*)a.dl_tab[0] : (const void*)a.blk_tab);
  const __amdgpu_buffer_rsrc_t rdl1 = rsrc_of(pr && a.dl_tab[1] ? (const void*)a.dl_tab[1] : (const void*)a.blk_tab);
  // other-rank neighbours' theta^j (ring slot `slot`) into tl / tr; false on a deadline
  auto poll_remote = [&](int slot, int j, double& tl, double& tr) -> bool {
    const unsigned tag = make_tag(a.epoch, j);
    const int so = slot * ring_slot_bytes;
    for (int spin = 0;; ++spin) {
      bool g0 = true;
      if (in) {
        if (rl) g0 &= load_granule<SYS>(rtab, ring_l + so, tag, &tl);
        if (rr) g0 &= load_granule<SYS>(rtab, ring_r + so, tag, &tr);
      }
      if (__all(g0)) return true;
      if ((spin & 7) == 7 && now_ticks() > deadline) return false;
      GADMM_POLL_PAUSE();
    }
  };
  // the hosted halo head's far neighbour's theta^j (ring slot `slot`) into tf; false on a deadline
  auto poll_far = [&](int slot, int j, double& tf) -> bool {
    const unsigned tag = make_tag(a.epoch, j);
    // ring row of the far neighbour (another rank's tail, pushed after its tail phase)
    const int so = slot * ring_slot_bytes + (int)((ring_base + (long)(hp + hd) * d + lane) * 16);
    for (int spin = 0;; ++spin) {
      const bool g0 = !in || load_granule<SYS>(rtab, so, tag, &tf);
      if (__all(g0)) return true;
      if ((spin & 7) == 7 && now_ticks() > deadline) return false;
      GADMM_POLL_PAUSE();
    }
  };
  // this edge position's theta^j into the neighbour ranks' rings (their row p, slot `slot`)
  auto push_remote = [&](int slot, int j) {
    const unsigned tag = make_tag(a.epoch, j);
    const int off = ring_p + slot * ring_slot_bytes;
    if (pl) store_granule<SYS>(rdl0, off, tag, th);
    if (pr) store_granule<SYS>(rdl1, off, tag, th);
  };
  bool ring_defer = false;
  int rslot = a.start_iter % a.ring;                  // == it % ring
  int dslot = (a.start_iter + 1 - a.lag) % a.ring;     // == (it + 1 - lag) % ring (>= 0 once polled)
  if (dslot < 0) dslot += a.ring;
  for (;; ++it, rslot = rslot + 1 == a.ring ? 0 : rslot + 1, dslot = dslot + 1 == a.ring ? 0 : dslot + 1) {
    if (ring_defer) {  // tails: theta^{it-1}, before a re-chain may replace th
      put_granule<SYS>(local, rtab, ring_p + (rslot == 0 ? a.ring - 1 : rslot - 1) * ring_slot_bytes,
                       make_tag(a.epoch, it - 1), th);
      ring_defer = false;
    }
    if (it > a.max_iter + a.lag) break;
    if (a.hard_stop > 0 && it > a.hard_stop) {  // D-GADMM chunk end: state = after the hard stop
      hard_stopped = true;
      break;
    }
    const bool stamp = TL && v == 0 && it - a.start_iter < a.timeline_iters;  // wave-uniform (SGPR stamps)
    if (stamp) ts[0] = (long long)now_ticks();
    if constexpr (DYN) {
      if (it == next_start) {  // ---- re-chain (dynamic_group_ADMM_closedForm.m:18-21)
        const unsigned tag = make_tag(a.epoch, it);
        const long eb = etab_base + (long)((ep + 1) & 1) * n * 2 * d;  // this switch's slot
        if (owned && in) {  // the worker's state after iteration it - 1 (a head's dual still pending)
          const long base = eb + (long)w * 2 * d;
          put_granule<SYS>(local, rtab, (int)((base + lane) * 16), tag, th);
          put_granule<SYS>(local, rtab, (int)((base + d + lane) * 16), tag, mu);
        }
        ++ep;
        next_start = ep + 1 < a.n_epochs ? el.st[ep + 1] : 0x7fffffff;
        if (active) {
          {
            const int4 s4 = el.sl[ep];
            sl.li = s4.x;
            sl.gid = s4.y;
          }
          // the new worker's old-chain neighbours when it was a head (pending-dual flush), -1: none
          const int2 of = el.fl[ep];
          li = sl.li;
          w = sl.gid;
          if (solver) {  // the new worker's inverse (lane-major padded image, coalesced unmasked loads)
                         // and b: issued before the state poll below, so they overlap the hand-off
            quad_load_image<QT>(Mq, a.minv_pad + ((long)li * a.nvar + a.deg_to_var[deg]) * (long)(512 * ((QT + 1) / 2)));
            bb = in ? a.b[(long)li * d + lane] : 0.0;
          }
          const bool fl = pending && of.x >= 0, fr = pending && of.y >= 0;  // it was a head: dual pending
          double t0 = 0.0, t1 = 0.0, tl = 0.0, tr = 0.0;
          bool ok = true;
          for (int spin = 0;; ++spin) {
            bool g0 = true;
            if (in) {
              const long b0 = eb + (long)w * 2 * d;
              g0 &= load_granule<SYS>(rtab, (int)((b0 + lane) * 16), tag, &t0);
              g0 &= load_granule<SYS>(rtab, (int)((b0 + d + lane) * 16), tag, &t1);
              if (fl) g0 &= load_granule<SYS>(rtab, (int)((eb + (long)of.x * 2 * d + lane) * 16), tag, &tl);
              if (fr) g0 &= load_granule<SYS>(rtab, (int)((eb + (long)of.y * 2 * d + lane) * 16), tag, &tr);
            }
            if (__all(g0)) break;
            if ((spin & 7) == 7 && now_ticks() > deadline) {
              ok = false;
              break;
            }
            GADMM_POLL_PAUSE();
          }
          if (!ok && lane == 0) abort_lds = 1;
          th = in ? t0 : 0.0;
          double m = in ? t1 : 0.0;
          if (fl) m = m - rho * (tl - th);  // the old chain's end-of-iteration dual
          if (fr) m = m + rho * (th - tr);
          mu = in ? m : 0.0;
          thS[u * 64 + lane] = th;
        }
        pending = 0;
        next_x = it + k;
        blk0 = it;
        lds_barrier();
        if (abort_lds) break;
      }
    }
    // ---- halo exchange every k iterations (state after iteration it - 1); the owned workers
    // published theirs during the tail phase of it - 1 (publish() below)
    if (!HALO && it == next_x) {  // (HALO: one workgroup per segment, no intra-rank exchange)
      if (active && !owned) {
        const unsigned tag = make_tag(a.epoch, it);
        const int sel = xc & 1;
        const int base = ((sel * n + p) * 2) * d;
        double t0 = 0.0, t1 = 0.0;
        bool ok = true;
        for (int spin = 0;; ++spin) {
          bool g0 = true;
          if (in) {
            g0 &= load_granule<SYS>(rtab, (base + lane) * 16, tag, &t0);
            g0 &= load_granule<SYS>(rtab, (base + d + lane) * 16, tag, &t1);
          }
          if (__all(g0)) break;
          if ((spin & 7) == 7 && now_ticks() > deadline) {
            ok = false;
            break;
          }
          GADMM_POLL_PAUSE();
        }
        if (!ok && lane == 0) abort_lds = 1;
        th = in ? t0 : 0.0;
        mu = in ? t1 : 0.0;
        thS[u * 64 + lane] = th;
      }
      lds_barrier();  // refreshed halo theta visible to the neighbouring waves
      if (abort_lds) break;
      blk0 = it;
      next_x = it + k;
      ++xc;
    }
    if (stamp) ts[1] = ts[2] = ts[3] = (long long)now_ticks();

    // ---- head phase
    const int slack = 2 * k - 1 - 2 * (it - blk0);  // head phase; the tail phase has slack - 1
    if (active && head && u >= uo_lo - slack && u <= uo_hi + slack) {
      double tl = nbl ? thL[lane] : 0.0, tr = nbr ? thR[lane] : 0.0;
      if (rl || rr) {  // the other ranks' tails' theta^{it-1} (their initial theta at the first iteration)
        if (it == a.start_iter) {
          if (rl && in) tl = a.theta[(long)(p - 1) * d + lane];
          if (rr && in) tr = a.theta[(long)(p + 1) * d + lane];
        } else if (!poll_remote(rslot == 0 ? a.ring - 1 : rslot - 1, it - 1, tl, tr) && lane == 0) {
          abort_lds = 1;
        }
      }
      double m = mu;
      if (pending) {  // lazy end-of-iteration dual (reference order)
        if (has_l) m = m - rho * (tl - th);
        if (has_r) m = m + rho * (th - tr);
      }
      mu = m;
      double r = bb - m;
      if (has_l) r = r + rho * tl;
      if (has_r) r = r + rho * tr;
      if (stamp) ts[6] = (long long)now_ticks();
      th = solve(r);
      if (stamp) {
        asm volatile("" ::"v"(th));
        ts[7] = (long long)now_ticks();
      }
      if (rpush && in) push_remote(rslot, it);  // first: the other rank's tail waits on it
      thS[u * 64 + lane] = th;
    }
    if (HALO && hq >= 0) {  // hosted halo head h: row group hq of its solve of iteration it
      double tf = 0.0;  // the far neighbour's theta^{it-1} (its initial theta at the first iteration)
      if (hd > 0 ? hsr : hsl) {
        if (it == a.start_iter) {
          if (in) tf = a.theta[(long)(hp + hd) * d + lane];
        } else if (!poll_far(rslot == 0 ? a.ring - 1 : rslot - 1, it - 1, tf) && lane == 0) {
          abort_lds = 1;
        }
      }
      const double tn = thS[(hp - hd - ra) * 64 + lane];  // the boundary tail's theta^{it-1}
      const double tl = hd > 0 ? tn : tf, tr = hd > 0 ? tf : tn;
      const double th_h = hst[lane];
      double m = hst[64 + (it & 1) * 64 + lane];
      if (pending) {  // lazy end-of-iteration dual (reference order)
        if (hsl) m = m - rho * (tl - th_h);
        if (hsr) m = m + rho * (th_h - tr);
      }
      if (hq == 0) hst[64 + ((it + 1) & 1) * 64 + lane] = m;  // parity buffers: no reader races the write
      double r = hst[192 + lane] - m;
      if (hsl) r = r + rho * tl;
      if (hsr) r = r + rho * tr;
      hst[256 + hq * 64 + lane] = quad_rowgroup_lds<QT>(Mh, hq, in ? r : 0.0, myx);
    }
    pending = 1;
    lds_barrier();
    if (stamp) ts[4] = (long long)now_ticks();

    // ---- tail phase; the (idle head) decision wave fetches decision[it + 1 - lag]
    // the next iteration starts with a regular exchange (DYN: unless it starts a new epoch)
    const bool xnext = !HALO && it + 1 == next_x && !(DYN && it + 1 == next_start);
    // tail-wave stamps (wave MAXW/2 by default), timeline row 128 + g: [start, rhs, gemv, stores, barrier]
    // (GADMM_BLK_DBG bits 4-6 pick another tail wave: MAXW/2 + ((dbg >> 4) & 7))
    const bool tstamp = TL && v == MAXW / 2 + ((a.dbg >> 4) & 7) && it - a.start_iter < a.timeline_iters && g < 128;
    long long tt[4] = {0, 0, 0, 0};
    if (active && !head && u >= uo_lo - (slack - 1) && u <= uo_hi + (slack - 1)) {
      if (tstamp) tt[0] = (long long)now_ticks();
      double tl = nbl ? thL[lane] : 0.0, tr = nbr ? thR[lane] : 0.0;
      if (HALO && hdir != 0) {  // the hosted halo head's theta^it: fold the four row-group partials
        double pq[4] = {hst[256 + lane], hst[320 + lane], hst[384 + lane], hst[448 + lane]};
        const double y = quad_reduce(pq);
        const double th_h = in ? y : 0.0;
        hst[lane] = th_h;  // read by the next head phase (after this phase's barrier)
        if (hdir > 0) tr = th_h;
        else tl = th_h;
      }
      if ((rl || rr) && !poll_remote(rslot, it, tl, tr) && lane == 0) abort_lds = 1;  // other ranks' heads' theta^it
      double r = bb - mu;
      if (has_l) r = r + rho * tl;
      if (has_r) r = r + rho * tr;
      if (tstamp) {
        asm volatile("" ::"v"(r));
        tt[1] = (long long)now_ticks();
      }
      const double tn = solve(r);
      if (tstamp) {
        asm volatile("" ::"v"(tn));
        tt[2] = (long long)now_ticks();
      }
      double m = mu;
      if (has_l) m = m - rho * (tl - tn);
      if (has_r) m = m + rho * (tn - tr);
      mu = m;
      th = tn;
      if (rpush && in) push_remote(rslot, it);  // first: the other rank's next head phase waits on it
      thS[u * 64 + lane] = th;
      if (owned && in && xnext) publish(it);
      ring_defer = ring_post;
      if (a.rres && owned) {  // K4 primal residual of the tail's two edges (after the publish)
        double rp = 0.0;
        if (in && has_l) rp = fma(tl - tn, tl - tn, rp);
        if (in && has_r) rp = fma(tn - tr, tn - tr, rp);
        const double rs = wave_sum_f64(rp);
        if (lane == 0 && it - 1 < a.max_iter) a.rres[(long)(it - 1) * n + w] = rs;
      }
      if (tstamp) tt[3] = (long long)now_ticks();
    } else if (active && owned && in) {  // heads: theta^it and the (still pending) mu are final
      if (xnext) publish(it);
      if (ring_post) put_granule<SYS>(local, rtab, ring_p + rslot * ring_slot_bytes, make_tag(a.epoch, it), th);
    }
    if (TL && g < 8 && it - a.start_iter < a.timeline_iters && lane == 0) {
      const long long t_end = (long long)now_ticks();  // this wave's tail-phase work done
      a.timeline[((long)(160 + g * MAXW + v) * a.timeline_iters + (it - a.start_iter)) * 8] = t_end;
    }
    if (!(TL && (a.dbg & 1)) && dec_wave && !(active && !head) && lane == 0 && it + 1 - a.start_iter >= a.lag) {
      const int jdec = it + 1 - a.lag;
      const unsigned tj = make_tag(a.epoch, jdec);
      // loaded during the previous iteration's tail phase: its L2 round trip (~0.7 us) is off the
      // critical path; a decision that was not yet published then is re-polled here
      unsigned long long dv = dv_pref;
      if ((unsigned)(dv >> 32) != tj) dv = load_dec<SYS>(&a.decg[dslot]);
      for (int spin = 0; (unsigned)(dv >> 32) != tj; ++spin) {
        if ((spin & 7) == 7 && now_ticks() > deadline) {
          abort_lds = 1;
          break;
        }
        GADMM_POLL_PAUSE();
        dv = load_dec<SYS>(&a.decg[dslot]);
      }
      const unsigned code = (unsigned)(dv & 0xffffffffu);
      if (code && (unsigned)(dv >> 32) == tj) {
        stop_lds = (int)code;
        stop_iter_lds = jdec;
      }
      dv_pref = load_dec<SYS>(&a.decg[dslot + 1 == a.ring ? 0 : dslot + 1]);
    }
    lds_barrier();
    if (tstamp && lane == 0) {
      long long* tl = a.timeline + ((long)(128 + g) * a.timeline_iters + (it - a.start_iter)) * 8;
      for (int q = 0; q < 4; ++q) tl[q] = tt[q];
      tl[4] = (long long)now_ticks();
    }
    if (stamp && lane == 0) {
      long long* tl = a.timeline + ((long)g * a.timeline_iters + (it - a.start_iter)) * 8;
      for (int q = 0; q < 5; ++q) tl[q] = ts[q];
      tl[5] = (long long)now_ticks();
      tl[6] = ts[6];
      tl[7] = ts[7];
    }
    if (abort_lds || stop_lds) {
      ++it;  // the next iteration to run
      break;
    }
  }

  if (ring_defer)  // the last iteration's tails (it was advanced past it on a stop)
    put_granule<SYS>(local, rtab, ring_p + ((it - 1) % a.ring) * ring_slot_bytes, make_tag(a.epoch, it - 1), th);
  if (owned && in) {
    a.theta[(long)w * d + lane] = th;
    a.mu[(long)li * d + lane] = mu;
  }
  if (threadIdx.x == 0) {
    if (abort_lds) {
      a.ctl->done = 4;
    } else if (g == 0 && stop_lds) {
      a.ctl->done = stop_lds;
      a.ctl->conv_iter = stop_iter_lds;
      a.ctl->iter = it;
      a.ctl->pending = 1;
      a.ctl->monitored = stop_iter_lds;
    } else if (g == 0 && hard_stopped) {  // done / conv_iter come from the monitor
      a.ctl->iter = it;
      a.ctl->pending = 1;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Paired-wave variant (PW = 2, opt-in: GADMM_BLOCK_PW=2): a workgroup of PWW = 8 waves computes up to 16 chain positions, wave
// v the adjacent pair (2v, 2v + 1) = one head + one tail, with BOTH rows of (A + deg rho I)^{-1} in
// VGPRs (2 x 52 doubles at 2 waves per SIMD). Every phase then runs exactly one GEMV per wave, two
// per SIMD on all four SIMDs (the 12-wave kernel runs 2,2,1,1), and 16 positions allow k = 3
// (L = 4 owned + 2 x 6 halo): one cross-CU (or cross-GPU) exchange per 3 iterations instead of 2.
// Same arithmetic and stop protocol as chain_blocked_kernel (bit-identical traces).
constexpr int PWW = 8;            // waves per workgroup
constexpr int PCAP = 2 * PWW;     // computed positions per workgroup

template <int DB, bool SYS>
__global__ void __launch_bounds__(64 * PWW) chain_blocked_pair_kernel(PersistArgs a) {
  constexpr int QT = DB / 4;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int abort_lds, stop_lds, stop_iter_lds;
  const int d = a.d, n = a.n;
  const int lane = threadIdx.x & 63;
  const int v = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int k = a.blk_k, L = a.blk_len, H = 2 * a.blk_k;
  const bool multi = a.nranks > 1;
  const int seg_lo = multi ? a.seg_lo : 0, seg_hi = multi ? a.seg_hi : n - 1;
  const int nseg = seg_hi - seg_lo + 1;
  const int W = (nseg + L - 1) / L;
  const int Wo = (nseg + PWW - 1) / PWW;
  const unsigned long long deadline = now_ticks() + (unsigned long long)a.timeout_ticks;
  const __amdgpu_buffer_rsrc_t rob = rsrc_of(a.objg);
  const __amdgpu_buffer_rsrc_t rtab = rsrc_of(a.blk_tab);
  if (threadIdx.x == 0) {
    abort_lds = 0;
    stop_lds = 0;
    stop_iter_lds = 0;
  }
  lds_barrier();
  if ((int)blockIdx.x == W + Wo) {
    blocked_monitor<SYS, false>(a, lds, v, lane, deadline, rob, (int)blockIdx.x);
    return;
  }
  const long ring_base = 2L * n * 2 * d;
  if ((int)blockIdx.x >= W) {
    const int q = seg_lo + ((int)blockIdx.x - W) * PWW + v;
    if (q <= seg_hi) blocked_objective<QT, SYS>(a, lds, v, lane, q, deadline, rob, rtab);
    return;
  }

  // ---------------------------------------------------------------------- worker workgroup
  const int g = blockIdx.x;
  const int s0 = seg_lo + g * L, e0 = min(seg_hi + 1, s0 + L) - 1;  // owned chain positions [s0, e0]
  const int ra = max(0, s0 - H), rb = min(n - 1, e0 + H);
  const int nv = rb - ra + 1;
  // this wave's head / tail local positions (ra + u is a head iff even)
  const int uA = 2 * v;
  const bool aHead = ((ra + uA) & 1) == 0;
  const int uH = aHead ? uA : uA + 1, uT = aHead ? uA + 1 : uA;
  const bool actH = uH < nv, actT = uT < nv;
  const int pH = ra + uH, pT = ra + uT;
  const bool ownH = actH && pH >= s0 && pH <= e0, ownT = actT && pT >= s0 && pT <= e0;
  const PhaseSlot slH = a.slots[actH ? pH : 0], slT = a.slots[actT ? pT : 0];
  const bool hlH = actH && slH.left >= 0, hrH = actH && slH.right >= 0;
  const bool hlT = actT && slT.left >= 0, hrT = actT && slT.right >= 0;
  const double rho = a.rho;
  const bool in = lane < d;
  // decision wave: one whose positions are both halo (no granule stores queue ahead of its load)
  int vdec = 0;
  for (int vv = PWW - 1; vv >= 0; --vv) {
    const int pa = ra + 2 * vv, pb = pa + 1;
    if (2 * vv + 1 < nv && (pa < s0 || pa > e0) && (pb < s0 || pb > e0)) vdec = vv;
  }
  const bool dec_wave = v == vdec;

  double* thS = lds;                        // [PCAP][64] theta of every computed position
  double* bbS = thS + PCAP * 64;            // [PCAP][64] b of every computed position
  double* myx = bbS + PCAP * 64 + v * QSTAGE;  // [PWW][QSTAGE] quad GEMV staging
  const bool nblH = hlH && uH > 0, nbrH = hrH && uH + 1 < nv;
  const bool nblT = hlT && uT > 0, nbrT = hrT && uT + 1 < nv;

  double MH[3][QT], MT[3][QT], M3[QT];  // paired layout: rows 48..51 of both in one shared block
  quad_load_pair<QT>(MH, MT, M3,
                     a.Minv + ((long)slH.li * a.nvar + a.deg_to_var[(int)hlH + (int)hrH]) * (long)d * d,
                     a.Minv + ((long)slT.li * a.nvar + a.deg_to_var[(int)hlT + (int)hrT]) * (long)d * d, d, actH,
                     actT);
  double thH = (actH && in) ? a.theta[(long)slH.gid * d + lane] : 0.0;
  double muH = (actH && in) ? a.mu[(long)slH.li * d + lane] : 0.0;
  double thT = (actT && in) ? a.theta[(long)slT.gid * d + lane] : 0.0;
  double muT = (actT && in) ? a.mu[(long)slT.li * d + lane] : 0.0;
  if (actH) {
    thS[uH * 64 + lane] = thH;
    bbS[uH * 64 + lane] = in ? a.b[(long)slH.li * d + lane] : 0.0;
  }
  if (actT) {
    thS[uT * 64 + lane] = thT;
    bbS[uT * 64 + lane] = in ? a.b[(long)slT.li * d + lane] : 0.0;
  }
  int pending = a.pending_in;
  lds_barrier();

  auto publish = [&](int j, int p, double th, double mu) {
    const unsigned tag = make_tag(a.epoch, j + 1);
    const int base = (((((j + 1 - a.start_iter) / k) & 1) * n + p) * 2) * d;
    store_granule<SYS>(rtab, (base + lane) * 16, tag, th);
    store_granule<SYS>(rtab, (base + d + lane) * 16, tag, mu);
    for (int q = 0; q < a.blk_npeer; ++q)
      if (p >= a.blk_peer_lo[q] && p <= a.blk_peer_hi[q]) {
        const __amdgpu_buffer_rsrc_t rpe = rsrc_of(a.blk_peer_tab[q]);
        store_granule<SYS>(rpe, (base + lane) * 16, tag, th);
        store_granule<SYS>(rpe, (base + d + lane) * 16, tag, mu);
      }
  };
  unsigned long long dv_pref = 0;
  int it = a.start_iter;
  for (;; ++it) {
    if (it > a.max_iter + a.lag) break;
    // ---- halo exchange every k iterations: both of the wave's halo positions in one poll loop
    if (it > a.start_iter && (it - a.start_iter) % k == 0) {
      const bool needH = actH && !ownH, needT = actT && !ownT;
      if (needH || needT) {
        const unsigned tag = make_tag(a.epoch, it);
        const int bsel = ((it - a.start_iter) / k) & 1;
        const int baseH = ((bsel * n + pH) * 2) * d, baseT = ((bsel * n + pT) * 2) * d;
        double h0 = 0.0, h1 = 0.0, t0 = 0.0, t1 = 0.0;
        bool ok = true;
        for (int spin = 0;; ++spin) {
          bool g0 = true;
          if (in && needH) {
            g0 &= load_granule<SYS>(rtab, (baseH + lane) * 16, tag, &h0);
            g0 &= load_granule<SYS>(rtab, (baseH + d + lane) * 16, tag, &h1);
          }
          if (in && needT) {
            g0 &= load_granule<SYS>(rtab, (baseT + lane) * 16, tag, &t0);
            g0 &= load_granule<SYS>(rtab, (baseT + d + lane) * 16, tag, &t1);
          }
          if (__all(g0)) break;
          if ((spin & 7) == 7 && now_ticks() > deadline) {
            ok = false;
            break;
          }
          GADMM_POLL_PAUSE();
        }
        if (!ok && lane == 0) abort_lds = 1;
        if (needH) {
          thH = in ? h0 : 0.0;
          muH = in ? h1 : 0.0;
          thS[uH * 64 + lane] = thH;
        }
        if (needT) {
          thT = in ? t0 : 0.0;
          muT = in ? t1 : 0.0;
          thS[uT * 64 + lane] = thT;
        }
      }
      lds_barrier();
      if (abort_lds) break;
    }

    // ---- head phase: every wave solves its head
    if (actH) {
      const double tl = nblH ? thS[(uH - 1) * 64 + lane] : 0.0, tr = nbrH ? thS[(uH + 1) * 64 + lane] : 0.0;
      double m = muH;
      if (pending) {  // lazy end-of-iteration dual (reference order)
        if (hlH) m = m - rho * (tl - thH);
        if (hrH) m = m + rho * (thH - tr);
      }
      muH = m;
      double r = bbS[uH * 64 + lane] - m;
      if (hlH) r = r + rho * tl;
      if (hrH) r = r + rho * tr;
      const double y = quad_gemv_pair<QT>(MH, M3, 0, in ? r : 0.0, myx);
      thH = in ? y : 0.0;
      thS[uH * 64 + lane] = thH;
      if (ownH && in)
        store_granule<SYS>(rtab, (int)((ring_base + ((long)(it % a.ring) * n + pH) * d + lane) * 16),
                           make_tag(a.epoch, it), thH);
    }
    pending = 1;
    lds_barrier();

    // ---- tail phase: every wave solves its tail; owned heads publish at an exchange boundary
    const bool xnext = (it + 1 - a.start_iter) % k == 0;
    if (actT) {
      const double tl = nblT ? thS[(uT - 1) * 64 + lane] : 0.0, tr = nbrT ? thS[(uT + 1) * 64 + lane] : 0.0;
      double r = bbS[uT * 64 + lane] - muT;
      if (hlT) r = r + rho * tl;
      if (hrT) r = r + rho * tr;
      const double y = quad_gemv_pair<QT>(MT, M3, 1, in ? r : 0.0, myx);
      const double tn = in ? y : 0.0;
      double m = muT;
      if (hlT) m = m - rho * (tl - tn);
      if (hrT) m = m + rho * (tn - tr);
      muT = m;
      thT = tn;
      thS[uT * 64 + lane] = thT;
      if (ownT && in) {
        store_granule<SYS>(rtab, (int)((ring_base + ((long)(it % a.ring) * n + pT) * d + lane) * 16),
                           make_tag(a.epoch, it), thT);
        if (xnext) publish(it, pT, thT, muT);
      }
      if (a.rres && ownT) {  // K4 primal residual of the tail's two edges
        double rp = 0.0;
        if (in && hlT) rp = fma(tl - tn, tl - tn, rp);
        if (in && hrT) rp = fma(tn - tr, tn - tr, rp);
        const double rs = wave_sum_f64(rp);
        if (lane == 0 && it - 1 < a.max_iter) a.rres[(long)(it - 1) * n + slT.gid] = rs;
      }
    }
    if (ownH && xnext && in) publish(it, pH, thH, muH);  // theta^it and the (still pending) mu are final
    if (dec_wave && lane == 0 && it + 1 - a.start_iter >= a.lag) {
      const int jdec = it + 1 - a.lag;
      const unsigned tj = make_tag(a.epoch, jdec);
      unsigned long long dvv = dv_pref;  // prefetched one iteration ahead
      if ((unsigned)(dvv >> 32) != tj) dvv = load_dec<SYS>(&a.decg[jdec % a.ring]);
      for (int spin = 0; (unsigned)(dvv >> 32) != tj; ++spin) {
        if ((spin & 7) == 7 && now_ticks() > deadline) {
          abort_lds = 1;
          break;
        }
        GADMM_POLL_PAUSE();
        dvv = load_dec<SYS>(&a.decg[jdec % a.ring]);
      }
      const unsigned code = (unsigned)(dvv & 0xffffffffu);
      if (code && (unsigned)(dvv >> 32) == tj) {
        stop_lds = (int)code;
        stop_iter_lds = jdec;
      }
      dv_pref = load_dec<SYS>(&a.decg[(jdec + 1) % a.ring]);
    }
    lds_barrier();
    if (abort_lds || stop_lds) {
      ++it;
      break;
    }
  }

  if (ownH && in) {
    a.theta[(long)slH.gid * d + lane] = thH;
    a.mu[(long)slH.li * d + lane] = muH;
  }
  if (ownT && in) {
    a.theta[(long)slT.gid * d + lane] = thT;
    a.mu[(long)slT.li * d + lane] = muT;
  }
  if (threadIdx.x == 0) {
    if (abort_lds) {
      a.ctl->done = 4;
    } else if (g == 0 && stop_lds) {
      a.ctl->done = stop_lds;
      a.ctl->conv_iter = stop_iter_lds;
      a.ctl->iter = it;
      a.ctl->pending = 1;
      a.ctl->monitored = stop_iter_lds;
    }
  }
}

// out[b][e] = src[e] >= 0 ? M[b][src[e]] : 0 -- the lane-major inverse image of the dynamic mode
// (engine/chain_engine.py:quad_pad_image) rebuilt in place after a refresh, one launch
__global__ void __launch_bounds__(256) pad_image_kernel(const double* __restrict__ M, long mstride,
                                                        const long long* __restrict__ src, long n_el, int batch,
                                                        double* __restrict__ out) {
  const long tot = n_el * batch;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < tot; e += (long)gridDim.x * 256) {
    const long b = e / n_el, k = e - b * n_el;
    const long long s = src[k];
    out[e] = s >= 0 ? M[b * mstride + s] : 0.0;
  }
}

extern "C" {

// Pick (k, L) for n workers; returns the number of worker workgroups, 0 if not applicable.
int gadmm_chain_blocked_plan(int n, int d, int want_k, int* k_out, int* len_out) {
  if (d > 52 || n < 2) return 0;  // DB = 64 rows spill at 3 waves per SIMD: the per-worker kernel covers d <= 64
  int k = want_k > 0 ? want_k : 2;
  int len = MAXW - 4 * k;
  while (len < 1 && k > 1) {
    --k;
    len = MAXW - 4 * k;
  }
  if (len < 1) return 0;
  // Owned positions per workgroup: the fewest whose launch (W worker + objective + monitor
  // workgroups, one per CU) still fits on ONE XCD, so it can be packed there (PersistArgs::xcd).
  // With the halo GEMVs skipped where unused, a shorter segment means lighter phases: at N = 24,
  // L = 1 / 2 / 4 ran 1.94 / 1.98 / 2.07 ms (profiles/r02_halo_skip).
  int cus_xcd = 32;
  const int cus = gadmm_cu_count();
  if (cus >= 8) cus_xcd = cus / 8;
  for (int l = 1; l < len; ++l)
    if ((n + l - 1) / l + (n + MAXW - 1) / MAXW + 1 <= cus_xcd) {
      len = l;
      break;
    }
  if (const char* e = getenv("GADMM_BLOCK_L")) {  // owned positions per workgroup (tuning runs)
    const int want_len = atoi(e);
    if (want_len >= 1 && want_len <= MAXW - 4 * k) len = want_len;
  }
  if (len > n) len = n;
  const int W = (n + len - 1) / len;
  if (W + (n + MAXW - 1) / MAXW + 1 > 256) return 0;
  *k_out = k;
  *len_out = len;
  return W;
}

// Plan with the wave layout: pw = 1 (default: the 12-wave kernel, up to 12 positions per workgroup,
// k = 2) or pw = 2 (GADMM_BLOCK_PW=2 or want_pw = 2: the paired 8-wave kernel, up to 16 positions,
// k = 3). Measured on MI355X (profiles/r01c_pair_layout): pw = 2 exchanges a third less often but
// its iteration is ~0.3 us longer (255 VGPRs, SGPR spills, the decision poll on a computing wave),
// 2.80 vs 2.40 ms per E1 solve on one GPU and 3.58 vs 3.02 ms in the 2-rank rehearsal.
int gadmm_chain_blocked_plan2(int n, int d, int want_k, int want_pw, int* k_out, int* len_out, int* pw_out) {
  int pw = want_pw;
  if (pw <= 0) {
    const char* e = getenv("GADMM_BLOCK_PW");
    pw = (e && e[0] == '2') ? 2 : 1;
  }
  if (pw == 1) {
    *pw_out = 1;
    return gadmm_chain_blocked_plan(n, d, want_k, k_out, len_out);
  }
  if (d > 52 || n < 2) return 0;
  int k = want_k > 0 ? want_k : 3;
  int len = PCAP - 4 * k;
  while (len < 1 && k > 1) {
    --k;
    len = PCAP - 4 * k;
  }
  if (len < 1) return 0;
  if (const char* e = getenv("GADMM_BLOCK_L")) {
    const int want_len = atoi(e);
    if (want_len >= 1 && want_len < len) len = want_len;
  }
  if (len > n) len = n;
  const int W = (n + len - 1) / len;
  if (W + (n + PWW - 1) / PWW + 1 > 256) return 0;
  *k_out = k;
  *len_out = len;
  *pw_out = 2;
  return W;
}

// Row length of PersistArgs::minv_pad for dimension d (the kernel instantiation's DB): the padded
// inverse image is [n_local][nvar][64][pad_dim].
int gadmm_chain_blocked_pad_dim(int d) { return d <= 32 ? 32 : 52; }
// Doubles per matrix of the lane-major image (quad_load_image): 4 x 64 x QT rounded up to even.
long gadmm_chain_blocked_pad_len(int d) {
  const int qt = gadmm_chain_blocked_pad_dim(d) / 4;
  return 512L * ((qt + 1) / 2);
}
// Epochs one launch of the blocked kernel's dynamic mode can take (its tables are staged in LDS).
int gadmm_chain_blocked_max_epochs() { return EPL; }

// The lane-major image of `batch` matrices (mstride doubles apart) into out [batch][n_el]: src[k] = the
// element index read for image slot k, < 0 for a zero slot (engine/chain_engine.py:quad_pad_image).
int gadmm_pad_image_f64(const double* M, long mstride, const long long* src, long n_el, int batch, double* out,
                        hipStream_t st) {
  if (!M || !src || !out || n_el < 1 || batch < 1) {
    gadmm_set_error("pad_image: bad arguments");
    return -1;
  }
  const long tot = n_el * batch;
  const int grid = (int)((tot + 255) / 256 < 4096 ? (tot + 255) / 256 : 4096);
  hipLaunchKernelGGL(pad_image_kernel, dim3(grid), dim3(256), 0, st, M, mstride, src, n_el, batch, out);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// Plan of the data-local multi-GPU mode for a segment of nseg positions: one workgroup computing the
// whole segment when it fits the 12 waves (no intra-rank exchange at all: k = 2^20 never comes), else
// the one-GPU plan inside the segment (k = 2, owned runs of L, halos clipped at the segment edges).
int gadmm_chain_blocked_plan_dl(int nseg, int d, int want_k, int* k_out, int* len_out) {
  if (d > 52 || nseg < 1) return 0;
  // GADMM_DL_PLAN=blocked (A/B): the one-GPU plan inside the segment even when one workgroup fits it
  const char* e = getenv("GADMM_DL_PLAN");
  const bool force_blocked = e && e[0] == 'b' && nseg >= 2;
  if (nseg <= MAXW && !force_blocked) {
    *k_out = 1 << 20;
    *len_out = nseg;
    return 1;
  }
  return gadmm_chain_blocked_plan(nseg, d, want_k, k_out, len_out);
}

long gadmm_chain_blocked_lds(int d, int len) {
  (void)d;
  (void)len;
  return (long)(MAXW * 64 + MAXW * QSTAGE) * 8;
}

// Granules of the blk_tab buffer: exchange table [2][n][2][d] + theta ring [ring][n][d]
// (+ the D-GADMM epoch table [2][n][2][d]: gadmm_chain_blocked_tab_granules_dyn).
long gadmm_chain_blocked_tab_granules(int n, int d, int ring) { return 2L * n * 2 * d + (long)ring * n * d; }
long gadmm_chain_blocked_tab_granules_dyn(int n, int d, int ring) { return 4L * n * 2 * d + (long)ring * n * d; }

long gadmm_resident_capacity(const void* fn, int threads, size_t shm);  // chain_persistent.hip
int gadmm_xcd_mode(const PersistArgs* a, int blocks, long cap_total);  // chain_persistent.hip
unsigned gadmm_next_xtag();  // chain_persistent.hip

int gadmm_chain_blocked_launch(const PersistArgs* args, hipStream_t st) {
  const PersistArgs& a = *args;
  const bool multi = a.nranks > 1;
  const bool dl = a.blk_dl != 0;
  if (dl) {  // data-local mode: SYS scope, 12-wave layout, static chain, every computed range within MAXW
    const int nseg_dl = a.seg_hi - a.seg_lo + 1;
    const int W_dl = nseg_dl > 0 && a.blk_len > 0 ? (nseg_dl + a.blk_len - 1) / a.blk_len : 0;
    const int nhalo = a.dl_halo ? (int)(a.seg_lo > 0 && a.seg_lo % 2 == 1) + (int)(a.seg_hi < a.n - 1 && a.seg_hi % 2 == 1) : 0;
    // one workgroup: segment + halo heads, or (hosted) a full segment whose one halo head the tails run
    const bool hosted_dl = a.dl_halo && nseg_dl + nhalo > MAXW;
    const long span = W_dl == 1 ? (hosted_dl ? nseg_dl : nseg_dl + nhalo) : (long)a.blk_len + 4L * a.blk_k;
    if (hosted_dl && (nhalo != 1 || nseg_dl < 8)) {
      gadmm_set_error("blocked chain kernel (data-local halo): a hosted halo needs one hosted side and >= 4 tails");
      return -1;
    }
    if (!multi || !a.sys_scope || a.blk_pw != 1 || a.n_epochs != 0 || a.blk_npeer != 0 || a.blk_k < 1 ||
        a.blk_len < 1 || nseg_dl < 1 || span > MAXW || (W_dl > 1 && a.ring < 2 * a.blk_k + 4) ||
        (a.seg_lo > 0 && !a.dl_tab[0]) || (a.seg_hi < a.n - 1 && !a.dl_tab[1]) ||
        (a.dl_halo && (W_dl != 1 || nseg_dl < 2 || a.d > 52))) {
      gadmm_set_error("blocked chain kernel (data-local): unsupported configuration (seg %d..%d, L=%d, k=%d)",
                      a.seg_lo, a.seg_hi, a.blk_len, a.blk_k);
      return -1;
    }
  }
  if (a.blk_k < 1 || a.blk_len < 1 || (!dl && a.blk_len + 4 * a.blk_k > (a.blk_pw == 2 ? PCAP : MAXW)) || a.d > 52 ||
      !a.blk_tab || !a.dec_push ||
      (!multi && (!a.has_monitor || a.n != a.n_local)) ||
      (multi && (a.seg_lo < 0 || a.seg_hi < a.seg_lo || a.seg_hi >= a.n || a.blk_npeer < 0 || a.blk_npeer > 8 ||
                 (a.blk_npeer > 0 && !a.blk_peer_tab) || a.start_iter != 1 || a.pending_in != 0 || !a.sys_scope))) {
    gadmm_set_error("blocked chain kernel: unsupported configuration");
    return -1;
  }
  if (a.lag < 1 || a.ring <= a.lag + 1 || a.start_iter + a.max_iter + a.lag >= (1 << 20)) {
    gadmm_set_error("blocked chain kernel: ring/lag/tag range");
    return -1;
  }
  const int nseg = multi ? a.seg_hi - a.seg_lo + 1 : a.n;
  const int W = (nseg + a.blk_len - 1) / a.blk_len;
  if (a.blk_pw == 2 && a.n_epochs == 0) {  // paired-wave kernel (static chains only)
    if (a.blk_len + 4 * a.blk_k > PCAP || a.timeline) {
      gadmm_set_error("blocked chain kernel (pw=2): L + 4k > %d or timeline requested", PCAP);
      return -1;
    }
    const int Wo2 = (nseg + PWW - 1) / PWW;
    const int blocks2 = W + Wo2 + (a.has_monitor ? 1 : 0);
    long lds2 = (long)(2 * PCAP * 64 + PWW * QSTAGE) * 8;
    if (lds2 < (long)a.n * 8) lds2 = (long)a.n * 8;
    const void* fn2 = a.sys_scope ? (a.d <= 32 ? (const void*)chain_blocked_pair_kernel<32, true>
                                               : (const void*)chain_blocked_pair_kernel<52, true>)
                                  : (a.d <= 32 ? (const void*)chain_blocked_pair_kernel<32, false>
                                               : (const void*)chain_blocked_pair_kernel<52, false>);
    const long cap2 = gadmm_resident_capacity(fn2, 64 * PWW, (size_t)lds2);
    if (blocks2 > cap2) {  // every workgroup must be resident together (they spin on each other)
      gadmm_set_error("blocked chain kernel: %d workgroups but only %ld can be resident", blocks2, cap2);
      return -2;
    }
    if (lds2 > 65536) GADMM_CHECK(hipFuncSetAttribute(fn2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2));
    void* kargs2[] = {const_cast<PersistArgs*>(&a)};
    GADMM_CHECK(hipLaunchKernel(fn2, dim3(blocks2), dim3(64 * PWW), kargs2, (size_t)lds2, st));
    GADMM_CHECK(hipGetLastError());
    return 0;
  }
  const int Wo = (nseg + MAXW - 1) / MAXW;
  const int blocks = W + Wo + (a.has_monitor ? 1 : 0);
  long lds = gadmm_chain_blocked_lds(a.d, a.blk_len);
  if (lds < (long)a.n * 8) lds = (long)a.n * 8;
  if (lds > 160 * 1024) {
    gadmm_set_error("blocked chain kernel: %ld B of LDS", lds);
    return -1;
  }
  const void* fn;
  const bool tl = a.timeline != nullptr;
  if (a.n_epochs > 0) {  // D-GADMM in one launch: one GPU, 12-wave layout, no instrumentation
    if (multi || tl || a.sys_scope || !a.epoch_start || !a.ep_slots || !a.ep_pos || !a.minv_pad || !a.ep_flush ||
        a.hard_stop < 0 || (a.hard_stop > 0 && a.hard_stop < a.start_iter) || a.n_epochs > EPL) {
      gadmm_set_error("blocked chain kernel: dynamic epochs need one GPU, epoch tables (at most %d epochs per "
                      "launch), the padded inverse image (gadmm_chain_blocked_pad_len), no timeline", EPL);
      return -1;
    }
    lds = gadmm_chain_blocked_lds(a.d, a.blk_len) + DYN_LDS_BYTES;  // + the staged epoch tables
    fn = a.d <= 32 ? (const void*)chain_blocked_kernel<32, false, false, true>
                   : (const void*)chain_blocked_kernel<52, false, false, true>;
  } else if (a.sys_scope && dl && a.dl_halo) {
    if (tl) {
      gadmm_set_error("blocked chain kernel: no timeline build of the data-local halo mode");
      return -1;
    }
    fn = a.d <= 32 ? (const void*)chain_blocked_kernel<32, true, false, false, true>
                   : (const void*)chain_blocked_kernel<52, true, false, false, true>;
    lds += (long)(HIMG52 + 512) * 8;  // the hosted halo head's inverse image + state (segment + halo > MAXW)
  } else if (a.sys_scope) {
    if (tl) fn = a.d <= 32 ? (const void*)chain_blocked_kernel<32, true, true> : (const void*)chain_blocked_kernel<52, true, true>;
    else fn = a.d <= 32 ? (const void*)chain_blocked_kernel<32, true, false> : (const void*)chain_blocked_kernel<52, true, false>;
  } else {
    if (tl) fn = a.d <= 32 ? (const void*)chain_blocked_kernel<32, false, true> : (const void*)chain_blocked_kernel<52, false, true>;
    else fn = a.d <= 32 ? (const void*)chain_blocked_kernel<32, false, false> : (const void*)chain_blocked_kernel<52, false, false>;
  }
  const long cap = gadmm_resident_capacity(fn, 64 * MAXW, (size_t)lds);
  if (blocks > cap) {  // every workgroup must be resident together (they spin on each other)
    gadmm_set_error("blocked chain kernel: %d workgroups but only %ld can be resident", blocks, cap);
    return -2;
  }
  const int xcd = gadmm_xcd_mode(&a, blocks, cap);
  const int grid = xcd > 0 ? 8 * blocks : blocks;
  if (lds > 65536) GADMM_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  PersistArgs ka = a;
  {
    const char* e = getenv("GADMM_BLK_DBG");  // experiment bits: 1 no stop polling, 2 no objective ring stores
    ka.dbg = e ? atoi(e) : 0;
  }
  ka.xcd = xcd;
  ka.xtag = (int)gadmm_next_xtag();  // fresh placement-check tag: no memset of xchk
  void* kargs[] = {&ka};
  GADMM_CHECK(hipLaunchKernel(fn, dim3(grid), dim3(64 * MAXW), kargs, (size_t)lds, st));
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"
