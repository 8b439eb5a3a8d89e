"""Temporally blocked GADMM across GPUs (one process per GPU, xGMI fabric).

Each rank owns a contiguous chain segment [seg_lo, seg_hi] and runs ``chain_blocked_kernel<SYS>``
(csrc/kernels/chain_blocked.hip). Two modes:

* ``data_local=True`` (the multi-GPU default, ``engine/multigpu.py``): the rank holds ONLY its own
  workers' shards. Its workgroups compute its segment, temporally blocked inside it exactly as on one
  GPU (one workgroup for the whole segment when it fits 12 waves, else owned runs + halos clipped at
  the segment edges, one intra-rank exchange per k iterations). The two positions at the segment
  edges exchange theta with the neighbouring ranks' edge positions every phase -- the owner pushes
  theta^j into the neighbour GPU's theta ring right after its solve, the reader polls its own ring --
  which is the reference's exchange (group_ADMM_closedForm.m:18-27, 62-70): theta only, d doubles per
  boundary per phase, no mu, no shard. Payload per solve: 2 (ranks - 1) d 8 B per iteration.
* ``data_local=False`` (opt-in ``--engine replicated-halo``): the workgroups also compute a halo of
  H = 2k positions of the neighbouring ranks (whose Gram / inverse come from their shards, held
  here: ``replicated_shard_bytes``) and every k iterations each rank pushes the (theta, mu) of its
  owned workers into the exchange tables of the peers whose computed range contains them: one
  cross-GPU hand-off per k iterations instead of two per iteration, at the price of the shards.

Objective waves on every rank evaluate f_n of the owned workers and push them to rank 0's monitor
ring; rank 0's monitor pushes the stop decision into every rank's ring (as in the per-worker fabric,
parallel/xgmi.py). Hand-offs are tagged granules salted per solve, so correctness never depends on
timing; every spin has a deadline and a stalled peer surfaces as ``done == 4`` (callers fall back).
Identity chain (the static GADMM of the headline benchmark).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops import native
from ..ops.linalg import gram, spd_inverse
from ..parallel.topology import Placement
from ..parallel.xgmi import _Buf, device_identity, preflight
from ..utils.env import getenv


MAXW = 12  # waves (computed positions) per workgroup of chain_blocked_kernel


def halo_heads(lo: int, hi: int, n: int) -> list:
    """The other ranks' boundary heads a rank owning chain positions [lo, hi] solves in the halo mode:
    the neighbour of each boundary of its segment whose near side is a tail (odd position)."""
    return ([lo - 1] if lo > 0 and lo % 2 == 1 else []) + ([hi + 1] if hi < n - 1 and hi % 2 == 1 else [])


def dl_halo_eligible(segs, n: int, d: int) -> bool:
    """Whether the data-local halo mode can run on every rank: more than one rank, every segment >= 2
    positions and within one 12-wave workgroup. A halo head that does not fit a wave of its own (24
    workers on 2 ranks: 12 + 1) is hosted by the segment's tails (chain_blocked.hip: four tail waves
    run its row groups in the head phase, from its inverse in LDS; one hosted head per segment)."""
    def fits(lo, hi):
        nh = len(halo_heads(lo, hi, n))
        # one wave per position; or hosted: one halo head run by >= 4 of the segment's tails
        return hi - lo + 1 + nh <= MAXW or (hi - lo + 1 <= MAXW and nh == 1 and hi - lo + 1 >= 8)

    return (len(segs) > 1 and d <= 52 and all(hi - lo + 1 >= 2 for lo, hi in segs)
            and all(fits(lo, hi) for lo, hi in segs))


def dl_halo_hosted(lo: int, hi: int, n: int) -> bool:
    """Whether the segment [lo, hi] runs its halo heads hosted (segment + halo heads > 12 waves)."""
    return hi - lo + 1 + len(halo_heads(lo, hi, n)) > MAXW


def replicated_plans(n_total: int, placement: Placement, d: int, max_k: int = 6) -> List[Tuple[int, int]]:
    """Every (k, pw) the replicated-halo kernel admits for this chain (``gadmm_chain_blocked_plan2``
    with want_k = 1..max_k for both wave layouts, deduplicated): the engine tournament times each. A
    larger k exchanges (theta, mu) once per k iterations -- fewer cross-GPU hops per iteration -- at the
    cost of a 2k-position halo (more replicated shards, more halo GEMVs)."""
    lib = native.require()
    segs = [placement.local_workers(r) for r in range(placement.nranks)]
    nseg = max(len(s) for s in segs)
    out: List[Tuple[int, int]] = []
    for pw in (1, 2):
        for k in range(1, max_k + 1):
            kk, ll, pp = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(1)
            if int(lib.gadmm_chain_blocked_plan2(nseg, int(d), k, pw, ctypes.byref(kk), ctypes.byref(ll),
                                                 ctypes.byref(pp))) <= 0:
                continue
            if kk.value == k and pp.value == pw and (k, pw) not in out:
                out.append((k, pw))
    return out


class BlockedXgmiEngine:
    LAG = 8

    def __init__(self, X_all: torch.Tensor, y_all: torch.Tensor, n_total: int, placement: Placement, rank: int,
                 rho: float, obj0: float, tol: float, max_iter: int, device: torch.device, group=None,
                 want_k: int = 0, data_local: bool = False, dl_halo: Optional[bool] = None,
                 stream: Optional[torch.cuda.Stream] = None, want_pw: int = 0):
        """Collective over ``group``. ``data_local=False``: ``X_all`` / ``y_all`` hold the shards of at
        least this rank's computed range (indexable by global worker id); only those rows are read.
        ``data_local=True``: ``X_all`` / ``y_all`` are this rank's own shards, in segment order.
        ``dl_halo`` (data-local only; None: on unless GADMM_DL_HALO=0, when every segment has >= 2
        positions and fits one workgroup): the one-position halo mode -- at each rank boundary whose near
        side is a tail, this rank also holds the other rank's boundary head's shard (fetched once here
        from its owner) and solves it on one more wave, so only one cross-rank hop per iteration is on
        the critical cycle (chain_blocked.hip, PersistArgs::dl_halo). Needs every segment within one
        12-wave workgroup; a halo head beyond the 12 waves (2 ranks at 24 workers) is hosted by the
        boundary tail next to it."""
        self.lib = native.require()
        self.rank, self.nranks, self.device = rank, placement.nranks, device
        self.n, self.d = int(n_total), int(X_all.shape[2])
        self.rho, self.obj0, self.tol, self.max_iter = float(rho), float(obj0), float(tol), int(max_iter)
        self.data_local = bool(data_local)
        mine = placement.local_workers(rank)
        self.seg_lo, self.seg_hi = min(mine), max(mine)
        if mine != list(range(self.seg_lo, self.seg_hi + 1)):
            raise ValueError("blocked xgmi engine needs contiguous segments")
        segs = [(min(placement.local_workers(r)), max(placement.local_workers(r))) for r in range(self.nranks)]
        kk, ll, pp = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(1)
        if self.data_local:
            nseg = self.seg_hi - self.seg_lo + 1
            if int(X_all.shape[0]) != nseg:
                raise ValueError("data-local blocked engine: %d shards for a %d-position segment"
                                 % (int(X_all.shape[0]), nseg))
            if int(self.lib.gadmm_chain_blocked_plan_dl(nseg, self.d, int(want_k), ctypes.byref(kk),
                                                        ctypes.byref(ll))) <= 0:
                raise RuntimeError("data-local blocked engine: no plan for d=%d, %d positions" % (self.d, nseg))
        else:
            nseg = max(hi - lo + 1 for lo, hi in segs)
            if int(self.lib.gadmm_chain_blocked_plan2(nseg, self.d, int(want_k), int(want_pw), ctypes.byref(kk),
                                                      ctypes.byref(ll), ctypes.byref(pp))) <= 0:
                raise RuntimeError("blocked xgmi engine: no blocking plan for d=%d" % self.d)
            if want_k > 0 and kk.value != int(want_k):
                raise ValueError("blocked xgmi engine: k = %d is not admitted (plan gives k = %d, pw = %d)"
                                 % (want_k, kk.value, pp.value))
        self.k, self.L, self.pw = kk.value, ll.value, pp.value
        H = 0 if self.data_local else 2 * self.k
        self.H = H
        comp = [(max(0, lo - H), min(self.n - 1, hi + H)) for lo, hi in segs]
        self.ext_lo, self.ext_hi = comp[rank]
        self.halo = []  # data-local halo mode: the other ranks' boundary heads this rank solves too
        if self.data_local:
            ok_h = (dl_halo is not False and getenv("GADMM_DL_HALO", "1") != "0"
                    and self.L >= self.seg_hi - self.seg_lo + 1 and dl_halo_eligible(segs, self.n, self.d))
            if dl_halo and not ok_h:
                raise ValueError("data-local halo mode needs segments of >= 2 positions that fit one workgroup "
                                 "with their halo heads")
            self._halo_on = ok_h
            if ok_h:
                X_all, y_all = self._fetch_halo_shards(X_all, y_all, group)
        # stop-decision lag in iterations (GADMM_DL_LAG: A/B of the objective -> monitor -> decision
        # pipeline's slack; every rank must use the same value)
        self.LAG = int(getenv("GADMM_DL_LAG", str(self.LAG)))
        self.ring = self.LAG + 4
        torch.cuda.set_device(device)
        f64 = torch.float64
        ext = list(range(self.ext_lo, self.ext_hi + 1))
        if self.data_local:  # own shards (+ the halo heads' in the halo mode), in position order
            self.X = X_all.to(device).contiguous()
            self.y = y_all.to(device).contiguous()
        else:
            self.X = X_all[ext].to(device).contiguous()
            self.y = y_all[ext].to(device).contiguous()
        self.stream = stream if stream is not None else torch.cuda.Stream(device)
        with torch.cuda.stream(self.stream):
            self.A, self.b, self.yy = gram(self.X, self.y)
            self._inverses()
            self.theta = torch.zeros((self.n, self.d), dtype=f64, device=device)
            self.mu = torch.zeros((len(ext), self.d), dtype=f64, device=device)
            self.trace = torch.full((self.max_iter,), float("nan"), dtype=f64, device=device)
            self.ctl = torch.zeros((8,), dtype=torch.int32, device=device)
            # per-iteration decision clock (s_memrealtime, written by rank 0's monitor) when ``stamps``
            self.tstamp = torch.zeros((self.max_iter,), dtype=torch.int64, device=device)
            self.t0stamp = torch.zeros((1,), dtype=torch.int64, device=device)
            slots = []
            for p in range(self.n):  # position == worker id (identity chain); li indexes the ext arrays
                li = p - self.ext_lo if self.ext_lo <= p <= self.ext_hi else -1
                slots += [li, p, p - 1 if p > 0 else -1, p + 1 if p + 1 < self.n else -1]
            self.slots = torch.tensor(slots, dtype=torch.int32, device=device)
            self.pos = torch.arange(self.n, dtype=torch.int32, device=device)
        self.stream.synchronize()
        # ---- fabric: exchange table + theta ring (every rank), objective ring (rank 0), decision rings
        ng = int(self.lib.gadmm_chain_blocked_tab_granules(self.n, self.d, self.ring))
        self.tab = self.objg = self.decg = None
        self.opened = {}
        err = ""
        h = None
        try:
            self.tab = _Buf(self.lib, ng * 16)
            self.objg = _Buf(self.lib, self.ring * self.n * 16)
            self.decg = _Buf(self.lib, self.ring * 8)
            h = (bytes(self.tab.handle.raw), bytes(self.objg.handle.raw), bytes(self.decg.handle.raw))
        except Exception as e:  # pragma: no cover - box dependent
            err = "rank %d alloc: %s" % (rank, e)
        allh = [None] * self.nranks
        dist.all_gather_object(allh, (h, err, device_identity()), group=group)
        errs = [e for _, e, _ in allh if e]
        devs = [dv for _, _, dv in allh]
        ok = not errs
        self.peers: List[int] = []
        self.peer_ranges = []
        self.peer_ptrs: List[int] = []
        self.dl_ranks = [-1, -1]  # data-local: the ranks owning seg_lo - 1 / seg_hi + 1
        self.dl_ptrs = [0, 0]
        if self.data_local:
            owner = placement.owner
            if self.seg_lo > 0:
                self.dl_ranks[0] = int(owner[self.seg_lo - 1])
            if self.seg_hi < self.n - 1:
                self.dl_ranks[1] = int(owner[self.seg_hi + 1])
        if ok:
            try:
                touch = {q for q in self.dl_ranks if q >= 0} | ({0} if rank != 0 else set(range(self.nranks)))
                if not self.data_local:
                    touch |= {q for q in range(self.nranks)
                              if comp[q][1] >= self.seg_lo and comp[q][0] <= self.seg_hi}
                why = preflight(torch.cuda.current_device(), {q: devs[q] for q in touch if q != rank})
                if why:
                    raise RuntimeError("peer access pre-flight: " + why)
                for side, q in enumerate(self.dl_ranks):
                    if q >= 0:
                        self.dl_ptrs[side] = self._open(allh[q][0][0], ("tab", q)) if ("tab", q) not in self.opened \
                            else self.opened[("tab", q)].value
                for q in range(self.nranks):
                    if q == rank or self.data_local:
                        continue
                    lo, hi = comp[q]
                    if hi >= self.seg_lo and lo <= self.seg_hi:  # q computes some of my positions
                        self.peers.append(q)
                        self.peer_ranges.append((lo, hi))
                        self.peer_ptrs.append(self._open(allh[q][0][0], ("tab", q)))
                self.objg_mon = self.objg.ptr.value if rank == 0 else self._open(allh[0][0][1], ("objg", 0))
                self.dec_all = [self.decg.ptr.value if q == rank else self._open(allh[q][0][2], ("decg", q))
                                for q in range(self.nranks)] if rank == 0 else [self.decg.ptr.value]
            except Exception as e:  # pragma: no cover
                ok, err = False, str(e)
        flag = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64)
        dist.all_reduce(flag, group=group)
        if float(flag.item()) != 0.0:
            self.close()
            raise RuntimeError("blocked xgmi fabric failed on some rank (%s)" % ("; ".join(errs) or err or "remote"))
        if len(self.peers) > 8:
            self.close()
            raise RuntimeError("blocked xgmi engine: more than 8 peers")
        self.peer_tab_t = torch.tensor(self.peer_ptrs + [0], dtype=torch.int64, device=device)
        self.dec_push_t = torch.tensor(self.dec_all, dtype=torch.int64, device=device)
        self.epoch = 0
        self.stamps = False  # record the decision clock per iteration (entry runs: the time trace)
        if self.data_local:
            W = (self.seg_hi - self.seg_lo + self.L) // self.L
            hosted = self._halo_mode() and dl_halo_hosted(self.seg_lo, self.seg_hi, self.n)
            self.last_kernel = "blocked-dl%s(k=%s,L=%d,W=%d,nbr=%s)" % (
                ("-halo%s%s" % (self.halo, "-hosted" if hosted else "")) if self._halo_mode() else "",
                "inf" if W == 1 else self.k, self.L, W, self.dl_ranks)
        else:
            self.last_kernel = "blocked-xgmi(k=%d,L=%d,H=%d,pw=%d,peers=%s)" % (self.k, self.L, H, self.pw,
                                                                                self.peers)

    def _fetch_halo_shards(self, X_own: torch.Tensor, y_own: torch.Tensor, group):
        """Collective: the halo mode's one-time shard exchange. Every rank offers the shards of its
        boundary HEADS (a head at seg_lo > 0 / seg_hi < n - 1); a rank whose boundary position is a tail
        takes its neighbour's head. Returns this rank's ext-range shards (halo, own, halo) and sets
        ``ext_lo`` / ``ext_hi`` / ``halo``."""
        lo, hi, n = self.seg_lo, self.seg_hi, self.n
        offer = {}
        if lo > 0 and lo % 2 == 0:
            offer[lo] = (X_own[0].cpu().numpy(), y_own[0].cpu().numpy())
        if hi < n - 1 and hi % 2 == 0:
            offer[hi] = (X_own[-1].cpu().numpy(), y_own[-1].cpu().numpy())
        allo = [None] * self.nranks
        dist.all_gather_object(allo, offer, group=group)
        pool = {}
        for o in allo:
            pool.update(o)
        Xs, ys = [X_own.cpu()], [y_own.cpu()]
        for h in halo_heads(lo, hi, n):  # seg_lo / seg_hi is a tail: solve the neighbour rank's head too
            X_h, y_h = torch.from_numpy(pool[h][0]).unsqueeze(0), torch.from_numpy(pool[h][1]).unsqueeze(0)
            if h < lo:
                Xs.insert(0, X_h)
                ys.insert(0, y_h)
            else:
                Xs.append(X_h)
                ys.append(y_h)
            self.halo.append(h)
        self.ext_lo = lo - (1 if (lo - 1) in self.halo else 0)
        self.ext_hi = hi + (1 if (hi + 1) in self.halo else 0)
        return torch.cat(Xs).contiguous(), torch.cat(ys).contiguous()

    def _open(self, hbytes: bytes, key) -> int:
        p = ctypes.c_void_p()
        native.check(self.lib.gadmm_xgmi_open(ctypes.create_string_buffer(hbytes, 64), ctypes.byref(p)),
                     "xgmi_open %s" % (key,))
        self.opened[key] = p
        return p.value

    def _inverses(self, out: Optional[torch.Tensor] = None):
        sh = torch.tensor([self.rho, 2.0 * self.rho], dtype=torch.float64, device=self.device)
        if out is None:
            self.Minv = spd_inverse(self.A, sh)
        else:
            spd_inverse(self.A, sh, out=out, check_status=False)

    def refresh(self):
        """Recompute the Gram and cached inverses (the set-up of every solve)."""
        with torch.cuda.stream(self.stream):
            gram(self.X, self.y, out=(self.A, self.b, self.yy))
            self._inverses(out=self.Minv)

    def run(self, timeout_s: float = 20.0, timeline_iters: int = 0, dbg: int = 0):
        """Reset the state and solve; returns (iters, done, wall_ms). Collective in effect (every rank
        must run it; the kernels hand off to each other). ``timeline_iters > 0``: the instrumented
        kernel records s_memrealtime stamps (10 ns, one clock for the chip) of the first iterations
        into ``self.last_timeline`` (rows g: wave 0 of workgroup g [start, after exchange, -, -, after
        the head phase, after the tail phase, before / after its head solve]; rows 128 + g: the
        workgroup's tail wave MAXW/2 + ((dbg >> 4) & 7) [start, after its poll, after its solve, after
        its stores, after the phase barrier]); ``dbg``: PersistArgs::dbg experiment bits."""
        import time

        self.epoch = self.epoch % 4095 + 1
        pa = native.PersistArgs()
        pa.d, pa.n, pa.n_local, pa.start_iter, pa.max_iter = self.d, self.n, self.ext_hi - self.ext_lo + 1, 1, \
            self.max_iter
        pa.lag, pa.ring, pa.nvar, pa.obj_mode = self.LAG, self.ring, 2, 0
        pa.deg_to_var[0], pa.deg_to_var[1], pa.deg_to_var[2] = 0, 0, 1
        pa.pending_in, pa.has_monitor, pa.nranks, pa.sys_scope = 0, 1 if self.rank == 0 else 0, self.nranks, 1
        pa.epoch = self.epoch
        pa.rho, pa.obj0, pa.tol = self.rho, self.obj0, self.tol
        pa.timeout_ticks = int(timeout_s * 1e8)
        pa.slots, pa.pos = self.slots.data_ptr(), self.pos.data_ptr()
        pa.Minv, pa.A, pa.b, pa.yy = self.Minv.data_ptr(), self.A.data_ptr(), self.b.data_ptr(), self.yy.data_ptr()
        pa.theta, pa.mu = self.theta.data_ptr(), self.mu.data_ptr()
        pa.objg, pa.decg = self.objg_mon, self.decg.ptr.value
        pa.dec_push = self.dec_push_t.data_ptr()
        pa.trace, pa.ctl = self.trace.data_ptr(), self.ctl.data_ptr()
        pa.blk_k, pa.blk_len, pa.blk_pw = self.k, self.L, self.pw
        pa.blk_tab = self.tab.ptr.value
        pa.seg_lo, pa.seg_hi = self.seg_lo, self.seg_hi
        pa.blk_npeer = len(self.peers)
        for i, (lo, hi) in enumerate(self.peer_ranges):
            pa.blk_peer_lo[i], pa.blk_peer_hi[i] = lo, hi
        pa.blk_peer_tab = self.peer_tab_t.data_ptr()
        pa.blk_dl = 1 if self.data_local else 0
        pa.dl_halo = 1 if self._halo_mode() else 0
        pa.dl_tab[0], pa.dl_tab[1] = self.dl_ptrs[0] or None, self.dl_ptrs[1] or None
        pa.dbg = int(dbg)
        if self.stamps:
            pa.tstamp = self.tstamp.data_ptr()
        tl = None
        if timeline_iters > 0:
            tl = torch.zeros((256, int(timeline_iters), 8), dtype=torch.int64, device=self.device)
            pa.timeline, pa.timeline_iters = tl.data_ptr(), int(timeline_iters)
        with torch.cuda.stream(self.stream):
            self.theta.zero_()
            self.mu.zero_()
            self.ctl.zero_()
            if self.stamps:
                native.check(self.lib.gadmm_write_stamp(self.t0stamp.data_ptr(), self.stream.cuda_stream),
                             "write_stamp")
            t0 = time.perf_counter()
            native.check(self.lib.gadmm_chain_blocked_launch(ctypes.byref(pa), self.stream.cuda_stream),
                         "chain_blocked_launch")
            self.stream.synchronize()
            t1 = time.perf_counter()
        c = self.ctl.cpu().tolist()
        self.last_timeline = tl.cpu().numpy() if tl is not None else None
        if c[1] == 4:
            raise RuntimeError("blocked xgmi kernel timed out (hand-off never completed)")
        return c[2], c[1], (t1 - t0) * 1e3

    def exchange_bytes_per_solve(self, iters: int) -> int:
        """Payload this rank pushes over xGMI per solve (8 B per double; the granules on the wire carry
        16 B). Data-local: theta of each segment-edge worker to its other-rank neighbour, once per
        iteration (iterations 1..iters). Replicated halo: every k iterations, (theta, mu) of each owned
        worker that a peer computes, to that peer."""
        if self.data_local:
            return sum(1 for q in self.dl_ranks if q >= 0) * self.d * 8 * iters
        pushes = sum(1 for lo, hi in self.peer_ranges for p in range(self.seg_lo, self.seg_hi + 1) if lo <= p <= hi)
        return pushes * 2 * self.d * 8 * (iters // self.k)

    def monitor_bytes_per_solve(self, iters: int) -> int:
        """Stop-rule wire bytes leaving this rank: one 16-B objective granule per owned worker per
        iteration to rank 0's monitor (rank 0's own are local), and rank 0's 8-B decision to every
        other rank per iteration."""
        owned = self.seg_hi - self.seg_lo + 1
        return iters * (owned * 16 if self.rank != 0 else 8 * (self.nranks - 1))

    def _halo_mode(self) -> bool:
        """The halo mode is on for every rank together (a rank with no tail-side boundary holds no halo
        shard but still runs the halo kernel: its boundary heads stop pushing, their far neighbours push)."""
        return getattr(self, "_halo_on", False)

    def replicated_shard_bytes(self) -> int:
        """Bytes of OTHER ranks' shards this rank holds for its halo (X and y of the halo workers)."""
        if self.data_local:
            return len(self.halo) * int(self.X.shape[1]) * (self.d + 1) * 8
        halo = (self.ext_hi - self.ext_lo + 1) - (self.seg_hi - self.seg_lo + 1)
        return halo * int(self.X.shape[1]) * (self.d + 1) * 8

    def objective_trace(self, upto: int):
        return self.trace.cpu().numpy()[:upto]

    def time_trace(self, upto: int):
        """Seconds from the solve start to each iteration's stop decision (rank 0's monitor clock;
        needs ``stamps``; zeros on other ranks)."""
        import numpy as np
        t = self.tstamp[:upto].cpu().numpy().astype(np.int64)
        t0 = int(self.t0stamp.cpu().item())
        return np.maximum(t - t0, 0).astype(np.float64) / 1e8

    def close(self):
        for p in self.opened.values():
            self.lib.gadmm_xgmi_close(p)
        self.opened = {}
        for b in (self.tab, self.objg, self.decg):
            if b is not None:
                b.free()
        self.tab = self.objg = self.decg = None
