"""Python front-end of the persistent star-ADMM kernel (csrc/kernels/star_persistent.hip).

``standared_ADMM.m`` as one launch per GPU: every local worker (and the hub, worker
n-1, on the rank that owns it) is a resident wave holding its cached inverse and Gram in VGPRs; the
uploads (theta_n -> hub) and the broadcast (theta_hub -> every worker) are tagged granules, stored
device-initiated into the hub rank's / every rank's table; the stop rule runs on the device.
One GPU: the tables are plain device memory. Several GPUs: an ``XgmiFabric`` (parallel/xgmi.py)
supplies IPC-mapped fine-grained tables, and the same stores travel over xGMI.
"""
from __future__ import annotations

import ctypes
import time
from typing import Optional, Sequence

import numpy as np
import torch

from ..ops import native
from ..ops.linalg import gram, spd_inverse


class StarEngine:
    LAG = 4

    def __init__(self, X_loc: torch.Tensor, y_loc: torch.Tensor, local_ids: Sequence[int], n_total: int,
                 rho: float, obj0: float, tol: float, max_iter: int, hub_rank: int = 0, fabric=None,
                 precomputed=None):
        """``X_loc`` (n_local, m, d): this rank's shards (local order = ``local_ids``); the hub is worker
        ``n_total - 1``, owned by ``hub_rank``. ``fabric``: an ``XgmiFabric`` over every rank (multi-GPU)."""
        self.lib = native.require()
        self.device = X_loc.device
        self.local = [int(w) for w in local_ids]
        self.n, self.d = int(n_total), int(X_loc.shape[2])
        self.rho, self.obj0, self.tol, self.max_iter = float(rho), float(obj0), float(tol), int(max_iter)
        self.fabric = fabric
        self.rank = fabric.rank if fabric is not None else 0
        self.nranks = fabric.nranks if fabric is not None else 1
        self.hub_rank = int(hub_rank)
        self.ring = self.LAG + 4
        self.stream = torch.cuda.Stream(self.device)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        dev, f64 = self.device, torch.float64
        nl, d = len(self.local), self.d
        with torch.cuda.stream(self.stream):
            if precomputed is not None:
                self.A, self.b, self.yy = precomputed
            else:
                self.A, self.b, self.yy = gram(X_loc.to(f64), y_loc.to(f64))
            self._shifts = torch.tensor([[(self.n - 1) * self.rho if w == self.n - 1 else self.rho]
                                         for w in self.local], dtype=f64, device=dev)
            self.Minv = spd_inverse(self.A, self._shifts)
            # theta, lam and the hub's lam table in ONE buffer: a solve's reset is one fill
            # (each part starts on a 256-byte boundary, as its own allocation would)
            seg = (nl * d + 31) // 32 * 32
            self._state = torch.zeros((2 * seg + self.n * d,), dtype=f64, device=dev)
            self.theta = self._state[: nl * d].view(nl, d)
            self.lam = self._state[seg: seg + nl * d].view(nl, d)
            self.lam_hub = self._state[2 * seg: 2 * seg + self.n * d].view(self.n, d)
            self.trace = torch.full((self.max_iter,), float("nan"), dtype=f64, device=dev)
            self.tstamp = torch.zeros((self.max_iter,), dtype=torch.int64, device=dev)
            self.t0stamp = torch.zeros((1,), dtype=torch.int64, device=dev)
            self.ctl = torch.zeros((8,), dtype=torch.int32, device=dev)
            self.gid = torch.tensor(self.local, dtype=torch.int32, device=dev)
            if fabric is None:
                self._thg = torch.zeros((self.n * d * 4,), dtype=torch.int32, device=dev)
                self._objg = torch.zeros((self.ring * self.n * 4,), dtype=torch.int32, device=dev)
                self._decg = torch.zeros((self.ring,), dtype=torch.int64, device=dev)
                self.peer_thg = torch.tensor([self._thg.data_ptr()], dtype=torch.int64, device=dev)
                self.dec_push = torch.tensor([self._decg.data_ptr()], dtype=torch.int64, device=dev)
                self._ptrs = (self._thg.data_ptr(), self._objg.data_ptr(), self._decg.data_ptr())
                # XCD packing (one GPU; StarArgs::xcd): placement-check granules
                self._xchk = torch.zeros((256 * 4,), dtype=torch.int32, device=dev)
            else:
                self.peer_thg = torch.tensor(fabric.table_ptrs(), dtype=torch.int64, device=dev)
                self.dec_push = torch.tensor(fabric.dec_all if fabric.dec_all else [0], dtype=torch.int64,
                                             device=dev)
                self._ptrs = (fabric.thg.ptr.value, fabric.objg_mon, fabric.decg.ptr.value)
        self.stream.synchronize()
        self._epoch = 0
        self.last_kernel = "star-persistent"

    def refresh(self, X_loc: torch.Tensor, y_loc: torch.Tensor):
        """Recompute the set-up (Gram + cached inverses) from the raw shards, in place."""
        with torch.cuda.stream(self.stream):
            gram(X_loc, y_loc, out=(self.A, self.b, self.yy))
            spd_inverse(self.A, self._shifts, out=self.Minv, check_status=False)

    def _args(self, timeout_s: float) -> native.StarArgs:
        a = native.StarArgs()
        a.d, a.n, a.n_local, a.max_iter = self.d, self.n, len(self.local), self.max_iter
        a.lag, a.ring = self.LAG, self.ring
        a.has_monitor = 1 if self.rank == 0 else 0
        a.nranks, a.sys_scope = self.nranks, 1 if self.fabric is not None else 0
        a.hub_rank, a.my_rank = self.hub_rank, self.rank
        a.rho, a.obj0, a.tol = self.rho, self.obj0, self.tol
        a.timeout_ticks = int(timeout_s * 1e8)
        a.gid, a.Minv, a.A, a.b, a.yy = (self.gid.data_ptr(), self.Minv.data_ptr(), self.A.data_ptr(),
                                         self.b.data_ptr(), self.yy.data_ptr())
        a.theta, a.lam, a.lam_hub = self.theta.data_ptr(), self.lam.data_ptr(), self.lam_hub.data_ptr()
        a.thg, a.objg, a.decg = self._ptrs
        a.peer_thg, a.dec_push = self.peer_thg.data_ptr(), self.dec_push.data_ptr()
        a.trace, a.tstamp, a.ctl = self.trace.data_ptr(), self.tstamp.data_ptr(), self.ctl.data_ptr()
        if self.fabric is None:
            a.xchk, a.xcd = self._xchk.data_ptr(), 2
        return a

    def eligible(self) -> bool:
        if self.d > 64:
            return False
        blocks = len(self.local) + (1 if self.rank == 0 else 0)
        return blocks <= int(self.lib.gadmm_star_capacity(ctypes.byref(self._args(1.0))))

    def run(self, timeout_s: float = 20.0, timeline_iters: int = 0):
        """Reset and solve. Returns (iters, done, wall_ms). Collective across ranks (the kernels hand
        off to each other). ``timeline_iters > 0``: s_memrealtime stamps of the first iterations into
        ``self.last_timeline`` [workgroup][iteration][wait start, inputs ready, published, objective
        posted] (the last row is the monitor: column 0 = decided)."""
        if self.fabric is not None:
            self._epoch = self.fabric.next_epoch()
        else:
            self._epoch = self._epoch % 4095 + 1
        a = self._args(timeout_s)
        a.epoch = self._epoch
        tl = None
        if timeline_iters > 0:
            tl = torch.zeros((len(self.local) + 1, int(timeline_iters), 4), dtype=torch.int64, device=self.device)
            a.timeline, a.timeline_iters = tl.data_ptr(), int(timeline_iters)
        self._host_n = 0
        with torch.cuda.stream(self.stream):
            self._state.zero_()
            self.ctl.zero_()
            native.check(self.lib.gadmm_write_stamp(self.t0stamp.data_ptr(), self.stream.cuda_stream), "write_stamp")
            t0 = time.perf_counter()
            rc = int(self.lib.gadmm_star_launch(ctypes.byref(a), self.stream.cuda_stream))
            native.check(rc, "star_launch")
            # control block, the first K trace / clock entries and the start stamp come back behind the
            # kernel in one pinned copy batch: one blocking round trip per solve instead of four
            K = min(self.max_iter, 4096)
            if getattr(self, "_host", None) is None:
                self._host = (torch.empty((8,), dtype=torch.int32, pin_memory=True),
                              torch.empty((2 * K + 1,), dtype=torch.int64, pin_memory=True))
            hc, ht = self._host
            hc.copy_(self.ctl, non_blocking=True)
            ht[:K].copy_(self.trace[:K].view(torch.int64), non_blocking=True)
            ht[K:2 * K].copy_(self.tstamp[:K], non_blocking=True)
            ht[2 * K:].copy_(self.t0stamp, non_blocking=True)
            self.stream.synchronize()
            t1 = time.perf_counter()
            self._host_n = K
        self.last_timeline = tl.cpu().numpy() if tl is not None else None
        c = self._host[0].tolist()
        if c[1] == 4:
            from .chain_engine import HandoffTimeout
            raise HandoffTimeout("star kernel timed out (hand-off never completed)")
        return c[2], c[1], (t1 - t0) * 1e3

    def bytes_per_solve(self, iters: int):
        """(theta payload, wire, monitor) bytes this rank puts on the fabric for iterations 1..iters:
        uploads of local workers whose hub is on another rank, the hub's broadcast to every other rank,
        objective granules to rank 0, decisions from rank 0."""
        if self.fabric is None:
            return 0, 0, 0
        hub = self.n - 1
        ups = sum(1 for w in self.local if w != hub) if self.rank != self.hub_rank else 0
        down = (self.nranks - 1) if hub in self.local else 0
        pay = iters * (ups + down) * self.d * 8
        mon = iters * (len(self.local) * 16 if self.rank != 0 else 8 * (self.nranks - 1))
        return pay, 2 * pay, mon

    def objective_trace(self, upto: int) -> np.ndarray:
        if 0 <= upto <= getattr(self, "_host_n", 0):  # the pinned copy of the last run
            return self._host[1].numpy()[:upto].view(np.float64).copy()
        return self.trace[:upto].cpu().numpy()

    def time_trace(self, upto: int) -> np.ndarray:
        K = getattr(self, "_host_n", 0)
        if 0 <= upto <= K:
            h = self._host[1].numpy()
            t, t0 = h[K:K + upto], int(h[2 * K])
        else:
            t = self.tstamp[:upto].cpu().numpy().astype(np.int64)
            t0 = int(self.t0stamp.cpu().item())
        return np.where(t > 0, (t - t0) * 1e-8, 0.0)

    def close(self):
        pass
