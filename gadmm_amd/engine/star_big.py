"""Front-end of the large-d star ADMM (``csrc/kernels/star_big.hip``): ``standared_ADMM.m`` at d > 64,
the comparator of BASELINE configs[4] (the 10M x 10k real-shaped config, "vs standard-ADMM baseline").

Per iteration: the local non-hub workers' closed-form solves (HBM-streaming GEMVs with their cached
inverses), ``[sum lam_i, sum theta_i]`` reduced to the hub's rank, the hub's solve, ``theta_hub``
broadcast to every rank, the dual updates and the objective, all-reduced; the stop rule runs on the
device (``ctl.done``) and every kernel of later iterations returns at once, so the host enqueues
``block`` iterations between two looks at ``ctl`` instead of synchronising every iteration.

Collectives go through the run's comm on the engine stream: on one rank (``LocalComm``) they are
no-ops, across GPUs ``RcclComm`` issues ``ncclReduce`` / ``ncclBroadcast`` / ``ncclAllReduce`` (the
star's reduce + broadcast of SURVEY.md C5; 2d + d doubles per non-hub rank and iteration), and
``IpcComm`` runs the same three as device kernels over IPC-mapped mailboxes (``ipc_coll_kernel``:
tagged granules pushed straight into the hub's / every rank's memory, sums in rank order). The IPC
path needs no RCCL, so it also runs with several ranks sharing one GPU (the rehearsal of BASELINE
configs[4] on a one-GPU box) and is an RCCL-free data plane on a node.
"""
from __future__ import annotations

import contextlib
import ctypes
import time
from typing import Optional, Sequence

import numpy as np
import torch

from ..ops import native
from ..ops.linalg import spd_inverse, sym_pack


class StarBigArgs(ctypes.Structure):
    """Mirror of StarBigArgs in csrc/kernels/star_big.hip."""
    _fields_ = [
        ("d", ctypes.c_int), ("n_total", ctypes.c_int), ("n_local", ctypes.c_int), ("hub_li", ctypes.c_int),
        ("max_iter", ctypes.c_int), ("obj_mode", ctypes.c_int), ("pad0", ctypes.c_int), ("pad1", ctypes.c_int),
        ("rho", ctypes.c_double), ("obj0", ctypes.c_double), ("tol", ctypes.c_double),
        ("Minv", ctypes.c_void_p), ("A", ctypes.c_void_p), ("b", ctypes.c_void_p), ("yy", ctypes.c_void_p),
        ("theta", ctypes.c_void_p), ("lam", ctypes.c_void_p), ("th_hub", ctypes.c_void_p), ("agg", ctypes.c_void_p),
        ("rbuf", ctypes.c_void_p), ("objw", ctypes.c_void_p), ("objp", ctypes.c_void_p), ("trace", ctypes.c_void_p),
        ("ctl", ctypes.c_void_p), ("tstamp", ctypes.c_void_p), ("gid", ctypes.c_void_p),
    ]


def comm_ok(comm) -> bool:
    """Comms whose collectives are stream-ordered device operations: one rank, RCCL, or the IPC
    device-copy transport."""
    return comm is None or comm.nranks == 1 or getattr(comm, "backend", "") in ("rccl", "ipc")


class StarBigEngine:
    """One model's star solve state (cached inverses, buffers); ``run`` is one solve from zero."""

    def __init__(self, model, local_ids: Sequence[int], n_total: int, rho: float, comm=None, hub_rank: int = 0,
                 exact_objective: bool = False):
        self.lib = native.require()
        for fn, args in (("gadmm_star_big_workers", 2), ("gadmm_star_big_hub", 2), ("gadmm_star_big_post", 2),
                         ("gadmm_star_big_finish", 2)):
            f = getattr(self.lib, fn)
            f.restype, f.argtypes = ctypes.c_int, [ctypes.POINTER(StarBigArgs), ctypes.c_void_p]
        self.lib.gadmm_star_big_rstride.restype = ctypes.c_long
        self.lib.gadmm_star_big_rstride.argtypes = [ctypes.c_int]
        self.model, self.comm = model, comm
        self.device = model.device
        self.local = [int(w) for w in local_ids]
        self.n, self.d, self.rho = int(n_total), int(model.d), float(rho)
        self.hub = self.n - 1
        self.hub_li = self.local.index(self.hub) if self.hub in self.local else -1
        self.hub_rank = int(hub_rank)
        self.exact = bool(exact_objective)
        nl, d, f64, dev = len(self.local), self.d, torch.float64, self.device
        self.stream = torch.cuda.Stream(dev)
        self.stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(self.stream):
            shifts = torch.tensor([[(self.n - 1) * self.rho if w == self.hub else self.rho] for w in self.local],
                                  dtype=f64, device=dev)
            t0 = time.perf_counter()
            full = spd_inverse(model.A, shifts)  # (nl, 1, d, d): K2 on the device
            self.Minv = sym_pack(full)  # (nl, packed): the block-packed lower triangles the kernels stream
            del full
            self.stream.synchronize()
            self.setup_s = time.perf_counter() - t0
            self.theta = torch.zeros((nl, d), dtype=f64, device=dev)
            self.lam = torch.zeros((nl, d), dtype=f64, device=dev)
            self.th_hub = torch.zeros((d,), dtype=f64, device=dev)
            self.agg = torch.zeros((2 * d,), dtype=f64, device=dev)
            self.rbuf = torch.zeros((nl * int(self.lib.gadmm_star_big_rstride(d)),), dtype=f64, device=dev)
            self.objw = torch.zeros((nl,), dtype=f64, device=dev)
            self.objp = torch.zeros((self.n,), dtype=f64, device=dev)  # per global worker (exact all-reduce)
            self.gid = torch.tensor(self.local, dtype=torch.int32, device=dev)
            self.ctl = torch.zeros((8,), dtype=torch.int32, device=dev)
            self.t0stamp = torch.zeros((1,), dtype=torch.int64, device=dev)
            self.trace = self.tstamp = None
        self.last_kernel = "star-big(%s objective)" % ("exact" if self.exact else "identity")

    def _args(self, obj0: float, tol: float, max_iter: int) -> StarBigArgs:
        a = StarBigArgs()
        a.d, a.n_total, a.n_local, a.hub_li = self.d, self.n, len(self.local), self.hub_li
        a.max_iter, a.obj_mode = int(max_iter), 0 if self.exact else 1
        a.rho, a.obj0, a.tol = self.rho, float(obj0), float(tol)
        m = self.model
        a.Minv, a.A, a.b, a.yy = self.Minv.data_ptr(), m.A.data_ptr(), m.b.data_ptr(), m.yy.data_ptr()
        a.theta, a.lam, a.th_hub, a.agg = (self.theta.data_ptr(), self.lam.data_ptr(), self.th_hub.data_ptr(),
                                           self.agg.data_ptr())
        a.rbuf, a.objw, a.objp = self.rbuf.data_ptr(), self.objw.data_ptr(), self.objp.data_ptr()
        a.trace, a.ctl, a.tstamp = self.trace.data_ptr(), self.ctl.data_ptr(), self.tstamp.data_ptr()
        a.gid = self.gid.data_ptr()
        return a

    def run(self, obj0: float, tol: float, max_iter: int, block: int = 8):
        """One solve from theta = lam = 0. Returns (iters, done, wall_s); traces in ``self.trace``.
        Collective across the comm's ranks (every rank enqueues the same iterations)."""
        multi = self.comm is not None and self.comm.nranks > 1
        ipc = multi and getattr(self.comm, "backend", "") == "ipc"
        dev = self.device
        self.trace = torch.full((int(max_iter),), float("nan"), dtype=torch.float64, device=dev)
        self.tstamp = torch.zeros((int(max_iter),), dtype=torch.int64, device=dev)
        a = self._args(obj0, tol, max_iter)
        st = self.stream.cuda_stream
        cur = torch.cuda.current_stream(dev)
        self.stream.wait_stream(cur)
        ch = native.check
        t0 = time.perf_counter()
        with torch.cuda.stream(self.stream):
            self.theta.zero_()
            self.lam.zero_()
            self.th_hub.zero_()
            self.ctl.zero_()
            self.ctl[0] = 1  # iter
            native.check(self.lib.gadmm_write_stamp(self.t0stamp.data_ptr(), st), "write_stamp")
            if ipc:
                self.comm.new_epoch(st)
                coll = self.comm.device_collective
                reduce = lambda t, root: coll("reduce", t, root, self.ctl, st)  # noqa: E731
                bcast = lambda t, root: coll("broadcast", t, root, self.ctl, st)  # noqa: E731
                allred = lambda t: coll("allreduce", t, 0, self.ctl, st)  # noqa: E731
            elif multi:
                reduce, bcast, allred = self.comm.reduce_sum, self.comm.broadcast, self.comm.allreduce_sum
            # RCCL: the collectives are enqueued without a host wait each (batched) and the block's one
            # host look goes through the communicator's bounded wait (its watchdog aborts a hung block)
            rccl_wait = getattr(self.comm, "wait", None) if (multi and not ipc) else None
            batch = self.comm.batched() if rccl_wait is not None else contextlib.nullcontext()
            it = 0
            done = 0
            while it < max_iter and not done:
                with batch:
                    for _ in range(min(block, max_iter - it)):
                        ch(self.lib.gadmm_star_big_workers(ctypes.byref(a), st), "star_big_workers")
                        if multi:
                            reduce(self.agg, self.hub_rank)
                        ch(self.lib.gadmm_star_big_hub(ctypes.byref(a), st), "star_big_hub")
                        if multi:
                            bcast(self.th_hub, self.hub_rank)
                        ch(self.lib.gadmm_star_big_post(ctypes.byref(a), st), "star_big_post")
                        if multi:
                            allred(self.objp)
                        ch(self.lib.gadmm_star_big_finish(ctypes.byref(a), st), "star_big_finish")
                        it += 1
                if rccl_wait is not None:
                    rccl_wait(st)
                done = int(self.ctl[1].item())  # one host look per block (synchronises the stream)
            c = self.ctl.cpu().tolist()
        wall = time.perf_counter() - t0
        cur.wait_stream(self.stream)
        done, conv = int(c[1]), int(c[2])
        iters = conv if done else it
        return iters, done, wall

    def objective_trace(self, iters: int) -> np.ndarray:
        return self.trace[:iters].cpu().numpy()

    def time_trace(self, iters: int) -> np.ndarray:
        """Measured device clock (s) at each iteration's stop rule, from the solve's start stamp."""
        return (self.tstamp[:iters] - self.t0stamp).cpu().numpy().astype(np.float64) / 1e8

    def coll_bytes_per_iteration(self) -> int:
        """Collective payload leaving this rank per iteration: [sum lam, sum theta] to the hub (2d
        doubles, non-hub ranks), theta_hub to every other rank (d doubles, hub rank), the per-worker
        objective slots (N doubles; the IPC all-reduce pushes them to every other rank)."""
        if self.comm is None or self.comm.nranks == 1:
            return 0
        R = self.comm.nranks
        obj = 8 * self.n * ((R - 1) if getattr(self.comm, "backend", "") == "ipc" else 1)
        if self.comm.rank == self.hub_rank:
            return self.d * 8 * (R - 1) + obj
        return 2 * self.d * 8 + obj
