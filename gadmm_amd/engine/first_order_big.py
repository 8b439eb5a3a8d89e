"""Large-d first-order comparators on the device (``csrc/kernels/first_order_big.hip``).

GD, DGD, LAG-PS / LAG-WK, cyclic / randomized IAG and dual averaging (GD_DGD_LAG.m, dual_averaging.m;
SURVEY.md A8, A10) at d > 128, where ``engine/first_order.py``'s persistent kernels (operands in
VGPRs / LDS) do not apply: the real-shaped 10k data of BASELINE configs[4] and
``LinearRegression_Real.m:66-69``'s baseline bundle on it. The torch loop it replaces paid a host round
trip per iteration; here the host enqueues ``block`` iterations at a time and the stop rule runs on
the device (``ChainCtl.done``: every later kernel returns at once).

Every Gram is stored as its block-packed lower triangle (``ops.linalg.sym_pack``, half the bytes
of the full matrix) and multiplied by the symmetric GEMV of ``csrc/include/sym_gemv.h``; an
iteration costs one GEMV per worker that the algorithm refreshes (GD and IAG: the local Gram sum for
the server objective, one GEMV).

Ranks: GD (all-reduce of the local A_sum th, d doubles per iteration), DGD (boundary gradients to the
chain neighbours' ranks) and IAG (the refreshing worker's row broadcast from its owner, the objective
partials all-reduced) run across ranks over the run's communicator -- RCCL, or the IPC device
transport (``parallel/ipc.py``: also with ranks sharing one GPU). LAG-PS / LAG-WK and dual averaging
run across ranks over the IPC transport:
* LAG (GD_DGD_LAG.m:184-327): every rank keeps the server's gradient table and theta replicated; each
  iteration its workers decide their triggers on the device and a CONDITIONAL row all-gather
  (``ipc_cond_rows_kernel``) pushes a 16-byte flag per worker and the gradient row only for the
  workers that upload -- the reference's conditional uploads, with the flag as the control message;
* dual averaging (dual_averaging.m:15-70): the Gauss-Seidel sweep as a cross-rank pipeline -- a rank
  receives its left neighbour's boundary Z of the current sweep before sweeping and sends its own last
  row on after it; the right neighbour's first row of the previous sweep arrives at the pass start
  (Jacobi: both boundary rows of the previous sweep, before the sweep).
Both stay bit-identical to one rank: the server sums its table in worker order, objectives are
all-reduced per worker, and the sweep reads exactly the values the one-rank sweep reads.
"""
from __future__ import annotations

import ctypes
import time
from typing import Dict, Optional

import numpy as np
import torch

from ..ops import native
from ..ops.linalg import sym_pack
from ..parallel.topology import chain_plan

TRIG = 10
TICKS_PER_S = 1e8
MULTI_ALGS = ("GD", "DGD", "IAG", "LAG-PS", "LAG-WK", "DualAvg")
IPC_ONLY = ("LAG-PS", "LAG-WK", "DualAvg")  # device-side conditional / pipelined exchanges

_SIGS = {
    "gadmm_symv_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_long,
                                        ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    "gadmm_symv_work_doubles": (ctypes.c_long, [ctypes.c_int]),
    "gadmm_sym_padded": (ctypes.c_long, [ctypes.c_int]),
    "gadmm_fob_gd": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                    ctypes.c_double, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "gadmm_fob_dgd_grad": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "gadmm_fob_dgd_update": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                            ctypes.c_void_p, ctypes.c_void_p]),
    "gadmm_fob_server": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                        ctypes.c_void_p, ctypes.c_void_p]),
    "gadmm_fob_iag_refresh": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "gadmm_fob_lag": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "gadmm_fob_lag_rows": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p]),
    "gadmm_ipc_cond_rows": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    "gadmm_fob_worker_obj": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_void_p]),
    "gadmm_fob_objw": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "gadmm_fob_da_sweep": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_void_p]),
    "gadmm_fob_finish": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_double,
                                        ctypes.c_double, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
}


def _lib():
    lib = native.require()
    if not getattr(lib, "_fob_sigs", False):
        for name, (res, args) in _SIGS.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        lib._fob_sigs = True
    return lib


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


class FirstOrderBigEngine:
    """One model's large-d first-order state (packed Grams, padded vectors, control block)."""

    def __init__(self, model, comm=None, placement=None, n_total: Optional[int] = None):
        self.lib = _lib()
        self.model, self.comm, self.placement = model, comm, placement
        self.multi = comm is not None and comm.nranks > 1
        self.rank = comm.rank if self.multi else 0
        self.nranks = comm.nranks if self.multi else 1
        self.device = model.device
        self.d, self.nl = int(model.d), int(model.n_local)
        self.n = int(n_total) if n_total is not None else self.nl
        self.local = placement.local_workers(self.rank) if self.multi else list(range(self.n))
        self.w_lo = int(self.local[0]) if self.local else 0
        self.dp = int(self.lib.gadmm_sym_padded(self.d))
        self.nblk = (self.d + 127) // 128
        self.stream = torch.cuda.Stream(self.device)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        f64, dev, d, nl = torch.float64, self.device, self.d, self.nl
        with torch.cuda.stream(self.stream):
            self.Ap = sym_pack(model.A)                         # (nl, packed)
            self.Asum = sym_pack(model.A.sum(0, keepdim=True))  # (1, packed): this rank's Gram sum
            self.b = model.b.contiguous()
            self.yy = model.yy.contiguous()
            self.bsum_loc = self.b.sum(0).contiguous()
            yl = float(self.yy.sum().item())
            self.work = torch.zeros((max(nl, 1) * int(self.lib.gadmm_symv_work_doubles(d)),), dtype=f64, device=dev)
            self.ctl = torch.zeros((8,), dtype=torch.int32, device=dev)
        self.stream.synchronize()
        bsum = self.bsum_loc.clone()
        ysum = torch.tensor([yl], dtype=f64, device=dev)
        if self.multi:  # one-time: the global b and y'y sums (GD's server gradient and objective)
            self.comm.allreduce_sum(bsum)
            self.comm.allreduce_sum(ysum)
        self.bsum, self.yysum = bsum, ysum
        self.yyloc_t = torch.tensor([yl], dtype=f64, device=dev)

    # ------------------------------------------------------------------------------------------
    @staticmethod
    def eligible(model, comm, n_total: int, local_ids=None, placement=None, alg: str = "GD") -> bool:
        multi = comm is not None and comm.nranks > 1
        ok = getattr(model, "kind", "") == "linear" and isinstance(getattr(model, "X", None), torch.Tensor) \
            and model.X.is_cuda and int(model.d) > 128 and float(getattr(model, "lam", 0.0)) == 0.0 \
            and native.available()
        if not ok:
            return False
        if not multi:
            return int(model.n_local) == int(n_total)
        ids = [int(w) for w in (local_ids if local_ids is not None else placement.local_workers(comm.rank))]
        backends = ("ipc",) if alg in IPC_ONLY else ("rccl", "ipc")
        return (alg in MULTI_ALGS and getattr(comm, "backend", "") in backends and placement is not None
                and ids == list(range(ids[0], ids[0] + len(ids))) and len(ids) == int(model.n_local))

    @staticmethod
    def get(model, comm=None, placement=None, n_total: Optional[int] = None) -> "FirstOrderBigEngine":
        key = "_fob_engine_mr" if (comm is not None and comm.nranks > 1) else "_fob_engine"
        eng = getattr(model, key, None)
        if eng is None:
            eng = FirstOrderBigEngine(model, comm, placement, n_total)
            setattr(model, key, eng)
        return eng

    # ---- collectives on the engine stream ------------------------------------------------------
    def _allreduce(self, t):
        if getattr(self.comm, "backend", "") == "ipc":
            self.comm.device_collective("allreduce", t, 0, self.ctl, self.stream.cuda_stream)
        else:
            self.comm.allreduce_sum(t)

    def _bcast(self, t, root: int):
        if getattr(self.comm, "backend", "") == "ipc":
            self.comm.device_collective("broadcast", t, root, self.ctl, self.stream.cuda_stream)
        else:
            self.comm.broadcast(t, root)

    def _xchg(self, table, ops, phase: int):
        if not ops:
            return
        if getattr(self.comm, "backend", "") == "ipc":
            self.comm.exchange_rows_dev(table, ops, phase, self.ctl, self.stream.cuda_stream)
        else:
            self.comm.exchange_rows(table, ops)

    # ------------------------------------------------------------------------------------------
    def run(self, alg: str, max_iter: int, step: float, obj0: float = 0.0, tol: Optional[float] = None,
            faithful: bool = True, jacobi: bool = False, thrd: float = 0.0, hsq: Optional[torch.Tensor] = None,
            sched: Optional[np.ndarray] = None, block: int = 16) -> Dict[str, object]:
        """One run from theta = 0 (``alg``: GD, DGD, LAG-PS, LAG-WK, IAG, DualAvg). Output as
        ``FirstOrderEngine.run``: obj / cnt / times traces, iters, converged, uploads, theta, bytes."""
        if self.multi and (alg not in MULTI_ALGS or (alg in IPC_ONLY and getattr(self.comm, "backend", "") != "ipc")):
            raise ValueError("large-d %s across ranks needs the IPC transport" % alg)
        lib, L, ctl = self.lib, self.lib, self.ctl.data_ptr()
        d, dp, nl, n, nblk = self.d, self.dp, self.nl, self.n, self.nblk
        f64, dev = torch.float64, self.device
        st = self.stream.cuda_stream
        ck = native.check
        tolv = float(tol) if tol is not None else -1.0
        replicated = alg in ("GD", "IAG") or alg.startswith("LAG")
        cur = torch.cuda.current_stream(dev)
        self.stream.wait_stream(cur)
        pay = []  # fabric payload bytes this rank enqueued, per iteration
        with torch.cuda.stream(self.stream):
            rows = 1 if replicated else max(nl, 1)
            th = torch.zeros((rows, dp), dtype=f64, device=dev)
            q = torch.zeros((max(nl, 1), dp), dtype=f64, device=dev)
            part = torch.zeros((max(nl, 1) * nblk,), dtype=f64, device=dev)
            dpart = torch.zeros((nblk,), dtype=f64, device=dev)
            objw = torch.zeros((n,), dtype=f64, device=dev)
            zeros_n = torch.zeros((n,), dtype=f64, device=dev)
            trace = torch.full((int(max_iter),), float("nan"), dtype=f64, device=dev)
            tstamp = torch.zeros((int(max_iter),), dtype=torch.int64, device=dev)
            cnt = torch.zeros((int(max_iter),), dtype=f64, device=dev)
            ring = torch.zeros((TRIG + 2,), dtype=f64, device=dev)
            # server / gradient tables start as ones (GD_DGD_LAG.m:44-67; the torch path's servers always),
            # DGD's only when faithful
            T = torch.zeros((n, d), dtype=f64, device=dev) if (alg == "DGD" and not faithful) else \
                torch.ones((n, d), dtype=f64, device=dev)
            self.ctl.zero_()
            self.ctl[0] = 1
            if getattr(self.comm, "backend", "") == "ipc" and self.multi:
                self.comm.new_epoch(st)
            t0s = torch.zeros((1,), dtype=torch.int64, device=dev)
            ck(lib.gadmm_write_stamp(t0s.data_ptr(), st), "write_stamp")
            if alg.startswith("LAG"):
                ps = 1 if alg == "LAG-PS" else 0
                GN = torch.zeros((nl, d), dtype=f64, device=dev)
                Gl = torch.ones((nl, d), dtype=f64, device=dev)
                thhat = torch.zeros((nl, d), dtype=f64, device=dev)
                mask = torch.zeros((nl,), dtype=torch.int32, device=dev)
                ddpart = torch.zeros((nl * nblk,), dtype=f64, device=dev)
                hsq_t = hsq.to(dev, f64).contiguous()
                rows_tr = torch.zeros((int(max_iter),), dtype=f64, device=dev)  # rows this rank sends
            if alg == "DualAvg":
                Z = torch.zeros((n, d), dtype=f64, device=dev)  # chain-wide table: own rows + ghosts
                Zp = torch.zeros((nl, d), dtype=f64, device=dev)
                if self.multi:
                    R_, r_ = self.nranks, self.rank
                    lo, hi = self.w_lo, self.w_lo + nl - 1
                    if jacobi:  # both boundary rows of the previous sweep, before the sweep
                        da_pre = ([(r_ - 1, lo, 1), (r_ - 1, lo - 1, 0)] if r_ > 0 else []) + \
                                 ([(r_ + 1, hi, 1), (r_ + 1, hi + 1, 0)] if r_ + 1 < R_ else [])
                        da_left, da_post = [], []
                    else:  # right ghost (previous sweep) at the pass start; left ghost of THIS sweep; send on
                        da_pre = ([(r_ - 1, lo, 1)] if r_ > 0 else []) + ([(r_ + 1, hi + 1, 0)] if r_ + 1 < R_ else [])
                        da_left = [(r_ - 1, lo - 1, 0)] if r_ > 0 else []
                        da_post = [(r_ + 1, hi, 1)] if r_ + 1 < R_ else []
                    pay_da = sum(1 for _, _, snd in da_pre + da_post if snd) * d * 8
            if alg == "DGD" and self.multi:
                plan = chain_plan(list(range(n)), self.placement, self.rank)
                xops = plan.xchg_head + plan.xchg_tail
                pay_it = sum(1 for _, _, s in xops if s) * d * 8
            symv = lib.gadmm_symv_batch
            work = self.work.data_ptr()
            packed = self.Ap.shape[1]
            t0 = time.perf_counter()
            it, done = 0, 0
            last = max_iter + (1 if alg == "DualAvg" else 0)  # dual averaging: one more pass for obj(th^max)
            while it < last and not done:
                for _ in range(min(block, last - it)):
                    it += 1
                    pay.append(0)
                    if alg == "GD":
                        ck(symv(self.Asum.data_ptr(), 0, th.data_ptr(), 0, q.data_ptr(), 0, work, 1, d, ctl, st), "symv")
                        if self.multi:
                            # the d real entries only (a contiguous view): the zero padding of q[0]
                            # would cross the fabric every iteration and the bytes would disagree with
                            # the reported payload
                            self._allreduce(q[0, :d])
                            pay[-1] += d * 8 * (self.nranks - 1)
                        ck(L.gadmm_fob_gd(q.data_ptr(), self.bsum.data_ptr(), th.data_ptr(), part.data_ptr(), d,
                                          float(step), int(faithful), ctl, st), "fob_gd")
                        ck(L.gadmm_fob_finish(part.data_ptr(), 1, nblk, self.yysum.data_ptr(), trace.data_ptr(),
                                              tstamp.data_ptr(), max_iter, float(obj0), tolv, 0, None, 0, None, ctl, st),
                           "finish")
                    elif alg == "DGD":
                        ck(symv(self.Ap.data_ptr(), packed, th.data_ptr(), dp, q.data_ptr(), dp, work, nl, d, ctl, st),
                           "symv")
                        ck(L.gadmm_fob_dgd_grad(q.data_ptr(), dp, self.b.data_ptr(), th.data_ptr(), T.data_ptr(),
                                                part.data_ptr(), d, nl, self.w_lo, int(faithful), ctl, st), "dgd_grad")
                        if self.multi:
                            self._xchg(T, xops, 0)
                            pay[-1] += pay_it
                        ck(L.gadmm_fob_objw(part.data_ptr(), nblk, self.yy.data_ptr(), objw.data_ptr(), nl, self.w_lo,
                                            n, ctl, st), "objw")
                        if self.multi:
                            self._allreduce(objw)
                        ck(L.gadmm_fob_dgd_update(th.data_ptr(), dp, T.data_ptr(), d, nl, self.w_lo, n,
                                                  float(step), ctl, st), "dgd_update")
                        ck(L.gadmm_fob_finish(objw.data_ptr(), n, 1, zeros_n.data_ptr(), trace.data_ptr(),
                                              tstamp.data_ptr(), max_iter, float(obj0), tolv, 0, None, 0, None, ctl, st),
                           "finish")
                    elif alg == "IAG":
                        w = int(sched[it - 1])
                        owner = int(self.placement.owner[w]) if self.multi else 0
                        if it > 1:
                            if owner == self.rank:
                                li = w - self.w_lo
                                ck(symv(self.Ap.data_ptr() + li * packed * 8, 0, th.data_ptr(), 0, q.data_ptr(), 0,
                                        work, 1, d, ctl, st), "symv")
                                ck(L.gadmm_fob_iag_refresh(q.data_ptr(), self.b.data_ptr(), T.data_ptr(), d, li, w,
                                                           ctl, st), "iag_refresh")
                            if self.multi:
                                self._bcast(T[w], owner)
                                if owner == self.rank:
                                    pay[-1] += d * 8 * (self.nranks - 1)
                        q1 = q[1] if nl > 1 else q[0]
                        ck(symv(self.Asum.data_ptr(), 0, th.data_ptr(), 0, q1.data_ptr(), 0, work, 1, d, ctl, st),
                           "symv")
                        bs = self.bsum_loc if self.multi else self.bsum
                        ck(L.gadmm_fob_server(q1.data_ptr(), bs.data_ptr(), th.data_ptr(), T.data_ptr(),
                                              part.data_ptr(), None, d, n, float(step), ctl, st), "server")
                        if self.multi:
                            self._allreduce(part[:nblk])
                        ck(L.gadmm_fob_finish(part.data_ptr(), 1, nblk, self.yysum.data_ptr(), trace.data_ptr(),
                                              tstamp.data_ptr(), max_iter, float(obj0), tolv, 0, None, 0, None, ctl, st),
                           "finish")
                    elif alg.startswith("LAG"):
                        ck(symv(self.Ap.data_ptr(), packed, th.data_ptr(), 0, q.data_ptr(), dp, work, nl, d, ctl, st),
                           "symv")
                        ck(L.gadmm_fob_lag(q.data_ptr(), dp, self.b.data_ptr(), th.data_ptr(), GN.data_ptr(),
                                           Gl.data_ptr(), thhat.data_ptr(), T.data_ptr(), part.data_ptr(),
                                           ddpart.data_ptr(), hsq_t.data_ptr(), ring.data_ptr(), mask.data_ptr(),
                                           cnt.data_ptr(), d, nl, self.w_lo, ps, float(thrd), int(faithful), ctl, st),
                           "lag")
                        if self.multi:  # the uploads: a flag per worker, the row only when it triggered
                            ck(L.gadmm_fob_lag_rows(mask.data_ptr(), nl, rows_tr.data_ptr(), ctl, st), "lag_rows")
                            ck(L.gadmm_ipc_cond_rows(self.comm.xport, T.data_ptr(), mask.data_ptr(), nl, self.w_lo, d,
                                                     2, 3, ctl, st), "ipc_cond_rows")
                        ck(L.gadmm_fob_objw(part.data_ptr(), nblk, self.yy.data_ptr(), objw.data_ptr(), nl, self.w_lo,
                                            n, ctl, st), "objw")
                        if self.multi:
                            self._allreduce(objw)
                        ck(L.gadmm_fob_server(None, None, th.data_ptr(), T.data_ptr(), None, dpart.data_ptr(), d, n,
                                              float(step), ctl, st), "server")
                        ck(L.gadmm_fob_finish(objw.data_ptr(), n, 1, zeros_n.data_ptr(), trace.data_ptr(),
                                              tstamp.data_ptr(), max_iter, float(obj0), tolv, 0, dpart.data_ptr(),
                                              nblk, ring.data_ptr(), ctl, st), "finish")
                    else:  # DualAvg: pass `it` evaluates th^{it-1} (its stop rule) and sweeps to th^it
                        ck(symv(self.Ap.data_ptr(), packed, th.data_ptr(), dp, q.data_ptr(), dp, work, nl, d, ctl, st),
                           "symv")
                        ck(L.gadmm_fob_worker_obj(q.data_ptr(), dp, self.b.data_ptr(), th.data_ptr(), part.data_ptr(),
                                                  d, nl, ctl, st), "worker_obj")
                        ck(L.gadmm_fob_objw(part.data_ptr(), nblk, self.yy.data_ptr(), objw.data_ptr(), nl, self.w_lo,
                                            n, ctl, st), "objw")
                        if self.multi:
                            self._allreduce(objw)
                        ck(L.gadmm_fob_finish(objw.data_ptr(), n, 1, zeros_n.data_ptr(), trace.data_ptr(),
                                              tstamp.data_ptr(), max_iter, float(obj0), tolv, 1, None, 0, None, ctl, st),
                           "finish")
                        if it <= max_iter:
                            if self.multi:
                                self._xchg(Z, da_pre, 1)
                                self._xchg(Z, da_left, 0)
                                pay[-1] += pay_da
                            ck(L.gadmm_fob_da_sweep(q.data_ptr(), dp, self.b.data_ptr(), th.data_ptr(), Z.data_ptr(),
                                                    Zp.data_ptr(), d, nl, self.w_lo, n, float(step),
                                                    int(bool(jacobi)), ctl, st), "da_sweep")
                            if self.multi:
                                self._xchg(Z, da_post, 0)
                done = int(self.ctl[1].item())  # one host look per block
            c = self.ctl.cpu().tolist()
            wall = time.perf_counter() - t0
        cur.wait_stream(self.stream)
        done, conv = int(c[1]), int(c[2])
        k = conv if done else min(it, max_iter)
        times = (tstamp[:k] - t0s).cpu().numpy().astype(np.float64) / TICKS_PER_S
        counts = cnt[:k].cpu().numpy()
        out = {"obj": trace[:k].cpu().numpy(), "cnt": counts, "times": times, "iters": k, "converged": done == 1,
               "uploads": float(counts.sum()), "theta": th[:, :d].clone(), "rows_pushed": 0, "flags_pushed": 0,
               "payload_bytes": 0, "wire_bytes": 0, "wall_s": wall}
        out["engine"] = "native-big"
        if self.multi:  # payload the iterations 1..k put on the fabric, all ranks (skipped ones moved nothing)
            import torch.distributed as dist
            grp = getattr(self.comm, "control_group", None)
            if alg.startswith("LAG"):
                # conditional uploads: the rows that travelled (to every other rank) + one flag per
                # worker per iteration; the upload counts are summed over ranks
                rows_sent = float(rows_tr[:k].sum().item())
                pay_lag = (rows_sent * d + float(k) * nl) * 8 * (self.nranks - 1)
                c = torch.from_numpy(np.ascontiguousarray(counts, dtype=np.float64))
                dist.all_reduce(c, group=grp)
                out["cnt"] = c.numpy()
                out["uploads"] = float(out["cnt"].sum())
                pay = [pay_lag]
            t = torch.tensor([float(sum(pay[:k]))], dtype=torch.float64)
            dist.all_reduce(t, group=grp)
            out["payload_bytes"] = int(round(float(t.item())))
            out["wire_bytes"] = out["payload_bytes"] * (2 if getattr(self.comm, "backend", "") == "ipc" else 1)
        return out
