"""Front-end of the persistent first-order baseline engine (``csrc/kernels/first_order.hip``).

One kernel launch per GPU runs a whole GD / DGD / LAG-PS / LAG-WK / IAG / dual-averaging run: every
logical worker is one resident workgroup, a monitor workgroup (rank 0) records the objective trace.

* One rank: all workers on one CUDA device; tables in ordinary device memory.
* Several ranks (one process per GPU, BASELINE "comparators reproduced on the same fabric"): every
  rank launches its contiguous segment of workers; the upload tables, the monitor's ring and the
  run-wide words live in IPC-exported fine-grained memory (``FoFabric``), and uploads are pushed into
  the readers' GPUs with system-scope granule stores over xGMI: GD / LAG / IAG replicate the server
  step on every rank (an upload goes to every rank: LAG's conditional uploads with a one-granule
  flag), DGD and dual averaging push rows to the chain neighbours' ranks (dual averaging's
  Gauss-Seidel sweep becomes a cross-GPU pipeline, dual_averaging.m:44).

``algorithms/baselines.py`` and ``algorithms/dual_averaging.py`` dispatch here when ``d <= 128``, the
model lives on a GPU and (several ranks) the segments are contiguous; the torch implementations
remain the fallback and the oracle the engine is tested against (tests/test_gpu.py,
tests/test_gpu_multirank.py).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..ops import native

ALG_IDS = {"GD": 0, "DGD": 1, "LAG-PS": 2, "LAG-WK": 3, "IAG": 4, "DualAvg": 5}
TICKS_PER_S = 1e8  # s_memrealtime runs at a constant 100 MHz
RING = 64
SLOTS = RING + 3  # upload-row slots of a table (IAG needs ring + 3; the lock-step algorithms use 2)


def _group(comm):
    return getattr(comm, "control_group", None)


def _all_ok(flag: bool, comm) -> bool:
    if comm is None or comm.nranks == 1:
        return flag
    t = torch.tensor([0.0 if flag else 1.0], dtype=torch.float64)
    dist.all_reduce(t, group=_group(comm))
    return float(t.item()) == 0.0


class FoFabric:
    """IPC fine-grained buffers of the multi-rank first-order engine. Collective over the comm's
    control group. Per rank: the upload table ([SLOTS][N][d] rows + [2][N] flags), the monitor's part ring
    (used on rank 0) and a 16-byte {progress, stop} word pair; the table has SLOTS row slots. Every rank maps every other rank's
    table (the server algorithms replicate the server: any worker's upload reaches every rank) and
    rank 0's ring; rank 0 also maps every rank's words."""

    def __init__(self, n_total: int, d: int, rank: int, nranks: int, device: torch.device, comm=None,
                 ring: int = RING):
        from ..parallel.xgmi import _Buf, device_identity, preflight

        self.lib = native.require()
        self.n, self.d, self.rank, self.nranks, self.ring = int(n_total), int(d), rank, nranks, ring
        self.opened: Dict[tuple, ctypes.c_void_p] = {}
        self.tab = self.part = self.words = None
        torch.cuda.set_device(device)
        mine, err = None, ""
        try:
            self.tab = _Buf(self.lib, int(self.lib.gadmm_fo_tab_granules(self.n, self.d, SLOTS)) * 16)
            self.part = _Buf(self.lib, ring * self.n * 2 * 16)
            self.words = _Buf(self.lib, 64)
            mine = (bytes(self.tab.handle.raw), bytes(self.part.handle.raw), bytes(self.words.handle.raw))
        except Exception as e:  # pragma: no cover - box dependent
            err = "rank %d alloc: %s" % (rank, e)
        allh = [None] * nranks
        dist.all_gather_object(allh, (mine, err, device_identity()), group=_group(comm))
        errs = [e for _, e, _ in allh if e]
        ok = not errs
        if ok:
            try:
                why = preflight(torch.cuda.current_device(), {r: allh[r][2] for r in range(nranks) if r != rank})
                if why:
                    raise RuntimeError("peer access pre-flight: " + why)
                self.tab_all = [self.tab.ptr.value if r == rank else self._open(allh[r][0][0], ("tab", r))
                                for r in range(nranks)]
                self.part_mon = self.part.ptr.value if rank == 0 else self._open(allh[0][0][1], ("part", 0))
                self.words_all = [self.words.ptr.value if r == rank else self._open(allh[r][0][2], ("words", r))
                                  for r in range(nranks)] if rank == 0 else [self.words.ptr.value]
            except Exception as e:  # pragma: no cover
                ok, err = False, str(e)
        if not _all_ok(ok, comm):
            self.close()
            raise RuntimeError("first-order fabric failed on some rank (%s)" % ("; ".join(errs) or err or "remote"))
        dv = torch.device("cuda", torch.cuda.current_device())
        self.tab_push_t = torch.tensor(self.tab_all, dtype=torch.int64, device=dv)
        self.wpush_t = torch.tensor(self.words_all, dtype=torch.int64, device=dv)

    def _open(self, h: bytes, key) -> int:
        p = ctypes.c_void_p()
        native.check(self.lib.gadmm_xgmi_open(ctypes.create_string_buffer(h, 64), ctypes.byref(p)),
                     "xgmi_open %s" % (key,))
        self.opened[key] = p
        return p.value

    def close(self):
        for p in self.opened.values():
            self.lib.gadmm_xgmi_close(p)
        self.opened = {}
        for b in (self.tab, self.part, self.words):
            if b is not None:
                b.free()
        self.tab = self.part = self.words = None


class FirstOrderEngine:
    """Device buffers for one model (re-used across runs; tags are epoch-salted, so the granule
    tables never need clearing between runs). Several ranks: ``comm`` / ``placement`` describe the
    run (every rank creates its engine in the same order: the tag epochs stay equal)."""

    def __init__(self, model, comm=None, placement=None, n_total: Optional[int] = None):
        self.model = model
        self.lib = native.require()
        self.dev = model.device
        self.kind = model.kind
        self.n_local, self.d = int(model.n_local), int(model.d)
        self.n = int(n_total) if n_total is not None else self.n_local
        self.m = int(model.X.shape[1])
        self.comm = comm
        self.nranks = comm.nranks if comm is not None else 1
        self.rank = comm.rank if comm is not None else 0
        self.fab: Optional[FoFabric] = None
        if self.nranks > 1:
            mine = placement.local_workers(self.rank)
            self.w_lo = int(min(mine))
            self.owner_t = torch.tensor([int(o) for o in placement.owner], dtype=torch.int32, device=self.dev)
            self.fab = FoFabric(self.n, self.d, self.rank, self.nranks, self.dev, comm)
            self.tab = self.part = None
            self.ctlw = None
        else:
            self.w_lo = 0
            self.owner_t = None
            self.tab = torch.zeros((int(self.lib.gadmm_fo_tab_granules(self.n, self.d, SLOTS)), 4),
                                   dtype=torch.int32, device=self.dev)
            self.part = torch.zeros((RING * self.n * 2, 4), dtype=torch.int32, device=self.dev)
        self.theta = torch.zeros((self.n_local, self.d), dtype=torch.float64, device=self.dev)
        self.ctl = torch.zeros(ctypes.sizeof(native.FoCtl) // 4, dtype=torch.int32, device=self.dev)
        self.pushc = torch.zeros((self.n_local, 2), dtype=torch.float64, device=self.dev)
        self.epoch = 0
        if self.kind == "linear":
            self.A, self.b, self.yy = model.A.contiguous(), model.b.contiguous(), model.yy.contiguous()
            self.X = self.Y = None
        else:
            self.X, self.Y = model.X.contiguous(), model.y.contiguous()
            self.A = self.b = self.yy = None
        self.stream = torch.cuda.Stream(device=self.dev)

    # ------------------------------------------------------------------------------------------
    @staticmethod
    def eligible(model, comm, n_total: int, local_ids=None, placement=None, alg: str = "GD") -> bool:
        """Collective when ``comm.nranks > 1`` (every rank must call it: the answer is agreed)."""
        multi = comm is not None and comm.nranks > 1
        ok = isinstance(getattr(model, "X", None), torch.Tensor) and model.X.is_cuda \
            and int(model.d) <= 128 and model.kind in ("linear", "logistic") and native.available()
        if ok and not multi:
            ok = int(model.n_local) == int(n_total)
        if ok and multi:
            ids = [int(w) for w in (local_ids if local_ids is not None else placement.local_workers(comm.rank))]
            ok = placement is not None and len(ids) == int(model.n_local) and \
                ids == list(range(ids[0], ids[0] + len(ids))) and \
                [int(w) for w in placement.local_workers(comm.rank)] == ids
        if ok:
            lib = native.require()
            lds = lib.gadmm_fo_lds(0 if model.kind == "linear" else 1, ALG_IDS.get(alg, 0), int(n_total),
                                   int(model.d), int(model.X.shape[1]))
            ok = lds <= 159 * 1024 and (alg in ("DGD", "DualAvg") or int(n_total) <= 256)
        return _all_ok(ok, comm) if multi else ok

    @staticmethod
    def get(model, comm=None, placement=None, n_total: Optional[int] = None) -> "FirstOrderEngine":
        multi = comm is not None and comm.nranks > 1
        key = "_fo_engine_mr" if multi else "_fo_engine"
        eng = getattr(model, key, None)
        if eng is None:
            eng = FirstOrderEngine(model, comm if multi else None, placement, n_total if multi else None)
            setattr(model, key, eng)
        return eng

    # ------------------------------------------------------------------------------------------
    def run(self, alg: str, max_iter: int, step: float, obj0: float = 0.0, tol: Optional[float] = None,
            faithful: bool = True, jacobi: bool = False, thrd: float = 0.0, hsq: Optional[torch.Tensor] = None,
            sched: Optional[np.ndarray] = None, timeout_s: Optional[float] = None) -> Dict[str, object]:
        """One run (collective over the ranks). Returns the monitor's traces on every rank, plus the
        run's exact fabric traffic: ``rows_pushed`` / ``flags_pushed`` granule rows stored into OTHER
        ranks' tables (all ranks), ``payload_bytes`` = rows x d x 8, ``wire_bytes`` (16-B granules)."""
        if max_iter >= (1 << 20):
            raise ValueError("first-order engine: max_iter must be < 2^20 (tag width)")
        multi = self.nranks > 1
        self.epoch = (self.epoch + 1) & 0xFFF
        if self.epoch == 0:  # tag space wrapped: clear the tables once, so no granule of epoch 1 survives
            if not multi:
                self.tab.zero_()
                self.part.zero_()
            else:
                # every rank zeroes its OWN tables (the peers' copies of this rank's rows live there),
                # then all meet: no rank starts the new epoch 1 while another's stale slots (e.g. IAG ring
                # slots a run of epoch 1 wrote and nothing overwrote since) could still match
                f = self.fab
                for buf in (f.tab, f.part, f.words):
                    native.check(self.lib.gadmm_memset_async(buf.ptr.value, 0, buf.nbytes, self.stream.cuda_stream),
                                 "fo epoch wrap: clear tables")
                self.stream.synchronize()
                dist.barrier(group=_group(self.comm))
            self.epoch = 1
        mon = self.rank == 0
        T = max_iter if mon else 1
        obj = torch.zeros(T, dtype=torch.float64, device=self.dev)
        cnt = torch.zeros(T, dtype=torch.float64, device=self.dev)
        tms = torch.zeros(T, dtype=torch.int64, device=self.dev)
        sched_t = None
        if sched is not None:
            sched_t = torch.as_tensor(np.asarray(sched, dtype=np.int32), device=self.dev)
        hsq_t = hsq.to(self.dev, torch.float64).contiguous() if hsq is not None else None
        a = native.FoArgs()
        a.alg, a.model, a.n, a.d, a.m = ALG_IDS[alg], 0 if self.kind == "linear" else 1, self.n, self.d, self.m
        a.max_iter, a.faithful, a.jacobi = int(max_iter), int(bool(faithful)), int(bool(jacobi))
        a.has_tol, a.ring, a.epoch = int(tol is not None), RING, self.epoch
        a.slots = SLOTS if alg == "IAG" else 2
        a.step, a.lam = float(step), float(self.model.lam)
        a.obj0, a.tol, a.thrd = float(obj0), float(tol if tol is not None else -1.0), float(thrd)
        if timeout_s is None:
            timeout_s = 30.0 + 50e-6 * max_iter
        a.timeout_ticks = int(timeout_s * TICKS_PER_S)
        a.A, a.b, a.yy = native.ptr(self.A), native.ptr(self.b), native.ptr(self.yy)
        a.X, a.Y = native.ptr(self.X), native.ptr(self.Y)
        a.hsq, a.sched = native.ptr(hsq_t), native.ptr(sched_t)
        a.obj_trace, a.cnt_trace, a.time_trace = obj.data_ptr(), cnt.data_ptr(), tms.data_ptr()
        a.theta_out, a.ctl = self.theta.data_ptr(), self.ctl.data_ptr()
        a.nranks, a.my_rank, a.w_lo, a.n_local = self.nranks, self.rank, self.w_lo, self.n_local
        a.has_monitor = 1 if mon else 0
        a.pushc = self.pushc.data_ptr()
        ctl_addr = self.ctl.data_ptr()
        if multi:
            a.tab, a.part = self.fab.tab.ptr.value, self.fab.part_mon
            a.owner, a.tab_push = self.owner_t.data_ptr(), self.fab.tab_push_t.data_ptr()
            a.wmon, a.wstop = self.fab.words.ptr.value, self.fab.words.ptr.value + 4
            a.wpush = self.fab.wpush_t.data_ptr() if mon else None
            a.xcd = 0
        else:
            a.tab, a.part = self.tab.data_ptr(), self.part.data_ptr()
            a.wmon, a.wstop = ctl_addr, ctl_addr + 4  # FoCtl::monitored, FoCtl::stop_iter
            if getattr(self, "_xchk", None) is None:  # XCD packing (FoArgs::xcd): placement-check granules
                self._xchk = torch.zeros((256 * 4,), dtype=torch.int32, device=self.dev)
            a.xchk, a.xcd = self._xchk.data_ptr(), 2
        cur = torch.cuda.current_stream(self.dev)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self.ctl.zero_()
            self.pushc.zero_()
            if multi:  # this rank's run-wide words (the monitor can only post after this rank's uploads)
                native.check(self.lib.gadmm_memset_async(self.fab.words.ptr.value, 0, 16, self.stream.cuda_stream),
                             "memset fo words")
            rc = self.lib.gadmm_fo_launch(ctypes.byref(a), self.stream.cuda_stream)
            if rc != 0:
                raise RuntimeError("gadmm_fo_launch refused the configuration (rc=%d)" % rc)
        self.stream.synchronize()
        cur.wait_stream(self.stream)
        raw = bytes(self.ctl.cpu().numpy().tobytes())
        ctl = native.FoCtl.from_buffer_copy(raw)
        pc = self.pushc.sum(0).cpu().numpy()
        rows, flags = float(pc[0]), float(pc[1])
        if not multi:
            if ctl.status == 4:
                raise RuntimeError("first-order engine timed out (alg=%s, iters=%d)" % (alg, ctl.iters))
            k = int(ctl.iters)
            return {"obj": obj[:k].cpu().numpy(), "cnt": cnt[:k].cpu().numpy(),
                    "times": tms[:k].cpu().numpy().astype(np.float64) / TICKS_PER_S, "iters": k,
                    "converged": ctl.status == 1, "uploads": float(ctl.uploads), "theta": self.theta.clone(),
                    "rows_pushed": 0, "flags_pushed": 0, "payload_bytes": 0, "wire_bytes": 0}
        # several ranks: agree on failure, then every rank takes the monitor's (rank 0's) result
        grp = _group(self.comm)
        bad = torch.tensor([1.0 if ctl.status == 4 else 0.0, rows, flags], dtype=torch.float64)
        st = bad.clone()
        dist.all_reduce(st, group=grp)
        if float(st[0]) > 0:
            raise RuntimeError("first-order engine timed out on some rank (alg=%s)" % alg)
        hdr = torch.tensor([float(ctl.iters), float(ctl.status), float(ctl.uploads)], dtype=torch.float64)
        dist.broadcast(hdr, src=0, group=grp)
        k = int(hdr[0])
        body = torch.stack([obj[:k].cpu(), cnt[:k].cpu(), tms[:k].cpu().double()]) if mon \
            else torch.zeros((3, k), dtype=torch.float64)
        dist.broadcast(body, src=0, group=grp)
        rows_all, flags_all = int(round(float(st[1]))), int(round(float(st[2])))
        return {"obj": body[0].numpy().copy(), "cnt": body[1].numpy().copy(), "times": body[2].numpy() / TICKS_PER_S,
                "iters": k, "converged": int(hdr[1]) == 1, "uploads": float(hdr[2]), "theta": self.theta.clone(),
                "rows_pushed": rows_all, "flags_pushed": flags_all, "payload_bytes": rows_all * self.d * 8,
                "wire_bytes": rows_all * self.d * 16 + flags_all * 16}

    def close(self):
        if self.fab is not None:
            self.fab.close()
            self.fab = None
