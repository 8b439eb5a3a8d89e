"""Front-end of the persistent first-order baseline engine (``csrc/kernels/first_order.hip``).

One kernel launch runs a whole GD / DGD / LAG-PS / LAG-WK / IAG / dual-averaging run on one GPU
(every logical worker is one resident workgroup, a monitor workgroup records the objective trace).
``algorithms/baselines.py`` and ``algorithms/dual_averaging.py`` dispatch here when all workers live
on one CUDA device (single rank) and ``d <= 128``; the torch implementations remain the multi-rank
path and the reference the engine is tested against (tests/test_gpu.py).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np
import torch

from ..ops import native

ALG_IDS = {"GD": 0, "DGD": 1, "LAG-PS": 2, "LAG-WK": 3, "IAG": 4, "DualAvg": 5}
TICKS_PER_S = 1e8  # s_memrealtime runs at a constant 100 MHz
RING = 64


class FirstOrderEngine:
    """Device buffers for one model (re-used across runs; tags are epoch-salted, so the granule
    tables never need clearing between runs)."""

    def __init__(self, model):
        self.model = model
        self.lib = native.require()
        self.dev = model.device
        self.kind = model.kind
        self.n, self.d = int(model.n_local), int(model.d)
        self.m = int(model.X.shape[1])
        self.tab = torch.zeros((2 * self.n * self.d, 4), dtype=torch.int32, device=self.dev)
        self.part = torch.zeros((RING * self.n * 2, 4), dtype=torch.int32, device=self.dev)
        self.theta = torch.zeros((self.n, self.d), dtype=torch.float64, device=self.dev)
        self.ctl = torch.zeros(ctypes.sizeof(native.FoCtl) // 4, dtype=torch.int32, device=self.dev)
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
    def eligible(model, comm, n_total: int) -> bool:
        if not (isinstance(getattr(model, "X", None), torch.Tensor) and model.X.is_cuda):
            return False
        if comm is not None and comm.nranks > 1:
            return False
        if int(model.n_local) != int(n_total) or int(model.d) > 128 or model.kind not in ("linear", "logistic"):
            return False
        if not native.available():
            return False
        lib = native.require()
        lds = lib.gadmm_fo_lds(0 if model.kind == "linear" else 1, int(model.d), int(model.X.shape[1]))
        return lds <= 159 * 1024

    @staticmethod
    def get(model) -> "FirstOrderEngine":
        eng = getattr(model, "_fo_engine", None)
        if eng is None:
            eng = FirstOrderEngine(model)
            model._fo_engine = eng
        return eng

    # ------------------------------------------------------------------------------------------
    def run(self, alg: str, max_iter: int, step: float, obj0: float = 0.0, tol: Optional[float] = None,
            faithful: bool = True, jacobi: bool = False, thrd: float = 0.0, hsq: Optional[torch.Tensor] = None,
            sched: Optional[np.ndarray] = None, timeout_s: Optional[float] = None) -> Dict[str, object]:
        if max_iter >= (1 << 20):
            raise ValueError("first-order engine: max_iter must be < 2^20 (tag width)")
        self.epoch = (self.epoch + 1) & 0xFFF
        if self.epoch == 0:  # tag space wrapped: clear the tables once
            self.tab.zero_()
            self.part.zero_()
            self.epoch = 1
        obj = torch.zeros(max_iter, dtype=torch.float64, device=self.dev)
        cnt = torch.zeros(max_iter, dtype=torch.float64, device=self.dev)
        tms = torch.zeros(max_iter, dtype=torch.int64, device=self.dev)
        sched_t = None
        if sched is not None:
            sched_t = torch.as_tensor(np.asarray(sched, dtype=np.int32), device=self.dev)
        hsq_t = hsq.to(self.dev, torch.float64).contiguous() if hsq is not None else None
        a = native.FoArgs()
        a.alg, a.model, a.n, a.d, a.m = ALG_IDS[alg], 0 if self.kind == "linear" else 1, self.n, self.d, self.m
        a.max_iter, a.faithful, a.jacobi = int(max_iter), int(bool(faithful)), int(bool(jacobi))
        a.has_tol, a.ring, a.epoch = int(tol is not None), RING, self.epoch
        a.step, a.lam = float(step), float(self.model.lam)
        a.obj0, a.tol, a.thrd = float(obj0), float(tol if tol is not None else -1.0), float(thrd)
        if timeout_s is None:
            timeout_s = 30.0 + 50e-6 * max_iter
        a.timeout_ticks = int(timeout_s * TICKS_PER_S)
        a.A, a.b, a.yy = native.ptr(self.A), native.ptr(self.b), native.ptr(self.yy)
        a.X, a.Y = native.ptr(self.X), native.ptr(self.Y)
        a.hsq, a.sched = native.ptr(hsq_t), native.ptr(sched_t)
        a.tab, a.part = self.tab.data_ptr(), self.part.data_ptr()
        a.obj_trace, a.cnt_trace, a.time_trace = obj.data_ptr(), cnt.data_ptr(), tms.data_ptr()
        a.theta_out, a.ctl = self.theta.data_ptr(), self.ctl.data_ptr()
        if getattr(self, "_xchk", None) is None:  # XCD packing (FoArgs::xcd): placement-check granules
            self._xchk = torch.zeros((256 * 4,), dtype=torch.int32, device=self.dev)
        a.xchk, a.xcd = self._xchk.data_ptr(), 2
        cur = torch.cuda.current_stream(self.dev)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self.ctl.zero_()
            rc = self.lib.gadmm_fo_launch(ctypes.byref(a), self.stream.cuda_stream)
            if rc != 0:
                raise RuntimeError("gadmm_fo_launch refused the configuration (rc=%d)" % rc)
        self.stream.synchronize()
        cur.wait_stream(self.stream)
        raw = bytes(self.ctl.cpu().numpy().tobytes())
        ctl = native.FoCtl.from_buffer_copy(raw)
        if ctl.status == 4:
            raise RuntimeError("first-order engine timed out (alg=%s, iters=%d)" % (alg, ctl.iters))
        k = int(ctl.iters)
        return {"obj": obj[:k].cpu().numpy(), "cnt": cnt[:k].cpu().numpy(),
                "times": tms[:k].cpu().numpy().astype(np.float64) / TICKS_PER_S, "iters": k,
                "converged": ctl.status == 1, "uploads": float(ctl.uploads), "theta": self.theta.clone()}
