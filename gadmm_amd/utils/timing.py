"""Timing helpers (SURVEY.md §5 Tracing/profiling).

* ``WallTimer``: host monotonic clock, synchronising the HIP device when one is in use.
* ``EventTimer``: HIP events around device work (``torch.cuda.Event``).
* ``modelled_time``: the reference's like-for-like clock model — ``2 * toc`` of worker 1's local
  solve per iteration, i.e. heads then tails each take one local-solve time
  (``group_ADMM_closedForm.m:39-42,53-55``). Useful to regenerate the paper's "clock time" panels;
  real wall time (including communication) is what the framework reports by default.
* ``roctx_range``: named ranges for rocprofv3 traces when roctx is available (no-op otherwise).
* ``host_stamp``: labelled host clock stamps at fixed points of the native solve path, recorded only
  while a tool has set ``HOST_STAMPS`` to a list (tools/dgadmm_host_stamps.py); a no-op otherwise.
"""
from __future__ import annotations

import ctypes
import os
import time
from typing import Optional

import numpy as np
import torch


HOST_STAMPS: Optional[list] = None


def host_stamp(label: str) -> None:
    if HOST_STAMPS is not None:
        HOST_STAMPS.append((label, time.perf_counter()))


class WallTimer:
    def __init__(self, device: Optional[torch.device] = None):
        self.device = device
        self.t0 = None
        self.elapsed = 0.0

    def _sync(self):
        if self.device is not None and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def __enter__(self):
        self._sync()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self._sync()
        self.elapsed = time.perf_counter() - self.t0


class EventTimer:
    def __init__(self, stream: Optional[torch.cuda.Stream] = None):
        self.stream = stream
        self.start = torch.cuda.Event(enable_timing=True)
        self.end = torch.cuda.Event(enable_timing=True)

    def __enter__(self):
        self.start.record(self.stream)
        return self

    def __exit__(self, *exc):
        self.end.record(self.stream)

    def ms(self) -> float:
        self.end.synchronize()
        return self.start.elapsed_time(self.end)


def modelled_time(per_solve_s: float, iters: int) -> np.ndarray:
    """Reference clock model: cumulative ``2 * t_local_solve`` per iteration (first entry 0:
    ``gadmm_time(i) = gadmm_time(i-1) + 2*toc`` for i > 1, group_ADMM_closedForm.m:39-42,53-55)."""
    t = np.arange(iters, dtype=np.float64) * 2.0 * per_solve_s
    return t


def reference_local_solve_s(model, rho: float, reps: int = 20) -> float:
    """The ``toc`` of the reference's clock model, measured on this device: worker 1's local solve
    from its raw shard, as the reference times it (tic/toc around one solve of the first worker).

    * linear: ``(H'H + rho I) \\ (H'Y + ...)`` -- Gram of the raw rows + dense solve
      (group_ADMM_closedForm.m:39-43; the head has one neighbour, so the shift is rho);
    * logistic: the exact prox (Newton to machine precision), the stand-in for the reference's CVX
      call (group_ADMM_logistic.m:48-58).
    Median of ``reps`` solves; device-synchronised around each."""
    dev = model.X.device
    idx = torch.zeros(1, dtype=torch.long, device=dev)
    H, Y = model.X[0], model.y[0]
    d = H.shape[-1]
    times = []
    for _ in range(max(1, reps)):
        with WallTimer(dev) as t:
            if getattr(model, "kind", "linear") == "linear":
                M = H.T @ H + rho * torch.eye(d, dtype=H.dtype, device=dev)
                x = torch.linalg.solve(M, H.T @ Y)
            else:
                z = torch.zeros((1, d), dtype=H.dtype, device=dev)
                x = model.newton_prox(idx, z, z, torch.full((1,), rho, dtype=H.dtype, device=dev), z)
            del x
        times.append(t.elapsed)
    return float(np.median(times))


_roctx = None


def _profiled() -> bool:
    """roctx ranges only under a profiler (rocprofv3 preloads its tool library and exports ROCPROF_*
    settings) or with GADMM_ROCTX=1: outside one a range push / pop is ~2 us of host time per solve for
    nothing (GADMM_ROCTX=0 forces them off)."""
    v = os.environ.get("GADMM_ROCTX")
    if v is not None:
        return v == "1"
    return "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ)


def _load_roctx():
    global _roctx
    if _roctx is None:
        if not _profiled():
            _roctx = False
            return None
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                _roctx = ctypes.CDLL(name)
                _roctx.roctxRangePushA.argtypes = [ctypes.c_char_p]
                break
            except OSError:
                _roctx = False
    return _roctx or None


class _RoctxRange:
    """A roctx push / pop pair (class-based: a generator context manager costs ~2-3 us per use, and a
    D-GADMM solve enters one on its host path)."""
    __slots__ = ("name",)

    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        lib = _load_roctx()
        if lib:
            lib.roctxRangePushA(self.name.encode())
        return self

    def __exit__(self, *exc):
        lib = _load_roctx()
        if lib:
            lib.roctxRangePop()
        return False


def roctx_range(name: str) -> _RoctxRange:
    """A named range in rocprofv3 --marker-trace timelines (no-op without roctx)."""
    return _RoctxRange(name)
