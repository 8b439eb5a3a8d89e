"""Distributed dual averaging over the chain — ``dual_averaging.m`` / ``dual_averaging_logisticReg.m``
(SURVEY.md A8, A9).

Per iteration the workers sweep the chain in order; worker n computes its local gradient g_n at its
current theta_n and mixes its neighbours' dual variables with no self weight:
    ends:    Z_n = Z_nbr + g_n              middles: Z_n = 1/2 Z_{n-1} + 1/2 Z_{n+1} + g_n
then theta_n = -alpha Z_n. ``Z_prev`` is overwritten in place during the sweep (:44), so worker n
sees the left neighbour's *current* Z and the right neighbour's *previous* Z — a Gauss-Seidel
wavefront. On several ranks this becomes a pipeline: rank r waits for Z of the last worker of rank
r-1 from the current sweep and uses Z of the first worker of rank r+1 from the previous sweep
(SURVEY.md C8). ``jacobi=True`` offers the documented parallel variant (all neighbours' previous Z).
On GPUs the whole run is one persistent kernel per GPU (``engine/first_order.py``), where the
wavefront is realised directly between worker workgroups (across GPUs: device-initiated Z pushes
into the neighbour rank's table over xGMI).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from ..parallel.comm import Comm, LocalComm
from ..parallel.topology import Placement
from .base import RunResult, Stopper, total_bytes, global_objective, run_bytes


def dual_averaging(model, local_ids: Sequence[int], n_total: int, alpha: float, obj0: float, tol: float,
                   max_iter: int, comm: Optional[Comm] = None, placement: Optional[Placement] = None,
                   jacobi: bool = False, name: str = "DualAvg", backend: str = "auto") -> RunResult:
    comm = comm if comm is not None else LocalComm()
    placement = placement if placement is not None else Placement.contiguous(n_total, comm.nranks)
    if backend != "torch":
        from ..engine.first_order import FirstOrderEngine

        if FirstOrderEngine.eligible(model, comm, n_total, local_ids, placement, "DualAvg"):
            out = FirstOrderEngine.get(model, comm, placement, n_total).run("DualAvg", max_iter, alpha, obj0, tol,
                                                                              jacobi=jacobi)
            obj = out["obj"]
            n = len(obj)
            return RunResult(algorithm=name, obj=obj, loss=np.abs(obj - obj0),
                             iters=out["iters"] if out["converged"] else n, converged=out["converged"],
                             wall_s=float(out["times"][-1]) if n else 0.0, time_trace=out["times"],
                             comm_units=np.arange(1, n + 1, dtype=np.float64) * n_total,
                             bytes_sent=int(out["payload_bytes"]), bytes_total=int(out["payload_bytes"]),
                             extra={"jacobi": jacobi, "nranks": comm.nranks, "engine": "native-persistent",
                                    "transport": "xgmi" if comm.nranks > 1 else "local",
                                    "rows_pushed": out["rows_pushed"], "wire_bytes": out["wire_bytes"],
                                    "model_bytes": n * n_total * model.d * 8, "dim": model.d})
        from ..engine.first_order_big import FirstOrderBigEngine
        big = FirstOrderBigEngine.eligible(model, comm, n_total, local_ids, placement, "DualAvg")
        if comm.nranks > 1 and getattr(model, "kind", "") == "linear" and int(model.d) > 128:
            from ..engine.first_order import _all_ok
            big = _all_ok(big, comm)  # collective: every rank takes the same path
        if big:
            # d > 128: the stream-ordered large-d engine (packed Grams, device stop rule); across ranks the
            # Gauss-Seidel sweep is a pipeline over the IPC transport (first_order_big.py)
            out = FirstOrderBigEngine.get(model, comm, placement, n_total).run("DualAvg", max_iter, alpha, obj0, tol,
                                                                                 jacobi=jacobi)
            obj = out["obj"]
            n = len(obj)
            return RunResult(algorithm=name, obj=obj, loss=np.abs(obj - obj0),
                             iters=out["iters"] if out["converged"] else n, converged=out["converged"],
                             wall_s=float(out["times"][-1]) if n else 0.0, time_trace=out["times"],
                             comm_units=np.arange(1, n + 1, dtype=np.float64) * n_total,
                             bytes_sent=int(out["payload_bytes"]), bytes_total=int(out["payload_bytes"]),
                             extra={"jacobi": jacobi, "nranks": comm.nranks, "engine": "native-big",
                                    "wire_bytes": out["wire_bytes"],
                                    "model_bytes": n * n_total * model.d * 8, "dim": model.d})
        if backend == "native":
            raise RuntimeError("native dual averaging needs GPU ranks with contiguous segments")
    dev, d = model.device, model.d
    local_ids = [int(w) for w in local_ids]
    if local_ids != sorted(local_ids) or (local_ids and local_ids[-1] - local_ids[0] + 1 != len(local_ids)):
        raise ValueError("dual averaging needs a contiguous chain segment per rank")
    first, last = local_ids[0], local_ids[-1]
    rank, R = comm.rank, comm.nranks
    nl = len(local_ids)
    theta = torch.zeros((nl, d), dtype=torch.float64, device=dev)
    Z = torch.zeros((nl, d), dtype=torch.float64, device=dev)
    z_left = torch.zeros(d, dtype=torch.float64, device=dev)   # Z of worker first-1
    z_right = torch.zeros(d, dtype=torch.float64, device=dev)  # Z of worker last+1 (previous sweep)
    stop = Stopper(obj0, tol, max_iter)
    snap = comm.stats.snapshot()
    iters, converged = max_iter, False
    for it in range(1, max_iter + 1):
        g_all = model.gradient(theta)
        if R > 1 and not jacobi:
            if rank > 0:
                comm.recv_tensor(z_left, rank - 1)          # current sweep
        Zprev = Z.clone()
        for k in range(nl):
            w = local_ids[k]
            left = Z[k - 1] if k > 0 else (z_left if w > 0 else None)
            if jacobi and k > 0:
                left = Zprev[k - 1]
            right = Zprev[k + 1] if k < nl - 1 else (z_right if w < n_total - 1 else None)
            if left is None and right is None:
                zn = g_all[k].clone()
            elif left is None:
                zn = right + g_all[k]
            elif right is None:
                zn = left + g_all[k]
            else:
                zn = 0.5 * right + 0.5 * left + g_all[k]
            Z[k] = zn
            theta[k] = -alpha * zn
        if R > 1:
            if jacobi:
                ops = []
                # exchange boundary Z (previous-sweep semantics for both sides)
                if rank + 1 < R:
                    comm.send_tensor(Z[nl - 1], rank + 1)
                if rank > 0:
                    comm.recv_tensor(z_left, rank - 1)
                if rank > 0:
                    comm.send_tensor(Z[0], rank - 1)
                if rank + 1 < R:
                    comm.recv_tensor(z_right, rank + 1)
            else:
                if rank + 1 < R:
                    comm.send_tensor(Z[nl - 1], rank + 1)   # feeds rank+1's current sweep
                if rank > 0:
                    comm.send_tensor(Z[0], rank - 1)        # feeds rank-1's next sweep
                if rank + 1 < R:
                    comm.recv_tensor(z_right, rank + 1)
        if stop.record(global_objective(comm, model.objective(theta), local_ids, n_total)):
            iters, converged = it, True
            break
    obj, loss, times = stop.arrays()
    n = len(obj)
    return RunResult(algorithm=name, obj=obj, loss=loss, iters=iters if converged else n, converged=converged,
                     wall_s=float(times[-1]) if n else 0.0, time_trace=times,
                     comm_units=np.arange(1, n + 1, dtype=np.float64) * n_total,
                     bytes_sent=run_bytes(comm, snap), bytes_total=total_bytes(comm, snap),
                     extra={"jacobi": jacobi, "nranks": R, "model_bytes": n * n_total * d * 8, "dim": d})
