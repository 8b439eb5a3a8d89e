"""Run results and small helpers shared by every algorithm."""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import numpy as np


@dataclass
class RunResult:
    """What every algorithm returns (the reference's ``[obj, loss, Iter, time(, com_cost)]`` plus
    the communication accounting the MI355X build adds).

    * ``obj``/``loss``: per-iteration global objective and ``|obj - obj0|`` (reference arrays);
    * ``iters``: the reference ``Iter`` (first iteration with loss < acc, else the budget);
    * ``comm_units``: cumulative reference communication units per iteration (1 per worker
      transmission: GADMM ``iter*N``, GD ``iter*N + iter``, LAG ``uploads + iter``;
      LinearRegression_Synthetic.m:100-142);
    * ``com_cost``: cumulative energy/distance cost where the reference tracks one (D-GADMM, E7);
    * ``wall_s``/``time_trace``: real wall clock (cumulative per iteration; native engines: the
      device's s_memrealtime at each iteration's stop decision);
    * ``model_time``: the reference's modelled clock, ``2 * toc`` of worker 1's local solve per
      iteration (utils/timing.py; group_ADMM_closedForm.m:39-42,53-55), when the caller sets it;
    * ``bytes_sent``: actual bytes this rank put on the fabric; ``bytes_total`` summed over ranks;
    * ``primal_res``: per-iteration consensus violation sum over chain edges ||th_n - th_right||^2
      (kernel K4's residual; chain algorithms).
    """

    algorithm: str
    obj: np.ndarray
    loss: np.ndarray
    iters: int
    converged: bool
    wall_s: float
    time_trace: np.ndarray = field(default_factory=lambda: np.zeros(0))
    comm_units: np.ndarray = field(default_factory=lambda: np.zeros(0))
    com_cost: Optional[np.ndarray] = None
    bytes_sent: int = 0
    bytes_total: int = 0
    extra: Dict[str, Any] = field(default_factory=dict)
    theta: Optional[np.ndarray] = None
    primal_res: Optional[np.ndarray] = None
    model_time: Optional[np.ndarray] = None

    def summary(self) -> Dict[str, Any]:
        return {
            "algorithm": self.algorithm,
            "iters": int(self.iters),
            "converged": bool(self.converged),
            "final_obj": float(self.obj[self.iters - 1]) if self.iters > 0 and len(self.obj) >= self.iters else None,
            "final_loss": float(self.loss[self.iters - 1]) if self.iters > 0 and len(self.loss) >= self.iters else None,
            "wall_s": float(self.wall_s),
            "comm_units": float(self.comm_units[self.iters - 1]) if len(self.comm_units) >= self.iters > 0 else None,
            "bytes_sent": int(self.bytes_sent),
            "bytes_total": int(self.bytes_total),
            "logical_bytes": (float(self.comm_units[self.iters - 1]) * 8 * int(self.extra["dim"])
                              if self.extra.get("dim") and len(self.comm_units) >= self.iters > 0
                              and not self.extra.get("energy_units") else None),
            **{k: v for k, v in self.extra.items() if isinstance(v, (int, float, str, bool))},
        }

    def first_below(self, tol: float) -> Optional[int]:
        idx = np.nonzero(self.loss < tol)[0]
        return int(idx[0]) + 1 if len(idx) else None


class Stopper:
    """Reference stop rule ``loss < acc`` -> Iter = i (group_ADMM_closedForm.m:105-108)."""

    def __init__(self, obj0: float, tol: float, max_iter: int):
        self.obj0, self.tol, self.max_iter = float(obj0), float(tol), int(max_iter)
        self.obj: List[float] = []
        self.loss: List[float] = []
        self.times: List[float] = []
        self.t0 = time.perf_counter()

    def record(self, obj: float) -> bool:
        self.obj.append(float(obj))
        self.loss.append(abs(float(obj) - self.obj0))
        self.times.append(time.perf_counter() - self.t0)
        return self.loss[-1] < self.tol

    def arrays(self):
        return np.asarray(self.obj), np.asarray(self.loss), np.asarray(self.times)


def run_bytes(comm, snap) -> int:
    """This rank's algorithm bytes since ``snap`` (p2p + algorithmic collectives, no monitoring)."""
    d = comm.stats.delta(snap)
    return int(d["bytes_sent"] + d["coll_bytes"])


def total_bytes(comm, snap=None) -> int:
    """Algorithm bytes summed over all ranks (one scalar all-reduce, outside any timed loop)."""
    import torch

    b = run_bytes(comm, snap) if snap is not None else int(comm.stats.bytes_sent) + int(comm.stats.coll_bytes)
    if comm.nranks <= 1:
        return b
    t = torch.tensor([float(b)], dtype=torch.float64)
    if getattr(comm, "backend", "").startswith("torch"):
        import torch.distributed as dist

        dist.all_reduce(t, group=comm.group)
    else:
        import torch.distributed as dist

        dist.all_reduce(t, group=getattr(comm, "control_group", None))
    return int(t.item())


def global_objective_and_residual(comm, f_local, r_local, local_ids, n_total: int):
    """``global_objective`` plus the summed primal residual in the same all-reduce (2N entries,
    one contributor each, summed in worker order)."""
    import torch

    full = torch.zeros((2, n_total), dtype=torch.float64, device=f_local.device)
    ids = torch.as_tensor(list(local_ids), dtype=torch.long, device=f_local.device)
    full[0, ids] = f_local
    full[1, ids] = r_local
    if comm is not None and comm.nranks > 1:
        comm.allreduce_sum(full)
        nb = full.numel() * full.element_size()
        comm.stats.coll_bytes -= nb
        comm.stats.monitor_bytes += nb
    s = full.sum(-1)
    return float(s[0].item()), float(s[1].item())


def global_objective(comm, f_local, local_ids, n_total: int) -> float:
    """Sum of per-worker objectives, identical for every rank count: the N-vector of worker
    objectives is all-reduced (each entry has one non-zero contributor, so the reduction is exact)
    and summed in worker order."""
    import torch

    full = torch.zeros(n_total, dtype=torch.float64, device=f_local.device)
    full[torch.as_tensor(list(local_ids), dtype=torch.long, device=f_local.device)] = f_local
    if comm is not None and comm.nranks > 1:
        comm.allreduce_sum(full)
        nb = full.numel() * full.element_size()
        comm.stats.coll_bytes -= nb       # monitoring, not algorithm traffic
        comm.stats.monitor_bytes += nb
    return float(full.sum().item())
