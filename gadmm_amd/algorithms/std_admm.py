"""Standard (star / parameter-server) ADMM — ``standared_ADMM.m``.

Worker N (the last one) is the hub and also owns a shard. Per iteration:
  1. workers 1..N-1 solve ``(A_i + rho I) x = b_i - lam_i + rho theta_hub``      (:42)
  2. the hub gathers ``sum lam_i`` and ``sum theta_i`` (RCCL reduce to the hub rank)  (:66-71)
  3. hub solves ``(A_N + (N-1) rho I) x = b_N + sum lam_i + rho sum theta_i``         (:73)
  4. hub broadcasts theta_hub (RCCL broadcast)
  5. ``lam_i += rho (theta_i - theta_hub)``                                           (:84-88)
Reference comm units: N-1 uploads + N-1 downloads per iteration.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from ..parallel.comm import Comm, LocalComm
from ..parallel.topology import Placement
from .base import RunResult, Stopper, total_bytes, global_objective, run_bytes


def standard_admm(model, local_ids: Sequence[int], n_total: int, rho: float, obj0: float, tol: float,
                  max_iter: int, comm: Optional[Comm] = None, placement: Optional[Placement] = None,
                  name: str = "ADMM(star)", backend: str = "auto", engine_opts: Optional[dict] = None) -> RunResult:
    """``backend``: 'native' = the persistent star kernel (csrc/kernels/star_persistent.hip, d <= 64; one
    GPU, or several with ``engine_opts={'fabric': XgmiFabric}``) or, for d > 64, the streaming large-d
    engine (csrc/kernels/star_big.hip: cached-inverse GEMVs, RCCL reduce / broadcast across GPUs, the
    stop rule on the device); 'torch' = batched torch ops with the comm's reduce/broadcast; 'auto' =
    native when it applies."""
    comm = comm if comm is not None else LocalComm()
    placement = placement if placement is not None else Placement.contiguous(n_total, comm.nranks)
    if model.kind != "linear":
        raise NotImplementedError("the reference star ADMM is closed-form linear only")
    opts = engine_opts or {}
    if backend in ("auto", "native") and model.device.type == "cuda" and model.d > 64:
        from ..engine.star_big import comm_ok
        from ..ops import native
        if comm_ok(comm) and native.available():
            return _standard_admm_big(model, local_ids, n_total, rho, obj0, tol, max_iter, comm, placement, name,
                                      opts)
        if backend == "native":
            raise RuntimeError("native large-d star ADMM needs one rank or an RCCL communicator")
    if backend in ("auto", "native") and model.device.type == "cuda" and model.d <= 64 \
            and (comm.nranks == 1 or opts.get("fabric") is not None):
        from ..ops import native
        if native.available():
            from ..utils.timing import roctx_range
            with roctx_range("%s native N=%d" % (name, n_total)):
                r = _standard_admm_native(model, local_ids, n_total, rho, obj0, tol, max_iter, comm, placement,
                                          name, opts)
            if r is not None:
                return r
        if backend == "native":
            raise RuntimeError("native star ADMM unavailable for this configuration")
    dev = model.device
    d = model.d
    hub = n_total - 1
    hub_rank = int(placement.owner[hub])
    local_ids = [int(w) for w in local_ids]
    lidx = {w: i for i, w in enumerate(local_ids)}
    workers = [w for w in local_ids if w != hub]
    wl = torch.tensor([lidx[w] for w in workers], dtype=torch.long, device=dev)
    lam = torch.zeros((len(local_ids), d), dtype=torch.float64, device=dev)
    theta = torch.zeros((len(local_ids), d), dtype=torch.float64, device=dev)
    theta_hub = torch.zeros(d, dtype=torch.float64, device=dev)
    stop = Stopper(obj0, tol, max_iter)
    snap = comm.stats.snapshot()
    iters, converged = max_iter, False
    for it in range(1, max_iter + 1):
        if len(workers):
            rhs = model.b.index_select(0, wl) - lam.index_select(0, wl) + rho * theta_hub
            theta[wl] = model.prox_solve(wl, rhs, torch.full((len(workers),), rho, dtype=torch.float64, device=dev))
        agg = torch.cat([lam.index_select(0, wl).sum(0), theta.index_select(0, wl).sum(0)]) if len(workers) \
            else torch.zeros(2 * d, dtype=torch.float64, device=dev)
        agg = agg.contiguous()
        if comm.nranks > 1:
            comm.reduce_sum(agg, hub_rank)
        if comm.rank == hub_rank:
            hl = torch.tensor([lidx[hub]], dtype=torch.long, device=dev)
            rhs = model.b[lidx[hub]] + agg[:d] + rho * agg[d:]
            th = model.prox_solve(hl, rhs.unsqueeze(0),
                                  torch.tensor([(n_total - 1) * rho], dtype=torch.float64, device=dev))[0]
            theta[lidx[hub]] = th
            theta_hub.copy_(th)
        if comm.nranks > 1:
            comm.broadcast(theta_hub, hub_rank)
        if len(workers):
            lam[wl] = lam.index_select(0, wl) + rho * (theta.index_select(0, wl) - theta_hub)
        if stop.record(global_objective(comm, model.objective(theta), local_ids, n_total)):
            iters, converged = it, True
            break
    obj, loss, times = stop.arrays()
    n = len(obj)
    return RunResult(algorithm=name, obj=obj, loss=loss, iters=iters if converged else n, converged=converged,
                     wall_s=float(times[-1]) if n else 0.0, time_trace=times,
                     comm_units=np.arange(1, n + 1, dtype=np.float64) * 2 * (n_total - 1),
                     bytes_sent=run_bytes(comm, snap), bytes_total=total_bytes(comm, snap),
                     extra={"hub": hub, "hub_rank": hub_rank, "nranks": comm.nranks})


def _standard_admm_native(model, local_ids, n_total, rho, obj0, tol, max_iter, comm, placement, name, opts):
    import time as _time
    from ..engine.star_engine import StarEngine

    fabric = opts.get("fabric")
    hub_rank = int(placement.owner[n_total - 1])
    key = ("star", n_total, tuple(int(w) for w in local_ids), float(rho), int(max_iter), id(fabric))
    cache = model.__dict__.setdefault("_star_engines", {})
    eng = cache.get(key)
    if eng is None:
        eng = StarEngine(model.X, model.y, local_ids, n_total, rho, obj0, tol, max_iter, hub_rank=hub_rank,
                         fabric=fabric, precomputed=(model.A, model.b, model.yy))
        ok = eng.eligible()
        if comm.nranks > 1:  # every rank's launch is needed: the choice is agreed (gloo)
            from ..parallel.node import agree
            ok = agree(ok, comm.nranks, getattr(comm, "control_group", None))
        if not ok:
            eng.close()
            return None
        cache[key] = eng
    elif opts.get("refresh"):
        eng.refresh(model.X, model.y)  # Gram + cached inverses from the raw shards, on the engine stream
    eng.obj0, eng.tol = float(obj0), float(tol)
    t0 = _time.perf_counter()
    iters, done, _ = eng.run(timeout_s=float(opts.get("timeout_s", 20.0)))
    wall = _time.perf_counter() - t0
    tr, tt = eng.objective_trace(iters), eng.time_trace(iters)
    if comm.nranks > 1:  # the monitor (rank 0) holds the trace: every rank returns the same result
        import torch.distributed as dist
        buf = torch.from_numpy(np.stack([tr, tt]).astype(np.float64))
        # a CPU tensor: the comm's gloo control group (the default group may be nccl under launch.py)
        dist.broadcast(buf, src=0, group=getattr(comm, "control_group", None))
        tr, tt = buf[0].numpy().copy(), buf[1].numpy().copy()
    pay, wire, mon = eng.bytes_per_solve(iters)
    return RunResult(algorithm=name, obj=tr, loss=np.abs(tr - obj0), iters=iters, converged=(done == 1), wall_s=wall,
                     time_trace=tt, comm_units=np.arange(1, iters + 1, dtype=np.float64) * 2 * (n_total - 1),
                     bytes_sent=int(pay), bytes_total=int(pay),
                     extra={"hub": n_total - 1, "hub_rank": hub_rank, "nranks": comm.nranks, "backend": "native",
                            "engine": eng.last_kernel, "wire_bytes": int(wire), "monitor_bytes": int(mon),
                            "transport": "xgmi" if fabric is not None else "local", "engine_obj": eng})


def _standard_admm_big(model, local_ids, n_total, rho, obj0, tol, max_iter, comm, placement, name, opts):
    """d > 64: the streaming star engine (engine/star_big.py), cached per (model, rho, N, ranks)."""
    from ..engine.star_big import StarBigEngine
    from ..utils.timing import roctx_range

    hub_rank = int(placement.owner[n_total - 1])
    exact = bool(opts.get("exact_objective", False))
    key = ("star_big", n_total, tuple(int(w) for w in local_ids), float(rho), comm.nranks, exact)
    cache = model.__dict__.setdefault("_star_engines", {})
    eng = cache.get(key)
    if eng is None:
        eng = StarBigEngine(model, local_ids, n_total, rho, comm, hub_rank=hub_rank, exact_objective=exact)
        cache[key] = eng
    snap = comm.stats.snapshot()
    with roctx_range("%s native-big N=%d" % (name, n_total)):
        iters, done, wall = eng.run(obj0, tol, max_iter, block=int(opts.get("block", 8)))
    tr, tt = eng.objective_trace(iters), eng.time_trace(iters)
    # the host enqueues whole blocks: collectives enqueued after the device-side stop are no-ops that
    # move nothing, so the bytes are the per-iteration payload times the iterations run (the comm's
    # enqueue counters, ``enqueued_coll_bytes``, include the skipped ones)
    coll = int(comm.stats.delta(snap).get("coll_bytes", 0)) if comm.nranks > 1 else 0
    sent = eng.coll_bytes_per_iteration() * iters
    return RunResult(algorithm=name, obj=tr, loss=np.abs(tr - obj0), iters=iters, converged=(done == 1), wall_s=wall,
                     time_trace=tt,
                     comm_units=np.arange(1, iters + 1, dtype=np.float64) * 2 * (n_total - 1),
                     bytes_sent=sent, bytes_total=sent,
                     extra={"hub": n_total - 1, "hub_rank": hub_rank, "nranks": comm.nranks, "backend": "native",
                            "engine": eng.last_kernel, "inverse_setup_s": eng.setup_s, "engine_obj": eng,
                            "transport": getattr(comm, "backend", "local"), "enqueued_coll_bytes": coll})
