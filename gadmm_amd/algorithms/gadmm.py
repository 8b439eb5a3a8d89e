"""Chain ADMM family: GADMM, D-GADMM, static-chain-with-cost, logistic variants.

Reference components:
  A1 ``group_ADMM_closedForm.m``        GADMM, linear, closed-form local solve
  A2 ``group_ADMM_logistic_GD.m``       GADMM, logistic, inexact local GD (A3 ``logReg_GD.m``)
  D2 ``group_ADMM_logistic.m``          GADMM, logistic, exact local solve (CVX) -> Newton here
  A4 ``dynamic_group_ADMM_closedForm.m``    D-GADMM (re-chain via findPath2 every coherence_Time)
  A5 ``dynamic_group_ADMM_closedForm_v0.m`` D-GADMM over pre-generated path/cost matrices
  A6 ``static_group_ADMM_closedForm.m``     identity chain, moving-node cost matrix

All of them are one algorithm on different chain schedules: heads (even chain positions) update in
parallel, their theta goes to the neighbouring tails, tails update, their theta goes back, and every
worker updates its aggregated dual ``mu_n`` (= lambda_n - lambda_{n-1}). Per-worker duals survive a
re-chain (dynamic_group_ADMM_closedForm.m:40-49 keeps the reset commented out).

Two executions of the same schedule:
* ``backend='torch'``: batched torch ops per phase on any device with any ``Comm`` (gloo CPU
  plumbing, torch.distributed on GPU, single process);
* ``backend='native'``: the C++/HIP chain engine (graph-replayed fused phase kernels with RCCL
  p2p, or the persistent single-launch kernel on one GPU). ``'auto'`` picks native on a HIP device.
"""
from __future__ import annotations

import time
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..parallel.comm import Comm, LocalComm
from ..parallel.topology import rechain_iterations, PathSchedule, Placement, chain_plan
from .base import global_objective_and_residual, RunResult, Stopper, total_bytes, global_objective, run_bytes
from ..utils import timing as _timing
from ..utils.timing import roctx_range
from ..utils.env import getenv


def _gather_rows(theta: torch.Tensor, ids: List[int]) -> torch.Tensor:
    idx = torch.tensor([max(i, 0) for i in ids], dtype=torch.long, device=theta.device)
    rows = theta.index_select(0, idx)
    mask = torch.tensor([1.0 if i >= 0 else 0.0 for i in ids], dtype=theta.dtype, device=theta.device)
    return rows * mask.unsqueeze(-1), mask


def chain_admm(model, local_ids: Sequence[int], n_total: int, rho: float, obj0: float, tol: float,
               max_iter: int, comm: Optional[Comm] = None, placement: Optional[Placement] = None,
               path: Optional[Sequence[int]] = None, schedule: Optional[PathSchedule] = None,
               local_solver: Optional[str] = None, step: float = 1.0, max_inner: int = 100,
               inner_tol: float = 1e-4, cost_quirk: bool = True, backend: str = "auto",
               name: str = "GADMM", record_theta: bool = False, engine_opts: Optional[dict] = None,
               state=None, check_exchange: Optional[bool] = None,
               failures: Optional[dict] = None) -> RunResult:
    """Run one chain-ADMM solve on this rank. ``model`` holds this rank's shards (local order =
    ``local_ids``). ``schedule`` (D-GADMM) overrides ``path``; ``cost_quirk`` reproduces the
    reference's per-head-worker accumulation of ``sum(pathCost)`` (dynamic_group_ADMM_closedForm.m:51-55).
    ``state``: optional ``(theta_table, mu, start_iter)`` to resume from a checkpoint (natively on one
    rank with a static chain; torch path otherwise).
    ``check_exchange`` (or ``GADMM_CHECK_EXCHANGE=1``): verify every ghost row against its owner after
    every exchange (debug/race.py; forces the torch path).
    ``failures``: ``{iteration: [worker ids]}`` - elastic recovery: at that iteration
    the workers drop out, the chain re-forms over the survivors, each failed worker's aggregated
    dual is handed to a surviving chain neighbour (keeping sum(mu) = 0, the consensus-dual
    invariant) and the stopping target becomes the survivors' optimum (linear models; natively on
    one rank with a static chain, ``_chain_admm_native_elastic``; torch path otherwise)."""

    comm = comm if comm is not None else LocalComm()
    if check_exchange is None:
        check_exchange = getenv("GADMM_CHECK_EXCHANGE", "0") == "1"
    placement = placement if placement is not None else Placement.contiguous(n_total, comm.nranks)
    if schedule is None:
        p0 = list(path) if path is not None else list(range(n_total))
        schedule = PathSchedule(n_total, p0, np.zeros(max(n_total - 1, 0)), coherence=0)
    if local_solver is None:
        local_solver = "closed" if model.kind == "linear" else "gd"
    dev = model.device
    use_native = False
    native_solver = local_solver in ("closed", "gd") or (
        local_solver == "newton" and model.kind == "logistic" and model.d <= 64 and model.m <= 64)
    # resume (``state``) and elastic recovery (``failures``) run natively on one rank with a static
    # chain; across ranks, with re-chaining, or under the exchange checker they take the torch path
    one_static = comm.nranks == 1 and _static_schedule(schedule, max_iter)
    native_state = state is None or one_static
    native_fail = not failures or (one_static and model.kind == "linear" and local_solver == "closed"
                                   and sorted(int(w) for w in local_ids) == list(range(n_total)))
    if backend in ("auto", "native") and dev.type == "cuda" and native_solver and native_state \
            and not check_exchange and native_fail:
        from ..ops import native

        if native.available() and (comm.nranks == 1 or getattr(comm, "backend", "") in ("rccl", "ipc")
                                   or (engine_opts or {}).get("fabric") is not None):
            use_native = True
        elif backend == "native":
            raise RuntimeError("native backend requested but unavailable for this comm/device")
    if use_native:
        # a named range per solve in rocprofv3 --marker-trace timelines (no-op without roctx)
        with roctx_range("%s native N=%d" % (name, n_total)):
            if failures:
                return _chain_admm_native_elastic(model, n_total, rho, obj0, tol, max_iter, schedule, cost_quirk,
                                                  name, engine_opts or {}, failures)
            return _chain_admm_native(model, local_ids, n_total, rho, obj0, tol, max_iter, comm, placement,
                                      schedule, local_solver, step, max_inner, inner_tol, cost_quirk, name,
                                      engine_opts or {}, state=state)
    return _chain_admm_torch(model, local_ids, n_total, rho, obj0, tol, max_iter, comm, placement, schedule,
                             local_solver, step, max_inner, inner_tol, cost_quirk, name, record_theta, state,
                             check_exchange, failures)


def _chain_admm_torch(model, local_ids, n_total, rho, obj0, tol, max_iter, comm, placement, schedule,
                      local_solver, step, max_inner, inner_tol, cost_quirk, name, record_theta, state,
                      check_exchange=False, failures=None):
    rank = comm.rank
    checker = None
    if check_exchange:
        from ..debug.race import ExchangeChecker

        checker = ExchangeChecker(comm, local_ids, n_total)
        owner = [int(o) for o in placement.owner]
    d = model.d
    dev = model.device
    local_ids = [int(w) for w in local_ids]
    if state is not None:
        theta = state[0].to(dev).clone()
        mu = state[1].to(dev).clone()
        start = int(state[2])
    else:
        theta = torch.zeros((n_total, d), dtype=torch.float64, device=dev)
        mu = torch.zeros((len(local_ids), d), dtype=torch.float64, device=dev)
        start = 1
    stop = Stopper(obj0, tol, max_iter)
    snap = comm.stats.snapshot()
    alive = np.ones(n_total, dtype=bool)
    failures = {int(k): [int(w) for w in v] for k, v in (failures or {}).items()}
    if failures and model.kind != "linear":
        raise NotImplementedError("elastic failures: linear models (the survivors' optimum is closed form)")
    lidx_of = {w: i for i, w in enumerate(local_ids)}
    plan = chain_plan(schedule.path, placement, rank)
    cc = 0.0
    com_cost: List[float] = []
    inner_used: List[float] = []
    primal: List[float] = []
    iters = max_iter
    converged = False
    for it in range(start, max_iter + 1):
        if it in failures:
            obj0 = _drop_workers(failures[it], alive, schedule, theta, mu, lidx_of, model, comm, n_total, dev)
            stop.obj0 = obj0
            plan = chain_plan([w for w in schedule.path if alive[w]], placement, rank)
            comm.exchange_rows(theta, plan.xchg_tail)  # new cross-rank neighbours
        if schedule.step(it):
            plan = chain_plan([w for w in schedule.path if alive[w]], placement, rank)
            # new cross-rank neighbours: heads need their (new) tails' current theta first
            comm.exchange_rows(theta, plan.xchg_tail)
            if checker is not None:
                checker.verify(theta, [r for _, r, s in plan.xchg_tail if not s], it, "re-chain", owner)
        n_heads = (n_total + 1) // 2
        cc += float(np.sum(schedule.cost)) * (n_heads if cost_quirk else 1)
        com_cost.append(cc)
        for slots, xchg in ((plan.head, plan.xchg_head), (plan.tail, plan.xchg_tail)):
            if slots:
                li = torch.tensor([s.li for s in slots], dtype=torch.long, device=dev)
                gid = [s.gid for s in slots]
                thl, ml = _gather_rows(theta, [s.left for s in slots])
                thr, mr = _gather_rows(theta, [s.right for s in slots])
                deg = ml + mr
                m_li = mu.index_select(0, li)
                if local_solver == "closed":
                    rhs = model.b.index_select(0, li) - m_li + rho * thl + rho * thr
                    new = model.prox_solve(li, rhs, deg * rho)
                elif local_solver == "gd":
                    thw = theta.index_select(0, torch.tensor(gid, device=dev))
                    shift = m_li + rho * (thw - thl) * ml.unsqueeze(-1) + rho * (thw - thr) * mr.unsqueeze(-1)
                    new, used = model.inexact_gd(li, thw, shift, step, max_inner, inner_tol)
                    inner_used.append(float(used.double().mean()))
                elif local_solver == "newton":
                    thw = theta.index_select(0, torch.tensor(gid, device=dev))
                    quad = deg * rho
                    center = (thl + thr) / torch.clamp(deg, min=1.0).unsqueeze(-1)
                    new = model.newton_prox(li, thw, m_li, quad, center)
                else:
                    raise ValueError("unknown local solver %r" % local_solver)
                theta[torch.tensor(gid, dtype=torch.long, device=dev)] = new
            comm.exchange_rows(theta, xchg)
            if checker is not None:
                checker.verify(theta, [r for _, r, s in xchg if not s], it,
                               "head" if xchg is plan.xchg_head else "tail", owner)
        # dual update, reference order: mu - rho (th_l - th) + rho (th - th_r)
        for slots in (plan.head, plan.tail):
            if not slots:
                continue
            li = torch.tensor([s.li for s in slots], dtype=torch.long, device=dev)
            thw = theta.index_select(0, torch.tensor([s.gid for s in slots], device=dev))
            thl, ml = _gather_rows(theta, [s.left for s in slots])
            thr, mr = _gather_rows(theta, [s.right for s in slots])
            m = mu.index_select(0, li)
            m = m - rho * (thl - thw) * ml.unsqueeze(-1)
            m = m + rho * (thw - thr) * mr.unsqueeze(-1)
            mu[li] = m
        th_loc = theta.index_select(0, torch.tensor(local_ids, dtype=torch.long, device=dev))
        f = model.objective(th_loc)
        if not alive.all():
            f = f * torch.as_tensor(alive[local_ids], dtype=f.dtype, device=dev)
        # consensus residual of the edges this rank's workers start (edge n -> right neighbour)
        res_loc = torch.zeros(len(local_ids), dtype=torch.float64, device=dev)
        for s_ in plan.head + plan.tail:
            if s_.right >= 0:
                dlt = theta[s_.gid] - theta[s_.right]
                res_loc[s_.li] = dlt @ dlt
        f_all, r_all = global_objective_and_residual(comm, f, res_loc, local_ids, n_total)
        primal.append(r_all)
        if stop.record(f_all):
            iters = it
            converged = True
            break
    obj, loss, times = stop.arrays()
    n_it = len(obj)
    res = RunResult(algorithm=name, obj=obj, loss=loss, iters=iters if converged else (start - 1 + n_it),
                    converged=converged, wall_s=float(times[-1]) if n_it else 0.0, time_trace=times,
                    comm_units=np.arange(start, start + n_it, dtype=np.float64) * n_total,
                    com_cost=np.asarray(com_cost), bytes_sent=run_bytes(comm, snap),
                    bytes_total=total_bytes(comm, snap),
                    extra={"backend": "torch", "rank": rank, "nranks": comm.nranks, "solver": local_solver,
                           "inner_steps_mean": float(np.mean(inner_used)) if inner_used else 0.0,
                           "monitor_bytes": int(comm.stats.delta(snap)["monitor_bytes"])},
                    primal_res=np.asarray(primal))
    res.extra["state"] = (theta, mu, (iters if converged else start - 1 + n_it) + 1)
    if record_theta:
        res.theta = theta.cpu().numpy()
    return res


_RECHAINS: dict = {}


def _rechains(max_iter: int, coherence) -> np.ndarray:
    """``rechain_iterations`` memoised per (max_iter, coherence) (read-only array)."""
    key = (int(max_iter), float(coherence))
    r = _RECHAINS.get(key)
    if r is None:
        r = rechain_iterations(max_iter, coherence)
        r.setflags(write=False)
        if len(_RECHAINS) < 64:
            _RECHAINS[key] = r
    return r


def _max_epochs(eng) -> int:
    """gadmm_chain_blocked_max_epochs (a constant of the build), asked once per engine."""
    v = eng.__dict__.get("_max_epochs")
    if v is None:
        v = eng._max_epochs = int(eng.lib.gadmm_chain_blocked_max_epochs())
    return v


def _dyn_early_draw(eng, schedule, max_iter, fabric, n_total):
    """``(saved schedule state, epochs drawn, join)`` for the first D-GADMM launch's chains started
    asynchronously (PathSchedule.prefetch_async), with the chunk / look-ahead rule of the launch loop in
    ``_chain_admm_native``; None when the dynamic persistent path or the native builder does not
    apply."""
    if not eng.dynamic_eligible(fabric):
        return None
    rechains = _rechains(max_iter, schedule.coherence)
    if len(rechains) >= (1 << 20):
        return None
    hints = eng.__dict__.get("_dyn_epoch_hint", {})
    hk = (float(schedule.coherence), schedule.kind, int(max_iter), int(n_total))
    chunk = max(16, int(hints[hk]) + 8) if hk in hints else 128
    if eng.dynamic_uses_blocked(fabric, schedule.coherence):
        chunk = min(chunk, _max_epochs(eng) - 1)
    E_total = 1 + len(rechains)
    e1 = min(chunk, E_total)
    look = e1 if e1 < E_total else e1 - 1
    if look <= 0:
        return None
    saved = schedule.save()
    join = schedule.prefetch_async(look)
    if join is None:
        return None
    return saved, look, join


def _static_schedule(schedule, max_iter) -> bool:
    return not schedule.coherence or not np.isfinite(schedule.coherence) or schedule.coherence <= 0 \
        or schedule.coherence >= max_iter + 1


def _chain_admm_native(model, local_ids, n_total, rho, obj0, tol, max_iter, comm, placement, schedule, local_solver,
                       step, max_inner, inner_tol, cost_quirk, name, opts, state=None):
    """``opts``: ``block`` (iterations per graph replay), ``persistent`` (auto/True/False), ``graph``,
    ``cache``, ``state``, ``refresh`` (recompute Gram + inverses from the raw shards first), ``fabric`` (an ``XgmiFabric``: the device-initiated multi-GPU persistent
    kernels; with ``table_slots >= lag + 4`` it also runs multi-rank D-GADMM in one launch),
    ``stop_iter`` (static chains: run no iteration past it, on the graph engine - the persistent
    kernels stop only at the decision).
    ``state``: ``(theta_table (n_total, d), mu (n_local, d), start_iter)`` - resume a static chain
    from a checkpoint (one rank): the engine's tables are loaded and the kernels start at
    ``start_iter`` with no pending head duals (a saved state has them applied); the result covers
    iterations ``start_iter..iters`` like the torch path's."""
    from ..engine.chain_engine import NativeChainEngine, ResidencyError, HandoffTimeout

    _timing.host_stamp("native:start")
    rank = comm.rank
    rcomm = comm if comm.nranks > 1 else None
    fabric = opts.get("fabric")
    kind = "linear" if local_solver == "closed" else "logistic"
    # iterations per replayed graph: a logistic phase is ~37 us, so the replays left over after the stop
    # decision cost more than the extra host round trips of short blocks (tools/logistic_block_sweep.py:
    # 6.78 / 6.81 / 6.88 / 7.11 ms for 8 / 16 / 32 / 64)
    block = int(opts.get("block", 16 if comm.nranks > 1 else (8 if kind == "logistic" else 32)))
    pre = (model.A, model.b, model.yy) if kind == "linear" else None
    # one engine per (model, configuration) on a single rank: repeated solves (rho sweeps, benchmarks,
    # D-GADMM re-runs) reuse its device buffers, cached inverses and captured graph
    key = (kind, local_solver, n_total, tuple(map(int, local_ids)), float(rho), int(max_iter), block,
           float(step), int(max_inner), float(inner_tol), float(getattr(model, "lam", 0.0)),
           opts.get("chord"), bool(opts.get("residual", True)))
    cache = getattr(model, "_chain_engines", None) if rcomm is None else None
    eng = cache.get(key) if cache is not None else None
    fresh = eng is None
    # ``refresh``: the solve starts from the raw shards -- the Gram (K1) and the cached inverses (K2) are
    # recomputed (benchmarks time the same set-up in every config: bench.py's headline does this too)
    refresh = bool(opts.get("refresh", False)) and kind == "linear"
    if eng is None and refresh:
        from ..ops.linalg import gram
        gram(model.X, model.y, out=(model.A, model.b, model.yy))  # the new engine inverts the fresh Gram
    # D-GADMM on a cached engine: the first launch's chains start drawing now (geometries from the
    # schedule's RNG here, greedy walks on the native host worker) and are joined where the launch's
    # tables are built, so the walks overlap the refresh / set_path / reset below
    early = None
    if eng is not None and state is None and not _static_schedule(schedule, max_iter) \
            and opts.get("persistent", "auto") in (True, "auto") and "epoch_chunk" not in opts \
            and getenv("GADMM_DGADMM_EARLY", "1") != "0":
        early = _dyn_early_draw(eng, schedule, max_iter, fabric, n_total)
        _timing.host_stamp("native:early_draw")
    try:
        if eng is not None and refresh:
            # in place on the engine's stream (Gram, then inverses), while the native worker walks the
            # early-drawn chains (launching the refresh before the draw exposed the walks at the join:
            # profiles/r06_dgadmm)
            eng.refresh(model.X, model.y)
            _timing.host_stamp("native:refresh")
        if eng is None:
            eng = NativeChainEngine(model.X, model.y, local_ids, n_total, kind, rho=rho, obj0=obj0, tol=tol,
                                    max_iter=max_iter, lam=getattr(model, "lam", 0.0), step=step, max_inner=max_inner,
                                    inner_tol=inner_tol, comm=rcomm, block=block, precomputed=pre,
                                    local_solver="newton" if local_solver == "newton" else "gd",
                                    chord=None if opts.get("chord") is None else float(opts["chord"]),
                                    residual=bool(opts.get("residual", True)),
                                    obj_mode=str(opts.get("obj_mode", "auto")))
            if rcomm is None and opts.get("cache", True):
                if cache is None:
                    cache = {}
                    model._chain_engines = cache
                cache[key] = eng
        else:
            eng.set_targets(obj0, tol)
        _timing.host_stamp("native:engine")
        eng.set_path(schedule.path, placement, rank)
        _timing.host_stamp("native:set_path")
        start = 1 if state is None else int(state[2])
        static = _static_schedule(schedule, max_iter)
        if state is not None and not (static and comm.nranks == 1):
            raise ValueError("native resume: one rank, static chain")

        def load_state():  # fresh solve state, or the checkpoint's tables at start_iter (no pending duals)
            eng.reset(start_iter=start)
            if state is not None:
                eng.stream.wait_stream(torch.cuda.current_stream(model.device))  # the state's producers
                with torch.cuda.stream(eng.stream):
                    eng.theta.copy_(state[0].to(eng.theta.device, torch.float64).reshape(eng.theta.shape))
                    eng.mu.copy_(state[1].to(eng.mu.device, torch.float64).reshape(eng.mu.shape))

        load_state()
        _timing.host_stamp("native:reset")
        stop_iter = int(opts.get("stop_iter", 0))
        if fresh or state is not None:
            # inputs made on other streams (a new engine's set-up, a loaded state) are complete before the
            # solve; a cached engine's inputs are, and its own stream orders the reset before the kernel
            torch.cuda.synchronize(model.device)
    except BaseException:
        # the early draw moved the schedule's RNG ahead of its chains: join the worker and rewind, so a
        # re-run of this schedule draws the same chain sequence (seeded D-GADMM reproducibility)
        if early is not None:
            early[2]()
            schedule.restore(early[0])
        raise
    if fabric is not None and comm.nranks > 1:
        # the device-initiated kernels need every rank's launch: their eligibility is agreed, and a rank
        # that cannot run them sends every rank to the graph engine over the session's data plane
        import torch.distributed as dist
        elig = opts.get("persistent", "auto") in (True, "auto") and (
            eng.persistent_eligible(fabric) if static else eng.dynamic_eligible(fabric))
        t = torch.tensor([0.0 if elig else 1.0], dtype=torch.float64)
        dist.all_reduce(t, group=getattr(comm, "control_group", None))
        if float(t.item()) != 0.0:
            eng.close()
            fb = opts.get("fallback_comm")
            if fb is None:
                raise RuntimeError("%s: the xGMI kernel is not eligible on some rank and no data-plane "
                                   "fallback was given" % name)
            o2 = {k: v for k, v in opts.items() if k not in ("fabric", "fallback_comm")}
            res = _chain_admm_native(model, local_ids, n_total, rho, obj0, tol, max_iter, fb, placement, schedule,
                                     local_solver, step, max_inner, inner_tol, cost_quirk, name, o2, state=state)
            res.extra["fabric_fallback"] = "xgmi kernel not eligible on some rank: %s" % getattr(fb, "backend", "")
            return res
    t0 = time.perf_counter()
    cc = 0.0
    com_cost = []
    n_heads = (n_total + 1) // 2
    p2p = 0
    mon = 0
    wire = 0
    want_persistent = opts.get("persistent", "auto") in (True, "auto")
    if static:
        r = None
        engine_kind = None
        if want_persistent and stop_iter <= 0 and eng.persistent_eligible(fabric):
            try:
                r = eng.run_persistent(fabric=fabric, start_iter=start, fetch_trace=True)
                engine_kind = "persistent"
            except (ResidencyError, HandoffTimeout) as e:
                # the device could not hold every workgroup, or a hand-off stalled: the graph engine
                # runs the same schedule without co-residency (single rank; several ranks must agree,
                # see bench.py, so they raise)
                if comm.nranks > 1:
                    raise
                load_state()
                engine_kind = "graph(fallback: %s)" % type(e).__name__
        if r is None:
            r = eng.run(stop_iter=stop_iter, use_graph=opts.get("graph", True))
            if engine_kind is None:
                engine_kind = "graph" if eng.graph_ok() else "eager"
        iters, done = r.iters, r.done
        p2p, mon, wire = r.p2p_bytes, r.monitor_bytes, r.wire_bytes
        per = float(np.sum(schedule.cost)) * (n_heads if cost_quirk else 1)
        com_cost = np.arange(1, iters - start + 2) * per
        if local_solver == "newton" and not opts.get("_exact_retry"):
            # chord-Newton safety net: a local solve that reached the 50-step cap unconverged (a stale
            # inverse can send the first chord steps far off: the derm-shaped E4 problem at rho = 0.02) means
            # the iterates are not the exact prox the spec asks for (group_ADMM_logistic.m:26-49) -- the
            # whole solve is re-run with exact Newton steps (every step refreshes its inverse), as torch does
            fails = int(eng.ctl[7].item())
            chord_used = eng.chord_persistent if engine_kind == "persistent" else eng.chord
            if comm.nranks > 1:
                import torch.distributed as dist
                t = torch.tensor([float(fails)], dtype=torch.float64)
                dist.all_reduce(t, group=getattr(comm, "control_group", None))
                fails = int(t.item())
            if fails > 0 and chord_used > 0.0:
                res2 = _chain_admm_native(model, local_ids, n_total, rho, obj0, tol, max_iter, comm, placement,
                                          schedule, local_solver, step, max_inner, inner_tol, cost_quirk, name,
                                          dict(opts, chord=0.0, cache=False, _exact_retry=fails), state=state)
                res2.extra["chord_fallback"] = "%d unconverged chord-Newton local solves: re-run exact" % fails
                return res2
    elif want_persistent and eng.dynamic_eligible(fabric) \
            and len(_rechains(max_iter, schedule.coherence)) < (1 << 20):
        # D-GADMM in persistent launches of up to `epoch_chunk` epochs each: the seeded chain sequence
        # is drawn a chunk ahead (batched, the identical RNG stream), every worker switches neighbours /
        # role at each epoch on the device. A chunk ends at a hard stop just before its last+1 epoch
        # (whose neighbours already receive theta); unless the monitor decided a stop, the next launch
        # continues with the same tag salt from there. Only the chains a solve reaches are drawn.
        engine_kind = "persistent-dynamic"
        rechains = _rechains(max_iter, schedule.coherence)
        # first launch: `epoch_chunk` epochs, each continuation twice the previous. Drawing a chain
        # costs ~0.75 us on the host, a launch + read-back ~0.25 ms: 128 keeps coherence-10 solves
        # (~51 epochs) to one launch with few spare chains, coherence-1 solves (~250) to two
        # Without an explicit chunk, a repeat of a schedule of the same shape (coherence, kind, max_iter,
        # N) on this engine sizes its first launch from the epochs the previous solve reached (+ margin):
        # chains beyond them would be drawn for nothing. Only the launch size follows the hint; the
        # chains and iterates do not (a shortfall costs a continuation launch).
        hint_key = (float(schedule.coherence), schedule.kind, int(max_iter), int(n_total))
        hints = eng.__dict__.setdefault("_dyn_epoch_hint", {})
        if "epoch_chunk" in opts:
            chunk = max(1, int(opts["epoch_chunk"]))
        elif hint_key in hints:
            chunk = max(16, int(hints[hint_key]) + 8)
        else:
            chunk = 128
        # the blocked kernel's dynamic mode stages a launch's epoch tables in LDS: at most
        # gadmm_chain_blocked_max_epochs rows per launch (this chunk + the look-ahead epoch)
        use_blk = eng.dynamic_uses_blocked(fabric, schedule.coherence)
        cap = _max_epochs(eng) - 1 if use_blk else 1 << 30
        chunk = min(chunk, cap)
        saved = early[0] if early is not None else schedule.save()
        E_total = 1 + len(rechains)
        # epoch e's chain is row e of one (E_total, N) table, filled as chains are drawn (epoch 0: the
        # initial chain); epoch e starts at iteration ep_start[e]
        Pall = np.empty((E_total, n_total), dtype=np.int64)
        Pall[0] = saved[1]
        ep_start = np.concatenate([np.ones(1, dtype=np.int64), rechains])
        drawn_C = []
        n_drawn = [1]

        pend = [early]

        def ensure(upto):  # epochs 0..upto drawn
            need = upto + 1 - n_drawn[0]
            if pend[0] is not None:  # the early draw covers epochs 1..early[1]
                e_ = pend[0]
                pend[0] = None
                if n_drawn[0] == 1 and need >= e_[1]:
                    Pn_, Cn_ = e_[2]()
                    Pall[1:1 + e_[1]] = Pn_
                    n_drawn[0] += e_[1]
                    drawn_C.append(Cn_)
                    need -= e_[1]
                else:  # not this shape (cannot happen: same chunk rule); the schedule restarts from it
                    e_[2]()
                    schedule.restore(e_[0])
            if need > 0:
                Pn_, Cn_ = schedule.prefetch_arrays(need)
                Pall[n_drawn[0]:n_drawn[0] + need] = Pn_
                n_drawn[0] += need
                drawn_C.append(Cn_)

        e0, start_iter, pending_in, cont = 0, 1, 0, False
        done = iters = 0
        last_launched = 0
        pre = {}
        ep_all = ep_start  # every epoch's first iteration (ep_start is truncated after the launches)

        def cost_arrays():
            """Per-epoch chain costs of every epoch drawn so far and the cumulative com_cost of each
            iteration they cover: needs no outcome, so it runs while the launch executes
            (run_persistent's on_enqueued) instead of after it."""
            nd = n_drawn[0]
            if pre.get("nd") == nd:
                return
            if drawn_C and any(c.dtype == object for c in drawn_C):
                Cn_ = np.empty(sum(len(c) for c in drawn_C), dtype=object)
                Cn_[:] = [c for cc in drawn_C for c in cc]
            else:
                Cn_ = np.concatenate(drawn_C) if drawn_C else np.zeros((0, max(n_total - 1, 0)))
            # per-epoch cost; the initial cost vector may be ragged (the v0 column-slice quirk)
            csum = Cn_.sum(axis=1) if (len(Cn_) and Cn_.dtype != object) else np.asarray([float(np.sum(c)) for c in Cn_])
            per_it_ = np.concatenate([[float(np.sum(saved[2]))], csum]) * (n_heads if cost_quirk else 1)
            span = int(ep_all[nd] - 1) if nd < E_total else int(max_iter)  # iterations the drawn epochs cover
            which_ = np.searchsorted(ep_all[:nd], np.arange(1, span + 1), side="right") - 1
            pre.update(nd=nd, Cn=Cn_, com=np.cumsum(per_it_[which_]))
        while True:
            e1 = min(e0 + chunk, E_total)  # this launch executes epochs e0 .. e1 - 1
            look = e1 if e1 < E_total else e1 - 1  # + the next epoch's chain (push targets of theta^hard_stop)
            _timing.host_stamp("dyn:chunk_setup")
            ensure(look)
            _timing.host_stamp("dyn:draws")
            hard_stop = ep_start[e1] - 1 if e1 < E_total else 0
            st_arr = ep_start[e0:look + 1]
            P_arr = Pall[e0:look + 1]
            timed_out = None
            try:
                r = eng.run_persistent(epochs=(st_arr, P_arr), fabric=fabric, start_iter=start_iter,
                                       pending_in=pending_in, hard_stop=hard_stop, cont=cont, fetch_trace=True,
                                       blocked_dyn=use_blk, on_enqueued=cost_arrays)
            except HandoffTimeout as e:
                if comm.nranks == 1:
                    raise
                timed_out = e  # agree with the other ranks first: they may be waiting on this chunk's outcome
                r = None
            done, iters = (int(r.done), int(r.iters)) if r is not None else (4, 0)
            if comm.nranks > 1:
                # every chunk ends in ONE collective on every rank: the monitor rank holds the outcome
                # (the workers may stop at the hard stop before the decision of its last lag iterations
                # reaches them), and a timeout on ANY rank is agreed in the same all-reduce, so all ranks
                # raise together instead of the others waiting in a broadcast until the group's timeout.
                # MAX over [rank 0's (done, iters) | -1 elsewhere, failed flag].
                import torch.distributed as dist
                mine = comm.rank == 0
                t = torch.tensor([float(done) if mine else -1.0, float(iters) if mine else -1.0,
                                  1.0 if timed_out is not None else 0.0], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=getattr(comm, "control_group", None))
                if float(t[2].item()) > 0:
                    raise HandoffTimeout("D-GADMM chunk: a persistent hand-off timed out on some rank"
                                         + (" (here: %s)" % timed_out if timed_out is not None else ""))
                done, iters = int(t[0].item()), int(t[1].item())
            p2p, mon, wire = p2p + r.p2p_bytes, mon + r.monitor_bytes, wire + r.wire_bytes
            last_launched = hard_stop if done == 5 else start_iter - 1 + int(r.iterations_launched)
            if done != 5:
                if done == 0:
                    raise RuntimeError("D-GADMM chunk ended without an outcome (hard stop %d)" % hard_stop)
                break
            start_iter, pending_in, cont = hard_stop + 1, 1, True
            e0 = e1 - 1  # epoch 0 of the next launch: this chunk's last (the flush of pending duals)
            chunk = min(2 * chunk, cap)
        _timing.host_stamp("dyn:launches_done")
        if done == 5:
            done = 2
        ep_start = ep_start[:n_drawn[0]]
        hints[hint_key] = int(np.searchsorted(ep_start, max(last_launched, 1), side="right"))
        Pn = Pall[1:n_drawn[0]]
        cost_arrays()  # already done while the last launch ran, unless it drew more epochs since
        Cn = pre["Cn"]
        starts = ep_start
        P = Pall[:n_drawn[0]]
        com_cost = pre["com"][:iters]
        # leave the schedule (and the engine's plan) where the epoch-by-epoch run would have left them --
        # unless nobody can look: a schedule private to this call (dynamic_group_admm builds one per solve)
        # with no state to flush (~6 us of host time per D-GADMM solve, profiles/r06_dgadmm)
        if not getattr(schedule, "private", False) or opts.get("state", True):
            schedule.skip(saved, Pn, Cn, int(np.searchsorted(rechains, iters, side="right")))  # rechains ascend
            eng.set_path(P[int(np.searchsorted(starts, max(last_launched, 1), side="right") - 1)], placement, rank)
    else:
        # D-GADMM: run epoch by epoch; at a re-chain iteration flush the heads' pending duals with the
        # old chain, install the new chain, continue. Every rank draws the same chain sequence.
        if early is not None:  # (not reached with an early draw: it requires the dynamic path) undo it
            early[2]()
            schedule.restore(early[0])
        engine_kind = "epochs"
        it = 1
        done = 0
        iters = 0
        while it <= max_iter and not done:
            nxt = it + 1
            while nxt <= max_iter and not _is_rechain(nxt, schedule.coherence):
                nxt += 1
            per = float(np.sum(schedule.cost)) * (n_heads if cost_quirk else 1)
            r = eng.run(stop_iter=nxt - 1, use_graph=False)
            p2p += r.p2p_bytes
            mon += r.monitor_bytes
            wire += r.wire_bytes
            ran_to = r.iters
            for _ in range(it, ran_to + 1):
                cc += per
                com_cost.append(cc)
            done = r.done
            iters = ran_to
            if done or nxt > max_iter:
                break
            eng.flush_duals()
            schedule.step(nxt)
            eng.set_path(schedule.path, placement, rank)
            if comm.nranks > 1:
                eng.exchange("tail")  # refresh ghost rows of the new cross-rank neighbours
            it = nxt
    _timing.host_stamp("native:solved")
    if engine_kind not in ("persistent", "persistent-dynamic"):  # those synchronised after their launch
        eng.stream.synchronize()
    wall = time.perf_counter() - t0
    tr, tt = eng.traces(iters)
    if start > 1:  # a resumed solve reports iterations start..iters (as the torch path does)
        tr, tt = tr[start - 1:], tt[start - 1:]
    if fabric is not None and comm.nranks > 1:
        # the xGMI kernels decide on rank 0's monitor only: give every rank the same trace and clock
        import torch.distributed as dist

        buf = torch.from_numpy(np.stack([tr, tt]).astype(np.float64))
        dist.broadcast(buf, src=0, group=getattr(comm, "control_group", None))
        tr, tt = buf[0].numpy().copy(), buf[1].numpy().copy()
    loss = np.abs(tr - obj0)
    pres = eng.primal_residual(iters)  # K4, emitted by the kernels' tails (this rank's edges)
    if pres is not None and start > 1:
        pres = pres[start - 1:]
    if pres is not None and comm.nranks > 1:
        import torch.distributed as dist

        buf = torch.from_numpy(pres.astype(np.float64))
        dist.all_reduce(buf, group=getattr(comm, "control_group", None))
        pres = buf.numpy()
    bytes_tot = p2p
    if comm.nranks > 1:
        import torch.distributed as dist

        t = torch.tensor([float(p2p)], dtype=torch.float64)
        dist.all_reduce(t, group=getattr(comm, "control_group", None))
        bytes_tot = int(t.item())
    res = RunResult(algorithm=name, obj=tr, loss=loss, iters=iters, converged=(done == 1), wall_s=wall,
                    time_trace=tt,  # measured on the device: decision time of each iteration
                    comm_units=np.arange(start, iters + 1, dtype=np.float64) * n_total,
                    com_cost=np.asarray(com_cost[:iters - start + 1]), bytes_sent=int(p2p), bytes_total=bytes_tot,
                    primal_res=pres,
                    extra={"backend": "native", "engine": engine_kind, "rank": rank, "nranks": comm.nranks,
                           "solver": local_solver, "monitor_bytes": int(mon), "wire_bytes": int(wire),
                           "transport": getattr(comm, "backend", "local") if fabric is None else "xgmi",
                           # effective settings (engine-dependent defaults): the objective
                           # evaluation of the phase kernels and, for Newton, the chord threshold used
                           "obj_mode": eng.obj_mode_name})
    if local_solver == "newton":
        res.extra["chord"] = eng.chord_persistent if str(engine_kind).startswith("persistent") else eng.chord
    res.extra["engine_obj"] = eng
    _timing.host_stamp("native:result")
    if opts.get("state", True):
        # resumable state for checkpoints: (theta, mu) after the STOPPING iteration, whatever engine ran.
        # A persistent kernel learns the monitor's decision `lag` iterations late and leaves its tables
        # there; the same schedule is then replayed on the graph engine with no iteration past the stop
        # (bit-identical to the persistent kernels on the linear chains, tests/test_gpu.py), so every engine
        # hands back the state -- and next iteration -- of the graph engine (group_ADMM_closedForm.m:105-108)
        state_from = engine_kind
        if engine_kind == "persistent" and comm.nranks == 1 and static and done in (1, 2) \
                and int(eng.ctl_state()["iter"]) != iters + 1:
            load_state()
            r2 = eng.run(stop_iter=iters, use_graph=opts.get("graph", True))
            state_from = "graph replay to iteration %d" % iters
            if int(r2.iters) != iters:
                state_from += " (replay stopped at %d)" % int(r2.iters)
        res.extra["state_from"] = state_from
        # apply the heads' pending (lazy) duals with the current chain, so (theta, mu) is the reference
        # state after iteration next-1
        eng.flush_duals()
        eng.stream.synchronize()  # the flush runs on the engine's stream; the copies below do not
        nxt = int(eng.ctl_state()["iter"])
        res.extra["state"] = (eng.theta.clone(), eng.mu.clone(), nxt)
    return res


def _chain_admm_native_elastic(model, n_total, rho, obj0, tol, max_iter, schedule, cost_quirk, name, opts,
                               failures) -> RunResult:
    """Elastic recovery (``failures = {iteration: [worker ids]}``) on the native engine: one rank, a
    static chain, closed-form local solves. Same semantics as the torch path's ``failures``: at the
    failure iteration each dead worker's aggregated dual goes to its nearest surviving chain
    neighbour (``_drop_workers``), the chain re-forms over the survivors and the target becomes the
    survivors' optimum. The solve runs in segments: the current survivors' chain runs natively up to
    the iteration before the next failure (graph engine, ``stop_iter``), its state (pending head
    duals applied) goes back into the full tables, the duals are handed on, and the survivors - a
    smaller engine over their shards (``LinearRegression.subset``), ids renumbered in worker order -
    resume natively from the failure iteration (persistent kernel, ``start_iter``)."""
    dev = model.device
    d = model.d
    alive = np.ones(n_total, dtype=bool)
    theta = torch.zeros((n_total, d), dtype=torch.float64, device=dev)
    mu = torch.zeros((n_total, d), dtype=torch.float64, device=dev)
    lidx_of = {w: w for w in range(n_total)}
    events = sorted((int(k), [int(w) for w in v]) for k, v in failures.items() if 1 <= int(k) <= max_iter)
    start, cur_obj0 = 1, float(obj0)
    segs: List[RunResult] = []
    seg_info = []

    def run_segment(stop: int) -> RunResult:
        S = [w for w in range(n_total) if alive[w]]
        if len(S) < 2:
            raise ValueError("elastic recovery: fewer than two workers survive")
        new_of = {w: i for i, w in enumerate(S)}
        sub = model.subset(S)
        sch = PathSchedule(len(S), [new_of[w] for w in schedule.path if alive[w]], np.zeros(len(S) - 1), coherence=0)
        ix = torch.as_tensor(S, dtype=torch.long, device=dev)
        st = None if start == 1 else (theta.index_select(0, ix), mu.index_select(0, ix), start)
        o = dict(opts, cache=False, state=True)
        if stop > 0:
            o["stop_iter"] = stop
        r = _chain_admm_native(sub, list(range(len(S))), len(S), rho, cur_obj0, tol, max_iter, LocalComm(),
                               Placement.contiguous(len(S), 1), sch, "closed", 1.0, 1, 0.0, cost_quirk, name, o,
                               state=st)
        th_s, mu_s, _ = r.extra["state"]
        theta[ix] = th_s
        mu[ix] = mu_s
        seg_info.append({"first": start, "last": int(r.iters), "workers": len(S), "engine": r.extra.get("engine")})
        segs.append(r)
        return r

    finished = False
    for f, dead in events:
        if f > start:
            r = run_segment(f - 1)
            if r.converged or r.iters >= max_iter:
                finished = True
                break
            start = f
        cur_obj0 = _drop_workers(dead, alive, schedule, theta, mu, lidx_of, model, LocalComm(), n_total, dev)
    if not finished:
        run_segment(0)
    last = segs[-1]
    iters = int(last.iters)
    obj = np.concatenate([s.obj for s in segs])
    loss = np.concatenate([s.loss for s in segs])
    offs = np.cumsum([0.0] + [float(s.wall_s) for s in segs[:-1]])
    tt = np.concatenate([np.asarray(s.time_trace) + o for s, o in zip(segs, offs)])
    pres = None
    if all(s.primal_res is not None for s in segs):
        pres = np.concatenate([np.asarray(s.primal_res) for s in segs])
    per = float(np.sum(schedule.cost)) * ((n_total + 1) // 2 if cost_quirk else 1)
    res = RunResult(algorithm=name, obj=obj, loss=loss, iters=iters, converged=bool(last.converged),
                    wall_s=float(sum(s.wall_s for s in segs)), time_trace=tt,
                    comm_units=np.arange(1, iters + 1, dtype=np.float64) * n_total,
                    com_cost=np.arange(1, iters + 1) * per, bytes_sent=0, bytes_total=0, primal_res=pres,
                    extra={"backend": "native", "engine": "elastic", "segments": seg_info, "rank": 0, "nranks": 1,
                           "solver": "closed", "obj0_final": cur_obj0,
                           "state": (theta, mu, int(last.extra["state"][2]))})
    res.theta = theta.cpu().numpy()
    return res


def _drop_workers(dead, alive, schedule, theta, mu, lidx_of, model, comm, n_total, dev) -> float:
    """Remove ``dead`` workers (elastic recovery): hand each one's aggregated dual to its nearest
    surviving neighbour on the current chain (sum(mu) = 0 is the dual-feasibility invariant of the
    consensus problem; ADMM's dual steps preserve it, a lost dual would break it), mark it dead, and
    return the survivors' optimal objective. Collective: every rank calls it with the same list."""
    d = theta.shape[1]
    path = [w for w in schedule.path if alive[w]]
    lost = torch.zeros((n_total, d), dtype=torch.float64, device=dev)
    for w in dead:
        if w in lidx_of:
            lost[w] = mu[lidx_of[w]]
    if comm.nranks > 1:
        comm.allreduce_sum(lost)
    for w in dead:
        if not alive[w]:
            continue
        pos = path.index(w)
        heir = None
        for q in list(range(pos - 1, -1, -1)) + list(range(pos + 1, len(path))):  # nearest survivor, left first
            if alive[path[q]] and path[q] not in dead:
                heir = path[q]
                break
        if heir is not None and heir in lidx_of:
            mu[lidx_of[heir]] += lost[w]
        if w in lidx_of:
            mu[lidx_of[w]].zero_()
    for w in dead:
        alive[w] = False
    # the survivors' optimum: all-reduced Gram of the alive workers (one-time, like SURVEY.md C10)
    keep = torch.as_tensor([alive[w] for w in lidx_of], dtype=torch.float64, device=dev)
    As = (model.A * keep.view(-1, 1, 1)).sum(0)
    bs = (model.b * keep.view(-1, 1)).sum(0)
    yy = (model.yy * keep).sum()
    buf = torch.cat([As.reshape(-1), bs, yy.reshape(1)]).contiguous()
    if comm.nranks > 1:
        comm.allreduce_sum(buf)
    As, bs, yy = buf[: d * d].reshape(d, d), buf[d * d: d * d + d], buf[-1]
    lam_tot = model.lam * int(alive.sum())
    x = torch.linalg.solve(As + lam_tot * torch.eye(d, dtype=torch.float64, device=dev), bs)
    return float(0.5 * x @ (As @ x) - bs @ x + 0.5 * yy + 0.5 * lam_tot * (x @ x))


def _is_rechain(it: int, coherence) -> bool:
    from ..parallel.topology import rechain_iteration

    return rechain_iteration(it, coherence)


# Convenience wrappers named after the reference functions -----------------------------------------

def group_admm_closed_form(model, rho, obj0, acc, max_iter, **kw) -> RunResult:
    """``group_ADMM_closedForm`` (A1) on all local workers (single rank unless comm given)."""
    n_total = kw.pop("n_total", model.n_local)
    local_ids = kw.pop("local_ids", list(range(model.n_local)))
    return chain_admm(model, local_ids, n_total, rho, obj0, acc, max_iter, name="GADMM", **kw)


def group_admm_logistic_gd(model, rho, obj0, acc, max_iter, step, **kw) -> RunResult:
    """``group_ADMM_logistic_GD`` (A2 + A3)."""
    n_total = kw.pop("n_total", model.n_local)
    local_ids = kw.pop("local_ids", list(range(model.n_local)))
    return chain_admm(model, local_ids, n_total, rho, obj0, acc, max_iter, local_solver="gd", step=step,
                      name="GADMM-logistic-GD", **kw)


def group_admm_logistic_exact(model, rho, obj0, acc, max_iter, **kw) -> RunResult:
    """``group_ADMM_logistic`` (D2, CVX exact local solves) via Newton."""
    n_total = kw.pop("n_total", model.n_local)
    local_ids = kw.pop("local_ids", list(range(model.n_local)))
    return chain_admm(model, local_ids, n_total, rho, obj0, acc, max_iter, local_solver="newton",
                      name="GADMM-logistic-exact", **kw)


def dynamic_group_admm(model, rho, obj0, acc, max_iter, path, path_cost, coherence, seed=1234,
                       kind="findPath2", **kw) -> RunResult:
    """``dynamic_group_ADMM_closedForm`` (A4): re-chain with findPath2 every ``coherence`` iterations."""
    n_total = kw.pop("n_total", model.n_local)
    local_ids = kw.pop("local_ids", list(range(model.n_local)))
    sched = PathSchedule(n_total, path, path_cost, coherence, kind=kind, seed=seed)
    sched.private = True  # never seen by the caller: the solve need not leave it at the stop
    return chain_admm(model, local_ids, n_total, rho, obj0, acc, max_iter, schedule=sched,
                      name="D-GADMM(coh=%s)" % coherence, **kw)


def dynamic_group_admm_v0(model, rho, obj0, acc, max_iter, path_matrix, cost_matrix, coherence,
                          faithful_initial_cost=True, **kw) -> RunResult:
    """``dynamic_group_ADMM_closedForm_v0`` (A5): consume pre-generated chains. With
    ``faithful_initial_cost`` the initial cost is the reference's column slice
    ``pathCost_matrix(:,1)`` (quirk 6, dynamic_group_ADMM_closedForm_v0.m:18)."""
    n_total = kw.pop("n_total", model.n_local)
    local_ids = kw.pop("local_ids", list(range(model.n_local)))
    cm = np.asarray(cost_matrix)
    c0 = cm[:, 0] if faithful_initial_cost else cm[0]
    sched = PathSchedule(n_total, path_matrix[0], c0, coherence, kind="matrix", path_matrix=path_matrix,
                         cost_matrix=cm)
    return chain_admm(model, local_ids, n_total, rho, obj0, acc, max_iter, schedule=sched,
                      name="D-GADMM-v0(coh=%s)" % coherence, **kw)


def static_group_admm(model, rho, obj0, acc, max_iter, coherence, cost_static_matrix, **kw) -> RunResult:
    """``static_group_ADMM_closedForm`` (A6): identity chain; its cost row changes with the node
    geometry every ``coherence`` iterations."""
    n_total = kw.pop("n_total", model.n_local)
    local_ids = kw.pop("local_ids", list(range(model.n_local)))
    cm = np.asarray(cost_static_matrix)
    ident = list(range(n_total))
    sched = PathSchedule(n_total, ident, cm[0], coherence, kind="matrix",
                         path_matrix=[ident] * cm.shape[0], cost_matrix=cm)
    return chain_admm(model, local_ids, n_total, rho, obj0, acc, max_iter, schedule=sched,
                      name="GADMM-static(coh=%s)" % coherence, **kw)
