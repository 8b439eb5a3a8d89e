"""Engine tournament for the multi-GPU headline (bench.py, untimed warm-up).

Which multi-GPU GADMM engine is fastest depends on the one-way hop latency between neighbour GPUs
(``parallel/hop_probe.py``) and on how many hops each engine leaves on the critical cycle per
iteration (group_ADMM_closedForm.m:18-27, 62-70): the data-local blocked kernel pays two, its halo mode
one, the replicated-halo kernel one per k iterations, the per-worker kernel two plus its own
intra-GPU hand-offs. Rules measured on one shared GPU cannot settle that for a real node, so every
eligible candidate is built and timed here and the ranks AGREE on the fastest:

* a candidate is built by its factory on every rank; a failure on any rank drops it on every rank;
* ``warm`` untimed solves, then ``solves`` timed ones between a device sync + barrier on both sides;
  the candidate's time is the MAX over ranks (an all-reduce), so every rank ranks the candidates
  from identical numbers and picks the same winner;
* a candidate counts only if every solve on every rank converged, in one iteration count that all
  ranks agree on (``ranks_agree``; ``expect`` when given: the reference count);
* the winner stays built, every other candidate is closed as soon as it loses.

Everything collective goes over the default (gloo) group, so this module runs unchanged on CPU ranks
with stand-in solvers (tests/test_distributed_gloo.py).
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def _agree_ok(flag: bool, world: int) -> bool:
    if world == 1:
        return bool(flag)
    t = torch.tensor([0.0 if flag else 1.0], dtype=torch.float64)
    dist.all_reduce(t)
    return float(t.item()) == 0.0


def _max(v: float, world: int) -> float:
    if world == 1:
        return float(v)
    t = torch.tensor([float(v)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def ranks_agree(v: int, world: int) -> bool:
    """Collective: every rank holds the same integer (an all-reduce of its min and max)."""
    if world == 1:
        return True
    t = torch.tensor([float(v), -float(v)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0]) == -float(t[1])


def engine_tournament(candidates: Sequence[Tuple[str, Callable[[], object]]], world: int, solves: int = 3,
                      warm: int = 1, expect: Optional[int] = None, sync: Optional[Callable[[], None]] = None,
                      log: Optional[Callable[[str], None]] = None) -> Tuple[Optional[str], object, List[Dict]]:
    """Collective. ``candidates``: (name, factory) in preference order (ties keep the earlier one);
    a factory builds a solver with ``guarded_solve() -> (iters, done, ...)`` and ``close()``, or
    raises. Returns ``(winner_name, winner_solver, table)`` -- ``(None, None, table)`` if no
    candidate ran -- with one table row per candidate: engine, ok, ms (max over ranks), iters, error."""
    sync = sync or (lambda: None)
    table: List[Dict] = []
    best: Optional[Tuple[float, str, object]] = None
    for name, factory in candidates:
        if log is not None:
            log("tournament: building %s" % name)  # progress (a stalled candidate takes its deadline)
        solver, err = None, ""
        try:
            solver = factory()
        except Exception as e:  # collective factories raise on every rank together; agreed below anyway
            err = "%s: %s" % (type(e).__name__, e)
        if not _agree_ok(solver is not None, world):
            if solver is not None:
                solver.close()
            table.append({"engine": name, "ok": False, "ms": None, "iters": None,
                          "error": err or "unavailable on another rank"})
            continue
        ok, its = True, set()
        for _ in range(max(0, int(warm))):
            out = solver.guarded_solve()
            ok &= int(out.done) == 1
        ok = _agree_ok(ok, world)
        ms = None
        if ok:
            sync()
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            for _ in range(max(1, int(solves))):
                out = solver.guarded_solve()
                ok &= int(out.done) == 1
                its.add(int(out.iters))
            sync()
            ms = (time.perf_counter() - t0) * 1e3 / max(1, int(solves))
            if world > 1:
                dist.barrier()
            ms = _max(ms, world)
            ok = _agree_ok(ok and len(its) == 1 and (expect is None or its == {int(expect)}), world)
            # the same count on EVERY rank, not just one count per rank
            ok = ok and ranks_agree(next(iter(its)), world)
        row = {"engine": name, "ok": bool(ok), "ms": round(ms, 4) if ms is not None else None,
               "iters": sorted(its)[0] if len(its) == 1 else sorted(its), "error": "" if ok else
               ("a solve failed or disagreed on some rank" if ms is not None else "warm-up solve failed")}
        table.append(row)
        if log is not None:
            log("tournament: %s %s" % (name, row))
        if ok and (best is None or ms < best[0]):
            if best is not None:
                best[2].close()
            best = (ms, name, solver)
        else:
            solver.close()
    if best is None:
        return None, None, table
    return best[1], best[2], table
