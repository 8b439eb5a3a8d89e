"""Race checker + fault injection: the exchange checker passes on a clean run (same
iterates as without it) and flags every injected drop / corruption / delay at the phase it happens,
on every rank together (gloo, 2 and 3 ranks)."""
import pytest

from gadmm_amd.parallel.launch import spawn


def _run(rank, world, fault, at, rechain):
    import numpy as np
    from gadmm_amd.data import linear_synthetic
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.parallel.comm import TorchDistComm
    from gadmm_amd.parallel.topology import Placement, PathSchedule, find_path
    from gadmm_amd.algorithms import chain_admm
    from gadmm_amd.debug import FaultyComm, FaultPlan, RaceError
    from gadmm_amd.oracle.reference import opt_linear

    n = 24
    ds = linear_synthetic(n)
    Xf, yf = ds.stacked()
    obj0 = opt_linear(Xf.numpy(), yf.numpy())
    pl = Placement.contiguous(n, world)
    local = pl.local_workers(rank)
    m = LinearRegression(ds.X[local], ds.y[local])
    base = TorchDistComm()
    plan = FaultPlan()
    if fault:
        getattr(plan, fault).add(at)
    comm = FaultyComm(base, plan)
    sched = None
    if rechain:
        p0, c0, _ = find_path(n, np.random.default_rng(5))
        sched = PathSchedule(n, p0, c0, 10, seed=99)
    try:
        r = chain_admm(m, local, n, 7.0, obj0, 1e-4, 300, comm=comm, placement=pl, schedule=sched, backend="torch",
                       check_exchange=True)
        return ("ok", r.iters, comm.injected)
    except RaceError as e:
        return ("race", str(e), comm.injected)


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_checker_clean_run(world):
    out = spawn(_run, world, None, 0, False)
    assert all(o[0] == "ok" and o[1] == 248 for o in out), out  # reference count at rho = 7


def test_exchange_checker_clean_run_with_rechaining():
    out = spawn(_run, 2, None, 0, True)
    assert all(o[0] == "ok" for o in out), out


@pytest.mark.parametrize("fault", ["drop", "corrupt", "delay"])
def test_exchange_checker_flags_injected_fault(fault):
    # exchange call 9 = iteration 5, tail phase (2 calls per iteration)
    out = spawn(_run, 2, fault, 9, False)
    assert all(o[0] == "race" for o in out), out
    assert any("iteration 5 (tail phase)" in o[1] for o in out), out
    assert sum(o[2] for o in out) >= 1
