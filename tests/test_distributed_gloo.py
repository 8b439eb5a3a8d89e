"""Multi-process (gloo, CPU) runs reproduce the single-process results: chain p2p schedule, star
reduce/broadcast, LAG server uploads, dual-averaging pipeline (BASELINE.json configs[0])."""
import numpy as np
import pytest

from gadmm_amd.parallel.launch import spawn


def _rank_fn(rank, world, algo, params):
    import torch
    from gadmm_amd.data import linear_synthetic, logistic_synthetic
    from gadmm_amd.models import LinearRegression, LogisticRegression
    from gadmm_amd.parallel.comm import TorchDistComm
    from gadmm_amd.parallel.topology import Placement
    from gadmm_amd import algorithms as A

    n = params.get("n", 24)
    comm = TorchDistComm()
    pl = Placement.contiguous(n, world)
    local = pl.local_workers(rank)
    if algo.startswith("log"):
        ds = logistic_synthetic(n)
        m = LogisticRegression(ds.X[local], ds.y[local], 1e-5)
    else:
        ds = linear_synthetic(n)
        m = LinearRegression(ds.X[local], ds.y[local])
    obj0 = params["obj0"]
    if algo == "gadmm":
        r = A.chain_admm(m, local, n, params["rho"], obj0, params["tol"], params["max_iter"], comm=comm,
                         placement=pl, backend="torch", record_theta=True)
    elif algo == "dgadmm":
        from gadmm_amd.parallel.topology import PathSchedule
        s = PathSchedule(n, params["path"], params["cost"], params["coh"], seed=params["seed"])
        r = A.chain_admm(m, local, n, params["rho"], obj0, params["tol"], params["max_iter"], comm=comm,
                         placement=pl, schedule=s, backend="torch")
    elif algo == "loggd":
        r = A.chain_admm(m, local, n, params["rho"], obj0, params["tol"], params["max_iter"], comm=comm,
                         placement=pl, local_solver="gd", step=2.2, backend="torch")
    elif algo == "star":
        r = A.standard_admm(m, local, n, 1.0, obj0, 1e-4, 1000, comm=comm, placement=pl)
    elif algo == "dualavg":
        c = A.global_constants(m, comm)
        r = A.dual_averaging(m, local, n, c["stepsize"], obj0, 1e-4, params["max_iter"], comm=comm, placement=pl)
    elif algo == "lag":
        c = A.global_constants(m, comm)
        from gadmm_amd.algorithms.baselines import _Ctx, _gather_hmax
        hm = _gather_hmax(_Ctx(m, local, n, comm, pl), c["hmax_local"])
        r = A.lag(m, local, n, params["max_iter"], obj0, c["stepsize"], hm, params["variant"], comm=comm, placement=pl)
    elif algo == "iag":
        c = A.global_constants(m, comm)
        from gadmm_amd.algorithms.baselines import _Ctx, _gather_hmax
        hm = _gather_hmax(_Ctx(m, local, n, comm, pl), c["hmax_local"])
        r = A.iag(m, local, n, params["max_iter"], obj0, c["stepsize"], params["mode"], hm, comm=comm, placement=pl)
    elif algo == "dgd":
        c = A.global_constants(m, comm)
        r = A.decentralized_gd(m, local, n, params["max_iter"], obj0, c["stepsize"], comm=comm, placement=pl)
    elif algo == "gd":
        c = A.global_constants(m, comm)
        r = A.gradient_descent(m, local, n, params["max_iter"], obj0, c["stepsize"], comm=comm, placement=pl)
    elif algo == "optimum":
        return m.optimum(comm, n_total=n)
    else:
        raise ValueError(algo)
    out = {"iters": r.iters, "obj": r.obj, "bytes": r.bytes_sent, "bytes_total": r.bytes_total,
           "extra": {k: v for k, v in r.extra.items() if isinstance(v, (int, float, str))}}
    if r.theta is not None:
        out["theta"] = r.theta
    return out


def _single(algo, params):
    """Same computation in one process (LocalComm)."""
    import torch.distributed as dist  # noqa: F401
    from gadmm_amd.data import linear_synthetic, logistic_synthetic
    from gadmm_amd.models import LinearRegression, LogisticRegression
    from gadmm_amd import algorithms as A
    n = params.get("n", 24)
    if algo == "gadmm":
        ds = linear_synthetic(n)
        m = LinearRegression(ds.X, ds.y)
        return A.chain_admm(m, list(range(n)), n, params["rho"], params["obj0"], params["tol"], params["max_iter"],
                            backend="torch", record_theta=True)
    raise ValueError(algo)


@pytest.mark.parametrize("world", [2, 3])
def test_gadmm_gloo_matches_single_process(world, lin_obj0):
    params = {"rho": 5.0, "tol": 1e-8, "max_iter": 2000, "obj0": lin_obj0}
    res = spawn(_rank_fn, world, "gadmm", params)
    single = _single("gadmm", params)
    for r in res:
        assert r["iters"] == single.iters == 758
        assert np.allclose(r["obj"], single.obj, rtol=1e-12)
    # local rows of theta are bit-identical to the single-process computation
    from gadmm_amd.parallel.topology import Placement
    pl = Placement.contiguous(24, world)
    for k, r in enumerate(res):
        loc = pl.local_workers(k)
        assert np.array_equal(r["theta"][loc], single.theta[loc])
    # bytes: 2 (world-1) boundary messages of d doubles per iteration
    assert sum(r["bytes"] for r in res) == 2 * (world - 1) * 50 * 8 * 758


def test_dgadmm_gloo(lin_obj0):
    from gadmm_amd.parallel import topology as T
    rng = np.random.default_rng(11)
    p0, c0, _ = T.find_path(24, rng)
    params = {"rho": 1.0, "tol": 1e-4, "max_iter": 800, "obj0": lin_obj0, "path": p0, "cost": c0, "coh": 10,
              "seed": 4}
    res = spawn(_rank_fn, 2, "dgadmm", params)
    from gadmm_amd.data import linear_synthetic
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import dynamic_group_admm
    ds = linear_synthetic(24)
    single = dynamic_group_admm(LinearRegression(ds.X, ds.y), 1.0, lin_obj0, 1e-4, 800, p0, c0, 10, seed=4,
                                backend="torch")
    assert res[0]["iters"] == res[1]["iters"] == single.iters
    assert np.allclose(res[0]["obj"], single.obj, rtol=1e-10)


def test_logistic_gd_gloo(log_obj0):
    res = spawn(_rank_fn, 2, "loggd", {"rho": 2e-4, "tol": 1e-4, "max_iter": 200, "obj0": log_obj0})
    assert res[0]["iters"] == res[1]["iters"] == 53


def test_star_admm_gloo(lin_obj0):
    res = spawn(_rank_fn, 3, "star", {"obj0": lin_obj0})
    assert all(r["iters"] == 348 for r in res)


def test_dual_averaging_pipeline_gloo(lin_obj0):
    from gadmm_amd.data import linear_synthetic
    from gadmm_amd.oracle import reference as R
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import global_constants
    res = spawn(_rank_fn, 3, "dualavg", {"obj0": lin_obj0, "max_iter": 150})
    ds = linear_synthetic(24)
    c = global_constants(LinearRegression(ds.X, ds.y))
    X, y = ds.numpy()
    o = R.dual_averaging(X, y, 150, lin_obj0, 1e-4, c["stepsize"])
    for r in res:
        assert np.allclose(r["obj"], o.obj, rtol=1e-11)


@pytest.mark.parametrize("variant", ["PS", "WK"])
def test_lag_server_uploads_gloo(variant, lin_obj0):
    from gadmm_amd.data import linear_synthetic
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import lag, global_constants
    res = spawn(_rank_fn, 2, "lag", {"obj0": lin_obj0, "max_iter": 400, "variant": variant})
    ds = linear_synthetic(24)
    m = LinearRegression(ds.X, ds.y)
    c = global_constants(m)
    single = lag(m, list(range(24)), 24, 400, lin_obj0, c["stepsize"], m.hmax(), variant)
    for r in res:
        assert np.allclose(r["obj"], single.obj, rtol=1e-9)
        assert r["extra"]["uploads"] == single.extra["uploads"]


def test_iag_dgd_gd_gloo(lin_obj0):
    from gadmm_amd.data import linear_synthetic
    from gadmm_amd.models import LinearRegression
    from gadmm_amd import algorithms as A
    ds = linear_synthetic(24)
    m = LinearRegression(ds.X, ds.y)
    c = A.global_constants(m)
    for algo, kw, single in (
            ("iag", {"mode": "random"}, lambda: A.iag(m, list(range(24)), 24, 200, lin_obj0, c["stepsize"], "random",
                                                      m.hmax())),
            ("dgd", {}, lambda: A.decentralized_gd(m, list(range(24)), 24, 200, lin_obj0, c["stepsize"])),
            ("gd", {}, lambda: A.gradient_descent(m, list(range(24)), 24, 200, lin_obj0, c["stepsize"]))):
        params = {"obj0": lin_obj0, "max_iter": 200, **kw}
        res = spawn(_rank_fn, 2, algo, params)
        s = single()
        for r in res:
            assert np.allclose(r["obj"], s.obj, rtol=1e-9), algo


def test_global_optimum_allreduce(lin_obj0):
    res = spawn(_rank_fn, 2, "optimum", {"obj0": lin_obj0})
    assert res[0] == pytest.approx(lin_obj0, rel=1e-12)


# ------------------------------------------------------------------------------------------------
# bench.py's multi-GPU engine tournament (gadmm_amd/engine/tournament.py): the agreement logic with
# stand-in solvers on gloo CPU ranks (no device).
class _FakeSolver:
    def __init__(self, rank, delays, fail_at=None, iters=10):
        self.rank, self.delays, self.fail_at, self.iters = rank, delays, fail_at, iters
        self.n, self.closed = 0, False

    def guarded_solve(self):
        import time
        from gadmm_amd.engine.multigpu import SolveOut
        time.sleep(self.delays[self.rank])
        self.n += 1
        done = 4 if self.fail_at is not None and self.n == self.fail_at[1] and self.rank == self.fail_at[0] else 1
        return SolveOut(self.iters, done, 0, 0, 0)

    def close(self):
        self.closed = True


def _tournament_rank(rank, world):
    from gadmm_amd.engine.tournament import engine_tournament
    made = {}

    def fac(name, delays, fail_at=None, raise_on=None, iters=10):
        def f():
            if raise_on is not None and rank == raise_on:
                raise RuntimeError("not eligible here")
            made[name] = _FakeSolver(rank, delays, fail_at, iters)
            return made[name]
        return (name, f)

    cands = [fac("slow-everywhere", [0.03, 0.03]),
             fac("fast-on-0-only", [0.002, 0.05]),       # max over ranks = 50 ms: must lose
             fac("missing-on-1", [0.001, 0.001], raise_on=1),
             fac("fails-a-solve", [0.001, 0.001], fail_at=(1, 2)),
             fac("wrong-iterations", [0.001, 0.001], iters=11),
             fac("steady", [0.012, 0.012])]
    name, sol, table = engine_tournament(cands, world, solves=3, warm=1, expect=10)
    return {"winner": name, "winner_is_made": sol is made.get(name), "table": table,
            "closed": {k: v.closed for k, v in made.items()}}


def test_engine_tournament_agreement_on_gloo_ranks():
    res = spawn(_tournament_rank, 2, timeout=120)
    for r in res:
        assert r["winner"] == "steady" and r["winner_is_made"]
        rows = {row["engine"]: row for row in r["table"]}
        assert [row["engine"] for row in r["table"]][:2] == ["slow-everywhere", "fast-on-0-only"]
        assert rows["fast-on-0-only"]["ok"] and rows["fast-on-0-only"]["ms"] >= 45  # max over ranks
        assert not rows["missing-on-1"]["ok"] and rows["missing-on-1"]["ms"] is None
        assert not rows["fails-a-solve"]["ok"]
        assert not rows["wrong-iterations"]["ok"]
        assert rows["steady"]["ok"] and rows["steady"]["iters"] == 10
        # every loser is closed as soon as it loses, the winner stays open
        assert all(v for k, v in r["closed"].items() if k != "steady") and not r["closed"]["steady"]
    # both ranks ranked from identical numbers
    assert [(x["engine"], x["ok"], x["ms"]) for x in res[0]["table"]] == \
        [(x["engine"], x["ok"], x["ms"]) for x in res[1]["table"]]


def _tournament_rank_noexpect(rank, world):
    from gadmm_amd.engine.tournament import engine_tournament

    cands = [("differs-by-rank", lambda: _FakeSolver(rank, [0.001, 0.001], iters=10 + rank)),
             ("agreed", lambda: _FakeSolver(rank, [0.004, 0.004], iters=12))]
    name, sol, table = engine_tournament(cands, world, solves=2, warm=1, expect=None)
    return {"winner": name, "table": table}


def test_engine_tournament_rejects_rank_disagreement_without_expected_count():
    """with no pinned count a candidate must still converge in the SAME count on every rank
    (an all-reduce of the min and max), not merely in one count per rank."""
    res = spawn(_tournament_rank_noexpect, 2, timeout=120)
    for r in res:
        rows = {row["engine"]: row for row in r["table"]}
        assert not rows["differs-by-rank"]["ok"] and rows["agreed"]["ok"]
        assert r["winner"] == "agreed"
