"""Elastic recovery (SURVEY.md §5 extension): workers drop out mid-run, the chain re-forms over the
survivors (duals persist, the failed workers' duals go to a surviving neighbour) and GADMM converges
to the SURVIVORS' optimum; one rank and two gloo ranks give the same iterates."""
import numpy as np

from gadmm_amd.parallel.launch import spawn

FAIL = {60: [5], 150: [17, 18]}


def _survivor_optimum(ds, dead):
    import torch
    alive = [w for w in range(ds.num_workers) if w not in dead]
    X = ds.X[alive].reshape(-1, ds.dim).numpy()
    y = ds.y[alive].reshape(-1).numpy()
    x = np.linalg.solve(X.T @ X, X.T @ y)
    r = X @ x - y
    return 0.5 * float(r @ r), x


def test_elastic_single_rank_converges_to_survivor_optimum(lin24, lin_obj0):
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import chain_admm
    m = LinearRegression(lin24.X, lin24.y)
    r = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 5000, failures=FAIL, backend="torch",
                   record_theta=True)
    f_star, x_star = _survivor_optimum(lin24, [5, 17, 18])
    assert r.converged
    assert abs(r.obj[-1] - f_star) < 1e-8
    alive = [w for w in range(24) if w not in (5, 17, 18)]
    assert np.max(np.abs(r.theta[alive] - x_star)) < 1e-3  # every survivor near the survivors' solution
    assert r.iters > 150


def _rank(rank, world):
    from gadmm_amd.data import linear_synthetic
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.parallel.comm import TorchDistComm
    from gadmm_amd.parallel.topology import Placement
    from gadmm_amd.algorithms import chain_admm
    from gadmm_amd.oracle.reference import opt_linear
    ds = linear_synthetic(24)
    Xf, yf = ds.stacked()
    obj0 = opt_linear(Xf.numpy(), yf.numpy())
    pl = Placement.contiguous(24, world)
    loc = pl.local_workers(rank)
    m = LinearRegression(ds.X[loc], ds.y[loc])
    r = chain_admm(m, loc, 24, 3.0, obj0, 1e-8, 5000, comm=TorchDistComm(), placement=pl, failures=FAIL,
                   backend="torch")
    return r.iters, list(r.obj)


def test_elastic_two_ranks_match_single_rank(lin24, lin_obj0):
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import chain_admm
    m = LinearRegression(lin24.X, lin24.y)
    one = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 5000, failures=FAIL, backend="torch")
    out = spawn(_rank, 2)
    for it, obj in out:
        assert it == one.iters
        assert np.allclose(obj, one.obj, rtol=1e-12)
