"""Batched torch algorithms (CPU) against the oracle and the reference's golden numbers."""
import numpy as np
import pytest
import torch

from gadmm_amd.algorithms import (group_admm_closed_form, group_admm_logistic_gd, group_admm_logistic_exact,
                                  dynamic_group_admm, dynamic_group_admm_v0, static_group_admm, standard_admm,
                                  dual_averaging, gradient_descent, lag, iag, global_constants, chain_admm)
from gadmm_amd.models import LinearRegression, LogisticRegression
from gadmm_amd.oracle import reference as R
from gadmm_amd.parallel import topology as T


@pytest.fixture(scope="module")
def lin_model(lin24):
    return LinearRegression(lin24.X, lin24.y)


@pytest.fixture(scope="module")
def log_model(log24):
    return LogisticRegression(log24.X, log24.y, 1e-5)


def test_models_match_direct_forms(lin_model, log_model):
    th = torch.randn(24, 50, dtype=torch.float64)
    assert torch.allclose(lin_model.objective(th), lin_model.objective_direct(th), rtol=1e-12)
    g = lin_model.gradient(th)
    th.requires_grad_(True)
    lin_model.objective_direct(th).sum().backward()
    assert torch.allclose(g, th.grad, rtol=1e-10)
    t2 = torch.randn(24, 50, dtype=torch.float64, requires_grad=True)
    log_model.objective(t2).sum().backward()
    assert torch.allclose(log_model.gradient(t2.detach()), t2.grad, rtol=1e-10, atol=1e-12)


def test_optima(lin_model, log_model, lin_obj0, log_obj0):
    assert lin_model.optimum() == pytest.approx(lin_obj0, rel=1e-12)
    assert log_model.optimum() == pytest.approx(log_obj0, rel=1e-12)


@pytest.mark.parametrize("rho,it8", [(3, 1373), (5, 758), (7, 428)])
def test_gadmm_linear(lin_model, lin_obj0, rho, it8):
    r = group_admm_closed_form(lin_model, rho, lin_obj0, 1e-8, 3000)
    assert r.converged and r.iters == it8
    assert r.comm_units[-1] == it8 * 24  # GADMM: N transmissions per iteration


def test_gadmm_trace_matches_oracle(lin24, lin_model, lin_obj0):
    r = group_admm_closed_form(lin_model, 3.0, lin_obj0, 1e-30, 60)
    X, y = lin24.numpy()
    o = R.gadmm_linear(X, y, 3.0, 60, lin_obj0, 1e-30)
    assert np.allclose(r.obj, o.obj, rtol=1e-12)


def test_gadmm_logistic_gd(log_model, log_obj0):
    r = group_admm_logistic_gd(log_model, 2e-4, log_obj0, 1e-4, 400, 2.2)
    assert r.iters == 53


def test_gadmm_logistic_exact_converges(log_model, log_obj0):
    # exact local solves (CVX variant) reach 1e-8 with a well-chosen rho
    r = group_admm_logistic_exact(log_model, 1e-3, log_obj0, 1e-8, 1000)
    assert r.converged and r.iters == 424, r.loss[-5:]


def test_dgadmm_identity_equals_gadmm(lin_model, lin_obj0):
    a = group_admm_closed_form(lin_model, 1.0, lin_obj0, 1e-4, 3000)
    b = dynamic_group_admm(lin_model, 1.0, lin_obj0, 1e-4, 3000, list(range(24)), np.ones(23), 1e9)
    assert a.iters == b.iters == 2425


def test_dgadmm_matches_oracle_with_rechaining(lin24, lin_model, lin_obj0):
    X, y = lin24.numpy()
    rng = np.random.default_rng(5)
    p0, c0, _ = T.find_path(24, rng)
    sched_rng = np.random.default_rng(99)
    seq = {}

    def rechain(it):
        if it not in seq:
            p, c, _, _, _ = T.find_path2(24, sched_rng)
            seq[it] = (p, c)
        return seq[it]

    o = R.dgadmm_linear(X, y, 1.0, 400, lin_obj0, 1e-4, p0, c0, 10, rechain)
    r = dynamic_group_admm(lin_model, 1.0, lin_obj0, 1e-4, 400, p0, c0, 10, seed=99)
    assert r.iters == o.iters
    assert np.allclose(r.obj, o.obj, rtol=1e-10)
    assert np.allclose(r.com_cost, o.com_cost, rtol=1e-12)


def test_static_with_cost_equals_gadmm(lin_model, lin_obj0):
    cm = np.ones((200, 23))
    a = static_group_admm(lin_model, 7.0, lin_obj0, 1e-4, 600, 10, cm)
    assert a.iters == 248
    assert a.com_cost[0] == pytest.approx(12 * 23)  # quirk: sum(pathCost) once per head worker


def test_dgadmm_v0_faithful_initial_cost(lin_model, lin_obj0):
    rng = np.random.default_rng(2)
    paths, costs = [], []
    for _ in range(5):
        p, c, _ = T.find_path(24, rng)
        paths.append(p)
        costs.append(c)
    cm = np.asarray(costs)
    r = dynamic_group_admm_v0(lin_model, 3.0, lin_obj0, 1e-4, 30, paths, cm, 10)
    assert r.com_cost[0] == pytest.approx(12 * cm[:, 0].sum())


def test_std_admm(lin_model, lin_obj0):
    r = standard_admm(lin_model, list(range(24)), 24, 1.0, lin_obj0, 1e-4, 1000)
    assert r.iters == 348


def test_dual_averaging_matches_oracle(lin24, lin_model, lin_obj0):
    c = global_constants(lin_model)
    r = dual_averaging(lin_model, list(range(24)), 24, c["stepsize"], lin_obj0, 1e-4, 200)
    X, y = lin24.numpy()
    o = R.dual_averaging(X, y, 200, lin_obj0, 1e-4, c["stepsize"])
    assert np.allclose(r.obj, o.obj, rtol=1e-12)


def test_dual_averaging_logistic_matches_oracle(log24, log_model, log_obj0):
    c = global_constants(log_model)
    r = dual_averaging(log_model, list(range(24)), 24, c["stepsize"], log_obj0, 1e-4, 100)
    X, y = log24.numpy()
    o = R.dual_averaging(X, y, 100, log_obj0, 1e-4, c["stepsize"], logistic_eta=1e-5)
    assert np.allclose(r.obj, o.obj, rtol=1e-12)


def test_constants(lin_model):
    c = global_constants(lin_model)
    assert c["cond"] == pytest.approx(7299.9, rel=1e-4)


def test_baselines_short_horizon(lin_model, lin_obj0):
    c = global_constants(lin_model)
    s = c["stepsize"]
    hm = lin_model.hmax()
    gd = gradient_descent(lin_model, list(range(24)), 24, 300, lin_obj0, s)
    # GD semantics: theta_2 = -s * ones (gradients start as ones), then full gradients
    assert gd.obj[0] == pytest.approx(lin_model.objective(torch.zeros(24, 50, dtype=torch.float64)).sum().item())
    th2 = -s * torch.ones(50, dtype=torch.float64)
    assert gd.obj[1] == pytest.approx(lin_model.objective(th2.expand(24, 50).contiguous()).sum().item(), rel=1e-12)
    ps = lag(lin_model, list(range(24)), 24, 300, lin_obj0, s, hm, "PS")
    wk = lag(lin_model, list(range(24)), 24, 300, lin_obj0, s, hm, "WK")
    # LAG tables start as N columns of ones: theta_2 = -s * N * ones (GD_DGD_LAG.m:44,238)
    th2l = -s * 24 * torch.ones(50, dtype=torch.float64)
    ref2 = lin_model.objective(th2l.expand(24, 50).contiguous()).sum().item()
    assert ps.obj[1] == pytest.approx(ref2, rel=1e-12) and wk.obj[1] == pytest.approx(ref2, rel=1e-12)
    assert wk.extra["uploads"] > 0 and ps.extra["uploads"] > 0
    ci = iag(lin_model, list(range(24)), 24, 300, lin_obj0, s, "cyclic")
    ri = iag(lin_model, list(range(24)), 24, 300, lin_obj0, s, "random", hm, seed=3)
    assert np.all(np.isfinite(ci.obj)) and np.all(np.isfinite(ri.obj))


@pytest.mark.slow
def test_baseline_bundle_golden(lin_model, lin_obj0):
    """GD reaches 1e-4 at 53,891; LAG-WK at 44,368 with ~58k uploads (60,000 iterations)."""
    c = global_constants(lin_model)
    s = c["stepsize"]
    gd = gradient_descent(lin_model, list(range(24)), 24, 60000, lin_obj0, s)
    assert gd.first_below(1e-4) == 53891
    wk = lag(lin_model, list(range(24)), 24, 60000, lin_obj0, s, lin_model.hmax(), "WK")
    assert wk.first_below(1e-4) == 44368
    assert wk.extra["uploads"] == 58186


def test_resume_from_state(lin_model, lin_obj0):
    full = chain_admm(lin_model, list(range(24)), 24, 5.0, lin_obj0, 1e-8, 3000, backend="torch")
    part = chain_admm(lin_model, list(range(24)), 24, 5.0, lin_obj0, 1e-8, 300, backend="torch")
    th, mu, nxt = part.extra["state"]
    rest = chain_admm(lin_model, list(range(24)), 24, 5.0, lin_obj0, 1e-8, 3000, backend="torch",
                      state=(th, mu, nxt))
    assert rest.iters == full.iters == 758
    assert np.allclose(rest.obj, full.obj[300:], rtol=1e-13)


def test_primal_residual_trace(lin_model, lin_obj0):
    """K4's consensus residual sum_edges ||th_n - th_right||^2 is recorded per iteration and vanishes
    at convergence."""
    r = group_admm_closed_form(lin_model, 3.0, lin_obj0, 1e-8, 3000, backend="torch")
    assert r.primal_res is not None and len(r.primal_res) == r.iters == 1373
    assert r.primal_res[-1] < 1e-6 * r.primal_res[:10].max()


def test_first_order_model_bytes_follow_reference_units(lin24):
    """GD / LAG / IAG / DGD / dual averaging report the reference's communication model
    in bytes (one d-row of f64 per comm unit: uploads + one broadcast down per server iteration), the
    byte axis shared with star ADMM and GADMM, next to the fabric bytes."""
    import numpy as np
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import gradient_descent, lag, iag, decentralized_gd, dual_averaging, global_constants
    m = LinearRegression(lin24.X, lin24.y)
    s = global_constants(m)["stepsize"]
    ids, n, d = list(range(24)), 24, 50
    gd = gradient_descent(m, ids, n, 40, 218.6486436261889, s)
    assert gd.extra["model_bytes"] == 40 * (n + 1) * d * 8  # N uploads + 1 broadcast per iteration
    lw = lag(m, ids, n, 40, 218.6486436261889, s, m.hmax(), "WK")
    assert lw.extra["model_bytes"] == int(round(lw.comm_units[-1])) * d * 8
    ia = iag(m, ids, n, 40, 218.6486436261889, s, "cyclic", None)
    assert ia.extra["model_bytes"] == 40 * 2 * d * 8
    dg = decentralized_gd(m, ids, n, 40, 218.6486436261889, s)
    assert dg.extra["model_bytes"] == 40 * n * d * 8
    da = dual_averaging(m, ids, n, s, 218.6486436261889, 1e-12, 40)
    assert da.extra["model_bytes"] == len(da.obj) * n * d * 8
    assert np.isfinite(gd.obj).all()


def test_lanczos_extreme_eigs():
    """extreme_eigs (large-d global_constants): Lanczos with full reorthogonalisation == a dense
    eigensolve on a real-shaped Gram (Gaussian rows: a clustered spectrum, the slow case for power
    iteration)."""
    import torch
    from gadmm_amd.algorithms.baselines import extreme_eigs
    g = torch.Generator().manual_seed(3)
    X = torch.randn(900, 300, generator=g, dtype=torch.float64)
    G = X.T @ X
    lo, hi = extreme_eigs(G)
    ev = torch.linalg.eigvalsh(G)
    assert abs(hi - float(ev[-1])) <= 1e-10 * float(ev[-1])
    assert abs(lo - float(ev[0])) <= 1e-8 * float(ev[-1])


def test_cg_oracle_solve_and_fallback():
    """The large-d optimum's CG attempt (models/linear.py:_cg_solve, torch path on the CPU): a tall
    well-conditioned Gram converges to LU's solution at 1e-13; a Gram with rows ~ d returns None, so
    _spd_solve falls back to a direct solve."""
    import torch
    from gadmm_amd.models.linear import _cg_solve, _spd_solve
    g = torch.Generator().manual_seed(11)
    d = 120
    b = torch.randn(d, dtype=torch.float64, generator=g)
    X = torch.randn(12000, d, dtype=torch.float64, generator=g)
    M = X.T @ X
    x = _cg_solve(M, b)
    ref = torch.linalg.solve(M, b)
    assert x is not None and float((x - ref).abs().max() / ref.abs().max()) < 1e-13
    assert torch.equal(_cg_solve(M, b), x)  # fixed operation sequence
    X = torch.randn(d + 5, d, dtype=torch.float64, generator=g)
    M = X.T @ X
    assert _cg_solve(M, b, maxit=16) is None
    xs = _spd_solve(M, b)
    assert float((M @ xs - b).abs().max()) < 1e-8 * float(b.abs().max()) * float(torch.linalg.cond(M))
