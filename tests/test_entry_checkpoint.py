"""Entry points (quick budgets, CPU) and per-worker checkpoint / resume."""
import json
import os

import numpy as np
import pytest
import torch

from gadmm_amd import entry
from gadmm_amd.config import get_preset, parse_overrides


@pytest.mark.parametrize("name", ["LinearRegression_Synthetic", "LogisticRegression_Synthetic",
                                  "LinearRegression_Real", "Dynamic_LinearRegression_Real",
                                  "LinearRegression_gadmm_vs_admm"])
def test_entry_quick(name, tmp_path):
    out = entry.get(name).main(["--quick", "--device", "cpu", "--out", str(tmp_path), "--no-plot"])
    summ = json.load(open(os.path.join(tmp_path, "summary.json")))
    assert summ["entry"] == name and summ["runs"]
    if name == "LinearRegression_Synthetic":
        assert out["runs"]["GADMM_rho7"]["iters"] == 248 and out["runs"]["GADMM_rho7"]["converged"]
    if name == "LogisticRegression_Synthetic":
        assert out["runs"]["GADMM_rho0.0002"]["iters"] == 53
    if name == "LinearRegression_gadmm_vs_admm":
        assert out["runs"]["ADMM(star)"]["iters"] == 348
    assert any(f.endswith(".jsonl") for f in os.listdir(tmp_path))


def test_entry_clock_panels(tmp_path):
    """Every GADMM run carries the measured wall clock AND the reference's modelled 2*toc clock
    (group_ADMM_closedForm.m:39-42,53-55): both in the JSONL trace, four panels in the figure."""
    entry.get("LinearRegression_Synthetic").main(["--quick", "--device", "cpu", "--out", str(tmp_path),
                                                  "--no-baselines", "--set", "rhos=7"])
    rows = [json.loads(l) for l in open(os.path.join(tmp_path, "GADMM_rho7.jsonl"))]
    assert len(rows) == 248
    mc = np.asarray([r["model_clock_s"] for r in rows])
    wall = np.asarray([r["wall_s"] for r in rows])
    assert mc[0] == 0.0 and np.all(np.diff(mc) > 0) and np.allclose(np.diff(mc), mc[1])  # 2*toc steps
    assert np.all(np.diff(wall) >= 0) and wall[-1] > 0
    assert [f for f in os.listdir(tmp_path) if f.endswith(".png")]


def test_dynamic_entry_quick(tmp_path):
    out = entry.get("Dynamic_LinearRegression_Synthetic").main(
        ["--quick", "--device", "cpu", "--out", str(tmp_path), "--set", "gadmm_iters=60", "coherences=1,10"])
    assert "D-GADMM_v0(coh=10)" in out["runs"] and "D-GADMM(coh=1)" in out["runs"]
    assert os.path.exists(os.path.join(tmp_path, "summary.json"))


def test_entry_two_gloo_ranks(tmp_path):
    out = entry.get("LinearRegression_Synthetic").main(
        ["--quick", "--cpu-ranks", "2", "--out", str(tmp_path), "--no-plot", "--no-baselines"])
    assert out["runs"]["GADMM_rho7"]["iters"] == 248
    assert out["runs"]["GADMM_rho7"]["bytes_total"] == 2 * 50 * 8 * 248  # one boundary edge, both directions


def test_overrides():
    c = parse_overrides(get_preset("LinearRegression_Synthetic"), ["rhos=1,2", "acc=1e-8", "num_workers=12"])
    assert c.rhos == [1.0, 2.0] and c.acc == 1e-8 and c.num_workers == 12


def test_checkpoint_resume_bit_exact(tmp_path, lin24, lin_obj0):
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import chain_admm
    from gadmm_amd.utils.checkpoint import save_checkpoint, load_checkpoint, edge_duals
    from gadmm_amd.oracle import reference as R

    m = LinearRegression(lin24.X, lin24.y)
    part = chain_admm(m, list(range(24)), 24, 5.0, lin_obj0, 1e-8, 200, backend="torch")
    theta, mu, nxt = part.extra["state"]
    save_checkpoint(str(tmp_path), 0, list(range(24)), theta, mu, nxt, list(range(24)), {"rho": 5.0})
    assert len([f for f in os.listdir(tmp_path) if f.startswith("worker_")]) == 24
    th2, mu2, nxt2, path, man = load_checkpoint(str(tmp_path), list(range(24)))
    assert nxt2 == 201 and man["rho"] == 5.0 and torch.equal(th2, theta) and torch.equal(mu2, mu)
    rest = chain_admm(m, list(range(24)), 24, 5.0, lin_obj0, 1e-8, 3000, backend="torch", state=(th2, mu2, nxt2))
    full = chain_admm(m, list(range(24)), 24, 5.0, lin_obj0, 1e-8, 3000, backend="torch")
    assert rest.iters == full.iters == 758
    assert np.array_equal(rest.obj, full.obj[200:])
    # per-worker duals convert to the reference's edge duals (group_ADMM_closedForm.m:93-95)
    X, y = lin24.numpy()
    o = R.gadmm_linear(X, y, 5.0, 200, lin_obj0, 1e-30)
    lam = edge_duals(mu.numpy(), list(range(24)))
    assert np.allclose(lam, o.dual[:23], rtol=1e-9, atol=1e-9)


def test_checkpoint_multi_rank_layout(tmp_path):
    from gadmm_amd.utils.checkpoint import save_checkpoint, load_checkpoint
    th = torch.randn(6, 4, dtype=torch.float64)
    mu = torch.randn(6, 4, dtype=torch.float64)
    save_checkpoint(str(tmp_path), 1, [3, 4, 5], th, mu[3:], 9, [0, 1, 2, 3, 4, 5])
    save_checkpoint(str(tmp_path), 0, [0, 1, 2], th, mu[:3], 9, [0, 1, 2, 3, 4, 5], {"algorithm": "GADMM"})
    t, m, nxt, path, man = load_checkpoint(str(tmp_path), [3, 4, 5])
    assert torch.equal(t, th) and torch.equal(m, mu[3:]) and nxt == 9 and man["algorithm"] == "GADMM"


def test_logistic_entry_reports_exact_runs(tmp_path):
    """Logistic entries also run GADMM with exact local solves (SURVEY.md §7.3 "report both")."""
    out = entry.get("LogisticRegression_Synthetic").main(
        ["--quick", "--device", "cpu", "--out", str(tmp_path), "--no-plot", "--no-baselines",
         "--set", "exact_iters=500"])
    r = out["runs"]["GADMM_exact_rho0.001"]
    assert r["iters"] == 424 and r["converged"]
