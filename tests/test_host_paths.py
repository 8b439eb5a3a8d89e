"""Host-side pieces of the native paths that need no GPU: the survivors' model of elastic recovery
(``LinearRegression.subset``), the memoised re-chain schedule, and the routing of resume / elastic
solves (CPU models always take the torch path)."""
import numpy as np
import torch


def test_linear_subset_shares_per_worker_statistics(lin24):
    from gadmm_amd.models import LinearRegression
    m = LinearRegression(lin24.X, lin24.y)
    keep = [0, 3, 4, 17, 23]
    sub = m.subset(keep)
    ref = LinearRegression(lin24.X[keep], lin24.y[keep])
    assert sub.n_local == len(keep) and (sub.m, sub.d) == (m.m, m.d)
    for a, b in ((sub.A, ref.A), (sub.b, ref.b), (sub.yy, ref.yy), (sub.X, ref.X), (sub.y, ref.y)):
        assert torch.equal(a, b)  # per-worker statistics: slicing == recomputing, bit for bit
    th = torch.randn(len(keep), m.d, dtype=torch.float64)
    assert torch.equal(sub.objective(th), ref.objective(th))


def test_rechains_memo_matches_schedule():
    from gadmm_amd.algorithms.gadmm import _rechains
    from gadmm_amd.parallel.topology import rechain_iterations
    for max_iter, coh in ((3000, 10), (3000, 1), (57, 7), (10, 50)):
        r1, r2 = _rechains(max_iter, coh), _rechains(max_iter, coh)
        assert r1 is r2  # memoised
        assert np.array_equal(r1, rechain_iterations(max_iter, coh))
        assert not r1.flags.writeable


def test_cpu_resume_and_elastic_take_the_torch_path(lin24, lin_obj0):
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import chain_admm
    m = LinearRegression(lin24.X, lin24.y)
    a = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-4, 3000)
    assert a.extra["backend"] == "torch" and a.iters == 784
    th, mu, nxt = a.extra["state"]
    b = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-30, nxt + 9, state=(th, mu, nxt))
    assert b.extra["backend"] == "torch" and len(b.obj) == 10
    c = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 400, failures={30: [5]})
    assert c.extra["backend"] == "torch"
