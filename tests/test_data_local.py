"""Data locality of the multi-GPU path ('a test asserts that no rank reads a non-local X').

bench.py / engine/multigpu.py build each rank's problem with benchmarks.headline_rank_problem: the
shard builder is asked only for the rank's own workers, and obj0 comes from one all-reduce of local
Grams + residual vectors, equal on every rank to the stacked single-process optimum."""
import numpy as np
import pytest


def _rank(rank, world, n):
    from gadmm_amd.benchmarks import headline_rank_problem
    from gadmm_amd.data import linear_synthetic
    asked = []

    def builder(n_total, worker_ids=None):
        asked.append(list(worker_ids))
        return linear_synthetic(n_total, worker_ids=worker_ids)

    X, y, local, pl, obj0 = headline_rank_problem(n, rank, world, builder=builder)
    return {"asked": asked, "local": local, "shape": tuple(X.shape), "obj0": obj0,
            "X": X.numpy(), "owner": [int(o) for o in pl.owner]}


@pytest.mark.parametrize("world,n", [(2, 24), (4, 24), (8, 8)])
def test_each_rank_builds_only_its_own_shards(world, n):
    from gadmm_amd.parallel.launch import spawn
    from gadmm_amd.data import linear_synthetic
    from gadmm_amd.oracle.reference import opt_linear
    res = spawn(_rank, world, n, timeout=300)
    full = linear_synthetic(n)
    Xf, yf = full.stacked()
    ref = opt_linear(Xf.numpy(), yf.numpy())
    seen = []
    for r, out in enumerate(res):
        assert out["asked"] == [out["local"]]  # one build, of exactly the local workers
        assert all(out["owner"][w] == r for w in out["local"])
        assert out["shape"][0] == len(out["local"])
        assert np.array_equal(out["X"], full.X.numpy()[out["local"]])
        assert abs(out["obj0"] - ref) <= 1e-12 * abs(ref)
        seen += out["local"]
    assert sorted(seen) == list(range(n))  # a partition: no worker is held twice
