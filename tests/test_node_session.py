"""Node rules of the multi-GPU entry sessions, on the CPU:

* device selection: ``local_rank % visible devices`` (a per-process HIP_VISIBLE_DEVICES leaves one device:
  every rank takes device 0), device 0 when the ranks share one GPU;
* the session plan: gloo control plane, the IPC transport as the default data plane, RCCL only on request
  and never with ranks sharing a GPU, xGMI fabrics tried unless a graph-engine plane was asked for;
* ``NodeFabrics``: the xGMI fabric is agreed by every rank (one rank failing gives None on all), the data
  plane is built once per shape; ``Session.chain_kw`` routes chain solves to the fabric with the data plane
  as fallback, and to the data plane alone when no fabric came up;
* bench.py's default engine tournament builds no RCCL communicator.
"""
import os
import types

import pytest
import torch

from gadmm_amd.parallel.launch import spawn
from gadmm_amd.parallel.node import select_device_index, session_plan, share_requested


@pytest.mark.parametrize("local_rank,share,count,want", [
    (0, False, 8, 0), (3, False, 8, 3), (7, False, 8, 7), (9, False, 8, 1),
    (3, False, 1, 0), (7, False, 1, 0),      # per-process HIP_VISIBLE_DEVICES: one visible device
    (5, True, 8, 0), (5, True, 1, 0)])       # ranks sharing one GPU
def test_select_device_index(local_rank, share, count, want):
    assert select_device_index(local_rank, share, count) == want


def test_select_device_index_no_device():
    with pytest.raises(RuntimeError):
        select_device_index(0, False, 0)


def test_share_requested_names():
    assert share_requested({"GADMM_SHARE_GPU": "1"})
    assert share_requested({"GADMM_BENCH_SHARE_GPU": "1"})
    assert not share_requested({})
    assert not share_requested({"GADMM_SHARE_GPU": "0"})


@pytest.mark.parametrize("device,world,fabric,share,want", [
    ("cuda", 1, "auto", False, ("local", False)),
    ("cpu", 2, "auto", False, ("gloo", False)),
    ("cuda", 2, "auto", False, ("ipc", True)),
    ("cuda", 8, "xgmi", False, ("ipc", True)),
    ("cuda", 4, "ipc", False, ("ipc", False)),
    ("cuda", 8, "rccl", False, ("rccl", False)),
    ("cuda", 4, "rccl", True, ("ipc", False)),   # RCCL refuses ranks on one device
    ("cuda", 4, "auto", True, ("ipc", True))])
def test_session_plan(device, world, fabric, share, want):
    p = session_plan(device, world, fabric, share)
    assert (p["data_plane"], p["xgmi"]) == want
    assert p["control"] == (None if world == 1 else "gloo")


def test_session_plan_rejects_unknown_fabric():
    with pytest.raises(ValueError):
        session_plan("cuda", 2, "nvlink", False)


def test_setup_rank_device_under_one_visible_device(monkeypatch):
    """setup_rank('node') with LOCAL_RANK=3 and one visible device picks cuda:0 (not cuda:3)."""
    import gadmm_amd.parallel.launch as L

    picked = []
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: picked.append(torch.device(d)))
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("LOCAL_RANK", "3")
    monkeypatch.delenv("GADMM_SHARE_GPU", raising=False)
    monkeypatch.delenv("GADMM_BENCH_SHARE_GPU", raising=False)
    rank, world, local_rank, dev, comm = L.setup_rank("node")
    assert dev == torch.device("cuda", 0) and picked == [torch.device("cuda", 0)]
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    picked.clear()
    assert L.setup_rank("node")[3] == torch.device("cuda", 3)


class _StubPlane:
    backend = "ipc"

    def __init__(self, n_total, d):
        self.n_total, self.d, self.closed = n_total, d, False
        self.selection = {"requested": "auto", "data_plane": "ipc", "reason": "stub"}

    def close(self):
        self.closed = True


def _node_rank(rank, world, fail_rank):
    """Rank body: NodeFabrics with stub device objects; one rank's xGMI fabric fails to come up."""
    import gadmm_amd.parallel.dataplane as DP
    import gadmm_amd.parallel.xgmi as X
    from gadmm_amd.entry.common import Session
    from gadmm_amd.parallel.comm import RankInfo
    from gadmm_amd.parallel.node import NodeFabrics, session_plan

    built = []

    class StubFabric:
        def __init__(self, n, d, ring, rank_, nranks, device, table_slots=1, **kw):
            if rank_ == fail_rank:
                raise RuntimeError("peer mapping failed")
            self.table_slots, self.closed = table_slots, False
            built.append(self)

        def close(self):
            self.closed = True

    X.XgmiFabric = StubFabric
    DP.make_data_plane = lambda fabric, world_, device, share, n, d, ring, **kw: _StubPlane(n, d)
    nodes = NodeFabrics(rank, world, torch.device("cpu"), session_plan("cuda", world, "auto", False), "auto",
                        False, log=lambda m: None)
    sess = Session(rank, world, torch.device("cpu"), None, nodes=nodes)
    plane = sess.ensure_plane(24, 50)
    again = sess.ensure_plane(24, 50)
    kw_static = sess.chain_kw(24, 50)
    kw_dyn = sess.chain_kw(24, 50, dynamic=True)
    out = {"same_plane": plane is again, "plane_shape": (plane.n_total, plane.d),
           "static_comm": type(kw_static["comm"]).__name__,
           "static_fabric": "engine_opts" in kw_static,
           "dyn_slots": (kw_dyn.get("engine_opts") or {}).get("fabric").table_slots
           if "engine_opts" in kw_dyn else None,
           "fallback_is_plane": (kw_static.get("engine_opts") or {}).get("fallback_comm") is plane,
           "built": len(built), "closed_after_disagree": [b.closed for b in built],
           "events": [w for w, _ in nodes.events]}
    assert isinstance(kw_static["comm"], (RankInfo, _StubPlane))
    sess.close()
    out["plane_closed"] = plane.closed
    return out


@pytest.mark.parametrize("fail_rank", [-1, 1])
def test_node_fabrics_agreed_and_chain_routing(fail_rank):
    res = spawn(_node_rank, 2, fail_rank, timeout=120)
    for rk, r in enumerate(res):
        assert r["same_plane"] and r["plane_shape"] == (24, 50) and r["plane_closed"]
        assert r["events"] == ["data_plane", "xgmi", "xgmi"]
        if fail_rank < 0:
            # every rank has its fabric: the persistent kernels, the data plane as fallback
            assert r["static_comm"] == "RankInfo" and r["static_fabric"] and r["fallback_is_plane"]
            assert r["dyn_slots"] == 8
        else:
            # one rank's fabric failed: NO rank uses one (agreed); the chain solves take the data plane
            assert r["static_comm"] == "_StubPlane" and not r["static_fabric"] and r["dyn_slots"] is None
            if rk != fail_rank:
                assert r["built"] == 2 and r["closed_after_disagree"] == [True, True]


def test_bench_default_tournament_builds_no_rccl(monkeypatch):
    """The default node run (--fabric auto) times no graph-rccl candidate; RCCL only on request."""
    import bench
    import gadmm_amd.engine.blocked_xgmi as B

    monkeypatch.setattr(B, "replicated_plans", lambda n, pl, d: [(1, 1), (2, 1)])
    from gadmm_amd.parallel.topology import Placement

    def names(fabric, share, env=None):
        if env:
            monkeypatch.setenv("GADMM_TOURNAMENT_RCCL", env)
        else:
            monkeypatch.delenv("GADMM_TOURNAMENT_RCCL", raising=False)
        args = types.SimpleNamespace(fabric=fabric, workers=24, rho=3.0, tol=1e-8, block=0, no_graph=False)
        X = torch.zeros((12, 50, 50), dtype=torch.float64)
        cands = bench._headline_candidates(args, X, X[:, :, 0], list(range(12)), Placement.contiguous(24, 2), 0, 2,
                                           torch.device("cpu"), share, 1.0)
        return [c["name"] for c in cands]

    default = names("auto", False)
    assert "graph-rccl" not in default and "graph-ipc" in default and "blocked-dl-halo" in default
    assert "graph-rccl" in names("auto", False, env="1")
    assert "graph-rccl" in names("rccl", False)
    assert "graph-rccl" not in names("rccl", True)  # never with ranks sharing one GPU
