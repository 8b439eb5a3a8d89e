"""Data-plane selection and the RCCL watchdog's fallback logic, on gloo CPU ranks
with stand-ins for the device transports: which plane each (fabric, ranks, shared GPU) gets, that an
RCCL communicator failing on ONE rank sends EVERY rank to the IPC transport, and that an RCCL graph
solve aborted by its watchdog (native.RcclDead on one rank) makes every rank fall back together, aborting
(never collectively destroying) the communicator."""
import pytest

from gadmm_amd.parallel.dataplane import choose_data_plane
from gadmm_amd.parallel.launch import spawn


@pytest.mark.parametrize("fabric,world,share,want", [
    ("auto", 1, False, "local"), ("rccl", 1, False, "local"),
    ("auto", 2, False, "ipc"), ("xgmi", 8, False, "ipc"), ("ipc", 4, False, "ipc"),
    ("rccl", 8, False, "rccl"), ("rccl", 2, True, "ipc"), ("auto", 4, True, "ipc")])
def test_choose_data_plane(fabric, world, share, want):
    assert choose_data_plane(fabric, world, share) == want


class _StubIpc:
    backend = "ipc"

    def __init__(self, n_total, d, ring, device, group=None, timeout_s=20.0):
        self.args = (n_total, d, ring, timeout_s)
        self.closed = False

    def close(self):
        self.closed = True


def _select_rank(rank, world, fail_rank):
    import gadmm_amd.parallel.comm as C
    import gadmm_amd.parallel.ipc as I
    from gadmm_amd.parallel.dataplane import make_data_plane

    made = []

    class StubRccl:
        backend = "rccl"

        def __init__(self, device, control_group=None, timeout_s=60.0, init_timeout_s=120.0):
            if rank == fail_rank:
                raise RuntimeError("rccl_init failed: set-up deadline passed")
            self.aborted = self.closed = False
            self.timeout_s = timeout_s
            made.append(self)

        def abort(self):
            self.aborted = True

        def close(self):
            self.closed = True

    C.RcclComm, I.IpcComm = StubRccl, _StubIpc
    c = make_data_plane("rccl", world, "cpu", False, 24, 50, 16, timeout_s=3.0, log=lambda m: None)
    auto = make_data_plane("auto", world, "cpu", False, 24, 50, 16, timeout_s=3.0)
    return {"kind": type(c).__name__, "sel": c.selection, "auto": auto.selection["data_plane"],
            "made": [(m.aborted, m.closed, m.timeout_s) for m in made]}


@pytest.mark.parametrize("fail_rank", [-1, 1])
def test_rccl_setup_failure_on_one_rank_moves_every_rank_to_ipc(fail_rank):
    res = spawn(_select_rank, 2, fail_rank, timeout=120)
    for rk, r in enumerate(res):
        assert r["auto"] == "ipc"  # the node default never builds RCCL
        if fail_rank < 0:
            assert r["kind"] == "StubRccl" and r["sel"]["data_plane"] == "rccl"
            assert r["made"] == [(False, False, 3.0)]
        else:
            assert r["kind"] == "_StubIpc" and r["sel"]["data_plane"] == "ipc"
            assert "RCCL unavailable" in r["sel"]["reason"]
            # the rank whose RCCL came up aborts it (a peer failed): no collective destroy
            assert r["made"] == ([] if rk == fail_rank else [(True, True, 3.0)])


def _watchdog_rank(rank, world):
    from gadmm_amd.engine.multigpu import DistributedChainSolver, SolveOut
    from gadmm_amd.ops import native

    class Eng:
        def __init__(self, dead_on):
            self.dead_on, self.closed = dead_on, False

        def refresh(self, X, y):
            pass

        def reset(self):
            pass

        def run(self, use_graph=True):
            if rank == self.dead_on:
                raise native.RcclDead("chain_engine_run failed (rc=-77): rccl_wait: deadline passed")
            class R:
                iters, done, p2p_bytes, wire_bytes, monitor_bytes = 1373, 1, 0, 0, 0
            return R()

        def close(self):
            self.closed = True

    class Comm:
        def __init__(self, kind):
            self.kind, self.aborted, self.closed = kind, False, False

        def abort(self):
            self.aborted = True

        def close(self):
            self.closed = True

    s = DistributedChainSolver.__new__(DistributedChainSolver)
    s.rank, s.world, s.persistent, s.kind, s.fallbacks = rank, world, False, "rccl", []
    s.blk = s.fab = None
    s.use_graph, s.delay_next_s, s.X, s.y = True, 0.0, None, None
    s.eng, s.comm = Eng(dead_on=1), Comm("rccl")
    old_comm = s.comm
    rebuilt = []

    def graph_engine(force_ipc=False):
        rebuilt.append(force_ipc)
        s.comm, s.kind, s.eng, s.persistent = Comm("ipc"), "ipc", Eng(dead_on=-1), False

    s._graph_engine = graph_engine
    assert s.can_fall_back()
    out = s.solve_agreed()
    return {"done": out.done, "iters": out.iters, "kind": s.kind, "rebuilt": rebuilt,
            "old": (old_comm.aborted, old_comm.closed), "fallbacks": s.fallbacks, "can": s.can_fall_back()}


def test_rccl_watchdog_abort_on_one_rank_falls_back_collectively():
    res = spawn(_watchdog_rank, 2, timeout=120)
    for r in res:
        assert r["done"] == 1 and r["iters"] == 1373 and r["kind"] == "ipc"
        assert r["rebuilt"] == [True]          # forced to the IPC transport
        assert r["old"] == (True, True)        # the RCCL communicator aborted, then closed
        assert len(r["fallbacks"]) == 1 and "rccl solve failed" in r["fallbacks"][0]
        assert r["can"] is False               # nothing further to fall back to


def _host_fallback_rank(rank, world):
    """IPC transport fails on rank 1 -> every rank gets the host-staged gloo plane, and the last-resort
    torch-path engine solves the headline problem over it (1373 iterations, like every engine)."""
    import gadmm_amd.parallel.ipc as I
    from gadmm_amd.parallel.dataplane import make_data_plane
    from gadmm_amd.engine.multigpu import TorchPathEngine
    from gadmm_amd.benchmarks import headline_rank_problem

    class FailIpc:
        def __init__(self, n_total, d, ring, device, group=None, timeout_s=20.0):
            if rank == 1:
                raise RuntimeError("hipIpcOpenMemHandle: invalid argument")
            self.closed = False

        def close(self):
            self.closed = True

    I.IpcComm = FailIpc
    c = make_data_plane("auto", world, "cpu", False, 24, 50, 16, timeout_s=3.0, log=lambda m: None)
    X, y, local, pl, obj0 = headline_rank_problem(24, rank, world)
    eng = TorchPathEngine(X, y, local, 24, pl, c, 3.0, obj0, 1e-8, 2000)
    eng.refresh(X, y)
    r = eng.run()
    return {"backend": c.backend, "sel": c.selection["data_plane"], "iters": r.iters, "done": r.done,
            "bytes": r.p2p_bytes}


def test_ipc_failure_falls_back_to_host_staged_plane():
    res = spawn(_host_fallback_rank, 2, timeout=300)
    for r in res:
        assert r["backend"] == "host-gloo" and r["sel"] == "host-gloo"
        assert r["iters"] == 1373 and r["done"] == 1
        assert r["bytes"] == 1373 * 50 * 8  # one boundary: each rank sends its edge worker's theta once per iteration
