"""One GADMM chain over several MI355X (one process per GPU): engine choice, byte accounting and the
collective fallback. Used by ``bench.py`` and the multi-rank tests.

Data-local by construction: the solver is given only this rank's shards (``X_loc``) and ships only
theta, to the ranks of its chain neighbours (group_ADMM_closedForm.m:18-27, 62-70). Engines, in the
order ``engine="auto"`` tries them:

1. ``xgmi(blocked-dl)`` -- the temporally blocked kernel run inside each rank's segment
   (chain_blocked.hip, data-local mode, engine/blocked_xgmi.py): the segment's intra-rank hand-offs
   are LDS barriers (one workgroup when the segment fits 12 waves) as on one GPU, and only the two
   segment-edge workers exchange theta with the neighbouring ranks, every phase, over xGMI. When every
   segment has >= 2 positions and fits one workgroup it runs in the one-position halo mode
   (``xgmi(blocked-dl-halo)``, GADMM_DL_HALO=0 disables it): at each boundary the rank holding the tail
   also solves the other rank's boundary head from that head's shard (20 KB, fetched once and reported
   as ``replicated_bytes``), which leaves one cross-rank hop per iteration on the critical cycle.
2. ``xgmi`` -- the per-worker persistent kernel (chain_persistent.hip, SYS scope): one workgroup per
   local worker, boundary theta stored straight into the neighbour GPU's table over xGMI, objective
   granules to rank 0's monitor, decisions fanned back out. One launch per solve.
3. ``ipc`` / ``rccl`` -- the graph-replayed phase kernels (chain_engine.cpp) with the device-copy
   transport (parallel/ipc.py; the default data plane, and the only one when ranks share one GPU), or
   with RCCL send/recv when ``fabric="rccl"`` is asked for (non-blocking communicator, bounded host
   waits: a hung RCCL graph is aborted and every rank moves to ``ipc``).

Every choice is agreed by all ranks (an all-reduce of a success flag), and so is every fallback: a
solve that fails on ANY rank (a stalled hand-off reaches its deadline: ``done == 4``) makes every
rank drop the persistent kernel and continue on the graph engine together.

``engine="replicated-halo"`` is the opt-in temporally blocked kernel across GPUs
(engine/blocked_xgmi.py): it needs the halo workers' shards (``halo_data``) and is reported as such.
"""
from __future__ import annotations

import sys
import time
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist


@dataclass
class SolveOut:
    iters: int
    done: int
    theta_bytes: int   # payload, 8 B per double
    wire_bytes: int    # on the fabric (granules: 16 B per double)
    monitor_bytes: int


def all_ok(flag: bool, world: int) -> bool:
    if world == 1:
        return flag
    t = torch.tensor([0.0 if flag else 1.0], dtype=torch.float64)
    dist.all_reduce(t)
    return float(t.item()) == 0.0


_STREAMS: dict = {}


def solver_stream(device: torch.device) -> torch.cuda.Stream:
    """One engine stream per process and device, shared by every DistributedChainSolver (the engine
    tournament builds several): persistent kernels of several ranks must run at the same time, and with
    ranks time-sharing one GPU every extra stream a process touches is one more hardware queue for the
    GPU's scheduler to multiplex -- past its slots, queues are time-sliced and cross-rank hand-offs stall
    until their deadline (8 ranks on one MI355X, the second tournament candidate on)."""
    key = torch.device(device).index
    st = _STREAMS.get(key)
    if st is None:
        st = torch.cuda.Stream(device)
        _STREAMS[key] = st
    return st


class DistributedChainSolver:
    def __init__(self, X_loc: torch.Tensor, y_loc: torch.Tensor, local: Sequence[int], n_total: int, placement,
                 rank: int, world: int, device: torch.device, rho: float, obj0: float, tol: float,
                 max_iter: int = 20000, engine: str = "auto", fabric: str = "auto", share: bool = False,
                 block: int = 0, halo_data=None, timeout_s: float = 20.0, use_graph: bool = True,
                 dl_halo: Optional[bool] = None, strict: bool = False, halo_k: int = 0, halo_pw: int = 0,
                 plane=None):
        """``dl_halo`` (data-local blocked engine): None = the halo mode where eligible, True = only the
        halo mode, False = never. ``strict``: raise (on every rank together) when the requested
        persistent engine cannot run instead of falling back to the graph engine (the engine
        tournament of bench.py builds each candidate this way). ``plane``: an existing data-plane comm
        (an entry session's, ``parallel/node.NodeFabrics.data_plane``) for the graph engine instead of a
        new one; it is the caller's, never closed here."""
        from .chain_engine import NativeChainEngine

        self.X, self.y = X_loc, y_loc
        self.local = [int(w) for w in local]
        self.n, self.placement, self.rank, self.world, self.device = n_total, placement, rank, world, device
        self.rho, self.obj0, self.tol, self.max_iter = rho, obj0, tol, max_iter
        self.share, self.fabric_req, self.timeout_s, self.use_graph = share, fabric, timeout_s, use_graph
        self.block = block if block > 0 else (32 if world == 1 else 16)
        self.d = int(X_loc.shape[2])
        self.path = list(range(n_total))
        self.eng = self.comm = self.fab = self.blk = None
        self.kind, self.persistent, self.replicated_bytes = "local", False, 0
        self.fallbacks = []
        self.dl_halo = dl_halo
        self.plane, self._own_comm = plane, True
        self.delay_next_s = 0.0  # test hook: sleep before the next launch (a slow / stalled peer)
        self._NCE = NativeChainEngine
        if world == 1:
            self.eng = self._engine(None)
            self.persistent = engine in ("auto", "persistent") and self.eng.persistent_eligible()
        elif engine == "replicated-halo":
            from .blocked_xgmi import BlockedXgmiEngine
            if halo_data is None:
                raise ValueError("replicated-halo needs the halo workers' shards (halo_data=(X_all, y_all))")
            self.blk = BlockedXgmiEngine(halo_data[0], halo_data[1], n_total, placement, rank, rho, obj0, tol,
                                         max_iter, device, stream=solver_stream(device), want_k=halo_k,
                                         want_pw=halo_pw)
            self.replicated_bytes = self.blk.replicated_shard_bytes()
            self.persistent = True
            self.kind = "xgmi(replicated-halo,k=%d,pw=%d)" % (self.blk.k, self.blk.pw)
        else:
            if fabric in ("auto", "xgmi") and engine in ("auto", "persistent", "blocked-dl"):
                self._try_blocked_dl()
            if self.blk is None and fabric in ("auto", "xgmi") and engine in ("auto", "persistent", "per-worker"):
                self._try_xgmi()
            if self.eng is None and self.blk is None:
                if strict and engine != "graph":
                    raise RuntimeError("engine %r unavailable on some rank" % engine)
                self._graph_engine()

    # ---------------------------------------------------------------------------------------------
    def _engine(self, comm):
        e = self._NCE(self.X, self.y, self.local, self.n, "linear", rho=self.rho, obj0=self.obj0, tol=self.tol,
                      max_iter=self.max_iter, comm=comm, block=self.block, stream=solver_stream(self.device))
        e.set_path(self.path, self.placement, self.rank)
        return e

    def _try_blocked_dl(self):
        """Collective: the data-local blocked kernel over the xGMI fabric, if every rank can run it."""
        from .blocked_xgmi import BlockedXgmiEngine

        lo, hi = min(self.local), max(self.local)
        eligible = self.local == list(range(lo, hi + 1)) and self.d <= 52 and self.n >= 2
        if not all_ok(eligible, self.world):
            return
        try:
            blk = BlockedXgmiEngine(self.X, self.y, self.n, self.placement, self.rank, self.rho, self.obj0, self.tol,
                                    self.max_iter, self.device, data_local=True, dl_halo=self.dl_halo,
                                    stream=solver_stream(self.device))
        except Exception as e:  # collective inside the constructor: every rank raises together
            if self.rank == 0:
                print("DistributedChainSolver: data-local blocked fabric unavailable (%s)" % e, file=sys.stderr)
            return
        self.blk, self.persistent = blk, True
        self.kind = "xgmi(blocked-dl-halo)" if blk._halo_mode() else "xgmi(blocked-dl)"
        self.replicated_bytes = blk.replicated_shard_bytes()  # halo mode: one neighbour head's shard per tail-side boundary

    def _try_xgmi(self):
        from ..parallel.comm import RankInfo
        from ..parallel.xgmi import XgmiFabric

        ok, err = False, ""
        eng = self._engine(RankInfo(self.rank, self.world))
        try:
            need = sorted({int(self.placement.owner[u]) for w in self.local for u in (w - 1, w + 1)
                           if 0 <= u < self.n} - {self.rank})
            self.fab = XgmiFabric(self.n, self.d, 8, self.rank, self.world, self.device, peers_needed=need)
            ok = eng.persistent_eligible(self.fab)
            err = "" if ok else "persistent kernel not eligible (residency)"
        except Exception as e:
            err = str(e)
        if all_ok(ok, self.world):
            self.eng, self.persistent, self.kind = eng, True, "xgmi"
            return
        if self.rank == 0:
            print("DistributedChainSolver: xgmi fabric unavailable (%s); graph engine" % (err or "another rank"),
                  file=sys.stderr)
        if self.fab is not None:
            self.fab.close()
        self.fab = None
        eng.close()

    def _graph_engine(self, force_ipc: bool = False):
        """The graph-replayed phase kernels over the data plane of ``parallel/dataplane.py``: the IPC
        transport by default (``--fabric auto`` / ``ipc``, and always with ranks sharing a GPU), RCCL
        only for ``--fabric rccl`` -- with its watchdog (the engine's bounded waits abort a hung
        communicator; ``fall_back`` then moves every rank to IPC). Collective."""
        from ..parallel.dataplane import make_data_plane
        fabric = "ipc" if force_ipc else self.fabric_req
        if getattr(self, "plane", None) is not None and not (force_ipc and getattr(self.plane, "backend", "") != "ipc"):
            self.comm, self._own_comm = self.plane, False
        else:
            self.comm, self._own_comm = make_data_plane(fabric, self.world, self.device, self.share, self.n,
                                                        self.d, self.block, timeout_s=self.timeout_s), True
        self.kind = self.comm.selection["data_plane"]
        if getattr(self.comm, "backend", "") == "host-gloo":  # no device transport came up anywhere
            self.eng = TorchPathEngine(self.X, self.y, self.local, self.n, self.placement, self.comm, self.rho,
                                       self.obj0, self.tol, self.max_iter)
        else:
            self.eng = self._engine(self.comm)
        self.persistent = False

    def can_fall_back(self) -> bool:
        """A persistent kernel (-> the graph engine) or an RCCL graph engine (-> the IPC transport)."""
        return self.world > 1 and (self.persistent or self.kind == "rccl")

    def fall_back(self, why: str):
        """Collective: every rank drops the persistent kernels for the graph engine, or the RCCL data
        plane for the IPC transport."""
        self.fallbacks.append(why)
        from_rccl = (not self.persistent) and self.kind == "rccl"
        if self.blk is not None:
            self.blk.close()
            self.blk = None
        if self.fab is not None:
            self.fab.close()
            self.fab = None
        if self.eng is not None:
            self.eng.close()
            self.eng = None
        if self.comm is not None:
            if from_rccl:
                self.comm.abort()  # peers may be gone or aborted: never a collective destroy
            own = getattr(self, "_own_comm", True)
            if own or from_rccl:
                self.comm.close()
            if not own:
                self.plane = None  # the caller's plane is dead: never hand it out again
            self.comm = None
        self._graph_engine(force_ipc=from_rccl)

    # ---------------------------------------------------------------------------------------------
    def solve(self) -> SolveOut:
        """One solve from the raw shards (Gram, inverses, iterations). Raises on a stalled hand-off."""
        if self.delay_next_s > 0:
            time.sleep(self.delay_next_s)
            self.delay_next_s = 0.0
        if self.blk is not None:
            self.blk.refresh()
            it, done, self.last_wall_ms = self.blk.run(timeout_s=self.timeout_s)
            if done == 4:
                raise RuntimeError("blocked kernel: a hand-off timed out")
            pay = self.blk.exchange_bytes_per_solve(it)
            return SolveOut(it, done, pay, 2 * pay, self.blk.monitor_bytes_per_solve(it))
        self.eng.refresh(self.X, self.y)
        self.eng.reset()
        if self.persistent:
            r = self.eng.run_persistent(fabric=self.fab, timeout_s=self.timeout_s)
        else:
            r = self.eng.run(use_graph=self.use_graph)
        self.last_wall_ms = float(getattr(r, "wall_ms", 0.0))
        return SolveOut(r.iters, r.done, r.p2p_bytes, r.wire_bytes, r.monitor_bytes)

    def guarded_solve(self) -> SolveOut:
        try:
            return self.solve()
        except RuntimeError as e:
            print("DistributedChainSolver[rank %d]: %s" % (self.rank, e), file=sys.stderr)
            return SolveOut(0, 4, 0, 0, 0)

    def solve_agreed(self) -> SolveOut:
        """Solve; if it failed on any rank while a persistent kernel was in use, every rank falls back
        to the graph engine and solves again. Collective."""
        out = self.guarded_solve()
        if all_ok(out.done == 1, self.world):
            return out
        if self.can_fall_back():
            self.fall_back("%s solve failed on some rank (done=%d here)" % (self.kind, out.done))
            out = self.guarded_solve()
        return out

    # ---------------------------------------------------------------------------------------------
    @property
    def kernel(self) -> Optional[str]:
        if not self.persistent:
            return None
        return self.blk.last_kernel if self.blk is not None else getattr(self.eng, "last_kernel", None)

    def engine_name(self) -> str:
        if self.persistent:
            return "persistent"
        return "graph" if (self.eng is not None and self.eng.graph_ok() and self.use_graph) else "eager"

    def objective_trace(self, iters: int):
        return self.blk.objective_trace(iters) if self.blk is not None else self.eng.objective_trace(iters)

    def close(self):
        for o in (self.eng, self.blk, self.fab, self.comm if getattr(self, "_own_comm", True) else None):
            if o is not None:
                o.close()
        self.eng = self.blk = self.fab = self.comm = None


class TorchPathEngine:
    """The last-resort engine of a multi-GPU solve (``HostStagedComm`` data plane: neither the IPC
    transport nor RCCL came up): the torch GADMM loop (algorithms/gadmm._chain_admm_torch, the executable
    spec of group_ADMM_closedForm.m) on the device shards, neighbour theta staged through host memory
    over gloo. Same interface as the parts of NativeChainEngine that DistributedChainSolver uses."""

    def __init__(self, X, y, local, n_total, placement, comm, rho, obj0, tol, max_iter):
        from ..models import LinearRegression
        self.X, self.y, self.local, self.n, self.placement, self.comm = X, y, list(local), n_total, placement, comm
        self.rho, self.obj0, self.tol, self.max_iter = rho, obj0, tol, max_iter
        self.model = LinearRegression(X, y)
        self.last = None

    def refresh(self, X, y):
        from ..ops.linalg import gram
        gram(X, y, out=(self.model.A, self.model.b, self.model.yy))
        self.model._chol = {}

    def reset(self, start_iter: int = 1):
        self.last = None

    def run(self, stop_iter: int = 0, use_graph: bool = True):
        import time as _t
        from ..algorithms.gadmm import chain_admm
        t0 = _t.perf_counter()
        snap = self.comm.stats.snapshot()
        r = chain_admm(self.model, self.local, self.n, self.rho, self.obj0, self.tol, self.max_iter, comm=self.comm,
                       placement=self.placement, backend="torch")
        self.last = r
        pay = int(self.comm.stats.delta(snap)["bytes_sent"])
        mon = int(self.comm.stats.delta(snap)["monitor_bytes"])

        class _R:
            pass
        o = _R()
        o.iters, o.done = int(r.iters), (1 if r.converged else 2)
        o.p2p_bytes, o.wire_bytes, o.monitor_bytes = pay, pay, mon
        o.wall_ms = (_t.perf_counter() - t0) * 1e3
        return o

    def objective_trace(self, upto=None):
        tr = self.last.obj if self.last is not None else np.zeros(0)
        return tr if upto is None else tr[:upto]

    def traces(self, upto: int):
        return self.objective_trace(upto), np.asarray(self.last.time_trace[:upto])

    def graph_ok(self) -> bool:
        return False

    def close(self):
        self.last = None


def node_chain_admm(model, local_ids: Sequence[int], n_total: int, placement, rank: int, world: int,
                    device: torch.device, rho: float, obj0: float, tol: float, max_iter: int,
                    fabric: str = "auto", share: bool = False, plane=None, timeout_s: float = 20.0,
                    name: str = "GADMM"):
    """GADMM with closed-form local solves on a static identity chain (group_ADMM_closedForm.m:13-108)
    over several GPUs, on the engines of the headline benchmark: this rank's contiguous segment of
    ``model``'s shards goes to ``DistributedChainSolver`` (data-local blocked kernel over xGMI, with its
    halo mode where eligible -> per-worker persistent kernel -> graph engine over the session's data
    plane ``plane``). One solve from the raw shards (Gram, inverses, iterations), agreed by every rank;
    a solve that fails on any rank (stalled hand-off) moves every rank to the next engine and runs again.
    Returns a ``RunResult`` like ``chain_admm``'s: the objective trace of rank 0's monitor (identical on
    every rank), the per-iteration decision clock, payload / wire / monitor bytes."""
    import numpy as np
    from ..algorithms.base import RunResult

    local = [int(w) for w in local_ids]
    sol = DistributedChainSolver(model.X, model.y, local, n_total, placement, rank, world, device, rho, obj0, tol,
                                 max_iter=max_iter, fabric=fabric, share=share, timeout_s=timeout_s, plane=plane)
    try:
        if sol.blk is not None:
            sol.blk.stamps = True
        out = sol.guarded_solve()
        if not all_ok(out.done in (1, 2), world) and sol.can_fall_back():
            sol.fall_back("%s solve failed on some rank (done=%d here)" % (sol.kind, out.done))
            out = sol.guarded_solve()
        if not all_ok(out.done in (1, 2), world):
            raise RuntimeError("node GADMM solve failed (done=%d here, engine %s)" % (out.done, sol.kind))
        iters = int(out.iters)
        if sol.blk is not None:
            tr, tt = sol.blk.objective_trace(iters), sol.blk.time_trace(iters)
        else:
            tr, tt = sol.eng.traces(iters)
        # rank 0's monitor decided: every rank reports its trace and clock
        buf = torch.from_numpy(np.stack([np.asarray(tr, np.float64), np.asarray(tt, np.float64)]))
        dist.broadcast(buf, src=0)
        tr, tt = buf[0].numpy().copy(), buf[1].numpy().copy()
        tot = torch.tensor([float(out.theta_bytes), float(out.wire_bytes), float(out.monitor_bytes),
                            float(sol.replicated_bytes)], dtype=torch.float64)
        dist.all_reduce(tot)
        transport = "xgmi" if sol.persistent else sol.kind
        res = RunResult(algorithm=name, obj=tr, loss=np.abs(tr - obj0), iters=iters, converged=(out.done == 1),
                        wall_s=float(getattr(sol, "last_wall_ms", 0.0)) / 1e3, time_trace=tt,
                        comm_units=np.arange(1, iters + 1, dtype=np.float64) * n_total,
                        com_cost=np.zeros(iters), bytes_sent=int(out.theta_bytes), bytes_total=int(tot[0].item()),
                        extra={"backend": "native", "engine": sol.engine_name(), "kernel": sol.kernel or "",
                               "engine_kind": sol.kind, "transport": transport, "rank": rank, "nranks": world,
                               "solver": "closed", "wire_bytes": int(out.wire_bytes),
                               "monitor_bytes": int(out.monitor_bytes),
                               "wire_bytes_all_ranks": int(tot[1].item()),
                               "monitor_bytes_all_ranks": int(tot[2].item()),
                               "replicated_shard_bytes": int(tot[3].item()),
                               "fallbacks": "; ".join(sol.fallbacks)})
        return res
    finally:
        sol.close()
