"""Communication topologies: chain (GADMM / D-GADMM), star (parameter server), node geometry.

Reference components:

* ``find_path``  — ``findPath.m``: N nodes uniform in a 50x50 square, greedy nearest-unvisited chain
  from node 1, hop cost = squared distance.
* ``find_path2`` — ``findPath2.m``: nodes in 250x250, radio-energy hop cost
  ``P(n,m) = d^2 * eta * B * 2^(R/B)``; also the star energies ``P_central(n) = 1/2 d_c^2 eta B 2^(2R/B)``
  towards the node nearest the area centre.
* ``calc_cost``  — ``calc_cost.m``: cost of a fixed chain under a new geometry.

The reference draws positions with MATLAB's unseeded ``rand``; here every draw comes from an explicit
``numpy.random.Generator`` so all ranks (and tests) reproduce the same paths without messages
("all ranks use a shared seeded RNG, with no message").

Indices are 0-based throughout (reference worker ``ii`` == our worker ``ii-1``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
from ..utils.env import getenv

ETA = 1e-6
RATE = 10e6
BANDWIDTH = 2e6


@dataclass
class Geometry:
    x: np.ndarray
    y: np.ndarray

    @property
    def d_square(self) -> np.ndarray:
        dx = self.x[:, None] - self.x[None, :]
        dy = self.y[:, None] - self.y[None, :]
        d2 = dx * dx + dy * dy
        np.fill_diagonal(d2, 0.0)
        return d2


def random_geometry(n: int, side: float, rng: np.random.Generator) -> Geometry:
    """Node positions; the reference draws x(n) then y(n) per node (findPath.m:3-6)."""
    xy = rng.random((n, 2)) * side
    return Geometry(x=xy[:, 0].copy(), y=xy[:, 1].copy())


def greedy_chain(d_square: np.ndarray, start: int = 0) -> List[int]:
    """Greedy nearest-unvisited path from ``start`` (findPath.m:16-30). Ties -> lowest index."""
    n = d_square.shape[0]
    path = [start]
    visited = np.zeros(n, dtype=bool)
    visited[start] = True
    while len(path) < n:
        cur = path[-1]
        row = np.where(visited, np.inf, d_square[cur])
        row[cur] = np.inf
        nxt = int(np.argmin(row))
        path.append(nxt)
        visited[nxt] = True
    return path


def greedy_chains(d_square: np.ndarray, start: int = 0) -> np.ndarray:
    """``greedy_chain`` for a batch of geometries (E, N, N) at once; same tie rule (lowest index)."""
    E, n, _ = d_square.shape
    paths = np.zeros((E, n), dtype=np.int64)
    paths[:, 0] = start
    visited = np.zeros((E, n), dtype=bool)
    visited[:, start] = True
    cur = np.full(E, start)
    ar = np.arange(E)
    for k in range(1, n):
        row = np.where(visited, np.inf, d_square[ar, cur])
        row[ar, cur] = np.inf
        nxt = np.argmin(row, axis=1)
        paths[:, k] = nxt
        visited[ar, nxt] = True
        cur = nxt
    return paths


def find_path(n: int, rng: np.random.Generator) -> Tuple[List[int], np.ndarray, np.ndarray]:
    """``[path, pathCost, d_square] = findPath(N)``: squared-distance hop costs, 50x50 area."""
    g = random_geometry(n, 50.0, rng)
    d2 = g.d_square
    path = greedy_chain(d2)
    cost = np.array([d2[path[k], path[k + 1]] for k in range(n - 1)])
    return path, cost, d2


def link_energy(d2: np.ndarray) -> np.ndarray:
    return d2 * ETA * BANDWIDTH * 2.0 ** (RATE / BANDWIDTH)


def find_path2(n: int, rng: np.random.Generator):
    """``[path, pathCost, d_square, P_central, center] = findPath2(N)`` (radio-energy costs)."""
    side = 250.0
    g = random_geometry(n, side, rng)
    dist_c = np.sqrt((g.x - side / 2) ** 2 + (g.y - side / 2) ** 2)
    center = int(np.argmin(dist_c))
    d2c = (g.x - g.x[center]) ** 2 + (g.y - g.y[center]) ** 2
    p_central = 0.5 * d2c * ETA * BANDWIDTH * 2.0 ** (2 * RATE / BANDWIDTH)
    d2 = g.d_square
    P = link_energy(d2)
    path = greedy_chain(d2)
    cost = np.array([P[path[k], path[k + 1]] for k in range(n - 1)])
    return path, cost, d2, p_central, center


def calc_cost(grid: np.ndarray, path0: Sequence[int]) -> np.ndarray:
    """Hop costs of the fixed chain ``path0`` under geometry ``grid`` (calc_cost.m:1-10)."""
    return np.array([grid[path0[k], path0[k + 1]] for k in range(len(path0) - 1)])


def star_cost(p_central: np.ndarray) -> float:
    """Per-iteration star energy = uplink sum + downlink max (LinearRegression_gadmm_vs_admm.m:84-87)."""
    return float(np.sum(p_central) + np.max(p_central))


def rechain_iteration(it: int, coherence: float) -> bool:
    """D-GADMM refresh rule ``i > 1 && mod(i, coherence_Time) == 0`` (dynamic_group_ADMM_closedForm.m:18)."""
    if coherence is None or coherence <= 0 or not np.isfinite(coherence):
        return False
    c = int(coherence)
    return it > 1 and c > 0 and it % c == 0


def rechain_iterations(max_iter: int, coherence: float) -> np.ndarray:
    """All iterations in [2, max_iter] at which ``rechain_iteration`` fires."""
    if coherence is None or coherence <= 0 or not np.isfinite(coherence) or int(coherence) <= 0:
        return np.zeros(0, dtype=np.int64)
    c = int(coherence)
    its = np.arange(c, max_iter + 1, c, dtype=np.int64)
    return its[its > 1]


def native_greedy_chains(uv: np.ndarray, side: float, energy: bool) -> Tuple[np.ndarray, np.ndarray]:
    """Greedy chains + hop costs for a batch of node-position draws ``uv`` (E, N, 2) in [0, 1) by the
    native C++ routine (csrc/runtime/topology.cpp), bit-identical to the numpy path."""
    from ..ops import native

    lib = native.load(build_if_missing=False)
    uv = np.ascontiguousarray(uv, dtype=np.float64)
    E, n, _ = uv.shape
    paths = np.empty((E, n), dtype=np.int64)
    costs = np.empty((E, max(n - 1, 0)), dtype=np.float64)
    rc = lib.gadmm_greedy_chains(uv.ctypes.data, E, n, float(side), int(energy), ETA, BANDWIDTH,
                                 2.0 ** (RATE / BANDWIDTH), paths.ctypes.data, costs.ctypes.data)
    if rc != 0:
        raise RuntimeError("gadmm_greedy_chains failed")
    return paths, costs


_ASYNC_KEEP = None  # buffers of the last asynchronous greedy-chain job (PathSchedule.prefetch_async)
_SEED_STATE: Dict[int, Tuple[int, int]] = {}  # seed -> (state, inc) of default_rng(seed)'s PCG64


_NATIVE_CHAINS = []  # [bool]: whether the built library has the chain builder (asked once)


def _native_chains_ok() -> bool:
    """The native chain builder is used when the library is already built (never builds it)."""
    if getenv("GADMM_NATIVE_TOPOLOGY", "1") == "0":
        return False
    if not _NATIVE_CHAINS:
        try:
            from ..ops import native

            lib = native.load(build_if_missing=False)
            ok = lib is not None and getattr(lib, "gadmm_greedy_chains", None) is not None
        except Exception:
            ok = False
        if not ok:
            return False  # not cached: a later build may provide it
        _NATIVE_CHAINS.append(True)
    return True


class PathSchedule:
    """Deterministic sequence of chains for D-GADMM.

    ``kind='findPath2'`` re-draws a geometry and greedy chain at every refresh (the reference's
    ``dynamic_group_ADMM_closedForm.m:20``); ``kind='matrix'`` consumes pre-generated rows
    (``dynamic_group_ADMM_closedForm_v0.m:16-26``).
    """

    def __init__(self, n: int, initial_path: Sequence[int], initial_cost: Sequence[float], coherence: float,
                 kind: str = "findPath2", seed: int = 1234, path_matrix=None, cost_matrix=None):
        self.n = n
        self.coherence = coherence
        self.kind = kind
        # The numpy Generator (default_rng(seed)) is built on first use: until then the stream position
        # is (seed, outputs consumed) -- a D-GADMM solve whose chains the native worker draws from that
        # state (prefetch_async) never needs it (building one costs ~10-20 us per solve).
        self._seed = seed
        self._rng = None
        self._ahead = 0
        if not isinstance(seed, (int, np.integer)):  # entropy / SeedSequence seeds: no lazy replay
            self._rng = np.random.default_rng(seed)
        self.path = list(initial_path)
        self.cost = np.asarray(initial_cost, dtype=np.float64)
        self.path_matrix = path_matrix
        self.cost_matrix = cost_matrix
        self.k = 1  # next row of the matrices

    @property
    def rng(self) -> np.random.Generator:
        if self._rng is None:
            g = np.random.default_rng(self._seed)
            if self._ahead:
                g.bit_generator.advance(self._ahead)
            self._rng = g
        return self._rng

    def _pcg_state(self):
        """(state, inc) of the PCG64 stream at the current position, as ints; the materialised
        Generator (if any) is NOT advanced."""
        if self._rng is not None:
            st = self._rng.bit_generator.state["state"]
            return st["state"], st["inc"], 0
        st = _SEED_STATE.get(self._seed)
        if st is None:
            st = np.random.default_rng(self._seed).bit_generator.state["state"]
            st = (st["state"], st["inc"])
            if len(_SEED_STATE) < 256:
                _SEED_STATE[self._seed] = st
        return st[0], st[1], self._ahead

    def _consume(self, outputs: int) -> None:
        if self._rng is None:
            self._ahead += outputs
        else:
            self._rng.bit_generator.advance(outputs)

    def save(self):
        rs = ("lazy", self._ahead) if self._rng is None else self._rng.bit_generator.state
        return (rs, list(self.path), self.cost.copy(), self.k)

    def restore(self, st) -> None:
        if isinstance(st[0], tuple) and st[0][0] == "lazy":
            self._rng, self._ahead = None, int(st[0][1])
        else:
            self.rng.bit_generator.state = st[0]
        self.path, self.cost, self.k = list(st[1]), st[2].copy(), st[3]

    def prefetch_arrays(self, count: int) -> Tuple[np.ndarray, np.ndarray]:
        """The next ``count`` chains as arrays ``(paths (count, N) int64, costs (count, N-1))``,
        exactly as ``count`` successive re-chains would draw them (same RNG stream: the geometries
        of all epochs come from one batched draw), vectorised over epochs. Advances the schedule
        past them."""
        n = self.n
        if count <= 0:
            return np.zeros((0, n), dtype=np.int64), np.zeros((0, max(n - 1, 0)))
        if self.kind == "matrix":
            rows = range(self.k, self.k + count)
            paths = np.asarray([list(self.path_matrix[k]) for k in rows], dtype=np.int64)
            cl = [np.asarray(self.cost_matrix[k], dtype=np.float64) for k in rows]
            if len({len(c) for c in cl}) == 1:
                costs = np.asarray(cl)
            else:  # ragged rows (the v0 quirk): a 1-D object array of cost vectors
                costs = np.empty(len(cl), dtype=object)
                costs[:] = cl
            self.k += count
        elif native_greedy_chains is not None and _native_chains_ok():
            side = 50.0 if self.kind == "findPath" else 250.0
            uv = self.rng.random((count, n, 2))   # == count sequential rng.random((n, 2))
            paths, costs = native_greedy_chains(uv, side, self.kind != "findPath")
        else:
            side = 50.0 if self.kind == "findPath" else 250.0
            xy = self.rng.random((count, n, 2)) * side   # == count sequential rng.random((n, 2))
            x, y = xy[..., 0], xy[..., 1]
            d2 = (x[:, :, None] - x[:, None, :]) ** 2 + (y[:, :, None] - y[:, None, :]) ** 2
            idx = np.arange(n)
            d2[:, idx, idx] = 0.0
            paths = greedy_chains(d2)
            hop = d2 if self.kind == "findPath" else link_energy(d2)
            costs = hop[np.arange(count)[:, None], paths[:, :-1], paths[:, 1:]]   # hop[e, p_k, p_{k+1}]
        self.path, self.cost = [int(v) for v in paths[-1]], np.asarray(costs[-1], dtype=np.float64)
        return paths, costs

    def prefetch_async(self, count: int):
        """Start drawing the next ``count`` chains on the native library's host worker thread: the
        geometries (numpy's PCG64 stream from the schedule's current position, ``gadmm_draw_chains_async``)
        and the greedy walks. The schedule's RNG position moves past them at once. Returns a callable
        giving ``(paths, costs)`` exactly as ``prefetch_arrays(count)`` would (the current chain moves
        at that call), or None where the native builder does not apply (the caller draws
        synchronously)."""
        if count <= 0 or self.kind == "matrix" or not _native_chains_ok():
            return None
        from ..ops import native

        lib = native.load(build_if_missing=False)
        if getattr(lib, "gadmm_draw_chains_async", None) is None:
            return None
        n = self.n
        side = 50.0 if self.kind == "findPath" else 250.0
        state, inc, ahead = self._pcg_state()
        uv = np.empty((count, n, 2), dtype=np.float64)
        paths = np.empty((count, n), dtype=np.int64)
        costs = np.empty((count, max(n - 1, 0)), dtype=np.float64)
        global _ASYNC_KEEP
        lib.gadmm_greedy_chains_wait()  # a previous job (never joined) is done with its buffers
        _ASYNC_KEEP = (uv, paths, costs)  # held until the next submit: the worker writes into them
        M = (1 << 64) - 1
        rc = lib.gadmm_draw_chains_async(state >> 64, state & M, inc >> 64, inc & M, ahead, uv.ctypes.data, count, n,
                                         side, int(self.kind != "findPath"), ETA, BANDWIDTH, 2.0 ** (RATE / BANDWIDTH),
                                         paths.ctypes.data, costs.ctypes.data)
        if rc != 0:
            raise RuntimeError("gadmm_draw_chains_async failed")
        self._consume(2 * n * count)
        box = []

        def join():
            if not box:
                if lib.gadmm_greedy_chains_wait() != 0:
                    raise RuntimeError("gadmm_greedy_chains failed")
                self.path, self.cost = [int(v) for v in paths[-1]], np.asarray(costs[-1], dtype=np.float64)
                box.append((paths, costs))
            return box[0]

        return join

    def prefetch(self, count: int):
        """``prefetch_arrays`` as a list ``[(path, cost), ...]``."""
        paths, costs = self.prefetch_arrays(count)
        return [([int(v) for v in p], c.copy()) for p, c in zip(paths, costs)]

    def skip(self, saved, paths: np.ndarray, costs: np.ndarray, count: int) -> None:
        """Put the schedule where ``count`` re-chains after the ``save()`` point ``saved`` leave
        it, given the chains ``prefetch_arrays`` drew from there (the RNG is advanced, not
        re-drawn: every findPath/findPath2 geometry consumes 2N doubles)."""
        self.restore(saved)
        if count <= 0:
            return
        if self.kind == "matrix":
            self.k += count
        else:
            self._consume(2 * self.n * count)
        self.path, self.cost = [int(v) for v in paths[count - 1]], np.asarray(costs[count - 1], dtype=np.float64)

    def step(self, it: int) -> bool:
        """Advance to iteration ``it``; returns True if the chain changed."""
        if not rechain_iteration(it, self.coherence):
            return False
        if self.kind == "matrix":
            self.path = list(self.path_matrix[self.k])
            self.cost = np.asarray(self.cost_matrix[self.k])
            self.k += 1
        elif self.kind == "findPath":
            p, c, _ = find_path(self.n, self.rng)
            self.path, self.cost = p, c
        else:
            p, c, _, _, _ = find_path2(self.n, self.rng)
            self.path, self.cost = p, c
        return True


# -------------------------------------------------------------------------------------------------
# Placement and per-rank phase plans
# -------------------------------------------------------------------------------------------------

_CONTIGUOUS: Dict[Tuple[int, int], "Placement"] = {}


@dataclass
class Placement:
    """Logical worker -> rank map. Default: contiguous blocks of workers per rank (so a static
    identity chain crosses a device boundary only at segment ends)."""

    owner: np.ndarray          # (N,) rank of each global worker
    nranks: int

    @staticmethod
    def contiguous(n_workers: int, nranks: int) -> "Placement":
        """Memoised per (n_workers, nranks): the same object on every call (placements are never
        mutated), so per-solve callers skip the construction and identity-keyed memos hit."""
        key = (int(n_workers), int(nranks))
        pl = _CONTIGUOUS.get(key)
        if pl is None:
            if nranks > n_workers:
                raise ValueError("more ranks (%d) than workers (%d)" % (nranks, n_workers))
            base, extra = divmod(n_workers, nranks)
            owner = []
            for r in range(nranks):
                owner += [r] * (base + (1 if r < extra else 0))
            pl = Placement(owner=np.asarray(owner, dtype=np.int64), nranks=nranks)
            pl.owner.setflags(write=False)
            _CONTIGUOUS[key] = pl
        return pl

    def local_workers(self, rank: int) -> List[int]:
        return [int(w) for w in np.nonzero(self.owner == rank)[0]]

    def local_index(self, rank: int) -> Dict[int, int]:
        return {w: i for i, w in enumerate(self.local_workers(rank))}


@dataclass
class Slot:
    li: int
    gid: int
    left: int
    right: int


@dataclass
class RankPlan:
    head: List[Slot] = field(default_factory=list)
    tail: List[Slot] = field(default_factory=list)
    # (peer, row, is_send) messages after the head / tail phase
    xchg_head: List[Tuple[int, int, int]] = field(default_factory=list)
    xchg_tail: List[Tuple[int, int, int]] = field(default_factory=list)

    def send_rows(self) -> int:
        return sum(1 for _, _, s in self.xchg_head if s) + sum(1 for _, _, s in self.xchg_tail if s)


def chain_plan(path: Sequence[int], placement: Placement, rank: int) -> RankPlan:
    """Head/tail slots of ``rank`` for the chain ``path`` (position -> worker) and the neighbour
    messages that must cross ranks after each phase.

    Heads are chain positions 0, 2, 4, ... (MATLAB ``jj = 1:2:N``), tails 1, 3, 5, ...
    After the head phase every head sends its fresh theta to each neighbour that lives on another
    rank (C2); after the tail phase every tail does the same (C1). One message per (worker, peer
    rank) pair even when both neighbours live on the same peer.
    """
    n = len(path)
    lidx = placement.local_index(rank)
    plan = RankPlan()
    for pos, w in enumerate(path):
        left = path[pos - 1] if pos > 0 else -1
        right = path[pos + 1] if pos < n - 1 else -1
        phase_is_head = (pos % 2 == 0)
        if w in lidx:
            s = Slot(li=lidx[w], gid=int(w), left=int(left), right=int(right))
            (plan.head if phase_is_head else plan.tail).append(s)
        # messages
        owner_w = int(placement.owner[w])
        peers = sorted({int(placement.owner[u]) for u in (left, right) if u >= 0} - {owner_w})
        lst = plan.xchg_head if phase_is_head else plan.xchg_tail
        for p in peers:
            if owner_w == rank:
                lst.append((p, int(w), 1))
            elif p == rank:
                lst.append((owner_w, int(w), 0))
    return plan


def chain_message_count(path: Sequence[int], placement: Placement) -> int:
    """Total cross-rank messages per GADMM iteration for ``path`` (all ranks)."""
    total = 0
    for pos, w in enumerate(path):
        nb = [path[pos - 1]] if pos > 0 else []
        if pos < len(path) - 1:
            nb.append(path[pos + 1])
        total += len({int(placement.owner[u]) for u in nb} - {int(placement.owner[w])})
    return total
