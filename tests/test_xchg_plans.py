"""The multi-rank exchange plans (``parallel/topology.py:chain_plan``) proven on the CPU, for every rank
at 2 / 4 / 8 ranks, static chains and D-GADMM re-plans ("next round" #6).

The graph engine hands each rank's per-phase op list ``(peer, row, is_send)`` to either RCCL
(``gadmm_rccl_exchange_rows``: ONE ncclGroupStart/End per phase, csrc/runtime/rccl_comm.cpp) or the
IPC device-copy transport (``ipc_xchg_kernel``: batches of up to MAX_BATCH ops, one wave per op, the
batches of a phase launched in order, csrc/kernels/ipc_xport.hip). Neither can be run with two real
GPUs here, so the properties they rely on are checked on the plans themselves:

* matching: for every phase and ordered rank pair (A, B), the rows A sends to B, in A's list order,
  equal the rows B receives from A, in B's list order (NCCL matches the k-th send with the k-th recv
  of a pair inside a group; the count is d on both sides);
* coverage: every cross-rank chain neighbour receives the row of every worker it reads in that phase
  (group_ADMM_closedForm.m:18-27, 62-70), exactly once, and nothing else crosses;
* no deadlock for the batched IPC transport: a simulation of its batch order (sends complete when
  their batch starts, a batch finishes when all of its recvs' sends have started) always drains.
"""
import os
import re

import numpy as np
import pytest

from gadmm_amd.parallel import topology as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _max_batch() -> int:
    src = open(os.path.join(ROOT, "csrc", "kernels", "ipc_xport.hip")).read()
    return int(re.search(r"constexpr int MAX_BATCH = (\d+);", src).group(1))


def _plans(path, placement):
    return [T.chain_plan(path, placement, r) for r in range(placement.nranks)]


def _check_matching(plans, phase):
    R = len(plans)
    for a in range(R):
        for b in range(R):
            if a == b:
                continue
            sends = [row for peer, row, s in getattr(plans[a], phase) if peer == b and s]
            recvs = [row for peer, row, s in getattr(plans[b], phase) if peer == a and not s]
            assert sends == recvs, (phase, a, b, sends, recvs)
    for r, p in enumerate(plans):
        assert all(peer != r for peer, _, _ in getattr(p, phase)), "self message"


def _check_coverage(path, placement, plans):
    n = len(path)
    owner = placement.owner
    want = {"xchg_head": set(), "xchg_tail": set()}
    for pos, w in enumerate(path):
        phase = "xchg_head" if pos % 2 == 0 else "xchg_tail"
        for u in (path[pos - 1] if pos > 0 else -1, path[pos + 1] if pos < n - 1 else -1):
            if u >= 0 and owner[u] != owner[w]:
                want[phase].add((int(owner[w]), int(owner[u]), int(w)))  # (from, to, row)
    for phase in want:
        got = [(r, peer, row) for r, p in enumerate(plans) for peer, row, s in getattr(p, phase) if s]
        assert len(got) == len(set(got)), "duplicate message"
        assert set(got) == want[phase], phase


def _ipc_drains(plans, phase, max_batch) -> bool:
    """Simulate the IPC transport: each rank runs its op list in batches of max_batch (all ops of a
    batch concurrently, batches in order). A recv completes once the matching send (same pair, same
    rank-in-pair order) has started; a send completes at once."""
    R = len(plans)
    ops = [getattr(p, phase) for p in plans]
    batches = [[ops[r][i:i + max_batch] for i in range(0, len(ops[r]), max_batch)] for r in range(R)]
    # index of the k-th send a->b in a's op list, and the batch it belongs to
    send_batch = {}
    for a in range(R):
        cnt = {}
        for i, (peer, row, s) in enumerate(ops[a]):
            if s:
                k = cnt.get(peer, 0)
                cnt[peer] = k + 1
                send_batch[(a, peer, k)] = i // max_batch
    cur = [0] * R  # batch each rank is executing
    recv_rank = []
    for b in range(R):
        cnt, lst = {}, []
        for i, (peer, row, s) in enumerate(ops[b]):
            if not s:
                k = cnt.get(peer, 0)
                cnt[peer] = k + 1
                lst.append((i // max_batch, peer, k))
        recv_rank.append(lst)
    for _ in range(sum(len(x) for x in batches) + 2):
        progressed = False
        for b in range(R):
            if cur[b] >= len(batches[b]):
                continue
            ready = all(cur[a] >= send_batch[(a, b, k)] for bi, a, k in recv_rank[b] if bi == cur[b])
            if ready:
                cur[b] += 1
                progressed = True
        if all(cur[r] >= len(batches[r]) for r in range(R)):
            return True
        if not progressed:
            return False
    return all(cur[r] >= len(batches[r]) for r in range(R))


def _check_all(path, placement, max_batch):
    plans = _plans(path, placement)
    for phase in ("xchg_head", "xchg_tail"):
        _check_matching(plans, phase)
        assert _ipc_drains(plans, phase, max_batch), phase
    _check_coverage(path, placement, plans)
    return plans


@pytest.mark.parametrize("ranks", [2, 4, 8])
@pytest.mark.parametrize("n", [8, 24, 50])
def test_static_chain_plans_match(ranks, n):
    placement = T.Placement.contiguous(n, ranks)
    plans = _check_all(list(range(n)), placement, _max_batch())
    # a contiguous identity chain crosses ranks only at the ranks - 1 segment boundaries: one row each
    # way per boundary per iteration (2 (ranks - 1) d 8 bytes: the payload formula of bench.py)
    sends = sum(p.send_rows() for p in plans)
    assert sends == 2 * (ranks - 1) == T.chain_message_count(list(range(n)), placement)


@pytest.mark.parametrize("ranks", [2, 4, 8])
@pytest.mark.parametrize("n,kind", [(24, "findPath2"), (50, "findPath"), (8, "findPath2")])
def test_dgadmm_replans_match(ranks, n, kind):
    """D-GADMM re-chains (the seeded findPath / findPath2 stream every rank draws identically): every
    epoch's plan (also used for the ghost-row refresh right after a re-chain, gadmm.py) matches."""
    placement = T.Placement.contiguous(n, ranks)
    sched = T.PathSchedule(n, list(range(n)), np.zeros(n - 1), 1, kind=kind, seed=2024 + ranks)
    P, _ = sched.prefetch_arrays(40)
    mb = _max_batch()
    for path in P:
        _check_all([int(v) for v in path], placement, mb)


def test_ipc_batch_simulation_detects_a_deadlock():
    """The drain simulation is not vacuous: with batches of one op, two ranks that each post their
    recv before their send to each other deadlock."""
    class P:  # two ranks, each: [recv from other, send to other] in one phase
        def __init__(self, other):
            self.xchg_head = [(other, 7, 0), (other, 3, 1)]
    plans = [P(1), P(0)]
    assert not _ipc_drains(plans, "xchg_head", 1)
    assert _ipc_drains(plans, "xchg_head", 2)


def test_random_placements_match():
    """Arbitrary (non-contiguous) worker -> rank maps on random chains: still matched and covered."""
    rng = np.random.default_rng(5)
    mb = _max_batch()
    for _ in range(30):
        n = int(rng.integers(4, 60))
        R = int(rng.integers(2, min(8, n) + 1))
        owner = np.concatenate([np.arange(R), rng.integers(0, R, n - R)])
        rng.shuffle(owner)
        placement = T.Placement(owner=owner.astype(np.int64), nranks=R)
        _check_all([int(v) for v in rng.permutation(n)], placement, mb)
