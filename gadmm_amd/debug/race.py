"""Exchange race checker for the chain schedule ("race detection").

The correctness invariant of GADMM on real ranks is the head/tail phase order: a tail must use its
heads' theta of THIS iteration and a head its tails' theta of the previous one. In this framework
that is enforced by stream/RCCL ordering (graph path) or by tagged granules (persistent kernels).
The checker verifies it at run time: after every exchange, each rank publishes a checksum of every
row it OWNS (an all-reduce of an N-vector with one contributor per entry, so exact), and every rank
compares the checksum of each ghost row it holds with the owner's. A stale, torn or misrouted
message shows up as a mismatch with the iteration, the row, its owner and the phase.

Cost: one 2N-double all-reduce (plus a scalar) per phase, counted as monitor bytes. Enabled with
``chain_admm(..., check_exchange=True)`` or ``GADMM_CHECK_EXCHANGE=1``.
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import torch


class RaceError(RuntimeError):
    pass


def row_checksums(theta: torch.Tensor, rows: Iterable[int]) -> torch.Tensor:
    """Bit-exact fingerprint of each row: the float64 bit patterns hashed with odd per-element
    multipliers (int64, wrapping), kept as two 31-bit halves so each fits a float64 exactly and
    survives the all-reduce (one contributor per entry). Any single-bit change of any element
    changes the hash. Returns (len(rows), 2) float64."""
    rows = list(rows)
    d = theta.shape[1]
    if not rows:
        return torch.zeros((0, 2), dtype=torch.float64, device=theta.device)
    sub = theta.index_select(0, torch.tensor(rows, dtype=torch.long, device=theta.device)).contiguous()
    bits = sub.view(torch.int64)
    k = torch.arange(d, dtype=torch.int64, device=theta.device) * 2654435761 + 40503  # odd multipliers
    k = k | 1
    h = (bits * k).sum(-1)
    lo = (h & 0x7FFFFFFF).to(torch.float64)
    hi = ((h >> 31) & 0x7FFFFFFF).to(torch.float64)
    return torch.stack([lo, hi], dim=-1)


class ExchangeChecker:
    def __init__(self, comm, local_ids: List[int], n_total: int):
        self.comm = comm
        self.local = [int(w) for w in local_ids]
        self.n = int(n_total)
        self.checks = 0

    def verify(self, theta: torch.Tensor, ghost_rows: Iterable[int], it: int, phase: str,
               owner: Optional[List[int]] = None) -> None:
        ghosts = sorted(set(int(r) for r in ghost_rows) - set(self.local))
        full = torch.zeros((self.n, 2), dtype=torch.float64, device=theta.device)
        full[torch.tensor(self.local, dtype=torch.long, device=theta.device)] = row_checksums(theta, self.local)
        if self.comm.nranks > 1:
            self.comm.allreduce_sum(full)
            self.comm.stats.coll_bytes -= full.numel() * 8      # debug traffic is monitoring, not algorithm
            self.comm.stats.monitor_bytes += full.numel() * 8
        self.checks += 1
        bad = []
        if ghosts:
            mine = row_checksums(theta, ghosts)
            ref = full.index_select(0, torch.tensor(ghosts, dtype=torch.long, device=theta.device))
            bad = (mine != ref).any(-1).nonzero().flatten().tolist()
        # every rank raises together (a lone raise would leave the others blocked in a collective)
        nbad = float(len(bad))
        if self.comm.nranks > 1:
            nbad_all = self.comm.allreduce_max_scalar(nbad)
        else:
            nbad_all = nbad
        if nbad_all and not bad:
            raise RaceError("exchange check failed at iteration %d (%s phase) on another rank" % (it, phase))
        if bad:
            r = ghosts[bad[0]]
            raise RaceError("exchange check failed at iteration %d (%s phase): rank %d holds a stale/corrupt copy "
                            "of row %d%s (%d row(s) differ)" % (it, phase, self.comm.rank, r,
                                                                " owned by rank %d" % owner[r] if owner else "",
                                                                len(bad)))
