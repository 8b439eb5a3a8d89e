"""Fault injection for the communication layer ("failure detection / fault injection").

``FaultyComm`` wraps any ``Comm`` and perturbs row exchanges according to a ``FaultPlan``:
* ``drop``:    the message is not delivered (the receiver keeps its stale row);
* ``corrupt``: the receiver's copy gets a one-ulp perturbation of one element;
* ``delay``:   the receiver gets the row of the PREVIOUS delivery from that sender (a late message).
Faults are keyed by the exchange call index on this rank (every phase is one call), so a test can
place a fault at a chosen iteration/phase deterministically. The exchange checker
(``debug.race``) must flag every injected fault at the phase it happens.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Set

import torch

from ..parallel.comm import Comm


@dataclass
class FaultPlan:
    drop: Set[int] = field(default_factory=set)      # exchange-call indices whose receives are dropped
    corrupt: Set[int] = field(default_factory=set)
    delay: Set[int] = field(default_factory=set)


class FaultyComm(Comm):
    def __init__(self, base: Comm, plan: FaultPlan):
        super().__init__()
        self.base = base
        self.plan = plan
        self.rank, self.nranks, self.backend = base.rank, base.nranks, "faulty-" + base.backend
        self.stats = base.stats
        self.calls = 0
        self.injected = 0
        self._last: Dict[int, torch.Tensor] = {}

    def exchange_rows(self, table, ops):
        k = self.calls
        self.calls += 1
        recv_rows = [row for _, row, snd in ops if not snd]
        before = {r: table[r].clone() for r in recv_rows}
        self.base.exchange_rows(table, ops)
        for r in recv_rows:
            if k in self.plan.drop:
                table[r].copy_(before[r])
                self.injected += 1
            elif k in self.plan.corrupt:
                v = table[r, 0].item()
                table[r, 0] = torch.nextafter(torch.tensor(v, dtype=torch.float64),
                                              torch.tensor(float("inf"), dtype=torch.float64)).item()
                self.injected += 1
            elif k in self.plan.delay and r in self._last:
                table[r].copy_(self._last[r])
                self.injected += 1
            self._last[r] = table[r].clone()

    # everything else is delegated unchanged
    def send_tensor(self, t, peer):
        return self.base.send_tensor(t, peer)

    def recv_tensor(self, t, peer):
        return self.base.recv_tensor(t, peer)

    def allreduce_sum(self, t):
        return self.base.allreduce_sum(t)

    def reduce_sum(self, t, root):
        return self.base.reduce_sum(t, root)

    def broadcast(self, t, root):
        return self.base.broadcast(t, root)

    def barrier(self):
        return self.base.barrier()

    def _allreduce_max(self, t):
        return self.base._allreduce_max(t)
