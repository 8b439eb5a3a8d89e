"""The node rules of a multi-GPU run: which device a rank takes, which planes it uses, and the lazily
built fabrics an entry-point session hands to the algorithms.

The reference runs every worker in one MATLAB process and moves theta by column reads
(group_ADMM_closedForm.m:18-27, 62-70); its entry scripts run GADMM sweeps, D-GADMM and the star
comparator back to back (LinearRegression_Synthetic.m:78-94, Dynamic_LinearRegression_Synthetic.m:142-173,
LinearRegression_gadmm_vs_admm.m:94-119). On an MI355X node the same scripts run as one process per
GPU, and every algorithm gets the engine the benchmark uses:

* control plane: gloo (rendezvous, agreement flags, IPC handle exchange) -- never a device collective;
* data plane (``parallel/dataplane.py``): the IPC device-copy transport by default, RCCL only when
  ``--fabric rccl`` asks for it on distinct GPUs (watchdog + collective fallback to IPC);
* device-initiated fabrics for the persistent kernels, built on demand and agreed by every rank:
  ``XgmiFabric`` (per-worker chain kernels, D-GADMM with a ring of table slots, the star kernel),
  and the data-local blocked kernel through ``engine/multigpu.DistributedChainSolver``.

Everything here that does not touch a device is a pure function, tested on the CPU
(tests/test_node_session.py).
"""
from __future__ import annotations

import os
import sys
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from .dataplane import choose_data_plane


def share_requested(env=None) -> bool:
    """Ranks rehearse on one GPU (device 0) -- the one-box rehearsal of the node path. Either name works:
    GADMM_SHARE_GPU=1 or the bench's GADMM_BENCH_SHARE_GPU=1."""
    env = os.environ if env is None else env
    return env.get("GADMM_SHARE_GPU") == "1" or env.get("GADMM_BENCH_SHARE_GPU") == "1"


def select_device_index(local_rank: int, share: bool, count: int) -> int:
    """The device ordinal a rank uses among the ``count`` devices its process can see. Sharing: device 0.
    Otherwise ``local_rank % count``: a node launched with every GPU visible gives rank r device r, and a
    launcher that sets a per-process HIP_VISIBLE_DEVICES (one visible device each) gives every rank its
    only device 0 -- never an ordinal the process cannot see."""
    if share:
        return 0
    if count <= 0:
        raise RuntimeError("no visible HIP device for local rank %d" % local_rank)
    return int(local_rank) % int(count)


def session_plan(device: str, world: int, fabric: str, share: bool) -> Dict[str, object]:
    """Pure rule of an entry session: ``control`` (None | 'gloo'), ``data_plane`` ('local' | 'gloo' |
    'ipc' | 'rccl') and ``xgmi`` (whether the persistent kernels' device-initiated fabrics are tried).
    CPU ranks exchange over gloo; GPU ranks follow ``choose_data_plane`` (IPC default, RCCL opt-in and
    never with ranks sharing a GPU) and try the xGMI fabrics unless a graph-engine plane was asked for."""
    if fabric not in ("auto", "xgmi", "ipc", "rccl"):
        raise ValueError("unknown fabric %r" % fabric)
    if world <= 1:
        return {"control": None, "data_plane": "local", "xgmi": False}
    if device == "cpu":
        return {"control": "gloo", "data_plane": "gloo", "xgmi": False}
    return {"control": "gloo", "data_plane": choose_data_plane(fabric, world, share),
            "xgmi": fabric in ("auto", "xgmi")}


def agree(flag: bool, world: int, group=None) -> bool:
    """True on every rank iff ``flag`` is True on every rank (gloo all-reduce)."""
    if world <= 1:
        return bool(flag)
    t = torch.tensor([0.0 if flag else 1.0], dtype=torch.float64)
    dist.all_reduce(t, group=group)
    return float(t.item()) == 0.0


class NodeFabrics:
    """The data plane and the xGMI fabrics of one GPU rank, built lazily (collectively: every rank asks
    for the same thing in the same order, which the entry bodies do -- they run the same script) and
    cached by shape. ``plan`` is ``session_plan``'s result."""

    def __init__(self, rank: int, world: int, device: torch.device, plan: Dict[str, object], fabric: str,
                 share: bool, timeout_s: float = 20.0, log=None):
        self.rank, self.world, self.device = rank, world, device
        self.plan, self.fabric_req, self.share, self.timeout_s = plan, fabric, share, float(timeout_s)
        self._planes: Dict[Tuple[int, int], object] = {}
        self._xgmi: Dict[Tuple[int, int, int], Optional[object]] = {}
        self.log = log or (lambda m: print(m, file=sys.stderr, flush=True))
        self.events = []  # (what, outcome) in build order: the session's record of its planes

    def data_plane(self, n_total: int, d: int, ring: int = 16):
        """The comm of the graph engines and the set-up / oracle collectives (IPC by default)."""
        key = (int(n_total), int(d))
        c = self._planes.get(key)
        if c is None:
            from .dataplane import make_data_plane
            c = make_data_plane(self.fabric_req, self.world, self.device, self.share, n_total, d, ring,
                                timeout_s=self.timeout_s, log=self.log if self.rank == 0 else (lambda m: None))
            self._planes[key] = c
            self.events.append(("data_plane", dict(getattr(c, "selection", {}) or {}, n_total=n_total, d=d)))
        return c

    def xgmi(self, n_total: int, d: int, table_slots: int = 1):
        """An ``XgmiFabric`` on every rank or None on every rank (agreed). None also when the session's
        plan does not try the xGMI fabrics (``--fabric ipc`` / ``rccl``)."""
        key = (int(n_total), int(d), int(table_slots))
        if key in self._xgmi:
            return self._xgmi[key]
        fab = None
        if self.plan.get("xgmi"):
            from .xgmi import XgmiFabric
            err = ""
            try:
                fab = XgmiFabric(n_total, d, 8, self.rank, self.world, self.device, table_slots=table_slots)
            except Exception as e:  # collective inside: every rank raises together
                err = "%s: %s" % (type(e).__name__, e)
            if not agree(fab is not None, self.world):
                if fab is not None:
                    fab.close()
                fab = None
                if self.rank == 0:
                    self.log("node: xgmi fabric (N=%d, d=%d, slots=%d) unavailable (%s); data plane instead"
                             % (n_total, d, table_slots, err or "another rank"))
        self._xgmi[key] = fab
        self.events.append(("xgmi", {"n_total": n_total, "d": d, "table_slots": table_slots,
                                     "built": fab is not None}))
        return fab

    def close(self):
        for f in self._xgmi.values():
            if f is not None:
                f.close()
        for c in self._planes.values():
            try:
                c.close()
            except Exception:
                pass
        self._xgmi, self._planes = {}, {}
