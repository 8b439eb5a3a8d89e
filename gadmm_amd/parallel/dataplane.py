"""Which data plane a multi-rank run uses between graph-replayed phases and for its collectives.

The reference exchanges theta only between chain neighbours (group_ADMM_closedForm.m:18-27, 62-70) and
its star comparator reduces to / broadcasts from a hub (standared_ADMM.m:57-88). On one node this
framework has three ways to move those bytes:

* ``xgmi``  -- device-initiated stores between persistent kernels (parallel/xgmi.py); chosen by the
  engines themselves where a persistent kernel exists;
* ``ipc``   -- the device-copy transport (parallel/ipc.py): tagged-granule stores into IPC-mapped
  mailboxes, every wait bounded by a deadline in the kernel. **The default** everywhere a data plane is
  needed (``--fabric auto``): it is the path rehearsed with 2..16 ranks;
* ``rccl``  -- the native RCCL communicator (parallel/comm.py: RcclComm). Opt-in (``--fabric rccl``) and
  a tournament candidate; built only when a body actually needs it, non-blocking with a watchdog
  (a deadline aborts the communicator and every rank falls back to ``ipc`` together). RCCL refuses two
  ranks on one device, so ranks sharing a GPU (the one-box rehearsal) never get it.

``choose_data_plane`` is the pure selection rule (CPU-tested); ``make_data_plane`` builds the comm
collectively, with the RCCL -> IPC fallback agreed over the gloo control plane, and -- if the IPC
transport itself fails on any rank -- a last-resort host-staged gloo comm (``HostStagedComm``) on which
the engines run their torch loops.
"""
from __future__ import annotations

import sys
from typing import Optional

import torch
import torch.distributed as dist


def choose_data_plane(fabric: str, world: int, share: bool) -> str:
    """'local' (one rank), 'rccl' (explicitly requested, ranks on distinct GPUs) or 'ipc' (everything
    else: the node default and the only option when ranks share a GPU)."""
    if world <= 1:
        return "local"
    if fabric == "rccl" and not share:
        return "rccl"
    return "ipc"


def _agree(flag: bool, world: int, group=None) -> bool:
    if world <= 1:
        return bool(flag)
    t = torch.tensor([0.0 if flag else 1.0], dtype=torch.float64)
    dist.all_reduce(t, group=group)
    return float(t.item()) == 0.0


def make_data_plane(fabric: str, world: int, device, share: bool, n_total: int, d: int, ring: int = 16,
                    timeout_s: float = 20.0, group=None, log=None):
    """Collective. The comm of ``choose_data_plane``; an RCCL communicator that fails to come up on any
    rank (set-up error or its watchdog deadline) makes every rank take the IPC transport instead. The
    returned comm carries ``selection`` = (requested fabric, chosen, reason)."""
    from .comm import LocalComm

    kind = choose_data_plane(fabric, world, share)
    if kind == "local":
        c = LocalComm()
        c.selection = {"requested": fabric, "data_plane": "local", "reason": "one rank"}
        return c
    reason = "node default (rehearsed IPC transport)" if fabric in ("auto", "ipc", "xgmi") else \
        ("ranks share one GPU: RCCL refuses it" if share else "")
    if kind == "rccl":
        from .comm import RcclComm
        comm, err = None, ""
        try:
            # set-up deadline: 30 s at least (topology discovery on an 8-GPU node takes seconds), the
            # per-operation watchdog: the caller's deadline
            comm = RcclComm(device, control_group=group, timeout_s=max(float(timeout_s), 1.0),
                            init_timeout_s=max(30.0, float(timeout_s)))
        except Exception as e:  # set-up error or the non-blocking set-up's deadline
            err = "%s: %s" % (type(e).__name__, e)
        if _agree(comm is not None, world, group):
            comm.selection = {"requested": fabric, "data_plane": "rccl", "reason": "requested"}
            return comm
        if comm is not None:
            comm.abort()  # a peer failed: never a collective destroy against it
            comm.close()
        reason = "RCCL unavailable on some rank (%s); IPC transport" % (err or "another rank")
        (log or (lambda m: print(m, file=sys.stderr, flush=True)))("data plane: " + reason)
    from .ipc import IpcComm
    c, err = None, ""
    try:
        c = IpcComm(n_total, d, ring, device, group=group, timeout_s=timeout_s)
    except Exception as e:  # collective inside: a failure anywhere raises on every rank
        err = "%s: %s" % (type(e).__name__, e)
    if _agree(c is not None, world, group):
        c.selection = {"requested": fabric, "data_plane": "ipc", "reason": reason}
        return c
    if c is not None:
        c.close()
    # last resort: the gloo control plane with device tensors staged through host memory -- slow, but
    # every algorithm still runs (the engines take their torch loops)
    from .comm import HostStagedComm
    (log or (lambda m: print(m, file=sys.stderr, flush=True)))(
        "data plane: IPC transport unavailable (%s); host-staged gloo" % (err or "another rank"))
    h = HostStagedComm(group)
    h.selection = {"requested": fabric, "data_plane": "host-gloo",
                   "reason": "IPC transport unavailable on some rank (%s)" % (err or "another rank")}
    return h
