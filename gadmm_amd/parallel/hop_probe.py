"""One-way hop latency between chain-neighbour GPUs (``ipc_hop_probe_kernel``, csrc/kernels/ipc_xport.hip).

The multi-GPU headline exchanges theta across every rank boundary twice per iteration
(group_ADMM_closedForm.m:18-27, 62-70), so its speed is set by the one-way latency of a tagged-granule
row store over xGMI followed by the neighbour's poll. ``hop_probe`` measures exactly that, between
each pair of chain-adjacent ranks (r, r + 1), with the persistent kernels' row format: one wave per
side, system-scope write-through stores into the peer's IPC-mapped fine-grained row, polls of the own
row, ``n`` timed round trips after one untimed round. Even boundaries run together, then odd ones
(a rank is in at most one pair at a time). With ranks sharing one GPU (the one-box rehearsal) it
measures the cross-process same-device hop instead; the caller labels it.

Collective over the default (gloo) group; never raises on one rank only. Returns
``{"hop_us": [per boundary], "ok": bool, "same_device": bool}`` on every rank (``None`` entries where
a probe timed out).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..ops import native
from .xgmi import _Buf, device_identity, preflight, same_physical_device


def hop_probe(rank: int, world: int, device: torch.device, n: int = 2000, timeout_s: float = 5.0,
              group=None, salt: int = 1) -> Dict[str, List[Optional[float]]]:
    if world < 2:
        return {"hop_us": [], "ok": True}
    lib = native.require()
    torch.cuda.set_device(device)
    buf, err = None, ""
    try:
        buf = _Buf(lib, 64 * 16)
        mine_h = bytes(buf.handle.raw)
    except Exception as e:  # pragma: no cover - box dependent
        mine_h, err = None, str(e)
    dev = torch.cuda.current_device()
    ident = device_identity(dev)
    allh = [None] * world
    dist.all_gather_object(allh, (mine_h, ident, err), group=group)
    opened = {}
    try:
        if any(e for _, _, e in allh):  # the same on every rank
            return {"hop_us": [None] * (world - 1), "ok": False,
                    "error": "; ".join(e for _, _, e in allh if e)}
        nbrs = [q for q in (rank - 1, rank + 1) if 0 <= q < world]
        why = preflight(dev, {q: allh[q][1] for q in nbrs})
        if not why:
            try:
                for q in nbrs:
                    p = ctypes.c_void_p()
                    native.check(lib.gadmm_xgmi_open(ctypes.create_string_buffer(allh[q][0], 64),
                                                     ctypes.byref(p)), "hop probe: open rank %d" % q)
                    opened[q] = p
            except Exception as e:  # pragma: no cover - box dependent
                why = str(e)
        flag = torch.tensor([1.0 if why else 0.0], dtype=torch.float64)
        dist.all_reduce(flag, group=group)  # every rank probes, or none does
        if float(flag.item()) != 0.0:
            return {"hop_us": [None] * (world - 1), "ok": False,
                    "error": why or "peer mapping failed on another rank"}
        mine: List[Optional[float]] = [None] * (world - 1)  # this rank's measurements (as initiator)
        out = (ctypes.c_ulonglong * 2)()
        for parity in (0, 1):
            role = None
            if rank % 2 == parity and rank + 1 < world:
                role = (1, rank + 1)          # initiator of boundary (rank, rank + 1)
            elif (rank - 1) % 2 == parity and rank >= 1:
                role = (0, rank - 1)          # responder of boundary (rank - 1, rank)
            dist.barrier(group=group)
            if role is None:
                continue
            init, q = role
            rc = lib.gadmm_ipc_hop_probe(buf.ptr, opened[q], init, int(n), (salt * 2 + parity) & 0xfff,
                                         float(timeout_s), out)
            if rc == 0 and init and out[0] > 0:
                mine[rank] = out[0] * 10.0 / (2.0 * n) / 1e3  # 100 MHz ticks -> us per one-way hop
        t = torch.tensor([(-1.0 if v is None else v) for v in mine], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        hops = [None if v < 0 else round(float(v), 4) for v in t.tolist()]
        # every rank on one PHYSICAL device (PCI address / UUID, not the ordinal -- per-process
        # HIP_VISIBLE_DEVICES makes every rank's GPU device 0): the one-GPU rehearsal
        return {"hop_us": hops, "ok": all(h is not None for h in hops),
                "same_device": same_physical_device(h[1] for h in allh),
                "devices": [h[1].split("|")[0] for h in allh]}
    finally:
        for p in opened.values():
            lib.gadmm_xgmi_close(p)
        dist.barrier(group=group)  # nobody frees its row while a peer still maps it
        if buf is not None:
            buf.free()
