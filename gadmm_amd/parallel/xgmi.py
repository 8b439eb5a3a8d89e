"""xGMI-direct fabric for the persistent chain kernel on several MI355X (one process per GPU).

The RCCL path (``RcclComm`` + graph-replayed phase kernels) pays a collective/p2p launch and a kernel
boundary per phase. At the reference problem sizes a phase is ~1 us of arithmetic, so on a single
node the framework can instead keep one persistent kernel per GPU and move the boundary theta
*device-initiated*: every GPU allocates fine-grained (uncached) granule buffers, exports them by IPC
(dmabuf; HSA_ENABLE_IPC_MODE_LEGACY=0), and maps its chain neighbours' buffers; a worker's kernel
writes its fresh theta granules straight into the neighbour GPU's table over xGMI (every pair of
MI355X in a node is one xGMI hop), objective granules into rank 0's monitor ring, and rank 0's
monitor writes each stop decision into every rank's ring. The hand-off protocol is the same tagged
granule protocol as on one GPU (tags salted per solve), so correctness does not depend on timing;
every spin is bounded, and a stalled peer surfaces as ``done == 4`` (the caller falls back to RCCL).

Handles travel over the gloo control plane (``dist.all_gather_object``).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..ops import native


class _Buf:
    def __init__(self, lib, nbytes: int):
        self.lib = lib
        self.ptr = ctypes.c_void_p()
        self.handle = ctypes.create_string_buffer(64)
        native.check(lib.gadmm_xgmi_alloc(nbytes, ctypes.byref(self.ptr), self.handle), "xgmi_alloc")
        self.nbytes = nbytes

    def free(self):
        if self.ptr:
            self.lib.gadmm_xgmi_free(self.ptr)
            self.ptr = ctypes.c_void_p()


class XgmiFabric:
    """Per-rank granule buffers + the peers' mapped buffers.

    theta table: (table_slots, N, d) x 16-B granules on every rank (one slot for static chains; a ring
    of iteration slots for D-GADMM, whose hand-offs change peers at every re-chain); objective ring:
    (ring, N) x 16 B (read on the monitor rank 0); decision ring: ring x 8 B on every rank."""

    def __init__(self, n_total: int, d: int, ring: int, rank: int, nranks: int, device: torch.device,
                 group=None, peers_needed: Optional[List[int]] = None, table_slots: int = 1):
        """Collective over ``group``: every rank must call it. Failures on any rank are raised on
        every rank (so callers can fall back together). ``peers_needed``: ranks whose theta table
        this rank writes into (default: all; D-GADMM needs all, any pair can become neighbours)."""
        self.lib = native.require()
        self.rank, self.nranks, self.device = rank, nranks, device
        self.n, self.d, self.ring = n_total, d, ring
        self.table_slots = int(table_slots)
        self.opened: Dict[tuple, ctypes.c_void_p] = {}
        self.thg = self.objg = self.decg = None
        torch.cuda.set_device(device)
        mine = None
        err = ""
        try:
            self.thg = _Buf(self.lib, self.table_slots * n_total * d * 16)
            self.objg = _Buf(self.lib, ring * n_total * 16)
            self.decg = _Buf(self.lib, ring * 8)
            mine = (bytes(self.thg.handle.raw), bytes(self.objg.handle.raw), bytes(self.decg.handle.raw))
        except Exception as e:
            err = "rank %d alloc: %s" % (rank, e)
        allh = [None] * nranks
        dist.all_gather_object(allh, (mine, err, device_identity()), group=group)
        errs = [e for _, e, _ in allh if e]
        if errs:
            self.close()
            raise RuntimeError("xgmi fabric: " + "; ".join(errs))
        devs = [dv for _, _, dv in allh]
        allh = [h for h, _, _ in allh]
        ok = True
        try:
            need_thg = set(peers_needed if peers_needed is not None else [r for r in range(nranks) if r != rank])
            touch = set(need_thg) | ({0} if rank != 0 else set(range(nranks)))  # + the monitor's / decision rings
            why = preflight(torch.cuda.current_device(), {r: devs[r] for r in touch if r != rank})
            if why:
                raise RuntimeError("peer access pre-flight: " + why)
            self.thg_peer: Dict[int, int] = {}
            for r in need_thg:
                self.thg_peer[r] = self._open(allh[r][0], ("thg", r))
            self.objg_mon = self.objg.ptr.value if rank == 0 else self._open(allh[0][1], ("objg", 0))
            self.dec_all: List[int] = []
            if rank == 0:
                for r in range(nranks):
                    self.dec_all.append(self.decg.ptr.value if r == 0 else self._open(allh[r][2], ("decg", r)))
        except Exception as e:
            ok = False
            err = str(e)
        flag = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64)
        dist.all_reduce(flag, group=group)
        if float(flag.item()) != 0.0:
            self.close()
            raise RuntimeError("xgmi fabric: peer mapping failed on some rank (%s)" % (err or "remote"))
        self.epoch = 0

    def _open(self, h: bytes, key) -> int:
        p = ctypes.c_void_p()
        native.check(self.lib.gadmm_xgmi_open(ctypes.create_string_buffer(h, 64), ctypes.byref(p)),
                     "xgmi_open %s" % (key,))
        self.opened[key] = p
        return p.value

    def table_ptrs(self) -> List[int]:
        """Every rank's theta table (own included) by rank: the D-GADMM push targets."""
        if len(self.thg_peer) != self.nranks - 1:
            raise RuntimeError("fabric was built for a subset of peers; D-GADMM needs peers_needed=None")
        return [self.thg.ptr.value if r == self.rank else self.thg_peer[r] for r in range(self.nranks)]

    def next_epoch(self) -> int:
        self.epoch = (self.epoch + 1) % 4095 + 1
        return self.epoch

    def close(self):
        for p in self.opened.values():
            self.lib.gadmm_xgmi_close(p)
        self.opened = {}
        for b in (self.thg, self.objg, self.decg):
            if b is not None:
                b.free()
        self.thg = self.objg = self.decg = None


def peer_access_ok(nranks: int) -> bool:
    """Every pair of the first ``nranks`` devices can access each other (hipDeviceCanAccessPeer)."""
    lib = native.require()
    n = torch.cuda.device_count()
    if n < 2:
        return True
    return all(lib.gadmm_device_can_access_peer(i, j) == 1 for i in range(min(n, nranks)) for j in range(min(n, nranks))
               if i != j)


_IDENT: Dict[int, str] = {}


def device_identity(index: Optional[int] = None) -> str:
    """A physical identity of a visible device: PCI domain:bus:device plus the UUID when the runtime
    reports one. Ranks compare THIS, never the logical ordinal: ranks launched with a per-process
    HIP_VISIBLE_DEVICES all see their GPU as device 0, while ranks sharing one GPU (the one-box
    rehearsal) see the same PCI address."""
    i = torch.cuda.current_device() if index is None else int(index)
    if i not in _IDENT:
        p = torch.cuda.get_device_properties(i)
        uuid = str(getattr(p, "uuid", "") or "")
        _IDENT[i] = "%04x:%02x:%02x|%s" % (int(getattr(p, "pci_domain_id", 0)), int(getattr(p, "pci_bus_id", 0)),
                                           int(getattr(p, "pci_device_id", 0)), uuid)
    return _IDENT[i]


def same_physical_device(idents) -> bool:
    """All the identities (``device_identity``) name one GPU."""
    return len({str(x) for x in idents}) == 1


def preflight(my_dev: int, peer_devs: Dict[int, str]) -> str:
    """Pre-flight of the IPC / xGMI mappings a rank is about to open: every peer rank's device (by its
    ``device_identity``) must be reachable from this rank's device (hipDeviceCanAccessPeer) before
    ``hipIpcOpenMemHandle`` (which would otherwise fail -- or worse, map -- on a box without the link).
    A peer on this rank's own physical device (the one-GPU rehearsal) needs no peer access. A peer
    device this process cannot see (per-process HIP_VISIBLE_DEVICES) cannot be checked here: it is
    allowed, and the IPC open that follows is the check (its failure falls back collectively).
    Returns '' or the reason."""
    lib = native.require()
    mine = device_identity(my_dev)
    visible = {device_identity(i): i for i in range(torch.cuda.device_count())}
    bad = []
    for r, ident in sorted(peer_devs.items()):
        if isinstance(ident, int):  # a bare ordinal (old callers): resolve it on this process
            ident = device_identity(ident)
        if ident == mine:
            continue
        j = visible.get(ident)
        if j is None:
            continue
        if int(lib.gadmm_device_can_access_peer(my_dev, j)) != 1:
            bad.append("rank %d (device %s)" % (r, ident.split("|")[0]))
    return ("device %s cannot access %s" % (mine.split("|")[0], ", ".join(bad))) if bad else ""
