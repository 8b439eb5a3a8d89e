"""Device-copy transport for the graph-replayed chain engine (``csrc/kernels/ipc_xport.hip``).

The native chain engine exchanges boundary theta rows after every phase and reduces the per-worker
objective ring at every block end. ``RcclComm`` does that with ncclSend/ncclRecv/ncclAllReduce;
``IpcComm`` does it with two small kernels over IPC-mapped fine-grained mailboxes (one per rank):
a sender stores its row as tagged 16-byte granules straight into the receiver's mailbox, and the
receiver's kernel polls its own mailbox and copies the row into its theta table. Both are plain
kernels, so the exchange is captured in the engine's hipGraph like the RCCL calls are.

Why it exists:
* RCCL refuses two ranks on one device, so the engine's multi-rank code (chain plans, ghost rows,
  the objective ring and monitor, D-GADMM re-plans, logistic across ranks) could never run on a
  one-GPU box. With this transport it runs with 2..16 processes sharing one MI355X.
* On a node it is the DEFAULT data plane between graph-replayed phases and for the set-up / oracle
  collectives (parallel/dataplane.py): every MI355X pair is one xGMI hop, the stores go straight over
  the link, and every wait has a deadline in the kernel (RCCL is opt-in, behind a watchdog).

Handles travel over the gloo control plane, like ``parallel/xgmi.py``.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import native
from .comm import Comm
from .xgmi import _Buf


class IpcTransport:
    """This rank's mailbox + every peer's mapped mailbox + the native transport handle.
    Collective over ``group``; a failure on any rank raises on every rank."""

    def __init__(self, n_total: int, d: int, ring: int, rank: int, nranks: int, device: torch.device,
                 group=None, timeout_s: float = 20.0):
        self.lib = native.require()
        self.rank, self.nranks = rank, nranks
        self.n_total, self.d, self.ring = int(n_total), int(d), int(ring)
        self.opened: List[ctypes.c_void_p] = []
        self.box: Optional[_Buf] = None
        self.handle = None
        torch.cuda.set_device(device)
        err, mine = "", None
        try:
            self.box = _Buf(self.lib, int(self.lib.gadmm_ipc_box_bytes(self.n_total, self.d, self.ring, nranks)))
            mine = bytes(self.box.handle.raw)
        except Exception as e:  # pragma: no cover - box dependent
            err = "rank %d mailbox: %s" % (rank, e)
        allh = [None] * nranks
        dist.all_gather_object(allh, (mine, err), group=group)
        errs = [e for _, e in allh if e]
        ptrs: List[int] = []
        if not errs:
            try:
                for r, (h, _) in enumerate(allh):
                    if r == rank:
                        ptrs.append(self.box.ptr.value)
                    else:
                        p = ctypes.c_void_p()
                        native.check(self.lib.gadmm_xgmi_open(ctypes.create_string_buffer(h, 64), ctypes.byref(p)),
                                     "ipc open mailbox of rank %d" % r)
                        self.opened.append(p)
                        ptrs.append(p.value)
                arr = (ctypes.c_void_p * nranks)(*ptrs)
                self.handle = self.lib.gadmm_ipc_xport_create(rank, nranks, self.d, self.n_total, self.ring,
                                                              self.box.ptr, arr, float(timeout_s))
                if not self.handle:
                    native.check(-1, "ipc_xport_create")
            except Exception as e:
                errs.append(str(e))
        flag = torch.tensor([1.0 if errs else 0.0], dtype=torch.float64)
        dist.all_reduce(flag, group=group)
        if float(flag.item()) != 0.0:
            self.close()
            raise RuntimeError("ipc transport: %s" % ("; ".join(errs) or "failed on another rank"))

    def counters(self) -> dict:
        out = (ctypes.c_longlong * 4)()
        self.lib.gadmm_ipc_counters(self.handle, out)
        return {"payload_bytes": out[0], "wire_bytes": out[1], "msgs": out[2], "obj_wire_bytes": out[3]}

    def close(self):
        if self.handle:
            self.lib.gadmm_ipc_xport_destroy(self.handle)
            self.handle = None
        for p in self.opened:
            self.lib.gadmm_xgmi_close(p)
        self.opened = []
        if self.box is not None:
            self.box.free()
            self.box = None


class IpcComm(Comm):
    """Rank identity + the device-copy transport, for ``NativeChainEngine(comm=...)`` /
    ``chain_admm(..., comm=...)``. Control-plane helpers (barrier, max) go over gloo."""

    backend = "ipc"

    def __init__(self, n_total: int, d: int, ring: int, device: torch.device, group=None, timeout_s: float = 20.0):
        super().__init__()
        self.group = group
        self.control_group = group
        self.rank = dist.get_rank(group)
        self.nranks = dist.get_world_size(group)
        self.device = torch.device(device)
        self.transport = IpcTransport(n_total, d, ring, self.rank, self.nranks, self.device, group, timeout_s)
        self.handle = None          # no RCCL communicator
        self.xport = self.transport.handle

    def barrier(self):
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)

    # host-called point-to-point (the torch loops: DGD / dual averaging / chain ADMM fallbacks), staged
    # through host memory over the gloo control plane; the engines use ``exchange_rows_dev``
    def exchange_rows(self, table, ops):
        if not ops:
            return
        p2p, recv_bufs = [], []
        for peer, row, snd in ops:
            if snd:
                buf = table[row].detach().to("cpu").contiguous()
                p2p.append(dist.P2POp(dist.isend, buf, int(peer), self.group))
                self.stats.bytes_sent += buf.numel() * buf.element_size()
                self.stats.msgs_sent += 1
            else:
                buf = torch.empty(table[row].shape, dtype=table.dtype)
                recv_bufs.append((row, buf))
                p2p.append(dist.P2POp(dist.irecv, buf, int(peer), self.group))
                self.stats.bytes_recv += buf.numel() * buf.element_size()
        for r in dist.batch_isend_irecv(p2p):
            r.wait()
        for row, buf in recv_bufs:
            table[row].copy_(buf)

    def send_tensor(self, t, peer):
        h = t.detach().to("cpu").contiguous()
        dist.send(h, int(peer), group=self.group)
        self.stats.bytes_sent += h.numel() * h.element_size()
        self.stats.msgs_sent += 1

    def recv_tensor(self, t, peer):
        h = torch.empty(t.shape, dtype=t.dtype)
        dist.recv(h, int(peer), group=self.group)
        t.copy_(h)
        self.stats.bytes_recv += h.numel() * h.element_size()

    def _allreduce_max(self, t):
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t

    # device collectives on a stream (csrc/kernels/ipc_xport.hip: ipc_coll_kernel), sums in rank order;
    # every rank must issue the same sequence. ``ctl``: the caller's ChainCtl (done skips, timeouts set 4)
    KIND = {"reduce": 0, "broadcast": 1, "allreduce": 2}

    def device_collective(self, kind: str, t, root: int, ctl, stream) -> None:
        from ..ops import native
        k = self.KIND[kind]
        seq = self._seq = getattr(self, "_seq", 0) + 1
        native.check(self.transport.lib.gadmm_ipc_collective(self.xport, k, int(root), t.data_ptr(), t.data_ptr(),
                                                             int(t.numel()), seq & 0xffffffff, ctl.data_ptr(),
                                                             stream), "ipc_collective(%s)" % kind)
        R, me = self.nranks, self.rank
        sent = (R - 1) if k == 2 else (1 if (k == 0 and me != root) else (R - 1 if (k == 1 and me == root) else 0))
        self.stats.coll_bytes += sent * t.numel() * t.element_size()

    def exchange_rows_dev(self, table, ops, phase: int, ctl, stream) -> None:
        """Grouped row exchange on a stream (the chain engine's ``gadmm_ipc_exchange_rows``): ``ops`` =
        (peer, row, is_send) over ``table`` (n_total, d); tags from ``4 * ctl.iter + phase``, so every rank
        must issue the same exchanges per iteration. Stalled peers set ctl.done = 4."""
        from ..ops import native
        lib = self.transport.lib
        fn = lib.gadmm_ipc_exchange_rows
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                       ctypes.c_void_p, ctypes.c_void_p]
        arr = (native.XchgOp * len(ops))()
        for i, (peer, row, snd) in enumerate(ops):
            arr[i].peer, arr[i].row, arr[i].is_send, arr[i].count = int(peer), int(row), int(snd), 0
        d = int(table.shape[1])
        native.check(fn(self.xport, ctypes.cast(arr, ctypes.c_void_p), len(ops), table.data_ptr(), d, int(phase),
                        ctl.data_ptr(), stream), "ipc_exchange_rows")
        for peer, row, snd in ops:
            if snd:
                self.stats.bytes_sent += d * 8
                self.stats.msgs_sent += 1
            else:
                self.stats.bytes_recv += d * 8

    def new_epoch(self, stream) -> None:
        """Start a new solve on this transport: granules of earlier solves stop matching (every rank)."""
        from ..ops import native
        native.check(self.transport.lib.gadmm_ipc_new_epoch(self.xport, stream), "ipc_new_epoch")

    def _device_collective_sync(self, kind: str, t, root: int) -> bool:
        """A host-called collective on a CUDA f64 tensor through the device collective (chunks of the
        coll row, 2 d + 8 doubles; no host staging of e.g. an 800 MB Gram at d = 10k), synchronised and
        checked. False: not eligible (the caller uses the gloo control plane)."""
        step = 2 * self.transport.d + 8
        if not (t.is_cuda and t.dtype == torch.float64 and t.is_contiguous() and t.numel() >= 64):
            return False
        if kind != "allreduce" and t.numel() > 4 * step:
            # a reduce / broadcast is not a rendezvous for its pushing ranks: more chunks than the
            # transport's collective slots (8) could lap a slow reader -- the control plane instead
            return False
        from ..ops import native
        st = torch.cuda.current_stream(self.device).cuda_stream
        if getattr(self, "_ctl", None) is None:
            self._ctl = torch.zeros((8,), dtype=torch.int32, device=self.device)
        self._ctl.zero_()
        self.new_epoch(st)
        flat = t.view(-1)
        for c0 in range(0, flat.numel(), step):
            self.device_collective(kind, flat[c0:c0 + step], root, self._ctl, st)
        if int(self._ctl[1].item()) != 0:
            native.check(-1, "ipc %s: a peer did not arrive (done=%d)" % (kind, int(self._ctl[1].item())))
        return True

    def allreduce_sum(self, t):
        """Set-up / oracle all-reduce (the distributed CG's d-vector products): CUDA f64
        tensors by the device collective, anything else over the gloo control plane."""
        if self._device_collective_sync("allreduce", t, 0):
            return t
        h = t.detach().cpu()
        dist.all_reduce(h, group=self.group)
        t.copy_(h)
        self.stats.coll_bytes += t.numel() * t.element_size()
        return t

    def reduce_sum(self, t, root: int):
        """Reduce to ``root`` (the star comparator's upload, standared_ADMM.m:66-71)."""
        if self._device_collective_sync("reduce", t, root):
            return t
        h = t.detach().cpu()
        dist.reduce(h, dst=root, group=self.group)
        if self.rank == root:
            t.copy_(h)
        self.stats.coll_bytes += t.numel() * t.element_size()
        return t

    def broadcast(self, t, root: int):
        """Broadcast from ``root`` (the star hub's theta, standared_ADMM.m:86)."""
        if self._device_collective_sync("broadcast", t, root):
            return t
        h = t.detach().cpu()
        dist.broadcast(h, src=root, group=self.group)
        t.copy_(h)
        self.stats.coll_bytes += t.numel() * t.element_size()
        return t

    def close(self):
        self.transport.close()
        self.xport = None
