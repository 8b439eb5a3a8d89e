"""Communication backends behind one small interface (SURVEY.md §2.6 call-site inventory).

* ``LocalComm``   — one rank owns every logical worker; neighbour "messages" are reads of the local
  theta table (the analogue of the reference's column reads, ``out(:,ii-1)``). No fabric bytes; the
  per-worker ("logical") traffic is reported from the reference communication units
  (``RunResult.summary()['logical_bytes']``).
* ``TorchDistComm`` — ``torch.distributed`` point-to-point + collectives. With the ``gloo`` backend
  this is the CPU plumbing config of BASELINE.json (configs[0]); with ``nccl`` (= RCCL on ROCm) it
  runs on MI355X ranks.
* ``RcclComm``    — the native RCCL communicator of ``libgadmm_native`` (one ``ncclComm_t`` per
  process, ops enqueued on a HIP stream, capturable into the engine's hipGraph). Fast path on GPU.

All exchange APIs move *rows of a row-major table* (theta or Z, shape (N_total, d)) so the same plan
(``topology.chain_plan``) drives every backend.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from ..utils.env import getenv

Op = Tuple[int, int, int]  # (peer, row, is_send)


class CommStats:
    """Per-rank byte counters. ``bytes_sent``: point-to-point payload; ``coll_bytes``: payload this
    rank contributed to collectives that belong to the algorithm (GD all-reduce, star reduce/bcast);
    ``monitor_bytes``: collectives of the stopping monitor only (global objective), which the
    reference computes for free in shared memory and a deployment would run every K iterations."""

    FIELDS = ("bytes_sent", "bytes_recv", "msgs_sent", "coll_bytes", "monitor_bytes")

    def __init__(self):
        for f in self.FIELDS:
            setattr(self, f, 0)

    def as_dict(self):
        return {f: getattr(self, f) for f in self.FIELDS}

    def snapshot(self):
        return self.as_dict()

    def delta(self, snap):
        return {f: getattr(self, f) - snap.get(f, 0) for f in self.FIELDS}


class Comm:
    rank: int = 0
    nranks: int = 1
    backend: str = "base"

    def __init__(self):
        self.stats = CommStats()

    # point to point on table rows
    def exchange_rows(self, table: torch.Tensor, ops: Sequence[Op]) -> None:
        raise NotImplementedError

    def send_tensor(self, t: torch.Tensor, peer: int) -> None:
        raise NotImplementedError

    def recv_tensor(self, t: torch.Tensor, peer: int) -> None:
        raise NotImplementedError

    # collectives
    def allreduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def reduce_sum(self, t: torch.Tensor, root: int) -> torch.Tensor:
        raise NotImplementedError

    def broadcast(self, t: torch.Tensor, root: int) -> torch.Tensor:
        raise NotImplementedError

    def barrier(self) -> None:
        pass

    def allreduce_max_scalar(self, v: float) -> float:
        t = torch.tensor([float(v)], dtype=torch.float64)
        return float(self._allreduce_max(t).item())

    def _allreduce_max(self, t):
        return t

    def close(self) -> None:
        pass


class RankInfo(Comm):
    """Rank identity without a data-plane communicator (the xGMI fabric moves the data)."""

    backend = "none"

    def __init__(self, rank: int, nranks: int):
        super().__init__()
        self.rank, self.nranks = rank, nranks
        self.handle = None


class LocalComm(Comm):
    backend = "local"

    def __init__(self):
        super().__init__()
        self.rank, self.nranks = 0, 1

    def exchange_rows(self, table, ops):
        if ops:
            raise RuntimeError("LocalComm cannot exchange with peers")

    def send_tensor(self, t, peer):
        raise RuntimeError("LocalComm has no peers")

    recv_tensor = send_tensor

    def allreduce_sum(self, t):
        return t

    def reduce_sum(self, t, root):
        return t

    def broadcast(self, t, root):
        return t


class TorchDistComm(Comm):
    """torch.distributed backend (gloo on CPU, nccl/RCCL on GPU)."""

    def __init__(self, group=None):
        super().__init__()
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised")
        self.group = group
        self.rank = dist.get_rank(group)
        self.nranks = dist.get_world_size(group)
        self.backend = "torch-" + str(dist.get_backend(group))

    def exchange_rows(self, table, ops):
        if not ops:
            return
        p2p = []
        recv_bufs = []
        for peer, row, snd in ops:
            if snd:
                buf = table[row].contiguous()
                p2p.append(dist.P2POp(dist.isend, buf, peer, self.group))
                self.stats.bytes_sent += buf.numel() * buf.element_size()
                self.stats.msgs_sent += 1
            else:
                buf = torch.empty_like(table[row])
                recv_bufs.append((row, buf))
                p2p.append(dist.P2POp(dist.irecv, buf, peer, self.group))
                self.stats.bytes_recv += buf.numel() * buf.element_size()
        for r in dist.batch_isend_irecv(p2p):
            r.wait()
        for row, buf in recv_bufs:
            table[row].copy_(buf)

    def send_tensor(self, t, peer):
        t = t.contiguous()
        dist.send(t, peer, group=self.group)
        self.stats.bytes_sent += t.numel() * t.element_size()
        self.stats.msgs_sent += 1

    def recv_tensor(self, t, peer):
        buf = torch.empty_like(t)
        dist.recv(buf, peer, group=self.group)
        t.copy_(buf)
        self.stats.bytes_recv += t.numel() * t.element_size()

    def allreduce_sum(self, t):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        self.stats.coll_bytes += t.numel() * t.element_size()
        return t

    def reduce_sum(self, t, root):
        dist.reduce(t, dst=root, op=dist.ReduceOp.SUM, group=self.group)
        self.stats.coll_bytes += t.numel() * t.element_size()
        return t

    def broadcast(self, t, root):
        dist.broadcast(t, src=root, group=self.group)
        self.stats.coll_bytes += t.numel() * t.element_size()
        return t

    def barrier(self):
        dist.barrier(group=self.group)

    def _allreduce_max(self, t):
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t


class HostStagedComm(TorchDistComm):
    """The last-resort data plane of a GPU run: torch.distributed over the gloo control plane, device
    tensors staged through host memory. Used only when neither the IPC transport nor RCCL comes up on
    every rank (parallel/dataplane.py); the engines then run the torch loops (slow, but a result)."""

    def __init__(self, group=None):
        super().__init__(group)
        self.backend = "host-gloo"
        self.control_group = group

    @staticmethod
    def _host(t):
        return t.detach().to("cpu").contiguous()

    def exchange_rows(self, table, ops):
        if not ops:
            return
        p2p, recv_bufs = [], []
        for peer, row, snd in ops:
            if snd:
                buf = self._host(table[row])
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
        h = self._host(t)
        dist.send(h, int(peer), group=self.group)
        self.stats.bytes_sent += h.numel() * h.element_size()
        self.stats.msgs_sent += 1

    def recv_tensor(self, t, peer):
        h = torch.empty(t.shape, dtype=t.dtype)
        dist.recv(h, int(peer), group=self.group)
        t.copy_(h)
        self.stats.bytes_recv += h.numel() * h.element_size()

    def allreduce_sum(self, t):
        h = self._host(t)
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
        t.copy_(h)
        self.stats.coll_bytes += t.numel() * t.element_size()
        return t

    def reduce_sum(self, t, root):
        h = self._host(t)
        dist.reduce(h, dst=root, op=dist.ReduceOp.SUM, group=self.group)
        if self.rank == root:
            t.copy_(h)
        self.stats.coll_bytes += t.numel() * t.element_size()
        return t

    def broadcast(self, t, root):
        h = self._host(t)
        dist.broadcast(h, src=root, group=self.group)
        t.copy_(h)
        self.stats.coll_bytes += t.numel() * t.element_size()
        return t


class RcclComm(Comm):
    """Native RCCL communicator (libgadmm_native). The unique id travels over an existing
    torch.distributed group (the gloo control plane).

    Watchdog (csrc/runtime/rccl_comm.cpp): the communicator is non-blocking, its set-up and every
    enqueue are bounded by ``timeout_s``, and host waits on RCCL work go through ``wait`` (or the chain
    engine's bounded waits). A deadline that passes aborts the communicator and raises
    ``native.RcclDead``; callers fall back to the IPC transport together (``parallel/dataplane.py``).
    Host-called collectives (set-up, oracles, the star comparator) wait after every call unless they
    run inside ``with comm.batched():`` (an engine loop that waits once per block)."""

    backend = "rccl"

    def __init__(self, device: torch.device, control_group=None, timeout_s: float = 60.0,
                 init_timeout_s: float = 120.0):
        super().__init__()
        from ..ops import native

        self.lib = native.require()
        self.native = native
        self.rank = dist.get_rank(control_group)
        self.nranks = dist.get_world_size(control_group)
        self.device = torch.device(device)
        self.timeout_s = float(timeout_s)
        self._batched = 0
        idbuf = ctypes.create_string_buffer(128)
        if self.rank == 0:
            native.check(self.lib.gadmm_rccl_unique_id(idbuf), "rccl_unique_id")
        obj = [bytes(idbuf.raw)]
        dist.broadcast_object_list(obj, src=0, group=control_group)
        idbytes = ctypes.create_string_buffer(obj[0], 128)
        self.control_group = control_group
        # the set-up (topology discovery, transports: seconds on an 8-GPU node) gets its own deadline;
        # every later enqueue / wait gets ``timeout_s``
        self.handle = self.lib.gadmm_rccl_init_timeout(idbytes, self.nranks, self.rank, self.device.index or 0,
                                                      max(float(init_timeout_s), self.timeout_s))
        if not self.handle:
            native.check(-1, "rccl_init")
        native.check(self.lib.gadmm_rccl_set_timeout(self.handle, self.timeout_s), "rccl_set_timeout")

    @property
    def alive(self) -> bool:
        return bool(self.handle) and int(self.lib.gadmm_rccl_alive(self.handle)) == 1

    def wait(self, stream=None, timeout_s: float = 0.0) -> None:
        """Bounded host wait for everything queued on ``stream`` (default: the current one). Raises
        native.RcclDead after aborting the communicator when the deadline passes."""
        st = stream if stream is not None else self._stream()
        self.native.check(self.lib.gadmm_rccl_wait(self.handle, st, float(timeout_s)), "rccl_wait")

    def abort(self) -> None:
        if self.handle:
            self.lib.gadmm_rccl_abort(self.handle)

    class _Batch:
        def __init__(self, c):
            self.c = c

        def __enter__(self):
            self.c._batched += 1
            return self.c

        def __exit__(self, *exc):
            self.c._batched -= 1
            return False

    def batched(self):
        return RcclComm._Batch(self)

    def _settle(self):
        if not self._batched:
            self.wait()

    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def exchange_rows(self, table, ops):
        if not ops:
            return
        arr = (self.native.XchgOp * len(ops))()
        for i, (peer, row, snd) in enumerate(ops):
            arr[i].peer, arr[i].row, arr[i].is_send, arr[i].count = peer, row, snd, 0
        d = table.shape[1]
        self.native.check(self.lib.gadmm_rccl_exchange_rows(self.handle, arr, len(ops), table.data_ptr(), d,
                                                            self._stream()), "rccl_exchange_rows")
        self._settle()
        for peer, row, snd in ops:
            if snd:
                self.stats.bytes_sent += d * 8
                self.stats.msgs_sent += 1
            else:
                self.stats.bytes_recv += d * 8

    def send_tensor(self, t, peer):
        self._raw([(peer, 1, t)])

    def recv_tensor(self, t, peer):
        self._raw([(peer, 0, t)])

    def _raw(self, items):
        n = len(items)
        peers = (ctypes.c_int * n)(*[p for p, _, _ in items])
        sends = (ctypes.c_int * n)(*[s for _, s, _ in items])
        bufs = (ctypes.c_void_p * n)(*[t.data_ptr() for _, _, t in items])
        counts = (ctypes.c_long * n)(*[t.numel() for _, _, t in items])
        fn = self.lib.gadmm_rccl_sendrecv_raw
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                       ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_long), ctypes.c_void_p]
        self.native.check(fn(self.handle, n, peers, sends, bufs, counts, self._stream()), "rccl_sendrecv")
        self._settle()
        for p, s, t in items:
            if s:
                self.stats.bytes_sent += t.numel() * 8
                self.stats.msgs_sent += 1
            else:
                self.stats.bytes_recv += t.numel() * 8

    def allreduce_sum(self, t):
        self.native.check(self.lib.gadmm_rccl_allreduce_sum_f64(self.handle, t.data_ptr(), t.data_ptr(), t.numel(),
                                                                self._stream()), "rccl_allreduce")
        self.stats.coll_bytes += t.numel() * 8
        self._settle()
        return t

    def reduce_sum(self, t, root):
        self.native.check(self.lib.gadmm_rccl_reduce_sum_f64(self.handle, t.data_ptr(), t.data_ptr(), t.numel(), root,
                                                             self._stream()), "rccl_reduce")
        self.stats.coll_bytes += t.numel() * 8
        self._settle()
        return t

    def broadcast(self, t, root):
        self.native.check(self.lib.gadmm_rccl_bcast_f64(self.handle, t.data_ptr(), t.numel(), root, self._stream()),
                          "rccl_bcast")
        self.stats.coll_bytes += t.numel() * 8
        self._settle()
        return t

    def barrier(self):
        self.wait()
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.control_group)

    def _allreduce_max(self, t):
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.control_group)
        return t

    def close(self):
        if getattr(self, "handle", None):
            self.lib.gadmm_rccl_destroy(self.handle)
            self.handle = None


def init_distributed(backend: Optional[str] = None):
    """Initialise torch.distributed from torchrun-style env vars (MASTER_ADDR defaults to 127.0.0.1).
    Returns (rank, world_size, local_rank)."""
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size(), int(getenv("LOCAL_RANK", "0"))
    world = int(getenv("WORLD_SIZE", "1"))
    rank = int(getenv("RANK", "0"))
    local_rank = int(getenv("LOCAL_RANK", str(rank)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if backend is None:
        backend = "gloo"
    dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local_rank
