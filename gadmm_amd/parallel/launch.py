"""Process launch helpers.

* ``spawn(fn, world_size)``: run ``fn(rank, world_size, *args)`` in ``world_size`` processes on this
  host with a gloo process group (127.0.0.1 rendezvous, free port). Used by the CPU multi-process
  tests (BASELINE.json configs[0]) and by ``python -m gadmm_amd ... --cpu-ranks N``.
* ``setup_rank(...)``: torchrun-style set-up for GPU jobs — the gloo control plane, one process per
  MI355X; data planes and fabrics come later, on demand (parallel/node.py).
"""
from __future__ import annotations

import os
import socket
import traceback
from typing import Any, Callable, List, Optional

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, fn, args, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    os.environ["LOCAL_RANK"] = str(rank)
    torch.set_num_threads(1)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world, init_method="tcp://127.0.0.1:%d" % port)
        out = fn(rank, world, *args)
        q.put((rank, "ok", out))
    except Exception:  # pragma: no cover - surfaced to the parent
        q.put((rank, "err", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


def spawn(fn: Callable, world_size: int, *args, timeout: float = 600.0) -> List[Any]:
    """Run ``fn`` on ``world_size`` gloo ranks; returns the per-rank return values (rank order)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world_size, port, fn, args, q), daemon=True)
             for r in range(world_size)]
    for p in procs:
        p.start()
    results: List[Any] = [None] * world_size
    errors = []
    try:
        for _ in range(world_size):
            rank, status, payload = q.get(timeout=timeout)
            if status == "ok":
                results[rank] = payload
            else:
                errors.append("rank %d:\n%s" % (rank, payload))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    if errors:
        raise RuntimeError("spawned ranks failed:\n" + "\n".join(errors))
    return results


def setup_rank(backend: str = "node", device: Optional[int] = None):
    """torchrun-style per-process set-up. Returns (rank, world, local_rank, device, comm).

    ``backend='node'`` (GPU ranks): the gloo control plane only -- the data plane and the xGMI fabrics
    are built on demand by ``parallel/node.NodeFabrics`` (IPC by default, RCCL opt-in); ``comm`` is None
    for several ranks until the caller builds it. The device is ``select_device_index``: device 0 when the
    ranks share one GPU (GADMM_SHARE_GPU / GADMM_BENCH_SHARE_GPU), else ``local_rank % visible devices``.
    ``'rccl'``: as 'node' plus an eager native RCCL communicator (explicit opt-in only);
    ``'nccl'``: torch.distributed nccl (= RCCL) process group used through TorchDistComm;
    ``'gloo'``: CPU plumbing."""
    from .comm import LocalComm, RcclComm, TorchDistComm
    from .node import select_device_index, share_requested

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    dev = torch.device("cpu")
    if backend in ("node", "rccl", "nccl"):
        idx = device if device is not None else select_device_index(local_rank, share_requested(),
                                                                    torch.cuda.device_count())
        dev = torch.device("cuda", idx)
        torch.cuda.set_device(dev)
    if world == 1:
        return rank, world, local_rank, dev, LocalComm()
    if not dist.is_initialized():
        dist.init_process_group("nccl" if backend == "nccl" else "gloo", rank=rank, world_size=world)
    if backend == "node":
        return rank, world, local_rank, dev, None
    if backend == "rccl":
        comm = RcclComm(dev)
    else:
        comm = TorchDistComm()
    return rank, world, local_rank, dev, comm
