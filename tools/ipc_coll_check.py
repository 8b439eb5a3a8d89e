"""IPC device collectives (ipc_coll_kernel) vs gloo, ranks sharing one GPU: python tools/ipc_coll_check.py [world]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def rank_fn(rank, world):
    import torch
    import torch.distributed as dist
    from gadmm_amd.parallel.ipc import IpcComm
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    d = 2048
    comm = IpcComm(8, d, 16, dev)
    out = {}
    for n in (4000, 4104, 4105, 9000, 4 * 1024 * 1024 + 2049):
        g = torch.Generator(device="cpu").manual_seed(1000 * rank + n % 97)
        h = torch.randn(n, generator=g, dtype=torch.float64)
        ref = h.clone()
        dist.all_reduce(ref)
        t = h.to(dev)
        comm.allreduce_sum(t)
        err = (t.cpu() - ref).abs()
        bad = torch.nonzero(err > 1e-12 * ref.abs().max()).flatten()
        out[n] = (float(err.max()), int(bad.numel()), bad[:8].tolist())
    comm.close()
    return out


if __name__ == "__main__":
    from gadmm_amd.parallel.launch import spawn
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    res = spawn(rank_fn, world, timeout=300)
    for r, o in enumerate(res):
        print("rank", r, o, flush=True)
