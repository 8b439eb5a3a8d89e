"""Diagnose the 4-rank large-d optimum: local Gram sums, IPC vs gloo all-reduce, vs the one-rank Gram."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rank_fn(rank, world, wpg, rows, dim):
    import torch
    import torch.distributed as dist
    from gadmm_amd.data import gaussian_regression
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.parallel.ipc import IpcComm
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = wpg * world
    ids = list(range(rank * wpg, (rank + 1) * wpg))
    ds = gaussian_regression(n, rows, dim, seed=0, labels="linear", device=dev, worker_ids=ids)
    m = LinearRegression(ds.X, ds.y)
    out = {"A_loc_sum": [float(m.A[i].double().sum()) for i in range(wpg)],
           "X_sum": [float(ds.X[i].sum()) for i in range(wpg)]}
    buf = torch.cat([m.A.sum(0).reshape(-1), m.b.sum(0), m.yy.sum().reshape(1)]).contiguous()
    ref = buf.cpu()
    dist.all_reduce(ref)
    comm = IpcComm(n, dim, 16, dev)
    t = buf.clone()
    comm.allreduce_sum(t)
    out["ipc_vs_gloo_max"] = float((t.cpu() - ref).abs().max())
    out["obj0"] = m.optimum(comm, n_total=n)
    if rank == 0:
        full = gaussian_regression(n, rows, dim, seed=0, labels="linear", device=dev)
        mf = LinearRegression(full.X, full.y)
        out["full_A_sums"] = [float(mf.A[i].double().sum()) for i in range(n)]
        out["full_X_sums"] = [float(full.X[i].sum()) for i in range(n)]
        tot = torch.cat([mf.A.sum(0).reshape(-1), mf.b.sum(0), mf.yy.sum().reshape(1)]).cpu()
        out["gloo_vs_full_max"] = float((ref - tot).abs().max())
        out["obj0_full"] = mf.optimum()
    comm.close()
    return out


if __name__ == "__main__":
    from gadmm_amd.parallel.launch import spawn
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    res = spawn(rank_fn, world, 2, 20000, 2048, timeout=300)
    for r, o in enumerate(res):
        print("rank", r, o, flush=True)
