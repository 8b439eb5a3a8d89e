"""The large-d optimum across ranks sharing one GPU, in the order the multi-rank test runs it (fresh
IpcComm, Gram still in flight when the chunked device all-reduce is enqueued), with the all-reduced
buffer checked against a gloo all-reduce of the same input: python tools/ipc_optimum_stress.py [world] [reps]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rank_fn(rank, world, reps):
    import torch
    import torch.distributed as dist
    from gadmm_amd.data import gaussian_regression
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.parallel.ipc import IpcComm
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wpg, rows, dim = 2, 20000, 2048
    n = wpg * world
    ids = list(range(rank * wpg, (rank + 1) * wpg))
    outs = []
    for rep in range(reps):
        ds = gaussian_regression(n, rows, dim, seed=0, labels="linear", device=dev, worker_ids=ids)
        m = LinearRegression(ds.X, ds.y)       # Gram enqueued, not waited for
        from gadmm_amd.ops.linalg import gram
        A2, b2, _ = gram(ds.X, ds.y)            # the same kernel again: bit for bit?
        At = torch.bmm(ds.X.transpose(1, 2), ds.X)  # rocBLAS
        gram_rep_equal = bool(torch.equal(A2, m.A) and torch.equal(b2, m.b))
        gram_vs_blas = float((At - m.A).abs().max() / At.abs().max())
        del A2, b2, At
        comm = IpcComm(n, dim, 16, dev)
        buf = torch.cat([m.A.sum(0).reshape(-1), m.b.sum(0), m.yy.sum().reshape(1)]).contiguous()
        src = buf.clone()
        comm.allreduce_sum(buf)
        ref = src.cpu()
        dist.all_reduce(ref)
        err = (buf.cpu() - ref).abs()
        tol = 1e-12 * float(ref.abs().max())
        bad = torch.nonzero(err > tol).flatten()
        step = 2 * dim + 8
        loc = src.cpu()
        only_local = int(((buf.cpu() - loc).abs() <= tol)[bad].sum()) if bad.numel() else 0
        chunks = sorted(set((bad // step).tolist()))
        o = {"rep": rep, "max_err": float(err.max()), "n_bad": int(bad.numel()), "bad_chunks": chunks[:12],
             "n_bad_chunks": len(chunks), "bad_equal_local": only_local, "first_bad": bad[:6].tolist()}
        o["gram_rep_equal"], o["gram_vs_blas"] = gram_rep_equal, gram_vs_blas
        o["obj0"] = m.optimum(comm, n_total=n)
        o["obj0_again"] = m.optimum(comm, n_total=n)
        o["obj0_local"] = m.optimum() if world == 1 else None
        comm.close()
        print("rank", rank, o, flush=True)
        outs.append(o)
    return outs


if __name__ == "__main__":
    from gadmm_amd.parallel.launch import spawn
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    if world == 1:  # one process, no comm: the Gram / oracle alone
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29571")
        dist.init_process_group("gloo", rank=0, world_size=1)
    res = spawn(rank_fn, world, reps, timeout=300) if world > 1 else [rank_fn(0, 1, reps)]
    for r, o in enumerate(res):
        for x in o:
            print("rank", r, x, flush=True)
