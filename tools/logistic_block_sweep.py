"""Graph block size (iterations per replayed hipGraph) of the logistic inner-GD engine: ms per solve
and iterations for several blocks on one GPU (bench config logistic). Usage:
python tools/logistic_block_sweep.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.data import logistic_synthetic  # noqa: E402
from gadmm_amd.models import LogisticRegression  # noqa: E402
from gadmm_amd.algorithms import chain_admm  # noqa: E402
from gadmm_amd.parallel.topology import Placement  # noqa: E402

dev = torch.device("cuda", 0)
n = 24
ds = logistic_synthetic(n)
pl = Placement.contiguous(n, 1)
local = pl.local_workers(0)
m = LogisticRegression(ds.X[local].to(dev).contiguous(), ds.y[local].to(dev).contiguous(), lam=1e-5)
obj0 = m.optimum(None, n_total=n)
for blk in (8, 16, 32, 64, 16, 32):
    def solve():
        return chain_admm(m, local, n, 2e-4, obj0, 1e-4, 400, placement=pl, local_solver="gd", step=2.2,
                          engine_opts={"block": blk})
    for _ in range(2):
        r = solve()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        r = solve()
    torch.cuda.synchronize()
    print("block %3d: %.3f ms per solve, %d iterations, engine %s" % (blk, (time.perf_counter() - t0) * 100, r.iters,
                                                                     r.extra.get("engine")), flush=True)
