"""Host-side profile of one D-GADMM solve (bench config dgadmm): cProfile of 20 solves, top entries by
cumulative time, plus the kernel-only time from the engine. Usage: python tools/dgadmm_host_profile.py"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.data import linear_synthetic  # noqa: E402
from gadmm_amd.models import LinearRegression  # noqa: E402
from gadmm_amd.algorithms import dynamic_group_admm  # noqa: E402
from gadmm_amd.parallel import topology as T  # noqa: E402
from gadmm_amd.oracle.reference import opt_linear  # noqa: E402

dev = torch.device("cuda", 0)
ds = linear_synthetic(24)
Xf, yf = ds.stacked()
obj0 = opt_linear(Xf.numpy(), yf.numpy())
m = LinearRegression(ds.X.to(dev).contiguous(), ds.y.to(dev).contiguous())
p0, c0, _ = T.find_path(24, np.random.default_rng(5))
COH = int(sys.argv[1]) if len(sys.argv) > 1 else 10


def solve():
    return dynamic_group_admm(m, 1.0, obj0, 1e-4, 3000, p0, c0, COH, seed=99, n_total=24, local_ids=list(range(24)),
                              engine_opts={"state": False, "residual": False})


for _ in range(3):
    r = solve()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    r = solve()
torch.cuda.synchronize()
print("ms per solve %.3f, iters %d, engine %s" % ((time.perf_counter() - t0) * 50, r.iters, r.extra.get("engine")))
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    solve()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(22)
pstats.Stats(pr).sort_stats("cumulative").print_stats(40)
