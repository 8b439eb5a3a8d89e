"""Host clock between labelled points of the inexact logistic bench step (bench.py --config logistic:
chain_admm with inner-GD local solves, the two-wave persistent kernel): the median time from each stamp
to the next over repeated solves (gadmm_amd.utils.timing.host_stamp).
Usage: python tools/lg_host_stamps.py [solves]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.algorithms import chain_admm  # noqa: E402
from gadmm_amd.data import logistic_synthetic  # noqa: E402
from gadmm_amd.models import LogisticRegression  # noqa: E402
from gadmm_amd.parallel.topology import Placement  # noqa: E402
from gadmm_amd.utils import timing  # noqa: E402

NS = int(sys.argv[1]) if len(sys.argv) > 1 else 30
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
n = 24
pl = Placement.contiguous(n, 1)
ds = logistic_synthetic(n)
m = LogisticRegression(ds.X.to(dev).contiguous(), ds.y.to(dev).contiguous(), lam=1e-5)
obj0 = m.optimum(None, n_total=n)


def solve():
    return chain_admm(m, list(range(n)), n, 2e-4, obj0, 1e-4, 400, placement=pl, local_solver="gd", step=2.2,
                      engine_opts={"state": False, "residual": False})


for _ in range(3):
    solve()
torch.cuda.synchronize()
segs, order = {}, []
for _ in range(NS):
    timing.HOST_STAMPS = [("solve:begin", time.perf_counter())]
    r = solve()
    timing.HOST_STAMPS.append(("solve:end", time.perf_counter()))
    st = timing.HOST_STAMPS
    timing.HOST_STAMPS = None
    for (a, ta), (b, tb) in zip(st[:-1], st[1:]):
        k = "%s -> %s" % (a, b)
        if k not in segs:
            segs[k] = []
            order.append(k)
        segs[k].append((tb - ta) * 1e6)
print("logistic inner GD, %d iterations, engine %s; median us per segment over %d solves:"
      % (r.iters, r.extra.get("engine"), NS))
tot = 0.0
for k in order:
    v = float(np.median(segs[k]))
    tot += v
    print("  %8.1f  %s" % (v, k))
print("  %8.1f  sum of medians" % tot)
