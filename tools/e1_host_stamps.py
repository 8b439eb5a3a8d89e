"""Host clock between labelled points of the headline solve (bench.py's E1 step on one GPU: the
DistributedChainSolver the bench times, Gram + inverses + iterations per solve): the median time from
each stamp to the next over repeated solves (gadmm_amd.utils.timing.host_stamp).
Usage: python tools/e1_host_stamps.py [solves]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.benchmarks import headline_rank_problem  # noqa: E402
from gadmm_amd.engine.multigpu import DistributedChainSolver  # noqa: E402
from gadmm_amd.utils import timing  # noqa: E402

NS = int(sys.argv[1]) if len(sys.argv) > 1 else 40
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
X, y, local, placement, obj0 = headline_rank_problem(24, 0, 1)
sol = DistributedChainSolver(X.to(dev).contiguous(), y.to(dev).contiguous(), local, 24, placement, 0, 1, dev, 3.0, obj0,
                             1e-8, engine="auto", fabric="auto", share=False, block=0, use_graph=True, timeout_s=20.0)
for _ in range(5):
    sol.guarded_solve()
torch.cuda.synchronize()
segs, order = {}, []
for _ in range(NS):
    timing.HOST_STAMPS = [("solve:begin", time.perf_counter())]
    r = sol.guarded_solve()
    timing.HOST_STAMPS.append(("solve:end", time.perf_counter()))
    st = timing.HOST_STAMPS
    timing.HOST_STAMPS = None
    for (a, ta), (b, tb) in zip(st[:-1], st[1:]):
        k = "%s -> %s" % (a, b)
        if k not in segs:
            segs[k] = []
            order.append(k)
        segs[k].append((tb - ta) * 1e6)
print("E1 headline, %d iterations (done %d), kernel %s; median us per segment over %d solves:"
      % (r.iters, r.done, sol.kernel, NS))
tot = 0.0
for k in order:
    v = float(np.median(segs[k]))
    tot += v
    print("  %8.1f  %s" % (v, k))
print("  %8.1f  sum of medians" % tot)
