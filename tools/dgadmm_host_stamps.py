"""Host clock between labelled points of a D-GADMM solve (the bench config): the median time from each
stamp to the next over repeated solves (gadmm_amd.utils.timing.host_stamp). Segment names are
"from -> to"; "solve:begin" / "solve:end" bracket the whole call.
Usage: python tools/dgadmm_host_stamps.py [coherence] [solves] [refresh]"""
import os
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
from gadmm_amd.utils import timing  # noqa: E402

dev = torch.device("cuda", 0)
ds = linear_synthetic(24)
Xf, yf = ds.stacked()
obj0 = opt_linear(Xf.numpy(), yf.numpy())
m = LinearRegression(ds.X.to(dev).contiguous(), ds.y.to(dev).contiguous())
p0, c0, _ = T.find_path(24, np.random.default_rng(5))
COH = int(sys.argv[1]) if len(sys.argv) > 1 else 10
NS = int(sys.argv[2]) if len(sys.argv) > 2 else 40
REFRESH = len(sys.argv) > 3 and sys.argv[3] == "refresh"  # the bench's step: Gram + inverses per solve


def solve():
    return dynamic_group_admm(m, 1.0, obj0, 1e-4, 3000, p0, c0, COH, seed=99, n_total=24, local_ids=list(range(24)),
                              engine_opts={"state": False, "residual": False, "refresh": REFRESH})


for _ in range(3):
    solve()
torch.cuda.synchronize()
segs = {}
order = []
for _ in range(NS):
    timing.HOST_STAMPS = [("solve:begin", time.perf_counter())]
    r = solve()
    timing.HOST_STAMPS.append(("solve:end", time.perf_counter()))
    st = timing.HOST_STAMPS
    timing.HOST_STAMPS = None
    for (a, ta), (b, tb) in zip(st[:-1], st[1:]):
        key = "%s -> %s" % (a, b)
        if key not in segs:
            segs[key] = []
            order.append(key)
        segs[key].append((tb - ta) * 1e6)
print("coherence %d, %d iterations, engine %s; median us per segment over %d solves:" % (COH, r.iters,
                                                                                         r.extra.get("engine"), NS))
tot = 0.0
for k in order:
    v = float(np.median(segs[k]))
    tot += v
    print("  %8.1f  %s" % (v, k))
print("  %8.1f  sum of medians" % tot)
