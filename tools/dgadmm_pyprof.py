"""cProfile of the host side of repeated D-GADMM solves (bench config, coherence 10): where the ~170 us
before the persistent launch go. Usage: python tools/dgadmm_pyprof.py [coherence] [refresh]"""
import cProfile
import os
import pstats
import sys

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
REFRESH = len(sys.argv) > 2 and sys.argv[2] == "refresh"  # the bench's step: Gram + inverses per solve
opts = {"state": False, "residual": False, "refresh": REFRESH}


def solve():
    return dynamic_group_admm(m, 1.0, obj0, 1e-4, 3000, p0, c0, COH, seed=99, n_total=24, engine_opts=opts)


for _ in range(5):
    solve()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    r = solve()
pr.disable()
print("engine", r.extra.get("engine"), "iters", r.iters)
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumulative").print_stats(45)
