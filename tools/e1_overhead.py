"""Where does one E1 bench step go besides the blocked kernel? (1 GPU)
    python tools/e1_overhead.py"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gadmm_amd.data import linear_synthetic
from gadmm_amd.oracle.reference import opt_linear
from gadmm_amd.engine.chain_engine import NativeChainEngine
from gadmm_amd.parallel.topology import Placement

dev = torch.device("cuda", 0)
ds = linear_synthetic(24)
Xf, yf = ds.stacked()
obj0 = opt_linear(Xf.numpy(), yf.numpy())
X, y = ds.X.to(dev).contiguous(), ds.y.to(dev).contiguous()
eng = NativeChainEngine(X, y, list(range(24)), 24, "linear", rho=3.0, obj0=obj0, tol=1e-8, max_iter=20000, block=32)
eng.set_path(list(range(24)), Placement.contiguous(24, 1), 0)
T = {"refresh": [], "reset": [], "run_persistent": [], "kernel_wall": [], "total": []}
for rep in range(30):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.refresh(X, y)
    t1 = time.perf_counter()
    eng.reset()
    t2 = time.perf_counter()
    r = eng.run_persistent()
    t3 = time.perf_counter()
    if rep >= 5:
        T["refresh"].append((t1 - t0) * 1e3)
        T["reset"].append((t2 - t1) * 1e3)
        T["run_persistent"].append((t3 - t2) * 1e3)
        T["kernel_wall"].append(r.wall_ms)
        T["total"].append((t3 - t0) * 1e3)
print({k: round(float(np.median(v)), 4) for k, v in T.items()}, "iters", r.iters)
