"""Small large-d engine run for kernel profiling (d = 4096, 2 workers x 65,536 rows)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gadmm_amd.data import gaussian_regression
from gadmm_amd.models import LinearRegression
from gadmm_amd.engine.chain_engine import NativeChainEngine
from gadmm_amd.parallel.topology import Placement
dev = torch.device("cuda", 0)
ds = gaussian_regression(2, 65536, 4096, seed=0, device=dev)
m = LinearRegression(ds.X, ds.y)
obj0 = m.optimum()
eng = NativeChainEngine(ds.X, ds.y, [0, 1], 2, "linear", rho=0.5 * 65536, obj0=obj0, tol=1e-8 * abs(obj0),
                        max_iter=200, precomputed=(m.A, m.b, m.yy), block=8)
eng.set_path([0, 1], Placement.contiguous(2, 1), 0)
for _ in range(3):
    eng.reset()
    r = eng.run()
print("iters", r.iters, "done", r.done)
