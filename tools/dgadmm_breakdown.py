"""Where does a D-GADMM solve's wall time go (E1 data, rho = 1, coherence 10, one GPU)?"""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gadmm_amd.data import linear_synthetic
from gadmm_amd.models import LinearRegression
from gadmm_amd.algorithms import dynamic_group_admm
from gadmm_amd.engine.chain_engine import NativeChainEngine
from gadmm_amd.parallel import topology as T
from gadmm_amd.oracle.reference import opt_linear

dev = torch.device("cuda", 0)
ds = linear_synthetic(24)
Xf, yf = ds.stacked()
obj0 = opt_linear(Xf.numpy(), yf.numpy())
m = LinearRegression(ds.X.to(dev), ds.y.to(dev))
p0, c0, _ = T.find_path(24, np.random.default_rng(5))
out = {}
for rep in range(3):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    r = dynamic_group_admm(m, 1.0, obj0, 1e-4, 3000, p0, c0, 10, seed=99)
    torch.cuda.synchronize(); out["solve_ms"] = (time.perf_counter() - t0) * 1e3
out["iters"], out["engine"] = r.iters, r.extra["engine"]
s = T.PathSchedule(24, p0, c0, 10, seed=99)
t0 = time.perf_counter(); s.prefetch(299); out["prefetch_299_ms"] = (time.perf_counter() - t0) * 1e3
torch.cuda.synchronize(); t0 = time.perf_counter()
eng = NativeChainEngine(m.X, m.y, list(range(24)), 24, "linear", rho=1.0, obj0=obj0, tol=1e-4, max_iter=3000,
                        precomputed=(m.A, m.b, m.yy))
eng.set_path(p0, T.Placement.contiguous(24, 1), 0); eng.reset()
torch.cuda.synchronize(); out["engine_create_ms"] = (time.perf_counter() - t0) * 1e3
eng.close()
print(json.dumps(out))
