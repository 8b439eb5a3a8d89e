"""Headline timings on one MI355X (development tool): E1 GADMM (persistent + graph), E3 logistic."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gadmm_amd.data import linear_synthetic, logistic_synthetic
from gadmm_amd.engine.chain_engine import NativeChainEngine
from gadmm_amd.parallel.topology import Placement
from gadmm_amd.oracle import reference as R

dev = torch.device("cuda", 0)
pl = Placement.contiguous(24, 1)
ds = linear_synthetic(24)
Xf, yf = ds.stacked()
obj0 = R.opt_linear(Xf.numpy(), yf.numpy())
X, y = ds.X.to(dev), ds.y.to(dev)
for rho in (3.0, 7.0):
    eng = NativeChainEngine(X, y, list(range(24)), 24, "linear", rho=rho, obj0=obj0, tol=1e-8, max_iter=3000, block=32)
    eng.set_path(list(range(24)), pl, 0)
    for mode in ("persistent", "graph"):
        ts = []
        for k in range(7):
            eng.refresh(X, y); eng.reset()
            torch.cuda.synchronize(); t0 = time.perf_counter()
            r = eng.run_persistent() if mode == "persistent" else eng.run()
            torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
        print("E1 rho=%g %-10s iters=%d  median %.3f ms  min %.3f ms  (%.2f us/iter)" % (
            rho, mode, r.iters, np.median(ts) * 1e3, min(ts) * 1e3, min(ts) * 1e6 / r.iters), flush=True)
    eng.close()
dl = logistic_synthetic(24)
Xlf, ylf = dl.stacked()
obj0l = R.logistic_optimum(Xlf.numpy(), ylf.numpy(), 24e-5)
Xl, yl = dl.X.to(dev), dl.y.to(dev)
for rho, want in ((2e-4, 53), (3e-4, 274)):
    eng = NativeChainEngine(Xl, yl, list(range(24)), 24, "logistic", rho=rho, obj0=obj0l, tol=1e-4, max_iter=400,
                            lam=1e-5, step=2.2, max_inner=100, inner_tol=1e-4, block=8)
    eng.set_path(list(range(24)), pl, 0)
    ts = []
    for k in range(3):
        eng.reset(); torch.cuda.synchronize(); t0 = time.perf_counter(); r = eng.run(); torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print("E3 logistic rho=%g iters=%d (want %d)  min %.3f ms  (%.1f us/iter), inner steps last=%s" % (
        rho, r.iters, want, min(ts) * 1e3, min(ts) * 1e6 / r.iters, eng.inner_iters[:4].tolist()), flush=True)
    eng.close()
