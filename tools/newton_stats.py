"""Newton local-solve statistics of the exact logistic GADMM (chain_newton.hip): Newton steps per
worker per phase over a whole solve, and wall time per solve. Usage: python tools/newton_stats.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.data import logistic_synthetic  # noqa: E402
from gadmm_amd.engine.chain_engine import NativeChainEngine  # noqa: E402
from gadmm_amd.models import LogisticRegression  # noqa: E402
from gadmm_amd.parallel.topology import Placement  # noqa: E402

dev = torch.device("cuda", 0)
ds = logistic_synthetic(24)
m = LogisticRegression(ds.X.to(dev), ds.y.to(dev), lam=1e-5)
obj0 = m.optimum(None, n_total=24)
eng = NativeChainEngine(ds.X.to(dev), ds.y.to(dev), list(range(24)), 24, "logistic", rho=1e-3, obj0=obj0, tol=1e-8,
                        max_iter=2000, lam=1e-5, local_solver="newton", block=8)
eng.set_path(list(range(24)), Placement.contiguous(24, 1), 0)
steps = []
for it in range(1, 430):  # one iteration per run: read the Newton step counts of both phases' workers
    if it == 1:
        eng.reset()
    r = eng.run(stop_iter=it, use_graph=False)
    steps.append(eng.inner_iters.cpu().numpy().copy())
    if r.done:
        break
steps = np.asarray(steps)
print("iterations", len(steps), "newton steps per worker: mean %.2f max %d; by iteration (first 10):"
      % (steps.mean(), steps.max()), steps[:10].mean(axis=1).round(2).tolist())
ts = []
for rep in range(5):
    eng.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = eng.run()
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3)
print("solve: %d iterations, done=%d, ms per solve %s" % (r.iters, r.done, [round(t, 2) for t in ts]))

# in-kernel breakdown (instrumented instantiation): one iteration, every worker of both phases
os.environ["GADMM_NEWTON_TL"] = "1"
eng2 = NativeChainEngine(ds.X.to(dev), ds.y.to(dev), list(range(24)), 24, "logistic", rho=1e-3, obj0=obj0, tol=1e-8,
                         max_iter=2000, lam=1e-5, local_solver="newton", block=8)
eng2.set_path(list(range(24)), Placement.contiguous(24, 1), 0)
eng2.reset()
eng2.run(stop_iter=20, use_graph=False)
eng2.run(stop_iter=21, use_graph=False)  # iteration 21: stamps of its two phases
tl = eng2.rbuf.cpu().numpy().reshape(-1, 50, 5).astype(np.float64)
used = eng2.inner_iters.cpu().numpy()
seg = []
for w in range(tl.shape[0]):
    for k in range(int(used[w])):
        st = tl[w, k]
        if st[0] > 0 and st[4] > st[0]:
            seg.append(np.diff(st) * 10e-3)  # 10 ns ticks -> us
seg = np.asarray(seg)
print("per Newton step (us, median over workers/steps of iteration 21): sigma %.2f | gradient+Hessian %.2f | "
      "Gauss-Jordan %.2f | update + test %.2f | total %.2f  (n=%d)"
      % tuple(list(np.median(seg, axis=0)) + [float(np.median(seg.sum(axis=1))), len(seg)]))
