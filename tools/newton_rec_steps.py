"""Per-step stamps of the persistent Newton pipeline kernel (chain_persistent_newton_rec_kernel): who
waits for whom inside a chord step. One exact-logistic solve (bench config logistic_exact) with
timeline_iters = 512; for the first 24 segments of workers 0-7, the median over steps k >= 1 of
  S period (s_k post -> s_{k+1} post), T period (y post -> y post), and the hand-off lags
  T got b_k - S posted s_k (H's b_k = B s_k between)   S got w_k - W posted w_k   W posted w - T posted y
(s_memrealtime, 10 ns).  python tools/newton_rec_steps.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from gadmm_amd.data import logistic_synthetic
from gadmm_amd.engine.chain_engine import NativeChainEngine
from gadmm_amd.oracle.reference import logistic_optimum
from gadmm_amd.parallel.topology import Placement

dev = torch.device("cuda", 0)
ds = logistic_synthetic(24)
Xf, yf = ds.stacked()
obj0 = logistic_optimum(Xf.numpy(), yf.numpy(), 24 * 1e-5)
eng = NativeChainEngine(ds.X.to(dev), ds.y.to(dev), list(range(24)), 24, "logistic", rho=1e-3, obj0=obj0, tol=1e-8,
                        max_iter=2000, lam=1e-5, local_solver="newton", chord=0.3, max_inner=100, inner_tol=1e-4)
eng.set_path(list(range(24)), Placement.contiguous(24, 1), 0)
for rep in range(3):
    eng.reset()
    r = eng.run_persistent(timeline_iters=512)
    print("solve %d: %d iterations, %.2f ms" % (rep, r.iters, r.wall_ms))
tl = eng.last_timeline[:8, 128:128 + 384, :].astype(np.float64).reshape(8, 24, 16, 8)
names = ["S period", "T period", "T got b - S posted s", "S posted s -> H posted b", "T posted y -> W posted w",
         "W posted w -> S got w", "S got w -> S posted next s"]
vals = {k: [] for k in names}
for w in range(8):
    for sg in range(24):
        st = tl[w, sg]
        for k in range(1, 15):
            a, b = st[k], st[k + 1]
            if a[0] > 0 and b[0] > 0:
                vals["S period"].append(b[0] - a[0])
            if a[1] > 0 and b[1] > 0:
                vals["T period"].append(b[1] - a[1])
            if a[5] > 0 and a[0] > 0:
                vals["T got b - S posted s"].append(a[5] - a[0])
            if a[0] > 0 and a[2] > 0:
                vals["S posted s -> H posted b"].append(a[2] - a[0])
            if a[1] > 0 and b[3] > 0:
                vals["T posted y -> W posted w"].append(b[3] - a[1])
            if a[3] > 0 and a[4] > 0:
                vals["W posted w -> S got w"].append(a[4] - a[3])
            if a[4] > 0 and b[0] > 0:
                vals["S got w -> S posted next s"].append(b[0] - a[4])
for k in names:
    v = np.array(vals[k]) * 10.0  # ns
    if len(v):
        print("%-28s median %7.0f ns  p10 %7.0f  p90 %7.0f  (n=%d)" % (k, np.median(v), np.percentile(v, 10),
                                                                    np.percentile(v, 90), len(v)))
