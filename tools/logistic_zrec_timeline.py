"""Per-step shader-cycle stamps of the two-wave logistic kernel (chain_persistent_logistic_zrec_kernel,
worker 0, its 3rd local solve): margins wave [top, sigmoid done, s posted, K s done], iterate wave
[top, s seen, X^T s done]. Usage: python tools/logistic_zrec_timeline.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.data import logistic_synthetic  # noqa: E402
from gadmm_amd.engine.chain_engine import NativeChainEngine  # noqa: E402
from gadmm_amd.models import LogisticRegression  # noqa: E402

dev = torch.device("cuda", 0)
ds = logistic_synthetic(24)
m = LogisticRegression(ds.X.to(dev), ds.y.to(dev), lam=1e-5)
obj0 = LogisticRegression(ds.X, ds.y, lam=1e-5).optimum()
eng = NativeChainEngine(m.X, m.y, list(range(24)), 24, "logistic", rho=2e-4, obj0=obj0, tol=1e-4, max_iter=400,
                        lam=1e-5, step=2.2, max_inner=100, inner_tol=1e-4)
from gadmm_amd.parallel.topology import Placement  # noqa: E402
eng.set_path(list(range(24)), Placement.contiguous(24, 1), 0)
for _ in range(2):
    eng.reset()
    r = eng.run_persistent(timeline_iters=64)
tl = eng.last_timeline.reshape(-1, 8)
mg = tl[0:64, :4].astype(np.float64)
it = tl[256:320, :3].astype(np.float64)
print("iterations", r.iters, "kernel", eng.last_kernel)
ok = mg[:, 0] > 0
if ok.sum() > 2:
    d = np.diff(mg[ok], axis=1)
    per = np.diff(mg[ok][:, 0])
    print("margins wave, median cycles: sigmoid %.0f | post s %.0f | K s GEMV %.0f | step period %.0f"
          % (np.median(d[:, 0]), np.median(d[:, 1]), np.median(d[:, 2]), np.median(per)))
oi = it[:, 0] > 0
if oi.sum() > 2:
    d = np.diff(it[oi], axis=1)
    per = np.diff(it[oi][:, 0])
    print("iterate wave, median cycles: wait for s %.0f | X^T s GEMV + release %.0f | step period %.0f"
          % (np.median(d[:, 0]), np.median(d[:, 1]), np.median(per)))
