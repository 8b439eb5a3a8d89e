"""Does the stop-rule monitor keep up with the blocked GADMM kernel? (E1, 1 GPU)

Per iteration j: worker workgroup 0 finishes iteration j at W_j; the monitor posts decision j at
M_j (both s_memrealtime, one chip clock). Prints the monitor's delay M_j - W_j over the run and the
solve time for several stop-rule lags.

    python tools/monitor_lag.py [iters=600]"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gadmm_amd.data import linear_synthetic
from gadmm_amd.engine.chain_engine import NativeChainEngine
from gadmm_amd.parallel.topology import Placement
from gadmm_amd.oracle.reference import opt_linear

K = int(sys.argv[1]) if len(sys.argv) > 1 else 600
dev = torch.device("cuda", 0)
ds = linear_synthetic(24)
Xf, yf = ds.stacked()
obj0 = opt_linear(Xf.numpy(), yf.numpy())
eng = NativeChainEngine(ds.X.to(dev), ds.y.to(dev), list(range(24)), 24, "linear", rho=3.0, obj0=obj0, tol=1e-8,
                        max_iter=5000)
eng.set_path(list(range(24)), Placement.contiguous(24, 1), 0)
res = {}
for lag in (8, 16, 32):
    ts = []
    for rep in range(5):
        eng.reset()
        r = eng.run_persistent(lag=lag)
        ts.append(r.wall_ms)
    res["lag%d_ms" % lag] = float(np.median(ts))
    res["lag%d_iters" % lag] = r.iters
eng.reset()
r = eng.run_persistent(lag=8, timeline_iters=K)
k, L, W, _pw = eng.blocked_plan(timeline=True)
Wo = (24 + 11) // 12
T = eng.last_timeline.astype(np.float64) * 10e-3
work_end = T[0, :, 5]
mon = T[W + Wo, :, 0]
delay = mon - work_end
res["kernel"] = eng.last_kernel
res["monitor_delay_us"] = {str(j): round(float(delay[j]), 2) for j in (10, 50, 100, 200, 300, 400, 500, K - 10) if j < K}
res["worker_period_us"] = float(np.median(np.diff(work_end[20:K - 2])))
res["monitor_period_us"] = float(np.median(np.diff(mon[20:K - 2])))
print(json.dumps(res, indent=1))
