"""In-kernel timeline of the temporally blocked GADMM kernel (E1). Per workgroup and iteration:
[start, after exchange, decision ready, after decision barrier, after head phase, after tail phase].

    GADMM_BLOCK_K=2 python tools/blocked_timeline.py [iters=300]"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gadmm_amd.data import linear_synthetic
from gadmm_amd.engine.chain_engine import NativeChainEngine
from gadmm_amd.parallel.topology import Placement
from gadmm_amd.oracle.reference import opt_linear

K = int(sys.argv[1]) if len(sys.argv) > 1 else 300
dev = torch.device("cuda", 0)
ds = linear_synthetic(24)
Xf, yf = ds.stacked()
obj0 = opt_linear(Xf.numpy(), yf.numpy())
eng = NativeChainEngine(ds.X.to(dev), ds.y.to(dev), list(range(24)), 24, "linear", rho=3.0, obj0=obj0, tol=1e-8,
                        max_iter=5000)
eng.set_path(list(range(24)), Placement.contiguous(24, 1), 0)
for rep in range(3):
    eng.reset()
    r = eng.run_persistent(timeline_iters=K, timeout_s=float(os.environ.get("TL_TIMEOUT", "20")))
k, L, W, _pw = eng.blocked_plan(timeline=True)
T = eng.last_timeline[: W + 1].astype(np.float64) * 10e-3
ks = np.arange(20, K - 2)
res = {"kernel": eng.last_kernel, "iters": r.iters, "us_per_iter_wall": r.wall_ms * 1e3 / max(r.iters, 1)}
res["period_us_median"] = float(np.median(np.diff(T[0, :, 0])[ks]))
names = ["exchange", "decision_wait", "decision_barrier", "head_phase", "tail_phase"]
for q, nm in enumerate(names):
    dd = np.concatenate([T[g, ks, q + 1] - T[g, ks, q] for g in range(W)])
    res[nm + "_us_median"] = float(np.median(dd))
    exch = np.concatenate([T[g, ks, 1] - T[g, ks, 0] for g in range(W)])
res["wave0_head_rhs_us_median"] = float(np.median(T[0, ks, 6] - T[0, ks, 3]))
res["wave0_head_gemv_us_median"] = float(np.median(T[0, ks, 7] - T[0, ks, 6]))
res["wave0_head_after_gemv_to_barrier_us_median"] = float(np.median(T[0, ks, 4] - T[0, ks, 7]))
res["exchange_us_mean_per_iter"] = float(np.mean(exch))
res["exchange_us_max"] = float(np.max(exch))
Tt = eng.last_timeline[128: 128 + W].astype(np.float64) * 10e-3
for q, nm in enumerate(["tail_rhs", "tail_gemv", "tail_dual_stores", "tail_to_barrier_end"]):
    dd = np.concatenate([Tt[g, ks, q + 1] - Tt[g, ks, q] for g in range(W)])
    res["tailwave_" + nm + "_us_median"] = float(np.median(dd))
dd = np.concatenate([Tt[g, ks, 0] - T[g, ks, 4] for g in range(W)])
res["tailwave_start_after_head_barrier_us_median"] = float(np.median(dd))
# per-wave end of tail-phase work (rows 160 + g*12 + v): which wave closes the tail barrier?
Tw = eng.last_timeline[160: 160 + 12 * min(W, 8)].astype(np.float64).reshape(min(W, 8), 12, K, 8)[..., 0] * 10e-3
late = []
for g in range(min(W, 8)):
    e = Tw[g][:, ks]                       # (12, iters)
    valid = e.min(axis=1) > 0
    rel = e - e[valid].min(axis=0, keepdims=True)
    late.append([round(float(np.median(rel[v])), 2) if valid[v] else None for v in range(12)])
res["tail_work_end_rel_us_median[g][wave]"] = late
print(json.dumps(res, indent=1))
