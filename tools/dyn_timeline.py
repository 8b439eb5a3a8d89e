"""Timeline of the one-launch D-GADMM kernel (E1, rho = 1, coherence argv[1], default 10): iteration
period inside and at epoch boundaries, per-phase compute and hand-off."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gadmm_amd.data import linear_synthetic
from gadmm_amd.engine.chain_engine import NativeChainEngine
from gadmm_amd.parallel import topology as T
from gadmm_amd.oracle.reference import opt_linear

dev = torch.device("cuda", 0)
ds = linear_synthetic(24)
Xf, yf = ds.stacked()
obj0 = opt_linear(Xf.numpy(), yf.numpy())
p0, c0, _ = T.find_path(24, np.random.default_rng(5))
COH = int(sys.argv[1]) if len(sys.argv) > 1 else 10
s = T.PathSchedule(24, p0, c0, COH, seed=99)
rech = [it for it in range(2, 3001) if T.rechain_iteration(it, COH)]
pre = s.prefetch(len(rech))
epochs = [(1, list(p0))] + [(it, pc[0]) for it, pc in zip(rech, pre)]
eng = NativeChainEngine(ds.X.to(dev), ds.y.to(dev), list(range(24)), 24, "linear", rho=1.0, obj0=obj0, tol=1e-4,
                        max_iter=3000)
eng.set_path(p0, T.Placement.contiguous(24, 1), 0)
K = 200
for rep in range(2):
    eng.reset()
    r = eng.run_persistent(epochs=epochs, timeline_iters=K)
T_ = eng.last_timeline[:25].astype(np.float64) * 10e-3
per = np.diff(T_[0, :, 0])
bound = np.array([it for it in range(2, K) if T.rechain_iteration(it, COH)]) - 1  # 0-based boundary index
inner = np.setdiff1d(np.arange(5, K - 1), np.concatenate([bound - 1, bound]))
if len(inner) == 0:
    inner = np.arange(5, K - 1)
print(json.dumps({"coherence": COH, "iters": r.iters, "wall_ms": r.wall_ms, "us_per_iter": r.wall_ms * 1e3 / r.iters,
                  "period_median_inside_epoch_us": float(np.median(per[inner])),
                  "period_median_at_boundary_us": float(np.median(per[bound[bound < K - 1] - 1])),
                  "ready_minus_start_median_us": float(np.median(T_[:24, 5:K - 1, 1] - T_[:24, 5:K - 1, 0])),
                  "pub_minus_ready_median_us": float(np.median(T_[:24, 5:K - 1, 2] - T_[:24, 5:K - 1, 1]))}))
