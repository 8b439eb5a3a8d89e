"""Where does a persistent-kernel GADMM iteration go? In-kernel s_memrealtime timeline (10 ns ticks)
of the E1 solve (N = 24, d = 50, rho = 3) on one MI355X.

    python tools/persist_timeline.py [iters=400]

Per iteration k and worker: start, ready (neighbours' theta + stop decision in hand), published
(theta granules issued), end (objective granule issued). Reports the iteration period, per-phase
compute, the hand-off latency (consumer ready - last producer publish) and the monitor's lag."""
import json, os, sys
os.environ.setdefault("GADMM_BLOCKED", "0")  # the per-worker kernel (the blocked one: blocked_timeline.py)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gadmm_amd.data import linear_synthetic
from gadmm_amd.models import LinearRegression
from gadmm_amd.engine.chain_engine import NativeChainEngine
from gadmm_amd.parallel.topology import Placement
from gadmm_amd.oracle.reference import opt_linear

K = int(sys.argv[1]) if len(sys.argv) > 1 else 400
dev = torch.device("cuda", 0)
ds = linear_synthetic(24)
Xf, yf = ds.stacked()
obj0 = opt_linear(Xf.numpy(), yf.numpy())
eng = NativeChainEngine(ds.X.to(dev), ds.y.to(dev), list(range(24)), 24, "linear", rho=3.0, obj0=obj0, tol=1e-8,
                        max_iter=5000)
eng.set_path(list(range(24)), Placement.contiguous(24, 1), 0)
for rep in range(3):
    eng.reset()
    r = eng.run_persistent(timeline_iters=K)
T = eng.last_timeline.astype(np.float64) * 10e-3  # us
slots = eng.last_timeline_slots
n = len(slots)
gid_row = {g: i for i, (g, p) in enumerate(slots)}
head = {g: (p % 2 == 0) for g, p in slots}
ks = np.arange(20, K - 1)
period = np.diff(T[gid_row[0], :, 0])[ks]
comp = {"head": [], "tail": []}
hop_ht, hop_th = [], []
for g, p in slots:
    row = T[gid_row[g]]
    comp["head" if head[g] else "tail"].append(row[ks, 2] - row[ks, 1])
    nbrs = [u for u in (g - 1, g + 1) if 0 <= u < 24]
    if head[g]:  # ready at k+1 after tails published theta^k
        prod = np.max([T[gid_row[u], ks, 2] for u in nbrs], axis=0)
        hop_th.append(T[gid_row[g], ks + 1, 1] - prod)
    else:  # tail ready at k after heads published theta^k
        prod = np.max([T[gid_row[u], ks, 2] for u in nbrs], axis=0)
        hop_ht.append(row[ks, 1] - prod)
last_end = np.max(T[:n, ks, 3], axis=0)
mon = T[n, ks, 0] - last_end
res = {"iters": r.iters, "us_per_iter_wall": r.wall_ms * 1e3 / r.iters,
       "period_us_median": float(np.median(period)),
       "head_compute_us_median": float(np.median(np.concatenate(comp["head"]))),
       "tail_compute_us_median": float(np.median(np.concatenate(comp["tail"]))),
       "hop_head_to_tail_us_median": float(np.median(np.concatenate(hop_ht))),
       "hop_tail_to_head_us_median": float(np.median(np.concatenate(hop_th))),
       "hop_head_to_tail_us_p90": float(np.percentile(np.concatenate(hop_ht), 90)),
       "hop_tail_to_head_us_p90": float(np.percentile(np.concatenate(hop_th), 90)),
       "monitor_after_last_worker_us_median": float(np.median(mon)),
       "end_minus_pub_us_median": float(np.median(np.concatenate([T[i, ks, 3] - T[i, ks, 2] for i in range(n)]))),
       "barrier_minus_ready_us_median": float(np.median(np.concatenate([T[i, ks, 4] - T[i, ks, 1] for i in range(n)]))),
       "gemv_minus_barrier_us_median": float(np.median(np.concatenate([T[i, ks, 5] - T[i, ks, 4] for i in range(n)]))),
       "pub_minus_gemv_us_median": float(np.median(np.concatenate([T[i, ks, 2] - T[i, ks, 5] for i in range(n)]))),
       "ready_minus_start_us_median_tail": float(np.median(np.concatenate(
           [T[gid_row[g], ks, 1] - T[gid_row[g], ks, 0] for g, p in slots if not head[g]])))}
print(json.dumps(res, indent=1))
