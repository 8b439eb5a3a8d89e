"""Star ADMM kernel (star_persistent.hip) on 1 GPU: ms per solve and us per iteration vs the stop-rule
lag, plus the per-iteration decision clock. Usage: python tools/star_sweep.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.benchmarks import headline_rank_problem  # noqa: E402
from gadmm_amd.engine.star_engine import StarEngine  # noqa: E402
from gadmm_amd.models import LinearRegression  # noqa: E402

dev = torch.device("cuda", 0)
X, y, loc, pl, obj0 = headline_rank_problem(24, 0, 1)
m = LinearRegression(X.to(dev), y.to(dev))
for lag in (2, 4, 8, 16):
    StarEngine.LAG = lag
    eng = StarEngine(m.X, m.y, loc, 24, 1.0, obj0, 1e-4, 20000, precomputed=(m.A, m.b, m.yy))
    eng.run()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        it, done, _ = eng.run()
        ts.append((time.perf_counter() - t0) * 1e3)
    tt = eng.time_trace(it)
    per = np.diff(tt) * 1e6
    print("lag %2d: %d iterations done=%d, ms per solve %s, decision period us: median %.2f p10 %.2f p90 %.2f"
          % (lag, it, done, [round(t, 3) for t in ts], np.median(per), np.percentile(per, 10), np.percentile(per, 90)),
          flush=True)

# in-kernel timeline of iterations 50..249 (lag 4): per-iteration hub / worker phases, in us
StarEngine.LAG = 4
eng = StarEngine(m.X, m.y, loc, 24, 1.0, obj0, 1e-4, 20000, precomputed=(m.A, m.b, m.yy))
eng.run()
eng.run(timeline_iters=300)
T = eng.last_timeline.astype(np.float64) * 1e-2  # 10 ns ticks -> us
hub, mon = 23, 24
its = np.arange(50, 250)
hub_wait = T[hub, its, 1] - T[hub, its, 0]
hub_work = T[hub, its, 2] - T[hub, its, 1]
hub_obj = T[hub, its, 3] - T[hub, its, 2]
# worker side: hub publish of iteration i -> worker ready at i + 1 -> upload
wk_seen = T[:hub, its + 1, 1] - T[hub, its, 2][None, :]
wk_work = T[:hub, its + 1, 2] - T[:hub, its + 1, 1]
last_up = T[:hub, its + 1, 2].max(axis=0) - T[hub, its, 2]
hub_ready = T[hub, its + 1, 1] - T[:hub, its + 1, 2].max(axis=0)
period = np.diff(T[hub, its, 2])
print("timeline (median us): period %.2f | hub: wait %.2f, solve+publish %.2f, objective %.2f | "
      "worker: sees hub row %.2f after publish (max over workers %.2f), solve+upload %.2f | "
      "last upload %.2f after publish | hub ready %.2f after the last upload"
      % (np.median(period), np.median(hub_wait), np.median(hub_work), np.median(hub_obj), np.median(wk_seen),
         np.median(wk_seen.max(axis=0)), np.median(wk_work), np.median(last_up), np.median(hub_ready)), flush=True)
