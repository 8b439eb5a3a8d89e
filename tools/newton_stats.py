"""Newton local-solve statistics of the exact logistic GADMM (chain_newton.hip), per chord threshold
(0 = a fresh inverse Hessian every Newton step): Newton steps per worker per phase over a whole
solve, wall time per solve, and the in-kernel breakdown of refresh vs chord steps.
Usage: python tools/newton_stats.py [chord ...]"""
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
chords = [float(c) for c in sys.argv[1:]] or [0.0, 0.02, 0.05, 0.1, 0.2, 0.4]


def engine(chord, tl):
    os.environ["GADMM_NEWTON_TL"] = "1" if tl else "0"
    e = NativeChainEngine(ds.X.to(dev), ds.y.to(dev), list(range(24)), 24, "logistic", rho=1e-3, obj0=obj0,
                          tol=1e-8, max_iter=2000, lam=1e-5, local_solver="newton", block=8, chord=chord)
    e.set_path(list(range(24)), Placement.contiguous(24, 1), 0)
    return e


for chord in chords:
    eng = engine(chord, False)
    ts = []
    for rep in range(5):
        eng.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = eng.run()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    print("chord %.3g: %d iterations, done=%d, ms per solve %s" % (chord, r.iters, r.done, [round(t, 2) for t in ts]),
          flush=True)
    # per-iteration step counts + in-kernel stamps (instrumented instantiation), one iteration per run
    eng2 = engine(chord, True)
    eng2.reset()
    steps, seg_ref, seg_chord, nref = [], [], [], []
    for it in range(1, r.iters + 1):
        eng2.run(stop_iter=it, use_graph=False)
        used = eng2.inner_iters.cpu().numpy().copy()
        steps.append(used)
        tl = eng2.rbuf.cpu().numpy().reshape(-1, 50, 5)
        refr = 0
        for w in range(tl.shape[0]):
            for k in range(int(used[w])):
                st = tl[w, k].astype(np.float64)
                if st[0] > 0 and st[4] > st[0]:
                    is_ref = int(tl[w, k, 4]) & 1
                    refr += is_ref
                    (seg_ref if is_ref else seg_chord).append(np.diff(st) * 10e-3)  # 10 ns ticks -> us
        nref.append(refr)
    steps = np.asarray(steps)
    print("  steps per worker-solve: mean %.2f max %d; inverse refreshes per iteration: mean %.2f (of %d solves)"
          % (steps.mean(), steps.max(), float(np.mean(nref)), steps.shape[1]), flush=True)
    for name, seg in (("refresh", seg_ref), ("chord", seg_chord)):
        if seg:
            seg = np.asarray(seg)
            print("  %-7s steps (n=%d), median us: sigma %.2f | gradient(+Hessian) %.2f | inverse %.2f | "
                  "apply + test %.2f | total %.2f" % tuple([name, len(seg)] + list(np.median(seg, axis=0))
                                                         + [float(np.median(seg.sum(axis=1)))]), flush=True)
    eng.close()
    eng2.close()
