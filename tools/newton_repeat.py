"""Repeat the exact-logistic native solve (chord 0 and 0.02) and report iterations / NaN per run:
a check for run-to-run non-determinism of chain_newton.hip. Usage: python tools/newton_repeat.py [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.data import logistic_synthetic  # noqa: E402
from gadmm_amd.models import LogisticRegression  # noqa: E402
from gadmm_amd.algorithms.gadmm import group_admm_logistic_exact  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda", 0)
ds = logistic_synthetic(24)
m = LogisticRegression(ds.X.to(dev), ds.y.to(dev), lam=1e-5)
obj0 = 0.7177269844827424
bad = 0
for chord in (0.0, 0.02):
    its = []
    for _ in range(reps):
        r = group_admm_logistic_exact(m, 1e-3, obj0, 1e-8, 1000, engine_opts={"chord": chord, "cache": False})
        its.append((r.iters, bool(np.isnan(r.obj).any())))
        bad += r.iters != 424
    print("chord %g: %s" % (chord, its), flush=True)
print("bad runs:", bad)
sys.exit(1 if bad else 0)
