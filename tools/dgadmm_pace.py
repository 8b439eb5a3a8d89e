"""Per-iteration pace of a D-GADMM solve from the device clock the monitor stamps at every decision
(s_memrealtime, 10 ns): mean decision-to-decision time by offset inside an epoch (offset 0 = the
re-chain iteration), the first decision after the reset, and the last one. Whichever kernel the
environment selects (GADMM_BLOCKED_DYN=1: the blocked kernel's dynamic mode).
Usage: python tools/dgadmm_pace.py [coherence] [solves]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.data import linear_synthetic  # noqa: E402
from gadmm_amd.models import LinearRegression  # noqa: E402
from gadmm_amd.algorithms import dynamic_group_admm  # noqa: E402
from gadmm_amd.parallel import topology as T  # noqa: E402
from gadmm_amd.oracle.reference import opt_linear  # noqa: E402

dev = torch.device("cuda", 0)
ds = linear_synthetic(24)
Xf, yf = ds.stacked()
obj0 = opt_linear(Xf.numpy(), yf.numpy())
m = LinearRegression(ds.X.to(dev).contiguous(), ds.y.to(dev).contiguous())
p0, c0, _ = T.find_path(24, np.random.default_rng(5))
COH = int(sys.argv[1]) if len(sys.argv) > 1 else 10
NS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
opts = {"state": False, "residual": False}


def solve():
    return dynamic_group_admm(m, 1.0, obj0, 1e-4, 3000, p0, c0, COH, seed=99, n_total=24, local_ids=list(range(24)),
                              engine_opts=opts)


for _ in range(3):
    solve()
acc = np.zeros(COH)
cnt = np.zeros(COH)
firsts, lasts = [], []
for _ in range(NS):
    r = solve()
    t = np.asarray(r.time_trace) * 1e6
    firsts.append(t[0])
    lasts.append(t[-1])
    dt = np.diff(t)  # dt[j]: iteration j + 2, decision(j + 2) - decision(j + 1)
    its = np.arange(2, len(t) + 1)
    off = its % COH  # re-chains at iterations e * COH (offset 0; topology.rechain_iterations)
    for o in range(COH):
        sel = off == o
        acc[o] += dt[sel].sum()
        cnt[o] += sel.sum()
print("coherence %d, %d iterations, engine %s, kernel env GADMM_BLOCKED_DYN=%s"
      % (COH, r.iters, r.extra.get("engine"), os.environ.get("GADMM_BLOCKED_DYN", "0")))
print("reset -> first decision: median %.1f us; reset -> last decision: median %.1f us"
      % (np.median(firsts), np.median(lasts)))
print("mean us per iteration by offset in the epoch (0 = re-chain iteration):")
print("  " + "  ".join("%d:%.2f" % (o, acc[o] / max(cnt[o], 1)) for o in range(COH)))
