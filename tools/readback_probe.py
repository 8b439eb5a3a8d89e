"""Back-to-back persistent logistic solves on fresh engines (tests/test_gpu.py::test_postfence_stress's
pattern): per solve the wall time, the control block the host read back, and the device's own copy,
so a timed-out hand-off (device done == 4 after ~timeout_s) is told apart from a stale host read.
Usage: python tools/readback_probe.py [solves] [newton]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.data import logistic_synthetic  # noqa: E402
from gadmm_amd.engine.chain_engine import NativeChainEngine, HandoffTimeout  # noqa: E402
from gadmm_amd.parallel import topology as T  # noqa: E402

dev = torch.device("cuda", 0)
ds = logistic_synthetic(24)
X, Y = ds.X.to(dev).contiguous(), ds.y.to(dev).contiguous()
NS = int(sys.argv[1]) if len(sys.argv) > 1 else 32
newton = len(sys.argv) > 2 and sys.argv[2] == "newton"
bad = 0
for i in range(NS):
    eng = NativeChainEngine(X, Y, list(range(24)), 24, "logistic", rho=1e-3 if newton else 2e-4, obj0=0.7177269844827424,
                            tol=1e-8 if newton else 1e-4, max_iter=2000 if newton else 400, lam=1e-5,
                            step=2.2, local_solver="newton" if newton else "gd")
    eng.set_path(list(range(24)), T.Placement.contiguous(24, 1), 0)
    eng.reset()
    t0 = time.perf_counter()
    try:
        r = eng.run_persistent(timeout_s=5.0)
        out = "iters %d done %d" % (r.iters, r.done)
    except HandoffTimeout as e:
        bad += 1
        out = "TIMEOUT (%s)" % e
    dt = time.perf_counter() - t0
    torch.cuda.synchronize()
    host = eng._ctl_host.tolist()
    devc = eng.ctl.cpu().tolist()
    print("%3d %8.2f ms  %-28s host ctl %s  device ctl %s  placed %d" % (i, dt * 1e3, out, host, devc, eng.last_placed),
          flush=True)
    eng.close()
print("timeouts: %d of %d" % (bad, NS))
