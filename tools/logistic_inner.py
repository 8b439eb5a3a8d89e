"""Inner-GD step cost of the GADMM logistic phase kernels (E3, N = 24, rho = 2e-4, step 2.2).
Run under rocprofv3 --kernel-trace --stats; prints the solve time and the inner steps used by the
workers in the last phase (the reference's all-coordinates break rarely fires, so ~100).

    python tools/logistic_inner.py"""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gadmm_amd.data import logistic_synthetic
from gadmm_amd.models import LogisticRegression
from gadmm_amd.algorithms import chain_admm

dev = torch.device("cuda", 0)
ds = logistic_synthetic(24)
m = LogisticRegression(ds.X.to(dev), ds.y.to(dev), lam=1e-5)
obj0 = m.optimum()
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = chain_admm(m, list(range(24)), 24, 2e-4, obj0, 1e-4, 400, local_solver="gd", step=2.2)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
eng = r.extra.get("engine_obj")
inner = eng.inner_iters.cpu().tolist() if eng is not None and hasattr(eng, "inner_iters") else None
print(json.dumps({"iters": r.iters, "ms": (t1 - t0) * 1e3, "engine": r.extra.get("engine"),
                  "last_phase_inner_steps": inner}))
