"""E4 (LogisticRegression_Real, derm-shaped stand-in: N = 10, d = 34, m = 35) exact-Newton GADMM at
rho = 0.02: torch path vs the persistent Newton kernel vs the graph engine, 60 iterations, one GPU."""
import sys
import numpy as np
import torch

sys.path.insert(0, ".")
from gadmm_amd.config import get_preset
from gadmm_amd.entry.common import full_dataset
from gadmm_amd.models import make_model
from gadmm_amd.algorithms import chain_admm

cfg = get_preset("LogisticRegression_Real")
ds = full_dataset(cfg)
dev = torch.device("cuda", 0)
m = make_model("logistic", ds.X.to(dev).contiguous(), ds.y.to(dev).contiguous(), lam=cfg.lam)
obj0 = m.optimum(None, n_total=ds.num_workers)
print("N=%d m=%d d=%d obj0=%.12f" % (ds.num_workers, ds.rows_per_worker, ds.dim, obj0))
n = ds.num_workers
out = {}
for name, kw in (("torch", dict(backend="torch")), ("persistent", dict(engine_opts={"cache": False})),
                 ("graph", dict(engine_opts={"cache": False, "persistent": False})),
                 ("persistent-exact", dict(engine_opts={"cache": False, "chord": 0.0})),
                 ("graph-exact", dict(engine_opts={"cache": False, "persistent": False, "chord": 0.0}))):
    r = chain_admm(m, list(range(n)), n, 0.02, obj0, 1e-8, 60, local_solver="newton", **kw)
    out[name] = r
    print(name, r.extra.get("engine"), r.iters, "obj[:5]", np.array2string(r.obj[:5], precision=10),
          "final gap %.4g" % r.loss[-1])
a, b = out["torch"].obj, out["persistent"].obj
k = int(np.argmax(np.abs(a - b) > 1e-9 * abs(obj0))) if np.any(np.abs(a - b) > 1e-9 * abs(obj0)) else -1
print("first persistent/torch divergence at iteration", k + 1 if k >= 0 else None)

for nm in ("graph", "persistent-exact", "graph-exact"):
    b = out[nm].obj
    bad = np.abs(a - b) > 1e-9 * abs(obj0)
    print(nm, "first divergence from torch at", int(np.argmax(bad)) + 1 if bad.any() else None,
          "max rel diff %.3g" % float(np.max(np.abs(a - b)) / abs(obj0)))
