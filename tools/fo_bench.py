"""Wall time of the reference baseline bundle on one MI355X: persistent native engine vs torch ops.

    python tools/fo_bench.py
"""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gadmm_amd.data import linear_synthetic, logistic_synthetic
from gadmm_amd.models import LinearRegression, LogisticRegression
from gadmm_amd.algorithms import gd_dgd_lag, dual_averaging, global_constants, gradient_descent
from gadmm_amd.oracle.reference import opt_linear

dev = torch.device("cuda", 0)
out = {}
ds = linear_synthetic(24)
Xf, yf = ds.stacked()
obj0 = opt_linear(Xf.numpy(), yf.numpy())
m = LinearRegression(ds.X.to(dev), ds.y.to(dev))
gd_dgd_lag(m, list(range(24)), 24, 100, obj0, backend="native")  # warm-up
t0 = time.perf_counter()
b = gd_dgd_lag(m, list(range(24)), 24, 60000, obj0, backend="native")
out["E1_bundle_native_s"] = time.perf_counter() - t0
out["E1_per_alg_us_per_iter"] = {k: b[k].wall_s / len(b[k].obj) * 1e6 for k in ("GD", "DGD", "LAG-PS", "LAG-WK", "cIAG", "R-IAG")}
step = global_constants(m)["stepsize"]
t0 = time.perf_counter()
da = dual_averaging(m, list(range(24)), 24, step, obj0, 1e-4, 60000, backend="native")
out["E1_dualavg_native_s"] = time.perf_counter() - t0
out["E1_dualavg_us_per_iter"] = da.wall_s / len(da.obj) * 1e6
t0 = time.perf_counter()
g = gradient_descent(m, list(range(24)), 24, 2000, obj0, step, backend="torch")
out["E1_GD_torch_us_per_iter"] = (time.perf_counter() - t0) / 2000 * 1e6
lg = logistic_synthetic(24)
ml = LogisticRegression(lg.X.to(dev), lg.y.to(dev), lam=1e-5)
t0 = time.perf_counter()
bl = gd_dgd_lag(ml, list(range(24)), 24, 100000, None, accuracy=1e-4, backend="native")
out["E3_bundle_native_s"] = time.perf_counter() - t0
out["E3_iters"] = {k: len(bl[k].obj) for k in ("GD", "DGD", "LAG-PS", "LAG-WK", "cIAG", "R-IAG")}
out["E3_per_alg_us_per_iter"] = {k: bl[k].wall_s / len(bl[k].obj) * 1e6 for k in ("GD", "DGD", "LAG-PS", "LAG-WK", "cIAG", "R-IAG")}
print(json.dumps(out, indent=1))
