"""Set-up breakdown of the real-shaped config on one GPU: 2 workers x 625K x 10k f64 (100 GB)."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gadmm_amd.data import gaussian_regression
from gadmm_amd.models import LinearRegression
from gadmm_amd.algorithms import chain_admm
from gadmm_amd.ops.linalg import spd_inverse

dev = torch.device("cuda", 0)
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 625000
dim = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
ds = gaussian_regression(2, rows, dim, seed=0, labels="linear", device=dev, worker_ids=[0, 1])
torch.cuda.synchronize()
out = {}
def t(name, fn):
    torch.cuda.synchronize(); t0 = time.perf_counter(); r = fn(); torch.cuda.synchronize()
    out[name] = round(time.perf_counter() - t0, 4); return r
m = t("gram_s", lambda: LinearRegression(ds.X, ds.y))
obj0 = t("optimum_s", lambda: m.optimum())
rho = 0.5 * rows
t("inverses_s", lambda: spd_inverse(m.A, torch.tensor([rho, 2 * rho], dtype=torch.float64, device=dev)))
r = t("chain_admm_s", lambda: chain_admm(m, [0, 1], 2, rho, obj0, 1e-8 * abs(obj0), 2000))
out["iters"] = r.iters
r = t("chain_admm_cached_s", lambda: chain_admm(m, [0, 1], 2, rho, obj0, 1e-8 * abs(obj0), 2000))
print(json.dumps(out))
