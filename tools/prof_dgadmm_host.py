import cProfile, pstats, sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from gadmm_amd.data import linear_synthetic
from gadmm_amd.models import LinearRegression
from gadmm_amd.algorithms import dynamic_group_admm
from gadmm_amd.parallel import topology as T
from gadmm_amd.oracle.reference import opt_linear
dev = torch.device("cuda", 0)
n = 24
ds = linear_synthetic(n)
Xf, yf = ds.stacked()
obj0 = opt_linear(Xf.numpy(), yf.numpy())
m = LinearRegression(ds.X.to(dev).contiguous(), ds.y.to(dev).contiguous())
p0, c0, _ = T.find_path(n, np.random.default_rng(5))
def solve():
    return dynamic_group_admm(m, 1.0, obj0, 1e-4, 3000, p0, c0, 10, seed=99, n_total=n, local_ids=list(range(n)))
for _ in range(3): r = solve()
torch.cuda.synchronize()
t0 = time.perf_counter(); r = solve(); torch.cuda.synchronize(); print("solve ms", (time.perf_counter()-t0)*1e3, r.iters, r.extra["engine"], "wall_s(kernel)", r.wall_s*1e3)
pr = cProfile.Profile(); pr.enable(); r = solve(); torch.cuda.synchronize(); pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
