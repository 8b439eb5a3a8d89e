"""Quick on-GPU correctness + timing check of the native path (development tool)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gadmm_amd.data import linear_synthetic, logistic_synthetic
from gadmm_amd.ops import linalg, native
from gadmm_amd.engine.chain_engine import NativeChainEngine
from gadmm_amd.parallel.topology import Placement
from gadmm_amd.oracle import reference as R

dev = torch.device("cuda:0")
print("device", torch.cuda.get_device_name(0), flush=True)
ds = linear_synthetic(24)
X, y = ds.X.to(dev), ds.y.to(dev)
A, b, yy = linalg.gram(X, y)
A0, b0, yy0 = linalg.gram_torch(ds.X, ds.y)
print("gram err", (A.cpu() - A0).abs().max().item(), (b.cpu() - b0).abs().max().item(), (yy.cpu() - yy0).abs().max().item())
# tall shard split-K check
g = torch.Generator().manual_seed(0)
Xt = torch.randn(3, 5000, 70, dtype=torch.float64, generator=g); yt = torch.randn(3, 5000, dtype=torch.float64, generator=g)
A1, b1, yy1 = linalg.gram(Xt.to(dev), yt.to(dev)); A2, b2, yy2 = linalg.gram_torch(Xt, yt)
print("gram tall err", ((A1.cpu() - A2).abs().max() / A2.abs().max()).item(), ((b1.cpu() - b2).abs().max() / b2.abs().max()).item())
Minv = linalg.spd_inverse(A, torch.tensor([3.0, 6.0], dtype=torch.float64, device=dev))
Mref = linalg.spd_inverse_torch(A0, torch.tensor([[3.0, 6.0]] * 24, dtype=torch.float64))
print("inv err", ((Minv.cpu() - Mref).abs().max() / Mref.abs().max()).item())
Xf, yf = ds.stacked()
obj0 = R.opt_linear(Xf.numpy(), yf.numpy())
pl = Placement.contiguous(24, 1)
for rho, e4, e8 in ((3, 784, 1373), (5, 434, 758), (7, 248, 428)):
    eng = NativeChainEngine(X, y, list(range(24)), 24, "linear", rho=rho, obj0=obj0, tol=1e-4, max_iter=3000, block=16)
    eng.set_path(list(range(24)), pl, 0)
    eng.reset()
    r4 = eng.run()
    eng.set_targets(obj0, 1e-8); eng.reset()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    r8 = eng.run()
    torch.cuda.synchronize(); t1 = time.perf_counter()
    print("rho", rho, "iters 1e-4", r4.iters, "(want", e4, ") 1e-8", r8.iters, "(want", e8, ") wall_ms", round((t1 - t0) * 1e3, 3),
          "engine_ms", round(r8.wall_ms, 3), "graph", eng.graph_ok(), "launched", r8.iterations_launched, flush=True)
    tr = eng.objective_trace(r8.iters)
    ref = R.gadmm_linear(ds.X.numpy(), ds.y.numpy(), rho, 40, obj0, 1e-30)
    print("   trace max rel diff first 40:", np.max(np.abs(tr[:40] - np.array(ref.obj)) / np.abs(np.array(ref.obj))))
    eng.close()
# eager
eng = NativeChainEngine(X, y, list(range(24)), 24, "linear", rho=3, obj0=obj0, tol=1e-8, max_iter=3000, block=16)
eng.set_path(list(range(24)), pl, 0); eng.reset()
t0 = time.perf_counter(); r = eng.run(use_graph=False); torch.cuda.synchronize(); print("eager iters", r.iters, "ms", (time.perf_counter()-t0)*1e3)
# logistic
dl = logistic_synthetic(24)
Xl, yl = dl.X.to(dev), dl.y.to(dev)
Xlf, ylf = dl.stacked()
obj0l = R.logistic_optimum(Xlf.numpy(), ylf.numpy(), 24e-5)
for rho, want in ((2e-4, 53), (3e-4, 274)):
    eng = NativeChainEngine(Xl, yl, list(range(24)), 24, "logistic", rho=rho, obj0=obj0l, tol=1e-4, max_iter=400,
                            lam=1e-5, step=2.2, max_inner=100, inner_tol=1e-4, block=8)
    eng.set_path(list(range(24)), pl, 0); eng.reset()
    torch.cuda.synchronize(); t0 = time.perf_counter(); r = eng.run(); torch.cuda.synchronize()
    print("logistic rho", rho, "iters", r.iters, "want", want, "ms", round((time.perf_counter() - t0) * 1e3, 3), flush=True)
print("OK")
# persistent
for rho, e4, e8 in ((3, 784, 1373), (5, 434, 758), (7, 248, 428)):
    eng = NativeChainEngine(X, y, list(range(24)), 24, "linear", rho=rho, obj0=obj0, tol=1e-4, max_iter=3000, block=16)
    eng.set_path(list(range(24)), pl, 0)
    eng.reset(); r4 = eng.run_persistent()
    eng.set_targets(obj0, 1e-8)
    best = 1e9
    for k in range(5):
        eng.reset(); torch.cuda.synchronize(); t0 = time.perf_counter(); r8 = eng.run_persistent(); torch.cuda.synchronize(); best = min(best, time.perf_counter() - t0)
    tr = eng.objective_trace(r8.iters)
    ref = R.gadmm_linear(ds.X.numpy(), ds.y.numpy(), rho, 40, obj0, 1e-30)
    print("persistent rho", rho, "iters", r4.iters, r8.iters, "want", e4, e8, "best ms", round(best * 1e3, 3),
          "us/iter", round(best * 1e6 / r8.iters, 3), "trace diff", np.max(np.abs(tr[:40] - np.array(ref.obj)) / np.abs(np.array(ref.obj))), flush=True)
    eng.close()
print("OK2")
