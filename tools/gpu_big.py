"""Scale run of the real-shaped config on one MI355X: Gram throughput (f64 MFMA), inverse set-up,
large-d GADMM iteration time. Usage: python tools/gpu_big.py [workers rows dim]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gadmm_amd.data import gaussian_regression
from gadmm_amd.ops import linalg
from gadmm_amd.engine.chain_engine import NativeChainEngine
from gadmm_amd.parallel.topology import Placement
from gadmm_amd.models import LinearRegression

W = int(sys.argv[1]) if len(sys.argv) > 1 else 2
M = int(sys.argv[2]) if len(sys.argv) > 2 else 625_000
D = int(sys.argv[3]) if len(sys.argv) > 3 else 10_000
dev = torch.device("cuda", 0)
t0 = time.perf_counter()
ds = gaussian_regression(W, M, D, seed=0, device=dev)
torch.cuda.synchronize(); t1 = time.perf_counter()
print("generated %d x %d x %d f64 (%.1f GB) in %.2fs" % (W, M, D, W * M * D * 8 / 1e9, t1 - t0), flush=True)
for rep in range(2):
    torch.cuda.synchronize(); t1 = time.perf_counter()
    A, b, yy = linalg.gram(ds.X, ds.y)
    torch.cuda.synchronize(); t2 = time.perf_counter()
    fl = W * M * (D + 1) * (D + 1)  # lower triangle incl. augmented column: ~ m (d+1)^2 flops (x2/2)
    print("gram rep %d: %.3fs  %.1f TF/s (lower-triangle flops)" % (rep, t2 - t1, fl / (t2 - t1) / 1e12), flush=True)
Xs, ys = ds.X[:, :4096].contiguous(), ds.y[:, :4096].contiguous()
As, bs, _ = linalg.gram(Xs.contiguous(), ys.contiguous())
ref = torch.bmm(Xs.transpose(1, 2), Xs)
print("gram check (4096-row slice) rel err %.2e" % float((As - ref).abs().max() / ref.abs().max()), flush=True)
del Xs, ys, As, bs, ref
m = LinearRegression.__new__(LinearRegression)
m.X, m.y, m.lam, m.A, m.b, m.yy = ds.X, ds.y, 0.0, A, b, yy
m.n_local, m.m, m.d = W, M, D
m._chol = {}
torch.cuda.synchronize(); t3 = time.perf_counter()
obj0 = m.optimum()
torch.cuda.synchronize(); t4 = time.perf_counter()
print("optimum %.12e in %.2fs" % (obj0, t4 - t3), flush=True)
rho = 0.5 * M
for mode in ("exact", "identity"):
    torch.cuda.synchronize(); t5 = time.perf_counter()
    eng = NativeChainEngine(ds.X, ds.y, list(range(W)), W, "linear", rho=rho, obj0=obj0, tol=1e-8 * abs(obj0),
                            max_iter=500, precomputed=(A, b, yy), obj_mode=mode, block=8)
    torch.cuda.synchronize(); t6 = time.perf_counter()
    eng.set_path(list(range(W)), Placement.contiguous(W, 1), 0)
    eng.reset()
    r = eng.run()
    torch.cuda.synchronize(); t7 = time.perf_counter()
    print("[%s] inverses %.2fs; GADMM rho=%g: iters=%d done=%d, %.3f s total, %.3f ms/iter, final rel gap %.2e" % (
        mode, t6 - t5, rho, r.iters, r.done, t7 - t6, (t7 - t6) * 1e3 / max(r.iters, 1),
        abs(eng.objective_trace(r.iters)[-1] - obj0) / abs(obj0)), flush=True)
    eng.close()
    del eng
    torch.cuda.empty_cache()
