"""Gram (SYRK) throughput on one MI355X: python tools/gram_bench.py [workers rows dim]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gadmm_amd.ops import linalg
W = int(sys.argv[1]) if len(sys.argv) > 1 else 1
M = int(sys.argv[2]) if len(sys.argv) > 2 else 262144
D = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(W, M, D, dtype=torch.float64, device=dev, generator=g)
y = torch.randn(W, M, dtype=torch.float64, device=dev, generator=g)
for rep in range(3):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    A, b, yy = linalg.gram(X, y)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    fl = W * M * (D + 1) * (D + 2)  # lower triangle incl. diagonal, 2 flops per MAC
    print("gram %dx%dx%d: %.3f s  %.1f TF/s (SYRK flops m*d*(d+1)), %.1f%% of 78.6 TF f64 peak" % (
        W, M, D, t1 - t0, fl / (t1 - t0) / 1e12, fl / (t1 - t0) / 78.6e12 * 100), flush=True)
Xs = X[:, :8192].contiguous(); ys = y[:, :8192].contiguous()
As, bs, yys = linalg.gram(Xs, ys)
ref = torch.bmm(Xs.transpose(1, 2), Xs)
print("check rel err %.2e" % float((As - ref).abs().max() / ref.abs().max()))
