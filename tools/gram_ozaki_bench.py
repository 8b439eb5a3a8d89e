"""The int8 Ozaki Gram (csrc/kernels/gram_ozaki.hip) against the f64-MFMA Gram: accuracy (entries relative
to sqrt(A_aa A_bb), against an f64 reference) and time, at a given shard shape.
Usage: python tools/gram_ozaki_bench.py N m d [reps]"""
import os
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from gadmm_amd.ops.linalg import gram, gram_ozaki  # noqa: E402

N, m, d = (int(v) for v in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(0)
X = torch.randn((N, m, d), dtype=torch.float64, device=dev, generator=g)
y = torch.randn((N, m), dtype=torch.float64, device=dev, generator=g)


def timed(f):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = f()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts), out


os.environ["GADMM_GRAM_OZAKI"] = "0"  # gram() would dispatch large shards to the Ozaki path itself
t64, (A64, b64, yy64) = timed(lambda: gram(X, y))
del os.environ["GADMM_GRAM_OZAKI"]
toz, (Aoz, boz, yyoz) = timed(lambda: gram_ozaki(X, y))
flops = 2.0 * N * m * (d + 1) * (d + 2) / 2
scale = torch.sqrt(torch.diagonal(A64, dim1=1, dim2=2))
rel = ((Aoz - A64).abs() / (scale.unsqueeze(2) * scale.unsqueeze(1))).max().item()
relb = ((boz - b64).abs() / (scale * yy64.sqrt().unsqueeze(1))).max().item()
relyy = ((yyoz - yy64).abs() / yy64).max().item()
print("shape N=%d m=%d d=%d" % (N, m, d))
print("f64 MFMA gram : %.4f s  %.1f TF/s" % (t64, flops / t64 / 1e12))
print("ozaki int8    : %.4f s  %.1f TF/s-equivalent  (%.2fx)" % (toz, flops / toz / 1e12, t64 / toz))
print("max |A_oz - A_f64| / sqrt(A_aa A_bb) = %.3e   b: %.3e   yy: %.3e" % (rel, relb, relyy), flush=True)
if m * d <= 4e8:  # an independent reference: torch's f64 GEMM
    Ar = torch.bmm(X.transpose(1, 2), X)
    r64 = ((A64 - Ar).abs() / (scale.unsqueeze(2) * scale.unsqueeze(1))).max().item()
    roz = ((Aoz - Ar).abs() / (scale.unsqueeze(2) * scale.unsqueeze(1))).max().item()
    print("vs torch bmm: f64-MFMA %.3e   ozaki %.3e" % (r64, roz), flush=True)
