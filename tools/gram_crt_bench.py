"""A/B of the int8 Grams on one MI355X: the digit scheme (gram_ozaki) vs CRT slicing (gram_crt) vs the
f64-MFMA kernel, same data, best of ``reps`` after a warm-up, and the entrywise agreement of the two int8
results. Shapes: ``N x m x d`` arguments, default the real10m per-GPU shape (2 x 625000 x 10000)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from gadmm_amd.ops import linalg


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    shapes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]] or [(2, 625000, 10000)]
    dev = torch.device("cuda", 0)
    for N, m, d in shapes:
        g = torch.Generator(device=dev)
        g.manual_seed(0)
        X = torch.randn((N, m, d), dtype=torch.float64, device=dev, generator=g)
        y = torch.randn((N, m), dtype=torch.float64, device=dev, generator=g)
        reps = 2 if m * d > 1e9 else 4
        flop = 2.0 * N * m * (d + 1) * (d + 2) / 2
        out = {}
        for name, fn in (("crt", lambda: linalg.gram_crt(X, y)), ("digits", lambda: linalg.gram_ozaki(X, y)),
                         ("f64", lambda: linalg._gram_f64(X, y, None, None))):
            t = timed(fn, reps)
            out[name] = fn()[0]
            print("%dx%dx%d %-7s %8.4f s  %6.1f TF/s (f64-equivalent)" % (N, m, d, name, t, flop / t / 1e12), flush=True)
        sc = torch.sqrt(torch.diagonal(out["f64"], dim1=1, dim2=2))
        nrm = sc.unsqueeze(2) * sc.unsqueeze(1)
        for k in ("crt", "digits"):
            print("  %s vs f64-mfma: max |diff| / sqrt(A_aa A_bb) = %.3g" % (k, float(((out[k] - out["f64"]).abs() / nrm).max())))
        del X, y, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
