"""Stage times of the large-d optimum oracle (models/linear.py:LinearRegression.optimum) at the real10m
shape: python tools/optimum_timing.py [workers rows_per_worker dim]. Prints ms per stage (device-synced)
for three calls, and which solve path the CG attempt took."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from gadmm_amd.data import gaussian_regression
from gadmm_amd.models import LinearRegression
from gadmm_amd.models import linear as L


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 625000
    d = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
    dev = torch.device("cuda", 0)
    ds = gaussian_regression(n, rows, d, seed=0, labels="linear", device=dev)
    m = LinearRegression(ds.X, ds.y)
    torch.cuda.synchronize()

    def t():
        torch.cuda.synchronize()
        return time.perf_counter()

    for rep in range(3):
        t0 = t()
        As, bs = m.A.sum(0), m.b.sum(0)
        t1 = t()
        x = L._cg_solve(As, bs)
        t2 = t()
        path = "cg"
        if x is None:
            path = "gauss-jordan"
            x = L._spd_solve(As, bs)
        t3 = t()
        r = torch.matmul(m.X, x) - m.y
        f = float(0.5 * (r * r).sum())
        t4 = t()
        obj = m.optimum()
        t5 = t()
        print("rep %d: sums %.1f ms, %s %.1f ms (+ fallback %.1f), residual %.1f ms | optimum() %.1f ms, f %.10e / %.10e"
              % (rep, 1e3 * (t1 - t0), path, 1e3 * (t2 - t1), 1e3 * (t3 - t2), 1e3 * (t4 - t3), 1e3 * (t5 - t4), f, obj),
              flush=True)


if __name__ == "__main__":
    main()
