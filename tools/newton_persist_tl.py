"""In-kernel timeline of the persistent exact-logistic kernel (chain_persistent_newton.hip): the crew's
refresh stages and the solver's per-phase wait / solve times (s_memrealtime, 10 ns ticks).

    python tools/newton_persist_tl.py [--chord 0.02]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chord", type=float, default=0.02)
    ap.add_argument("--rho", type=float, default=1e-3)
    ap.add_argument("--bg", type=int, default=0, help="background-refresh step threshold (0: kernel default)")
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--gj", action="store_true", help="background refreshes by Gauss-Jordan (not Newton-Schulz)")
    args = ap.parse_args()
    if args.sweep:
        for gj in (False, True):
            for chord in (0.02, 0.1, 0.3):
                for bg in (1, 2):
                    run(chord, bg, args.rho, gj, brief=True)
        return
    run(args.chord, args.bg, args.rho, args.gj)


def run(chord, bg, rho, gj=False, brief=False):
    class A:
        pass
    args = A()
    args.chord, args.bg, args.rho = chord, bg, rho
    if brief:
        print("[%s] " % ("gj" if gj else "ns"), end="")
    from gadmm_amd.data import logistic_synthetic
    from gadmm_amd.engine.chain_engine import NativeChainEngine
    from gadmm_amd.models import LogisticRegression
    from gadmm_amd.parallel.topology import Placement
    from gadmm_amd.oracle.reference import logistic_optimum
    dev = torch.device("cuda", 0)
    ds = logistic_synthetic(24)
    Xf, yf = ds.stacked()
    obj0 = logistic_optimum(Xf.numpy(), yf.numpy(), 24 * 1e-5)
    eng = NativeChainEngine(ds.X.to(dev), ds.y.to(dev), list(range(24)), 24, "logistic", rho=args.rho, obj0=obj0,
                            tol=1e-8, max_iter=2000, lam=1e-5, local_solver="newton", chord=args.chord,
                            max_inner=args.bg if args.bg > 0 else 100, inner_tol=-1.0 if gj else 1e-4)
    eng.set_path(list(range(24)), Placement.contiguous(24, 1), 0)
    if brief:
        ms = []
        for rep in range(3):
            eng.reset()
            r = eng.run_persistent()
            ms.append(r.wall_ms)
        print("chord %.2f bg %d: %d iterations, %.2f ms (median of 3, timeline off), " % (chord, bg, r.iters,
                                                                                         float(np.median(ms))), end="")
        eng.reset()
        eng.run_persistent(timeline_iters=128)
    else:
        for rep in range(3):
            eng.reset()
            r = eng.run_persistent(timeline_iters=128)
            print("solve %d: %d iterations, done %d, %.2f ms" % (rep, r.iters, r.done, r.wall_ms))
    tl = eng.last_timeline[:24, :128, :].astype(np.float64)
    cr = tl[:, :64, :]
    ok = cr[:, :, 3] > 0
    hess = (cr[:, :, 1] - cr[:, :, 0])[ok] / 100.0
    gj = (cr[:, :, 2] - cr[:, :, 1])[ok] / 100.0
    wr = (cr[:, :, 3] - cr[:, :, 2])[ok] / 100.0
    tot = (cr[:, :, 3] - cr[:, :, 0])[ok] / 100.0
    if brief:
        so = tl[:, 64:128, :]
        oks = so[:, :, 2] > 0
        print("median solve %.2f us, steps %.1f, requests/64 it %.1f"
              % (np.median((so[:, :, 2] - so[:, :, 1])[oks]) / 100.0, np.median(so[:, :, 3][oks]),
                 np.mean(so[:, 63, 4])))
        return
    print("crew refresh (us) median / p90: hessian %.2f / %.2f, gauss-jordan %.2f / %.2f, write %.2f / %.2f, "
          "total %.2f / %.2f (%d refreshes)" % (np.median(hess), np.percentile(hess, 90), np.median(gj),
                                                 np.percentile(gj, 90), np.median(wr), np.percentile(wr, 90),
                                                 np.median(tot), np.percentile(tot, 90), ok.sum()))
    so = tl[:, 64:128, :]
    oks = so[:, :, 2] > 0
    wait = (so[:, :, 1] - so[:, :, 0])[oks] / 100.0
    solve = (so[:, :, 2] - so[:, :, 1])[oks] / 100.0
    steps = so[:, :, 3][oks]
    print("solver per phase (us) median / p90: wait-for-inverse %.2f / %.2f, chord solve %.2f / %.2f, steps %.1f / %.1f"
          % (np.median(wait), np.percentile(wait, 90), np.median(solve), np.percentile(solve, 90), np.median(steps),
             np.percentile(steps, 90)))
    # phase cadence: worker 0 (head) start-to-start
    st0 = so[0, :, 0][so[0, :, 0] > 0]
    print("worker 0 iteration period (us): median %.2f" % (np.median(np.diff(st0)) / 100.0))
    # the hop: a worker's phase start against its neighbours' previous solve end (their theta publish)
    if (so[:, :, 6] > 0).any():
        hn, hd, hs = [], [], []
        for w in range(1, 23):
            for i in range(2, 63):
                head = w % 2 == 0
                j = i - 1 if head else i  # the neighbours' phase this one waits for
                ref = max(so[w - 1, j, 2], so[w + 1, j, 2])
                if ref <= 0 or so[w, i, 6] <= 0 or so[w, i, 0] <= 0:
                    continue
                hn.append((so[w, i, 6] - ref) / 100.0)
                hd.append((so[w, i, 7] - ref) / 100.0 if so[w, i, 7] > 0 else np.nan)
                hs.append((so[w, i, 0] - ref) / 100.0)
        print("hop (us, median / p90): neighbours' theta seen %.2f / %.2f, decision seen %.2f / %.2f, phase start "
              "%.2f / %.2f" % (np.median(hn), np.percentile(hn, 90), np.nanmedian(hd), np.nanpercentile(hd, 90),
                               np.median(hs), np.percentile(hs, 90)))
    okl = oks & (so[:, :, 5] > 0)
    if okl.any():  # the pipeline kernel: end of the solve -> the next phase's matrix loaded
        ld = (so[:, :, 5] - so[:, :, 2])[okl] / 100.0
        print("pipeline: end of solve -> next inverse loaded (us) median / p90: %.2f / %.2f"
              % (np.median(ld), np.percentile(ld, 90)))
        per_step = ((so[:, :, 2] - so[:, :, 1]) / np.maximum(so[:, :, 3], 1))[oks] / 100.0
        print("pipeline: solve time per chord step (us) median: %.3f" % np.median(per_step))
    req = so[:, :, 4][oks]
    print("refresh requests per worker after 64 iterations: mean %.1f (1 per iteration = background only)"
          % (np.mean(so[:, 63, 4]) if so.shape[1] > 63 else float("nan")))


if __name__ == "__main__":
    main()
