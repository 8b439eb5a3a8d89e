"""Host (numpy, f64) emulation of the exact-logistic GADMM solve (bench config logistic_exact) with two
forms of the chord-Newton local solve, to check the margins recursion numerically before it runs on
the GPU (chain_persistent_newton.hip):

  direct   x' = x - P g(x),  g = -X^T (y sigma(-y X x)) + shift x + cv        (the one-wave kernel)
  rec      y_k = shift x_k + cv;  dx_k = P y_k - B s_k;  x' = x - dx_k;
           z' = z - XP y_k + XB s_k                       (B = P X^T, XP = X P, XB = X B, products once
                                                           per inverse; z_0 = X x_0 exact per solve)

P: the inverse Hessian at the worker's previous final iterate (exact), a fresh one when a step
contracts by less than `chord`. Prints the outer iterations to the 1e-8 gap and the chord steps.
Usage: python tools/newton_recursion_emul.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.data import logistic_synthetic  # noqa: E402
from gadmm_amd.oracle.reference import logistic_optimum  # noqa: E402

N, RHO, LAM, TOL, CHORD = 24, 1e-3, 1e-5, 1e-8, 0.3


def softplus(v):
    return np.logaddexp(0.0, v)


def run(mode):
    ds = logistic_synthetic(N)
    X = ds.X.numpy()
    Y = ds.y.numpy()
    Xf, yf = ds.stacked()
    obj0 = logistic_optimum(Xf.numpy(), yf.numpy(), N * LAM)
    d = X.shape[2]
    th = np.zeros((N, d))
    mu = np.zeros((N, d))
    pend = np.zeros(N, bool)
    Pinv = [None] * N
    steps_hist = []

    def hess_inv(n, x, shift):
        p = 1.0 / (1.0 + np.exp(Y[n] * (X[n] @ x)))
        w = p * (1 - p)
        H = X[n].T @ (X[n] * w[:, None]) + shift * np.eye(d)
        return np.linalg.inv(H)

    def solve(n, x0, cv, shift):
        Xn, yn = X[n], Y[n]
        if Pinv[n] is None:
            Pinv[n] = hess_inv(n, x0, shift)
        P = Pinv[n]
        B = P @ Xn.T
        XP = Xn @ P
        XB = Xn @ B
        x = x0.copy()
        z = Xn @ x
        nd_prev, fresh = 0.0, False
        for k in range(50):
            if mode == "direct":
                z = Xn @ x
            s = yn / (1.0 + np.exp(yn * z))
            if mode == "direct":
                g = -(Xn.T @ s) + shift * x + cv
                dx = P @ g
            else:
                yk = shift * x + cv
                dx = P @ yk - B @ s
                z = z - XP @ yk + XB @ s
            x = x - dx
            mdx = np.abs(dx).max()
            if mdx < 1e-13 * max(1.0, np.abs(x).max()):
                steps_hist.append(k + 1)
                break
            if not fresh and k > 0 and mdx > CHORD * nd_prev:
                P = Pinv[n] = hess_inv(n, x, shift)
                B = P @ Xn.T
                XP = Xn @ P
                XB = Xn @ B
                z = Xn @ x
                fresh, nd_prev = True, 0.0
                continue
            fresh, nd_prev = False, mdx
        else:
            steps_hist.append(50)
        Pinv[n] = hess_inv(n, x, shift)  # the background refresh at the final iterate
        return x

    for it in range(1, 2001):
        for parity in (0, 1):
            new = th.copy()
            for n in range(parity, N, 2):
                left, right = n - 1, n + 1
                tl = th[left] if left >= 0 else 0.0
                tr = th[right] if right < N else 0.0
                if parity == 0 and pend[n]:
                    if left >= 0:
                        mu[n] -= RHO * (tl - th[n])
                    if right < N:
                        mu[n] += RHO * (th[n] - tr)
                cv = mu[n].copy()
                if left >= 0:
                    cv -= RHO * tl
                if right < N:
                    cv -= RHO * tr
                shift = LAM + RHO * ((left >= 0) + (right < N))
                x = solve(n, th[n], cv, shift)
                new[n] = x
                if parity == 1:
                    if left >= 0:
                        mu[n] -= RHO * (tl - x)
                    if right < N:
                        mu[n] += RHO * (x - tr)
                else:
                    pend[n] = True
            th = new
        obj = sum(LAM * 0.5 * th[n] @ th[n] + softplus(-Y[n] * (X[n] @ th[n])).sum() for n in range(N))
        if abs(obj - obj0) < TOL:
            break
    return it, np.array(steps_hist), th


if __name__ == "__main__":
    res = {}
    for mode in ("direct", "rec"):
        it, st, th = run(mode)
        res[mode] = th
        print("%-6s %d iterations, chord steps per solve: median %.1f mean %.2f max %d"
              % (mode, it, np.median(st), st.mean(), st.max()))
    print("max |theta_rec - theta_direct| / max |theta| = %.3e"
          % (np.abs(res["rec"] - res["direct"]).max() / np.abs(res["direct"]).max()))
