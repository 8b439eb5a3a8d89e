"""Reference-semantics oracle (NumPy, float64, one Python loop iteration per logical worker).

This is the executable *specification* the rest of the framework is tested against: it follows
the reference algorithms step by step (including their quirks) with no batching, no devices and no
communication. It is deliberately slow and literal; the framework's batched torch path and the
HIP engine must reproduce its iteration counts and traces.

Citations are to the MATLAB reference at /root/reference.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np


@dataclass
class OracleResult:
    obj: List[float] = field(default_factory=list)
    loss: List[float] = field(default_factory=list)
    iters: int = 0
    com_cost: List[float] = field(default_factory=list)
    theta: Optional[np.ndarray] = None  # (N, d) final primal iterates
    dual: Optional[np.ndarray] = None   # (N, d) final duals (edge or per-worker form)


def _lin_obj(X, y, theta):
    r = X @ theta - y
    return 0.5 * float(r @ r)


def _log_obj(X, y, theta, lam):
    return lam * 0.5 * float(theta @ theta) + float(np.sum(np.log1p(np.exp(-y * (X @ theta)))))


def opt_linear(X_fede: np.ndarray, y_fede: np.ndarray) -> float:
    """Normal-equation optimum of the stacked least squares (``opt_sol_closedForm.m:2-3``)."""
    x = np.linalg.solve(X_fede.T @ X_fede, X_fede.T @ y_fede)
    return _lin_obj(X_fede, y_fede, x)


def gadmm_linear(X: np.ndarray, y: np.ndarray, rho: float, max_iter: int, obj0: float,
                 acc: float) -> OracleResult:
    """GADMM, closed-form local solve, edge duals (``group_ADMM_closedForm.m``).

    ``X``: (N, m, d), ``y``: (N, m). Worker n (0-based) is a head when n is even (MATLAB odd).
    Head/tail RHS ``H^T y + lam_{n-1} - lam_n + rho th_{n-1} + rho th_{n+1}`` (:15-29, :43-45),
    dual ``lam_n += rho (th_n - th_{n+1})`` (:93-95), objective/stop (:96-108).
    """
    N, m, d = X.shape
    lam = np.zeros((N, d))
    th = np.zeros((N, d))
    res = OracleResult(iters=max_iter)

    def solve(n):
        H, Y = X[n], y[n]
        rhs = H.T @ Y
        deg = 0
        if n > 0:
            rhs = rhs + lam[n - 1] + rho * th[n - 1]
            deg += 1
        if n < N - 1:
            rhs = rhs - lam[n] + rho * th[n + 1]
            deg += 1
        th[n] = np.linalg.solve(H.T @ H + deg * rho * np.eye(d), rhs)

    for it in range(1, max_iter + 1):
        for n in range(0, N, 2):
            solve(n)
        for n in range(1, N, 2):
            solve(n)
        for n in range(N - 1):
            lam[n] = lam[n] + rho * (th[n] - th[n + 1])
        obj = sum(_lin_obj(X[n], y[n], th[n]) for n in range(N))
        res.obj.append(obj)
        res.loss.append(abs(obj - obj0))
        if res.loss[-1] < acc:
            res.iters = it
            break
    res.theta, res.dual = th, lam
    return res


def _chain_neighbours(path: Sequence[int], pos: int):
    N = len(path)
    l = path[pos - 1] if pos > 0 else None
    r = path[pos + 1] if pos < N - 1 else None
    return l, r


def dgadmm_linear(X: np.ndarray, y: np.ndarray, rho: float, max_iter: int, obj0: float, acc: float,
                  path: Sequence[int], path_cost: Sequence[float], coherence: float,
                  rechain: Optional[Callable[[int], tuple]] = None) -> OracleResult:
    """D-GADMM with per-worker aggregated duals (``dynamic_group_ADMM_closedForm.m``).

    ``path``: 0-based permutation (chain position -> worker). Every ``coherence`` iterations
    (``i > 1 and i % coherence == 0``, :18-21) ``rechain(i)`` returns a new ``(path, path_cost)``.
    ``com_cost`` adds ``sum(path_cost)`` once per *head* worker per iteration (quirk, :51-55).
    RHS ``H^T y - mu + rho th_l + rho th_r`` (:84-86); dual update (:153-168).
    """
    N, m, d = X.shape
    mu = np.zeros((N, d))
    th = np.zeros((N, d))
    res = OracleResult(iters=max_iter)
    path = list(path)
    path_cost = list(path_cost)
    cc = 0.0
    for it in range(1, max_iter + 1):
        if it > 1 and coherence and it % coherence == 0 and rechain is not None:
            path, path_cost = rechain(it)
            path = list(path)
        for phase in (0, 1):
            for pos in range(phase, N, 2):
                w = path[pos]
                l, r = _chain_neighbours(path, pos)
                if phase == 0:
                    cc += float(np.sum(path_cost))
                H, Y = X[w], y[w]
                rhs = H.T @ Y - mu[w]
                deg = 0
                if l is not None:
                    rhs = rhs + rho * th[l]
                    deg += 1
                if r is not None:
                    rhs = rhs + rho * th[r]
                    deg += 1
                th[w] = np.linalg.solve(H.T @ H + deg * rho * np.eye(d), rhs)
            if phase == 0:
                pass
        for pos in range(N):
            w = path[pos]
            l, r = _chain_neighbours(path, pos)
            upd = np.zeros(d)
            if r is not None:
                upd += rho * (th[w] - th[r])
            if l is not None:
                upd -= rho * (th[l] - th[w])
            mu[w] = mu[w] + upd
        obj = sum(_lin_obj(X[n], y[n], th[n]) for n in range(N))
        res.obj.append(obj)
        res.loss.append(abs(obj - obj0))
        res.com_cost.append(cc)
        if res.loss[-1] < acc:
            res.iters = it
            break
    res.theta, res.dual = th, mu
    return res


def std_admm_linear(X: np.ndarray, y: np.ndarray, rho: float, max_iter: int, obj0: float,
                    acc: float) -> OracleResult:
    """Star ADMM with worker N as hub holding a shard (``standared_ADMM.m``)."""
    N, m, d = X.shape
    lam = np.zeros((N, d))
    th = np.zeros((N, d))
    hub = N - 1
    res = OracleResult(iters=max_iter)
    I = np.eye(d)
    for it in range(1, max_iter + 1):
        for n in range(N - 1):
            H, Y = X[n], y[n]
            th[n] = np.linalg.solve(H.T @ H + rho * I, H.T @ Y - lam[n] + rho * th[hub])
        H, Y = X[hub], y[hub]
        C1 = lam[: N - 1].sum(axis=0)
        t1 = rho * th[: N - 1].sum(axis=0)
        th[hub] = np.linalg.solve(H.T @ H + (N - 1) * rho * I, H.T @ Y + C1 + t1)
        for n in range(N - 1):
            lam[n] = lam[n] + rho * (th[n] - th[hub])
        obj = sum(_lin_obj(X[n], y[n], th[n]) for n in range(N))
        res.obj.append(obj)
        res.loss.append(abs(obj - obj0))
        if res.loss[-1] < acc:
            res.iters = it
            break
    res.theta, res.dual = th, lam
    return res


def logreg_gd(H, Y, x, C1, C2, t1, t2, lam, step, max_inner=100, tol=1e-4):
    """Local inexact solver (``logReg_GD.m``): <= 100 GD steps, stop when *all* |dx| < tol."""
    for _ in range(max_inner):
        g = -(H.T @ (Y / (1.0 + np.exp(Y * (H @ x))))) + lam * x - C1 + C2 + t1 + t2
        x_prev = x
        x = x - step * g
        if np.all(np.abs(x - x_prev) < tol):
            break
    return x


def gadmm_logistic_gd(X: np.ndarray, y: np.ndarray, rho: float, max_iter: int, obj0: float,
                      lam: float, acc: float, step: float) -> OracleResult:
    """GADMM logistic with frozen (linearised) prox terms (``group_ADMM_logistic_GD.m``)."""
    N, m, d = X.shape
    dual = np.zeros((N, d))
    th = np.zeros((N, d))
    res = OracleResult(iters=max_iter)
    z = np.zeros(d)

    def update(n):
        C1 = dual[n - 1] if n > 0 else z
        t1 = rho * (th[n] - th[n - 1]) if n > 0 else z
        C2 = dual[n] if n < N - 1 else z
        t2 = rho * (th[n] - th[n + 1]) if n < N - 1 else z
        th[n] = logreg_gd(X[n], y[n], th[n].copy(), C1, C2, t1, t2, lam, step)

    for it in range(1, max_iter + 1):
        for n in range(0, N, 2):
            update(n)
        for n in range(1, N, 2):
            update(n)
        for n in range(N - 1):
            dual[n] = dual[n] + rho * (th[n] - th[n + 1])
        obj = sum(_log_obj(X[n], y[n], th[n], lam) for n in range(N))
        res.obj.append(obj)
        res.loss.append(abs(obj - obj0))
        if res.loss[-1] < acc:
            res.iters = it
            break
    res.theta, res.dual = th, dual
    return res


def dual_averaging(X: np.ndarray, y: np.ndarray, max_iter: int, obj0: float, acc: float,
                   alpha: float, logistic_eta: Optional[float] = None) -> OracleResult:
    """Chain dual averaging with in-place (Gauss-Seidel) Z sweep (``dual_averaging.m:15-70``)."""
    N, m, d = X.shape
    th = np.zeros((N, d))
    Z = np.zeros((N, d))
    res = OracleResult(iters=max_iter)
    for it in range(1, max_iter + 1):
        for n in range(N):
            H, Y = X[n], y[n]
            if logistic_eta is None:
                g = H.T @ (H @ th[n]) - H.T @ Y
            else:
                g = -(H.T @ (Y / (1.0 + np.exp(Y * (H @ th[n]))))) + logistic_eta * th[n]
            if n == 0:
                zn = Z[1] + g
            elif n == N - 1:
                zn = Z[N - 2] + g
            else:
                zn = 0.5 * Z[n + 1] + 0.5 * Z[n - 1] + g
            th[n] = -alpha * zn
            Z[n] = zn
        if logistic_eta is None:
            obj = sum(_lin_obj(X[n], y[n], th[n]) for n in range(N))
        else:
            obj = sum(_log_obj(X[n], y[n], th[n], logistic_eta) for n in range(N))
        res.obj.append(obj)
        res.loss.append(abs(obj - obj0))
        if res.loss[-1] < acc:
            res.iters = it
            break
    res.theta = th
    return res


def logistic_optimum(X_fede: np.ndarray, y_fede: np.ndarray, lam_total: float,
                     iters: int = 100) -> float:
    """Newton's method on ``lam_total/2 |x|^2 + sum softplus(-y x^T a)`` (certified optimum
    replacing the reference's CVX ``opt_sol_logistic.m:13-24`` / last-GD-iterate oracle)."""
    d = X_fede.shape[1]
    x = np.zeros(d)
    for _ in range(iters):
        z = y_fede * (X_fede @ x)
        s = 1.0 / (1.0 + np.exp(z))
        g = -(X_fede.T @ (y_fede * s)) + lam_total * x
        w = s * (1 - s)
        Hs = X_fede.T @ (X_fede * w[:, None]) + lam_total * np.eye(d)
        dx = np.linalg.solve(Hs, g)
        x = x - dx
        if np.linalg.norm(dx) < 1e-15 * max(1.0, np.linalg.norm(x)):
            break
    return _log_obj(X_fede, y_fede, x, lam_total)
