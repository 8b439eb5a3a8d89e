"""L2-regularised logistic regression ``sum_n [lam/2 ||theta||^2 + sum_i log(1 + exp(-y_i x_i^T theta))]``
(the reference's logistic problem; objective ``group_ADMM_logistic_GD.m:114``, gradient
``logReg_GD.m:9``, Lipschitz constants ``LogisticRegression_Synthetic.m:43-46``).

Local solvers:
* ``inexact_gd``  — the reference's local step (``logReg_GD.m``): <= 100 GD steps with frozen prox
  shifts, stop when every coordinate moved < 1e-4 (kernel K8 on the GPU);
* ``newton_prox`` — the exact local solve of the dead CVX variant (``group_ADMM_logistic.m``,
  SURVEY.md D2), by damped Newton with the d x d Hessian; needed to reach 1e-8 robustly.
"""
from __future__ import annotations

import torch


def softplus(t: torch.Tensor) -> torch.Tensor:
    return torch.where(t > 30, t + torch.log1p(torch.exp(-t)), torch.log1p(torch.exp(torch.clamp(t, max=30))))


class LogisticRegression:
    kind = "logistic"

    def __init__(self, X: torch.Tensor, y: torch.Tensor, lam: float = 1e-5):
        self.X = X
        self.y = y
        self.lam = float(lam)
        self.n_local, self.m, self.d = X.shape

    @property
    def device(self):
        return self.X.device

    def margins(self, theta: torch.Tensor, idx=None) -> torch.Tensor:
        X = self.X if idx is None else self.X[idx]
        return torch.bmm(X, theta.unsqueeze(-1)).squeeze(-1)

    def objective(self, theta: torch.Tensor, idx=None) -> torch.Tensor:
        y = self.y if idx is None else self.y[idx]
        z = self.margins(theta, idx)
        return self.lam * 0.5 * (theta * theta).sum(-1) + softplus(-y * z).sum(-1)

    def gradient(self, theta: torch.Tensor, idx=None) -> torch.Tensor:
        X = self.X if idx is None else self.X[idx]
        y = self.y if idx is None else self.y[idx]
        z = torch.bmm(X, theta.unsqueeze(-1)).squeeze(-1)
        s = y / (1.0 + torch.exp(y * z))
        return -torch.bmm(X.transpose(1, 2), s.unsqueeze(-1)).squeeze(-1) + self.lam * theta

    def hmax(self) -> torch.Tensor:
        """``1/4 lambda_max(X_n^T X_n) + lam`` (LogisticRegression_Synthetic.m:43-46)."""
        G = torch.bmm(self.X.transpose(1, 2), self.X)
        return 0.25 * torch.linalg.eigvalsh(G)[:, -1].abs() + self.lam

    def hmin(self) -> torch.Tensor:
        return torch.full((self.n_local,), self.lam, dtype=torch.float64, device=self.X.device)

    # ---- local solvers ------------------------------------------------------------------------------
    def inexact_gd(self, idx: torch.Tensor, x0: torch.Tensor, shift: torch.Tensor, step: float,
                   max_inner: int = 100, tol: float = 1e-4):
        """``logReg_GD.m`` for a batch of workers: ``g = grad f(x) + shift``; ``x -= step g``; a worker
        stops when all |dx| < tol (MATLAB vector-`if` semantics). Returns (x, steps_used)."""
        X, y = self.X[idx], self.y[idx]
        Xt = X.transpose(1, 2)
        x = x0.clone()
        active = torch.ones(x.shape[0], dtype=torch.bool, device=x.device)
        used = torch.zeros(x.shape[0], dtype=torch.long, device=x.device)
        for _ in range(max_inner):
            if not bool(active.any()):
                break
            z = torch.bmm(X, x.unsqueeze(-1)).squeeze(-1)
            s = y / (1.0 + torch.exp(y * z))
            g = -torch.bmm(Xt, s.unsqueeze(-1)).squeeze(-1) + self.lam * x + shift
            xn = x - step * g
            conv = (xn - x).abs().lt(tol).all(-1)
            x = torch.where(active.unsqueeze(-1), xn, x)
            used = used + active.long()
            active = active & ~conv
        return x, used

    def newton_prox(self, idx: torch.Tensor, x0: torch.Tensor, lin: torch.Tensor, quad: torch.Tensor,
                    center: torch.Tensor, iters: int = 50, tol: float = 1e-13):
        """Exact argmin of ``f_n(x) + lin^T x + quad/2 ||x||^2 - quad * center^T x`` by Newton
        (CVX's exact local solve). ``quad``: (k,) total proximal weight deg*rho."""
        X, y = self.X[idx], self.y[idx]
        Xt = X.transpose(1, 2)
        x = x0.clone()
        eye = torch.eye(self.d, dtype=x.dtype, device=x.device)
        for _ in range(iters):
            z = torch.bmm(X, x.unsqueeze(-1)).squeeze(-1)
            p = 1.0 / (1.0 + torch.exp(y * z))  # sigma(-y z)
            g = -torch.bmm(Xt, (y * p).unsqueeze(-1)).squeeze(-1) + self.lam * x + lin + quad.unsqueeze(-1) * (x - center)
            w = p * (1 - p)
            H = torch.bmm(Xt * w.unsqueeze(1), X) + (self.lam + quad).view(-1, 1, 1) * eye
            dx = torch.linalg.solve(H, g.unsqueeze(-1)).squeeze(-1)
            x = x - dx
            if float(dx.abs().max()) < tol * max(1.0, float(x.abs().max())):
                break
        return x

    # ---- global oracle ------------------------------------------------------------------------------
    def optimum(self, comm=None, n_total=None, iters: int = 100) -> float:
        """Certified optimum of the stacked problem with ``N lam`` ridge (Newton with all-reduced
        gradient/Hessian; replaces the reference's 100k-iteration GD oracle,
        GD_DGD_LAG_logistic.m:131-133)."""
        d = self.d
        N = n_total if n_total is not None else self.n_local
        Xf = self.X.reshape(-1, d)
        yf = self.y.reshape(-1)
        x = torch.zeros(d, dtype=torch.float64, device=self.X.device)
        eye = torch.eye(d, dtype=torch.float64, device=self.X.device)
        for _ in range(iters):
            z = yf * (Xf @ x)
            p = 1.0 / (1.0 + torch.exp(z))
            g = -(Xf.T @ (yf * p))
            w = p * (1 - p)
            H = Xf.T @ (Xf * w.unsqueeze(-1))
            if comm is not None and comm.nranks > 1:
                buf = torch.cat([g, H.reshape(-1)]).contiguous()
                comm.allreduce_sum(buf)
                g, H = buf[:d], buf[d:].reshape(d, d)
            g = g + N * self.lam * x
            H = H + N * self.lam * eye
            dx = torch.linalg.solve(H, g)
            x = x - dx
            if float(dx.abs().max()) < 1e-15 * max(1.0, float(x.abs().max())):
                break
        z = yf * (Xf @ x)
        loss = softplus(-z).sum()
        if comm is not None and comm.nranks > 1:
            t = loss.reshape(1).clone()
            comm.allreduce_sum(t)
            loss = t[0]
        return float(N * self.lam * 0.5 * (x @ x) + loss)
