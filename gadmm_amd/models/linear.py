"""Least-squares consensus problem ``min sum_n 1/2 ||X_n theta - y_n||^2`` (the reference's linear
regression; objective ``group_ADMM_closedForm.m:96-101``, optimum ``opt_sol_closedForm.m:2-3``).

A model instance holds the *local* shards of one rank (``X``: (n_loc, m, d)) and the loop-invariant
sufficient statistics ``A_n = X_n^T X_n``, ``b_n = X_n^T y_n``, ``yy_n = y_n^T y_n`` (kernel K1). All
per-iteration quantities are O(d^2) in these, independent of the shard height m.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops.linalg import gram, spd_inverse, spd_inverse_blocked
from ..utils.env import getenv


def _cg_solve(M: torch.Tensor, r: torch.Tensor, tol: float = 1e-13, maxit: int = 96, check: int = 8):
    """Jacobi-preconditioned conjugate gradients for the SPD system M x = r: x once the TRUE residual
    ||r - M x|| <= tol ||r|| (tested every `check` iterations, one host sync each), None if that takes
    more than `maxit` iterations or a diagonal entry is not positive. Fixed operation sequence
    (deterministic). On a HIP device everything runs in native kernels (csrc/kernels/first_order_big.hip:
    cg_begin / cg_step / cg_resid, one workgroup each, and the block-packed symmetric GEMV for the
    products): a cold solve pays no first-use loading of rocBLAS or of a dozen torch kernels (~0.2 s /
    ~50 ms measured inside the timed set-up)."""
    d = int(M.shape[-1])
    if M.is_cuda:
        return _cg_solve_native(M.contiguous(), r.contiguous(), tol, maxit, check)
    diag = torch.diagonal(M)
    rn0 = float(torch.sqrt((r * r).sum()))
    if rn0 == 0.0:
        return torch.zeros_like(r)
    if not bool((diag > 0).all()):
        return None
    dinv = 1.0 / diag
    x = dinv * r
    res = r - torch.mv(M, x)
    z = dinv * res
    p = z.clone()
    rz = (res * z).sum()
    for k in range(1, maxit + 1):
        q = torch.mv(M, p)
        alpha = rz / (p * q).sum()
        x.add_(alpha * p)
        res.sub_(alpha * q)
        if k % check == 0:
            e = r - torch.mv(M, x)
            if float(torch.sqrt((e * e).sum())) <= tol * rn0:
                return x
        z = dinv * res
        rz_new = (res * z).sum()
        p = z + (rz_new / rz) * p
        rz = rz_new
    return None


def _cg_solve_native(M: torch.Tensor, r: torch.Tensor, tol: float, maxit: int, check: int, comm=None):
    """``comm`` (several ranks): the distributed CG of the large-d optimum -- ``M`` is this rank's LOCAL
    Gram sum and the system matrix is the sum of every rank's, which is never formed: each product is the
    local block-packed GEMV followed by an all-reduce of the d-vector (d-vector
    collectives instead of the one-time d x d all-reduce, 80 KB instead of 800 MB per collective at d =
    10k), and the Jacobi diagonal is all-reduced once. The all-reduced products are bit-identical on every
    rank (the collectives sum in rank order), so every rank runs the same iterations and stops together."""
    import ctypes
    from ..ops import native
    from ..ops.linalg import sym_pack, sym_padded, symv_packed, symv_work_doubles
    lib = native.require()
    P, I = ctypes.c_void_p, ctypes.c_int
    sigs = {"gadmm_cg_begin": [P, P, P, P, P, I, P], "gadmm_cg_begin_diag": [P, P, P, P, P, I, P],
            "gadmm_cg_begin2": [P, P, P, P, P, P, P, I, P],
            "gadmm_cg_step": [P, P, P, P, P, P, P, I, P], "gadmm_cg_resid": [P, P, P, I, P]}
    for name, args in sigs.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = ctypes.c_int, args
    d, dev, st = int(M.shape[-1]), M.device, native.stream_handle()
    dp = sym_padded(d)
    V = torch.zeros((7, dp), dtype=torch.float64, device=dev)  # zero padding: the GEMV reads whole blocks
    b, dinv, x, res, z, p, q = V.unbind(0)
    b[:d].copy_(r)
    sc = torch.zeros((3,), dtype=torch.float64, device=dev)
    ptr = native.ptr
    multi = comm is not None and comm.nranks > 1
    if multi:
        diag = torch.diagonal(M).contiguous()
        comm.allreduce_sum(diag)
        native.check(lib.gadmm_cg_begin_diag(ptr(diag), ptr(b), ptr(dinv), ptr(x), ptr(sc), d, st), "cg_begin_diag")
    else:
        native.check(lib.gadmm_cg_begin(ptr(M), ptr(b), ptr(dinv), ptr(x), ptr(sc), d, st), "cg_begin")
    Mp = sym_pack(M.unsqueeze(0))[0]
    work = torch.empty((symv_work_doubles(d),), dtype=torch.float64, device=dev)

    def symv(v, out):
        symv_packed(Mp, v, out, work, d)
        if multi:
            comm.allreduce_sum(out[:d])  # in place, contiguous view; the padding stays zero
        return out

    head = sc.cpu()
    if float(head[2]) > 0:
        return None
    rn0 = float(head[1]) ** 0.5
    if rn0 == 0.0:
        return torch.zeros_like(r)
    symv(x, q)
    native.check(lib.gadmm_cg_begin2(ptr(b), ptr(dinv), ptr(q), ptr(res), ptr(z), ptr(p), ptr(sc), d, st), "cg_begin2")
    for k in range(1, maxit + 1):
        symv(p, q)
        native.check(lib.gadmm_cg_step(ptr(q), ptr(dinv), ptr(x), ptr(res), ptr(z), ptr(p), ptr(sc), d, st), "cg_step")
        if k % check == 0:
            symv(x, q)
            native.check(lib.gadmm_cg_resid(ptr(b), ptr(q), ptr(sc), d, st), "cg_resid")
            if float(sc[1].item()) ** 0.5 <= tol * rn0:
                return x[:d].clone()
    return None


def _distributed_cg_ok(model) -> bool:
    """The large-d optimum runs the distributed CG (d-vector all-reduces) on HIP devices with d > 256
    (GADMM_OPT_DIST=0: the one-time d x d Gram all-reduce instead)."""
    return (model.A.is_cuda and model.d > 256 and getenv("GADMM_OPT_DIST", "1") != "0"
            and getenv("GADMM_OPT_SOLVER", "native") != "rocsolver"
            and getenv("GADMM_OPT_CG", "1") != "0")


def _resid_sq(X: torch.Tensor, y: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """(1,) device tensor sum_rows (X_row . x - y_row)^2 over the local shards X (n_loc, m, d), f64:
    csrc/kernels/first_order_big.hip:gadmm_resid_sq (fixed-order partials: deterministic)."""
    import ctypes
    from ..ops import native
    lib = native.require()
    fn = lib.gadmm_resid_sq
    P = ctypes.c_void_p
    fn.restype, fn.argtypes = ctypes.c_int, [P, P, P, ctypes.c_long, ctypes.c_int, P, P, P]
    Xc, yc, xc = X.contiguous(), y.contiguous(), x.contiguous()
    rows = int(Xc.numel() // Xc.shape[-1])
    part = torch.empty((4096,), dtype=torch.float64, device=X.device)
    out = torch.empty((1,), dtype=torch.float64, device=X.device)
    native.check(fn(Xc.data_ptr(), yc.data_ptr(), xc.data_ptr(), rows, int(Xc.shape[-1]), part.data_ptr(),
                    out.data_ptr(), native.stream_handle()), "resid_sq")
    return out


def _spd_solve(M: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
    """Solve the SPD normal equations by Cholesky (half the flops of LU, no pivoting); LU only if
    the factorisation reports the matrix is not positive definite. On a HIP device with d > 256 (the
    real-shaped oracle, inside the timed set-up of the 10M x 10k config): Jacobi-preconditioned CG to a
    1e-13 relative residual when the Gram is well conditioned (a tall Gaussian shard: ~20 GEMVs of the
    d x d matrix, a few ms at d = 10k), else the native blocked Gauss-Jordan inverse (f64 MFMA,
    csrc/kernels/spd_inverse_blocked.hip, ~50 ms at d = 10k) and one GEMV. rocSOLVER's potrf / trsv
    spent ~0.3 s there, mostly first-call library loading between their kernels, and was not
    deterministic with ranks sharing a GPU (profiles/r04_real10m)."""
    native_ok = getenv("GADMM_OPT_SOLVER", "native") != "rocsolver"
    if M.is_cuda and M.shape[-1] > 256 and native_ok and getenv("GADMM_OPT_CG", "1") != "0":
        x = _cg_solve(M, r)
        if x is not None:
            return x
    if M.is_cuda and M.shape[-1] > 256 and native_ok:
        st = torch.zeros((1,), dtype=torch.int32, device=M.device)
        inv = spd_inverse_blocked(M.unsqueeze(0), torch.zeros((1, 1), dtype=torch.float64), check_status=False,
                                  status=st)[0, 0]
        if int(st.item()) == 0:
            return torch.mv(inv, r)
        del inv
    L, info = torch.linalg.cholesky_ex(M)
    if int(info.item()) != 0:
        return torch.linalg.solve(M, r)
    return torch.cholesky_solve(r.unsqueeze(-1), L).squeeze(-1)


class LinearRegression:
    kind = "linear"

    def __init__(self, X: torch.Tensor, y: torch.Tensor, lam: float = 0.0):
        self.X = X
        self.y = y
        self.lam = float(lam)  # ridge per worker (the reference uses lambda = 0: GD_DGD_LAG.m:83)
        self.A, self.b, self.yy = gram(X, y)
        self.n_local, self.m, self.d = X.shape
        self._chol = {}

    @property
    def device(self):
        return self.X.device

    def subset(self, idx) -> "LinearRegression":
        """The model of the local workers ``idx`` (in that order), sharing this model's Gram slices
        (no recomputation; the statistics are per worker). Used by elastic recovery: the survivors
        of a failure form a smaller chain on the same device."""
        ix = torch.as_tensor(list(idx), dtype=torch.long, device=self.X.device)
        sub = LinearRegression.__new__(LinearRegression)
        sub.X, sub.y = self.X.index_select(0, ix), self.y.index_select(0, ix)
        sub.lam = self.lam
        sub.A, sub.b, sub.yy = self.A.index_select(0, ix), self.b.index_select(0, ix), self.yy.index_select(0, ix)
        sub.n_local, sub.m, sub.d = int(ix.numel()), self.m, self.d
        sub._chol = {}
        return sub

    # ---- objective / gradient -------------------------------------------------------------------
    def objective(self, theta: torch.Tensor) -> torch.Tensor:
        """Per-worker ``1/2 ||X_n theta_n - y_n||^2 (+ lam/2 ||theta_n||^2)`` via the quadratic form.
        ``theta``: (n_loc, d)."""
        At = torch.bmm(self.A, theta.unsqueeze(-1)).squeeze(-1)
        f = 0.5 * (At * theta).sum(-1) - (self.b * theta).sum(-1) + 0.5 * self.yy
        if self.lam:
            f = f + 0.5 * self.lam * (theta * theta).sum(-1)
        return f

    def objective_direct(self, theta: torch.Tensor) -> torch.Tensor:
        r = torch.bmm(self.X, theta.unsqueeze(-1)).squeeze(-1) - self.y
        f = 0.5 * (r * r).sum(-1)
        if self.lam:
            f = f + 0.5 * self.lam * (theta * theta).sum(-1)
        return f

    def gradient(self, theta: torch.Tensor) -> torch.Tensor:
        """``X_n^T X_n theta_n - X_n^T y_n (+ lam theta_n)`` (GD_DGD_LAG.m:95)."""
        g = torch.bmm(self.A, theta.unsqueeze(-1)).squeeze(-1) - self.b
        if self.lam:
            g = g + self.lam * theta
        return g

    def hmax(self) -> torch.Tensor:
        """Per-worker Lipschitz constants ``lambda_max(X_n^T X_n)`` (LinearRegression_Synthetic.m:33)."""
        return torch.linalg.eigvalsh(self.A)[:, -1] + self.lam

    def hmin(self) -> torch.Tensor:
        return torch.linalg.eigvalsh(self.A)[:, 0] + self.lam

    # ---- closed-form prox: argmin f_n(x) + <mu, x> + rho/2 sum ||x - th_nbr||^2 -------------------
    def prox_factor(self, shift: float) -> torch.Tensor:
        """Cholesky factors of ``A_n + (lam + shift) I`` (cached per shift)."""
        key = float(shift)
        if key not in self._chol:
            eye = torch.eye(self.d, dtype=self.A.dtype, device=self.A.device)
            self._chol[key] = torch.linalg.cholesky(self.A + (self.lam + key) * eye)
        return self._chol[key]

    def prox_inverse(self, shift: float, worker: int) -> torch.Tensor:
        """Cached ``(A_n + (lam + shift) I)^{-1}`` of local worker ``worker`` (the blocked MFMA
        Gauss-Jordan of ops/linalg.py for d > 128), built on first use: a worker only pays for the
        shifts (chain degrees, star hub) it is actually solved with."""
        key = ("inv", float(shift), int(worker))
        if key not in self._chol:
            sh = torch.full((1, 1), self.lam + float(shift), dtype=torch.float64, device=self.A.device)
            self._chol[key] = spd_inverse(self.A[int(worker):int(worker) + 1], sh)[0, 0]
        return self._chol[key]

    def prox_solve(self, idx: torch.Tensor, rhs: torch.Tensor, shifts: torch.Tensor) -> torch.Tensor:
        """Solve ``(A_n + shift_n I) x = rhs_n`` for local workers ``idx``: batched Cholesky solves on
        the CPU / small d; on a HIP device with large d a GEMV with the cached inverse (two
        latency-bound 10k triangular solves per call would dominate), read in place (no gathered
        copy of the d x d inverse)."""
        out = torch.empty_like(rhs)
        use_inv = self.A.is_cuda and self.d > 256
        if use_inv:
            for k, (w, s) in enumerate(zip(idx.tolist(), shifts.tolist())):
                out[k] = torch.mv(self.prox_inverse(s, w), rhs[k])
            return out
        for s in torch.unique(shifts).tolist():
            sel = (shifts == s).nonzero().flatten()
            L = self.prox_factor(s)[idx[sel]]
            out[sel] = torch.cholesky_solve(rhs[sel].unsqueeze(-1), L).squeeze(-1)
        return out

    def inverses(self, shifts) -> torch.Tensor:
        return spd_inverse(self.A, torch.as_tensor(shifts, dtype=torch.float64, device=self.A.device))

    # ---- global oracle ----------------------------------------------------------------------------
    def optimum(self, comm=None, n_total=None) -> float:
        """Optimal objective of the stacked problem: ``x = (sum A_n)^{-1} sum b_n``, evaluated as ``1/2 ||X x - y||^2`` from the raw rows, as
        ``opt_sol_closedForm.m:2-3`` does (the quadratic form ``x'Ax/2 - b'x + y'y/2`` cancels badly:
        ~1e-10 absolute on the E1 problem, more than the margin of its 1e-8 stop).

        Across ranks: at d > 256 on HIP devices a distributed CG whose collectives are
        d-vectors (``_cg_solve_native(comm=...)``); otherwise, or if CG does not converge, the one-time
        all-reduce of the d x d Gram. ``last_optimum_path`` names the one taken."""
        self.last_optimum_path = "local" if comm is None or comm.nranks == 1 else "gram-allreduce"
        As = self.A.sum(0)
        bs = self.b.sum(0)
        yy = self.yy.sum()
        lam_tot = self.lam * (n_total if n_total is not None else self.n_local)
        x = None
        if comm is not None and comm.nranks > 1 and _distributed_cg_ok(self):
            # d-vector collectives only: b, the Jacobi diagonal and one product per CG iteration
            if lam_tot:
                As.diagonal().add_(lam_tot / comm.nranks)  # the ridge split evenly over the rank sums
            bs = bs.contiguous()
            comm.allreduce_sum(bs)
            x = _cg_solve_native(As.contiguous(), bs, 1e-13, 96, 8, comm=comm)
            self.last_optimum_path = "distributed-cg" if x is not None else "gram-allreduce"
            if x is None:  # ill-conditioned: the one-time d x d all-reduce below
                As, bs = self.A.sum(0), self.b.sum(0)
        if x is None and comm is not None and comm.nranks > 1:
            buf = torch.cat([As.reshape(-1), bs, yy.reshape(1)]).contiguous()
            comm.allreduce_sum(buf)
            d = self.d
            As = buf[: d * d].reshape(d, d)
            bs = buf[d * d: d * d + d]
            yy = buf[-1]
        if x is None:
            if lam_tot:  # ridge: the diagonal only (no d x d identity: 800 MB at d = 10k)
                As = As.clone()
                As.diagonal().add_(lam_tot)
            x = _spd_solve(As, bs)
        if self.X.is_cuda and self.d > 256 and self.X.dtype == torch.float64:
            f = 0.5 * _resid_sq(self.X, self.y, x)  # one native pass over the shard at HBM speed
        else:
            r = torch.matmul(self.X.to(x.dtype), x) - self.y.to(x.dtype)  # (n_loc, m) residuals
            f = (0.5 * (r * r).sum()).reshape(1)
        if comm is not None and comm.nranks > 1:
            comm.allreduce_sum(f)
        return float(f.item() + 0.5 * lam_tot * (x @ x).item())

    def optimum_point(self, comm=None) -> torch.Tensor:
        As, bs = self.A.sum(0), self.b.sum(0)
        if comm is not None and comm.nranks > 1:
            buf = torch.cat([As.reshape(-1), bs]).contiguous()
            comm.allreduce_sum(buf)
            As = buf[: self.d * self.d].reshape(self.d, self.d)
            bs = buf[self.d * self.d:]
        return _spd_solve(As, bs)
