"""First-order baselines of the reference: GD, DGD, LAG-PS, LAG-WK, cyclic IAG, randomized IAG
(``GD_DGD_LAG.m`` linear, ``GD_DGD_LAG_logistic.m`` logistic).

Realisation on the fabric:
* GD: the server step ``theta -= alpha * sum_n grad_n(theta)`` is an all-reduce of the local
  gradient sums; theta stays replicated on every rank.
* DGD: each worker steps on the average of its own and its chain neighbours' gradients; boundary
  gradients cross ranks by p2p (the same chain plan as GADMM).
* LAG-PS / LAG-WK: rank 0 plays the server and keeps the table of the latest uploaded gradient of
  every worker. Every iteration each rank sends a 1-double trigger count and, only if non-zero, the
  (row id, gradient) rows of its triggered workers (conditional, data-dependent uploads); the server
  steps with the table sum and broadcasts theta. Bytes are counted exactly.
* cIAG / RIAG: one worker refreshes per iteration and uploads its row to the server. RIAG's draw
  uses an RNG seeded identically on every rank (no message).

Native: when the workers live on GPUs and d <= 128, each algorithm runs as ONE persistent kernel
launch per GPU (``engine/first_order.py``, ``csrc/kernels/first_order.hip``): one rank, or several
ranks (contiguous segments) over the xGMI fabric, where every upload is a device-initiated push into
the reading GPUs (the replicated server's table on every rank; LAG's conditional uploads announced by
a one-granule flag; DGD rows to the chain neighbours' ranks) and the returned ``bytes_sent`` is the
exact payload that crossed between GPUs. ``backend="torch"`` forces the implementation below (the
test oracle, and the path for CPU ranks / non-contiguous placements).

Faithful quirks (``faithful=True``): gradients start as ``ones`` (GD_DGD_LAG.m:44-67);
LAG-PS refreshes worker 1 every iteration (timing side effect, :204-209); LAG does nothing before
``iter > triggerslot = 10``; a communication unit is still counted every 1000 quiet iterations
(:246-251); logistic GD's first step uses worker 1's gradient (GD_DGD_LAG_logistic.m:97); logistic
LAG/IAG stop at ``accuracy``, GD/DGD never stop early.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import numpy as np
import torch

from ..parallel.comm import Comm, LocalComm
from ..parallel.topology import Placement, chain_plan
from .base import RunResult, Stopper, total_bytes, global_objective, run_bytes

TRIGGERSLOT = 10


class _Ctx:
    def __init__(self, model, local_ids, n_total, comm, placement):
        self.model = model
        self.comm = comm if comm is not None else LocalComm()
        self.placement = placement if placement is not None else Placement.contiguous(n_total, self.comm.nranks)
        self.local_ids = [int(w) for w in local_ids]
        self.n_total = n_total
        self.d = model.d
        self.dev = model.device
        self.lidx = {w: i for i, w in enumerate(self.local_ids)}
        self.snap = self.comm.stats.snapshot()

    def allsum(self, t: torch.Tensor) -> torch.Tensor:
        t = t.contiguous()
        if self.comm.nranks > 1:
            self.comm.allreduce_sum(t)
        return t

    def grad_sum(self, theta: torch.Tensor) -> torch.Tensor:
        """sum over ALL workers of grad f_n(theta) (theta replicated)."""
        g = self.model.gradient(theta.unsqueeze(0).expand(len(self.local_ids), -1).contiguous()).sum(0)
        return self.allsum(g.clone())

    def obj(self, theta: torch.Tensor) -> float:
        f = self.model.objective(theta.unsqueeze(0).expand(len(self.local_ids), -1).contiguous())
        return global_objective(self.comm, f, self.local_ids, self.n_total)

    def obj_per_worker(self, theta_loc: torch.Tensor) -> float:
        return global_objective(self.comm, self.model.objective(theta_loc), self.local_ids, self.n_total)

    def worker_grad(self, w: int, theta: torch.Tensor) -> torch.Tensor:
        i = self.lidx[w]
        return self.model.gradient(theta.unsqueeze(0), idx=[i])[0] if self.model.kind == "logistic" \
            else (self.model.A[i] @ theta - self.model.b[i] + self.model.lam * theta)


def global_constants(model, comm: Optional[Comm] = None) -> Dict[str, object]:
    """Hmax per worker, Hmax_all and the GD step 1/Hmax_all (GD_DGD_LAG.m:19-47; logistic
    GD_DGD_LAG_logistic.m:24). One all-reduce of the d x d Gram / all-gather of Hmax."""
    comm = comm if comm is not None else LocalComm()
    big = int(model.d) > 128
    if big and model.kind == "linear":
        G = model.A.sum(0).contiguous()  # the cached Grams (K1): no second pass over a 100 GB shard
    else:
        G = torch.bmm(model.X.transpose(1, 2), model.X).sum(0).contiguous()
    if comm.nranks > 1:
        comm.allreduce_sum(G)
    if big:  # Lanczos instead of a dense eigensolve of a 10k x 10k matrix (K12 of SURVEY.md §2.5)
        lo, hi = extreme_eigs(G)
        ev = torch.tensor([lo, hi], dtype=torch.float64)
    else:
        ev = torch.linalg.eigvalsh(G)
    if model.kind == "linear":
        hmax_all = float(ev[-1])
    else:
        hmax_all = 0.25 * float(ev[-1]) + model.lam
    if big and model.kind == "linear":
        hmax_loc = torch.tensor([extreme_eigs(model.A[i])[1] for i in range(int(model.n_local))],
                                dtype=torch.float64, device=model.A.device) + model.lam
    else:
        hmax_loc = model.hmax()
    return {"hmax_local": hmax_loc, "hmax_all": hmax_all, "stepsize": 1.0 / hmax_all,
            "cond": float(ev[-1] / ev[0]) if float(ev[0]) > 0 else float("inf")}


def extreme_eigs(M: torch.Tensor, k: int = 96, seed: int = 0):
    """(lambda_min, lambda_max) of a symmetric matrix by Lanczos with full reorthogonalisation: ``k``
    GEMVs with M (on its device) and a k x k tridiagonal eigensolve. The extreme Ritz values converge
    first; at k = 96 they match a dense eigensolve to ~1e-12 relative on the real-shaped Grams
    (tests/test_algorithms.py::test_lanczos_extreme_eigs)."""
    d = int(M.shape[0])
    k = min(k, d)
    g = torch.Generator(device="cpu").manual_seed(seed)
    v = torch.randn(d, generator=g, dtype=torch.float64).to(M.device)
    v = v / torch.linalg.norm(v)
    V = torch.zeros((k, d), dtype=torch.float64, device=M.device)
    alpha = torch.zeros(k, dtype=torch.float64)
    beta = torch.zeros(k, dtype=torch.float64)
    m = k
    for j in range(k):
        V[j] = v
        w = M @ v
        a = float(w @ v)
        alpha[j] = a
        w = w - V[: j + 1].T @ (V[: j + 1] @ w)  # full reorthogonalisation (twice is enough)
        w = w - V[: j + 1].T @ (V[: j + 1] @ w)
        b = float(torch.linalg.norm(w))
        if j + 1 < k:
            beta[j] = b
            if b < 1e-300:
                m = j + 1
                break
            v = w / b
    Tm = torch.diag(alpha[:m]) + torch.diag(beta[: m - 1], 1) + torch.diag(beta[: m - 1], -1)
    ev = torch.linalg.eigvalsh(Tm)
    return float(ev[0]), float(ev[-1])


def _gather_hmax(ctx: _Ctx, hmax_local: torch.Tensor) -> torch.Tensor:
    full = torch.zeros(ctx.n_total, dtype=torch.float64, device=ctx.dev)
    for w, i in ctx.lidx.items():
        full[w] = hmax_local[i]
    return ctx.allsum(full)


def _fo_engine(ctx: _Ctx, backend: str, alg: str = "GD"):
    """The persistent first-order engine when this run can use it (None -> torch path). Collective
    on several ranks (the eligibility is agreed)."""
    if backend == "torch":
        return None
    from ..engine.first_order import FirstOrderEngine
    from ..engine.first_order_big import FirstOrderBigEngine

    ok = FirstOrderEngine.eligible(ctx.model, ctx.comm, ctx.n_total, ctx.local_ids, ctx.placement, alg)
    if ok:
        return FirstOrderEngine.get(ctx.model, ctx.comm, ctx.placement, ctx.n_total)
    # d > 128, linear: the stream-ordered large-d engine (packed Grams, device stop rule)
    big = getattr(ctx.model, "kind", "") == "linear" and int(ctx.model.d) > 128
    if big and ctx.comm.nranks > 1:  # collective: every rank takes the same path
        from ..engine.first_order import _all_ok
        big = _all_ok(FirstOrderBigEngine.eligible(ctx.model, ctx.comm, ctx.n_total, ctx.local_ids, ctx.placement,
                                                   alg), ctx.comm)
    elif big:
        big = FirstOrderBigEngine.eligible(ctx.model, ctx.comm, ctx.n_total, ctx.local_ids, ctx.placement, alg)
    if big:
        return FirstOrderBigEngine.get(ctx.model, ctx.comm, ctx.placement, ctx.n_total)
    if backend == "native":
        raise RuntimeError("native first-order engine needs GPU ranks with contiguous segments")
    return None


def model_bytes(units: np.ndarray, d: int) -> int:
    """The reference's communication model in bytes: every comm unit is one d-row transmission of f64
    (GD_DGD_LAG.m:102 and LinearRegression_Synthetic.m:100-142: a parameter-server iteration = the
    workers' uploads + ONE broadcast of theta down; DGD / dual averaging = one transmission per worker
    to its chain neighbours). This is the byte axis on which GD / LAG / IAG, star ADMM and GADMM compare
    (E1 / E7 curves), independent of how the fabric realises the server: the native engine replicates
    the server's table on every rank, so its FABRIC bytes (``bytes_sent``) grow with the rank count."""
    return int(round(float(units[-1]))) * int(d) * 8 if len(units) else 0


def _native_result(name, out, obj0, units, d: int, **extra) -> RunResult:
    """``extra['transport']``: 'xgmi' when the run spanned ranks (FoFabric: device-initiated granule pushes
    into IPC-mapped fine-grained memory), 'local' on one rank."""
    obj = out["obj"]
    n = len(obj)
    return RunResult(algorithm=name, obj=obj, loss=np.abs(obj - obj0), iters=out["iters"] if out["converged"] else n,
                     converged=out["converged"], wall_s=float(out["times"][-1]) if n else 0.0,
                     time_trace=out["times"], comm_units=units, bytes_sent=int(out.get("payload_bytes", 0)),
                     bytes_total=int(out.get("payload_bytes", 0)),
                     extra=dict(extra, engine=out.get("engine", "native-persistent"), rows_pushed=out.get("rows_pushed", 0),
                                flags_pushed=out.get("flags_pushed", 0), wire_bytes=out.get("wire_bytes", 0),
                                model_bytes=model_bytes(units, d)))


def _result(name, stop: Stopper, ctx: _Ctx, units: np.ndarray, converged: bool, iters: int, **extra):
    obj, loss, times = stop.arrays()
    return RunResult(algorithm=name, obj=obj, loss=loss, iters=iters, converged=converged,
                     wall_s=float(times[-1]) if len(times) else 0.0, time_trace=times, comm_units=units,
                     bytes_sent=run_bytes(ctx.comm, ctx.snap), bytes_total=total_bytes(ctx.comm, ctx.snap),
                     extra=dict(extra, model_bytes=model_bytes(units, ctx.d)))


# ------------------------------------------------------------------------------------------------- GD
def gradient_descent(model, local_ids, n_total, num_iter, obj0, stepsize, comm=None, placement=None,
                     faithful=True, tol: Optional[float] = None, backend: str = "auto") -> RunResult:
    ctx = _Ctx(model, local_ids, n_total, comm, placement)
    eng = _fo_engine(ctx, backend, "GD")
    if eng is not None:
        out = eng.run("GD", num_iter, stepsize, obj0, tol, faithful)
        n = len(out["obj"])
        return _native_result("GD", out, obj0, np.arange(1, n + 1, dtype=np.float64) * (n_total + 1), ctx.d,
                              final_theta=None, transport="xgmi" if ctx.comm.nranks > 1 else "local")
    d = ctx.d
    theta = torch.zeros(d, dtype=torch.float64, device=ctx.dev)
    stop = Stopper(obj0, tol if tol is not None else -1.0, num_iter)
    converged, iters = False, num_iter
    for it in range(1, num_iter + 1):
        if it == 1 and faithful:
            if model.kind == "linear":
                g = torch.ones(d, dtype=torch.float64, device=ctx.dev)
            else:  # GD_DGD_LAG_logistic.m:97: the first step uses worker 1's gradient only
                g = torch.zeros(d, dtype=torch.float64, device=ctx.dev)
                if 0 in ctx.lidx:
                    g = ctx.worker_grad(0, theta)
                g = ctx.allsum(g.clone())
        else:
            g = ctx.grad_sum(theta)
        hit = stop.record(ctx.obj(theta))
        theta = theta - stepsize * g
        if hit and tol is not None:
            converged, iters = True, it
            break
    n = len(stop.obj)
    units = np.arange(1, n + 1, dtype=np.float64) * (n_total + 1)
    return _result("GD", stop, ctx, units, converged, iters if converged else n, final_theta=None)


# ------------------------------------------------------------------------------------------------ DGD
def decentralized_gd(model, local_ids, n_total, num_iter, obj0, stepsize, comm=None, placement=None,
                     faithful=True, tol: Optional[float] = None, backend: str = "auto") -> RunResult:
    """DGD (GD_DGD_LAG.m:124-180): step stepsize/100 on the chain-neighbour average of gradients."""
    ctx = _Ctx(model, local_ids, n_total, comm, placement)
    eng = _fo_engine(ctx, backend, "DGD")
    if eng is not None:
        out = eng.run("DGD", num_iter, stepsize / 100.0, obj0, tol, faithful)
        n = len(out["obj"])
        return _native_result("DGD", out, obj0, np.arange(1, n + 1, dtype=np.float64) * n_total, ctx.d,
                              transport="xgmi" if ctx.comm.nranks > 1 else "local")
    d, dev = ctx.d, ctx.dev
    nl = len(ctx.local_ids)
    theta = torch.zeros((nl, d), dtype=torch.float64, device=dev)
    G = torch.ones((n_total, d), dtype=torch.float64, device=dev) if faithful else \
        torch.zeros((n_total, d), dtype=torch.float64, device=dev)
    plan = chain_plan(list(range(n_total)), ctx.placement, ctx.comm.rank)
    xchg = plan.xchg_head + plan.xchg_tail  # every boundary worker's gradient to its neighbour rank
    ids = torch.tensor(ctx.local_ids, dtype=torch.long, device=dev)
    step = stepsize / 100.0
    stop = Stopper(obj0, tol if tol is not None else -1.0, num_iter)
    converged, iters = False, num_iter
    for it in range(1, num_iter + 1):
        if it > 1 or not faithful:
            G[ids] = model.gradient(theta)
        ctx.comm.exchange_rows(G, xchg)
        hit = stop.record(ctx.obj_per_worker(theta))
        new = torch.empty_like(theta)
        for k, w in enumerate(ctx.local_ids):
            if n_total == 1:
                new[k] = theta[k] - step * G[w]
            elif w == 0:
                new[k] = theta[k] - 0.5 * step * (G[w] + G[w + 1])
            elif w == n_total - 1:
                new[k] = theta[k] - 0.5 * step * (G[w] + G[w - 1])
            else:
                new[k] = theta[k] - (1.0 / 3.0) * step * (G[w] + G[w + 1] + G[w - 1])
        theta = new
        if hit and tol is not None:
            converged, iters = True, it
            break
    n = len(stop.obj)
    return _result("DGD", stop, ctx, np.arange(1, n + 1, dtype=np.float64) * n_total, converged,
                   iters if converged else n)


# ------------------------------------------------------------------------------------------------ LAG
class _Server:
    """Rank 0 holds the server's table of the latest uploaded gradient of every worker
    (``grads`` in GD_DGD_LAG.m) and broadcasts theta; other ranks upload rows conditionally."""

    def __init__(self, ctx: _Ctx, init: torch.Tensor):
        self.ctx = ctx
        self.table = init.clone() if ctx.comm.rank == 0 else None  # (N, d)

    def upload(self, rows: torch.Tensor, vals: torch.Tensor) -> int:
        """Every rank calls with its triggered (global row ids, gradients). Returns the total count."""
        ctx, comm = self.ctx, self.ctx.comm
        d, dev = ctx.d, ctx.dev
        k = int(rows.numel())
        if comm.nranks == 1:
            if k:
                self.table[rows] = vals
            return k
        if comm.rank == 0:
            total = k
            if k:
                self.table[rows] = vals
            cnt = torch.zeros(1, dtype=torch.float64, device=dev)
            for r in range(1, comm.nranks):
                comm.recv_tensor(cnt, r)
                c = int(cnt.item())
                if c:
                    buf = torch.empty((c, d + 1), dtype=torch.float64, device=dev)
                    comm.recv_tensor(buf, r)
                    self.table[buf[:, 0].long()] = buf[:, 1:]
                total += c
            t = torch.tensor([float(total)], dtype=torch.float64, device=dev)
        else:
            comm.send_tensor(torch.tensor([float(k)], dtype=torch.float64, device=dev), 0)
            if k:
                comm.send_tensor(torch.cat([rows.double().unsqueeze(-1), vals], dim=1).contiguous(), 0)
            t = torch.zeros(1, dtype=torch.float64, device=dev)
        comm.broadcast(t, 0)
        return int(t.item())

    def step(self, theta: torch.Tensor, stepsize: float) -> torch.Tensor:
        """theta <- theta - stepsize * sum(grads, 2) on the server, broadcast to every rank."""
        comm = self.ctx.comm
        if comm.rank == 0:
            new = theta - stepsize * self.table.sum(0)
        else:
            new = torch.empty_like(theta)
        if comm.nranks > 1:
            comm.broadcast(new, 0)
        return new


def _lag_units(counts: np.ndarray) -> np.ndarray:
    """Reference communication units of LAG from the per-iteration upload counts (GD_DGD_LAG.m:246-251)."""
    comm_iter, out = 1.0, []
    for it, c in enumerate(counts, start=1):
        if c > 0:
            comm_iter += c
        elif it % 1000 == 0:
            comm_iter += 1
        out.append(comm_iter)
    return np.asarray(out) + np.arange(1, len(out) + 1)


def lag(model, local_ids, n_total, num_iter, obj0, stepsize, hmax_full: torch.Tensor, variant: str = "PS",
        comm=None, placement=None, faithful=True, tol: Optional[float] = None, backend: str = "auto") -> RunResult:
    """LAG-PS (server-side trigger) / LAG-WK (worker-side trigger), GD_DGD_LAG.m:184-327."""
    ctx = _Ctx(model, local_ids, n_total, comm, placement)
    d, dev = ctx.d, ctx.dev
    N = n_total
    thrd = (10.0 if variant == "PS" else 1.0) / (stepsize ** 2 * N ** 2) / TRIGGERSLOT
    eng = _fo_engine(ctx, backend, "LAG-" + variant)
    if eng is not None:
        out = eng.run("LAG-" + variant, num_iter, stepsize, obj0, tol, faithful, thrd=thrd,
                      hsq=hmax_full.to(dev, torch.float64) ** 2)
        return _native_result("LAG-" + variant, out, obj0, _lag_units(out["cnt"]), ctx.d,
                              uploads=int(round(out["uploads"])), transport="xgmi" if ctx.comm.nranks > 1 else "local")
    ids = torch.tensor(ctx.local_ids, dtype=torch.long, device=dev)
    nl = len(ctx.local_ids)
    server = _Server(ctx, torch.ones((N, d), dtype=torch.float64, device=dev))
    G = torch.ones((nl, d), dtype=torch.float64, device=dev)        # worker-side copy of its last upload
    theta_hat = torch.zeros((nl, d), dtype=torch.float64, device=dev)
    hloc = hmax_full[ids] ** 2
    hist = [torch.zeros(d, dtype=torch.float64, device=dev)]        # theta^{iter-11..iter}
    comm_iter = 1.0
    comm_final = []
    counts_trace = []
    uploads = 0
    stop = Stopper(obj0, tol if tol is not None else -1.0, num_iter)
    converged, iters = False, num_iter
    w0 = ctx.lidx.get(0)
    margin = float("inf")
    for it in range(1, num_iter + 1):
        theta = hist[-1]
        rows, vals = [], []
        grads_now = model.gradient(theta.unsqueeze(0).expand(nl, -1).contiguous())
        forced = None
        if variant == "PS" and faithful and it > 1 and w0 is not None:
            forced = grads_now[w0]  # worker-1 refresh side effect (quirk 4): no upload counted
        mask = torch.zeros(nl, dtype=torch.bool, device=dev)
        if it > TRIGGERSLOT:
            trig = sum(float((hist[-n] - hist[-n - 1]) @ (hist[-n] - hist[-n - 1])) for n in range(1, TRIGGERSLOT + 1))
            if variant == "PS":
                dd = ((theta_hat - theta) ** 2).sum(-1)
                lhs = hloc * dd
            else:
                dd = ((grads_now - G) ** 2).sum(-1)
                lhs = dd
            rhs = thrd * trig
            mask = lhs > rhs
            # the closest trigger decision of the run (relative): an engine whose reductions sum in
            # another order can only flip decisions whose margin is at rounding level
            rel = (lhs - rhs).abs() / torch.clamp(torch.maximum(lhs.abs(), torch.full_like(lhs, abs(rhs))), min=1e-300)
            margin = min(margin, float(rel.min()))
        if bool(mask.any()):
            sel = mask.nonzero().flatten()
            G[sel] = grads_now[sel]
            if variant == "PS":
                theta_hat[sel] = theta
        upd = mask.clone()
        if forced is not None:
            G[w0] = forced
            upd[w0] = True
        sel = upd.nonzero().flatten()
        server.upload(ids[sel], G[sel])
        count = int(mask.sum())
        c_all = count
        if ctx.comm.nranks > 1:
            t = torch.tensor([float(count)], dtype=torch.float64, device=dev)
            ctx.comm.allreduce_sum(t)
            c_all = int(t.item())
        uploads += c_all
        counts_trace.append(c_all)
        hit = stop.record(ctx.obj(theta))
        if c_all > 0:
            comm_iter += c_all
        elif it % 1000 == 0:
            comm_iter += 1
        comm_final.append(comm_iter)
        hist.append(server.step(theta, stepsize))
        if len(hist) > TRIGGERSLOT + 2:
            hist.pop(0)
        if hit and tol is not None:
            converged, iters = True, it
            break
    n = len(stop.obj)
    units = np.asarray(comm_final) + np.arange(1, n + 1)
    assert np.array_equal(units, _lag_units(np.asarray(counts_trace)))
    return _result("LAG-" + variant, stop, ctx, units, converged, iters if converged else n, uploads=uploads,
                   trigger_margin=margin)


# ------------------------------------------------------------------------------------------------ IAG
def iag_schedule(n_total: int, num_iter: int, mode: str, hmax_full=None, seed: int = 7) -> np.ndarray:
    """Refreshing worker of every iteration (index it-1): ``it mod N`` or a draw proportional to
    Hmax_i from a generator seeded identically on every rank."""
    its = np.arange(1, num_iter + 1)
    if mode == "cyclic":
        return (its % n_total).astype(np.int64)
    rng = np.random.default_rng(seed)
    prob = np.asarray(hmax_full.cpu().numpy(), dtype=np.float64)
    cum = np.cumsum(prob / prob.sum())
    return np.minimum(np.searchsorted(cum, rng.random(num_iter), side="left"), n_total - 1).astype(np.int64)


def iag(model, local_ids, n_total, num_iter, obj0, stepsize, mode: str = "cyclic", hmax_full=None, seed: int = 7,
        comm=None, placement=None, faithful=True, tol: Optional[float] = None, backend: str = "auto") -> RunResult:
    """Cyclic IAG (worker ``iter mod N`` refreshes) and non-uniform randomized IAG (worker drawn
    with probability proportional to Hmax_i); step alpha/N (GD_DGD_LAG.m:330-371)."""
    ctx = _Ctx(model, local_ids, n_total, comm, placement)
    name = "cIAG" if mode == "cyclic" else "R-IAG"
    sched = iag_schedule(n_total, num_iter, mode, hmax_full, seed)
    eng = _fo_engine(ctx, backend, "IAG")
    if eng is not None:
        out = eng.run("IAG", num_iter, stepsize / n_total, obj0, tol, faithful, sched=sched)
        n = len(out["obj"])
        return _native_result(name, out, obj0, np.arange(1, n + 1, dtype=np.float64) * 2, ctx.d,
                              transport="xgmi" if ctx.comm.nranks > 1 else "local")
    d, dev = ctx.d, ctx.dev
    N = n_total
    step = stepsize / N
    server = _Server(ctx, torch.ones((N, d), dtype=torch.float64, device=dev))
    theta = torch.zeros(d, dtype=torch.float64, device=dev)
    stop = Stopper(obj0, tol if tol is not None else -1.0, num_iter)
    converged, iters = False, num_iter
    empty_r = torch.zeros(0, dtype=torch.long, device=dev)
    empty_v = torch.zeros((0, d), dtype=torch.float64, device=dev)
    for it in range(1, num_iter + 1):
        w = int(sched[it - 1])
        if it > 1:
            if int(ctx.placement.owner[w]) == ctx.comm.rank:
                g = ctx.worker_grad(w, theta)
                server.upload(torch.tensor([w], dtype=torch.long, device=dev), g.unsqueeze(0))
            else:
                server.upload(empty_r, empty_v)
        hit = stop.record(ctx.obj(theta))
        theta = server.step(theta, step)
        if hit and tol is not None:
            converged, iters = True, it
            break
    n = len(stop.obj)
    return _result(name, stop, ctx, np.arange(1, n + 1, dtype=np.float64) * 2,
                   converged, iters if converged else n)


# ------------------------------------------------------------------------------------------- bundle
def gd_dgd_lag(model, local_ids, n_total, num_iter, obj0: Optional[float], comm=None, placement=None,
               faithful=True, accuracy: Optional[float] = None, which=("GD", "DGD", "LAG-PS", "LAG-WK", "cIAG", "R-IAG"),
               seed: int = 7, backend: str = "auto") -> Dict[str, object]:
    """The reference bundle: ``GD_DGD_LAG`` (linear, obj0 given) or ``GD_DGD_LAG_logistic`` (obj0 =
    final GD objective, returned as ``obj1``; LAG/IAG stop at ``accuracy``)."""
    comm = comm if comm is not None else LocalComm()
    consts = global_constants(model, comm)
    step = consts["stepsize"]
    ctx = _Ctx(model, local_ids, n_total, comm, placement)
    hmax_full = _gather_hmax(ctx, consts["hmax_local"])
    out: Dict[str, object] = {"stepsize": step, "hmax_all": consts["hmax_all"], "cond": consts["cond"]}
    logistic = model.kind == "logistic"
    if "GD" in which or logistic:
        gd = gradient_descent(model, local_ids, n_total, num_iter, obj0 if obj0 is not None else 0.0, step, comm,
                              placement, faithful, backend=backend)
        if logistic and obj0 is None:
            obj0 = float(gd.obj[-1])  # GD_DGD_LAG_logistic.m:131-133
            gd.loss = np.abs(gd.obj - obj0)
        out["GD"] = gd
    out["obj0"] = obj0
    tol_ = accuracy if logistic else None
    if "DGD" in which:
        out["DGD"] = decentralized_gd(model, local_ids, n_total, num_iter, obj0, step, comm, placement, faithful,
                                       backend=backend)
    if "LAG-PS" in which:
        out["LAG-PS"] = lag(model, local_ids, n_total, num_iter, obj0, step, hmax_full, "PS", comm, placement,
                            faithful, tol_, backend=backend)
    if "LAG-WK" in which:
        out["LAG-WK"] = lag(model, local_ids, n_total, num_iter, obj0, step, hmax_full, "WK", comm, placement,
                            faithful, tol_, backend=backend)
    if "cIAG" in which:
        out["cIAG"] = iag(model, local_ids, n_total, num_iter, obj0, step, "cyclic", None, seed, comm, placement,
                          faithful, tol_, backend=backend)
    if "R-IAG" in which:
        out["R-IAG"] = iag(model, local_ids, n_total, num_iter, obj0, step, "random", hmax_full, seed, comm,
                           placement, faithful, tol_, backend=backend)
    return out
