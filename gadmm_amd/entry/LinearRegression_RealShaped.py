"""BASELINE.json configs[4] — "LinearRegression_Real-shaped 10M x 10k sharded across 8 GPUs (288 GB HBM
sizing) vs standard-ADMM baseline".

Each rank generates its own shard(s) directly in HBM (Gaussian rows, y = X theta* + 0.1 noise; seeds
per worker, so no rank ever materialises another rank's data): with the defaults one worker of
1.25M x 10k f64 = 100 GB per MI355X, i.e. 10M x 10k over 8 GPUs (weak scaling: per-GPU shard fixed).
Set-up: augmented Gram on f64 MFMA (2.5e14 flop per GPU), cached inverses (A + c rho I)^{-1} (rocSOLVER
Cholesky), the global optimum from the all-reduced d x d Gram. Then GADMM over the chain of workers on
the row-blocked HIP engine (80 KB theta per boundary per phase over the session's data plane: the IPC
transport by default, RCCL with ``--fabric rccl``) until the relative gap
|obj - obj*| / |obj*| < tol, and the star ADMM of the reference on the same fabric for comparison.

    torchrun --nproc-per-node 8 -m gadmm_amd LinearRegression_RealShaped
    python -m gadmm_amd LinearRegression_RealShaped --set dim=2048 rows_per_worker=200000   # 1 GPU
    python -m gadmm_amd LinearRegression_RealShaped --set run_baselines=1 run_dualavg=1   # + the bundle
"""
import time

import numpy as np
import torch

from ..config import PRESETS, ExperimentConfig
from ..data import gaussian_regression
from .common import Problem, run_entry

ENTRY = "LinearRegression_RealShaped"

PRESETS.setdefault(ENTRY, ExperimentConfig(
    name=ENTRY, model="linear", data="gaussian", num_workers=0, rows_per_worker=1_250_000, dim=10_000,
    gadmm_iters=2000, rhos=[0.0], acc=1e-8, run_baselines=False, run_dualavg=False, run_star=True,
    baseline_iters=400,
    reference="BASELINE.json configs[4]; LinearRegression_Real.m shapes scaled to 10M x 10k"))


def body(cfg, sess, args, writer):
    from ..algorithms import chain_admm, standard_admm

    wpg = 1 if cfg.num_workers <= 0 else max(1, cfg.num_workers // sess.world)
    n_total = wpg * sess.world
    t0 = time.perf_counter()
    ids = list(range(sess.rank * wpg, (sess.rank + 1) * wpg))
    ds = gaussian_regression(n_total, cfg.rows_per_worker, cfg.dim, seed=cfg.seed, labels="linear",
                             device=sess.device, worker_ids=ids)
    if sess.device.type == "cuda":
        torch.cuda.synchronize(sess.device)
    t_gen = time.perf_counter() - t0

    class _Local:  # Problem over locally generated shards
        pass

    prob = _Local()
    prob.cfg, prob.n_total = cfg, n_total
    from ..parallel.topology import Placement
    from ..models import LinearRegression

    prob.placement = Placement.contiguous(n_total, sess.world)
    prob.local_ids = ids
    t1 = time.perf_counter()
    prob.model = LinearRegression(ds.X, ds.y)          # f64-MFMA Gram
    if sess.device.type == "cuda":
        torch.cuda.synchronize(sess.device)
    t_gram = time.perf_counter() - t1
    sess.ensure_plane(n_total, cfg.dim)  # several GPUs: the data plane (IPC default) of every solver below
    prob.obj0 = prob.model.optimum(sess.comm if sess.world > 1 else None, n_total=n_total)
    m = cfg.rows_per_worker
    rho = cfg.rhos[0] if cfg.rhos and cfg.rhos[0] > 0 else 0.5 * m   # A_n ~ m I for Gaussian rows
    tol_abs = cfg.acc * abs(prob.obj0)
    sess.log("  shards: %d x (%d x %d) f64 per rank (%.1f GB), gen %.2fs, Gram %.2fs (%.1f TF/s), obj* = %.10e"
             % (wpg, m, cfg.dim, wpg * m * cfg.dim * 8 / 1e9, t_gen, t_gram,
                wpg * 2.0 * m * (cfg.dim + 1) ** 2 / 2 / max(t_gram, 1e-9) / 1e12, prob.obj0))
    runs = {}
    g = chain_admm(prob.model, ids, n_total, rho, prob.obj0, tol_abs, cfg.gadmm_iters, comm=sess.comm,
                   placement=prob.placement, backend=args.backend, name="GADMM(rho=%g)" % rho)
    g.extra.pop("engine_obj", None)
    g.extra.pop("state", None)
    runs["GADMM"] = g
    out = {"runs": runs, "obj0": prob.obj0, "rho": rho, "tol_rel": cfg.acc, "t_generate_s": t_gen,
           "t_gram_s": t_gram, "rows_per_worker": m, "dim": cfg.dim, "n_workers": n_total,
           "dataset": {"d": cfg.dim, "N": n_total, "m": m}}
    if cfg.run_star and n_total > 1:
        s = standard_admm(prob.model, ids, n_total, rho, prob.obj0, tol_abs, min(cfg.gadmm_iters, 500),
                          comm=sess.comm, placement=prob.placement)
        runs["ADMM(star)"] = s
    if cfg.run_baselines:
        # the reference's baseline bundle on the real-shaped data (LinearRegression_Real.m:66-69, 78): at
        # d > 128 every algorithm runs on the stream-ordered large-d engine (engine/first_order_big.py;
        # GD / DGD / IAG across ranks, LAG and dual averaging on one rank, else the torch loop)
        from ..algorithms import gd_dgd_lag, dual_averaging, global_constants
        t2 = time.perf_counter()
        bl = gd_dgd_lag(prob.model, ids, n_total, cfg.baseline_iters, prob.obj0, comm=sess.comm,
                        placement=prob.placement, backend=args.backend)
        for k in ("GD", "DGD", "LAG-PS", "LAG-WK", "cIAG", "R-IAG"):
            if k in bl:
                runs[k] = bl[k]
        if cfg.run_dualavg:
            c = global_constants(prob.model, sess.comm)
            runs["DualAvg"] = dual_averaging(prob.model, ids, n_total, c["stepsize"], prob.obj0, tol_abs,
                                             cfg.dualavg_iters or cfg.baseline_iters, comm=sess.comm,
                                             placement=prob.placement, backend=args.backend)
        out["t_baselines_s"] = time.perf_counter() - t2
        sess.log("  baselines (%d iterations each): %.2fs" % (cfg.baseline_iters, out["t_baselines_s"]))
    out["figure_groups"] = {"10M x 10k real-shaped": runs}
    return out


def main(argv=None):
    return run_entry(ENTRY, body, argv)


if __name__ == "__main__":
    main()
