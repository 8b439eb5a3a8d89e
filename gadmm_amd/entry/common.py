"""Shared machinery of the entry points: process/device set-up, per-rank data, model, oracle,
GADMM sweeps, the baseline bundle, outputs.

Launch forms:
    python -m gadmm_amd LinearRegression_Synthetic                      # 1 process (GPU if present)
    python -m gadmm_amd LinearRegression_Synthetic --device cpu --cpu-ranks 2   # gloo plumbing
    torchrun --nproc-per-node 8 -m gadmm_amd LinearRegression_Synthetic      # 8 x MI355X
    GADMM_SHARE_GPU=1 torchrun --nproc-per-node 4 -m gadmm_amd ...          # rehearsal: 4 ranks, one GPU

Several GPU ranks (parallel/node.py): a gloo control plane, then per experiment the engines the
benchmarks use -- GADMM sweeps on the data-local blocked kernel over xGMI (engine/multigpu.py:
node_chain_admm), logistic / D-GADMM / star on their persistent kernels over an ``XgmiFabric``, the
baseline bundle on the first-order fabric, and the IPC device-copy transport (``--fabric auto``, the
default) or RCCL (``--fabric rccl``, opt-in) as the data plane of the graph engines and set-up
collectives. Every run's summary names its engine and transport.
"""
from __future__ import annotations

import argparse
import json
import os
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from ..config import ExperimentConfig, get_preset, parse_overrides
from ..data import ShardedDataset, linear_synthetic, logistic_synthetic, gaussian_regression
from ..data.sharding import from_stacked, split_workers
from ..models import make_model
from ..parallel.topology import Placement
from ..utils.metrics import RunWriter, plot_three_panel


class Session:
    def __init__(self, rank: int, world: int, device: torch.device, comm, nodes=None):
        self.rank, self.world, self.device, self.comm = rank, world, device, comm
        self.nodes = nodes  # parallel/node.NodeFabrics on GPU ranks (several), else None

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    @property
    def multi_gpu(self) -> bool:
        return self.nodes is not None

    def log(self, *a):
        if self.is_root:
            print(*a, flush=True)

    def ensure_plane(self, n_total: int, d: int):
        """The session's data-plane comm for this experiment's shape (GPU ranks: built on first use, IPC
        by default); set as ``self.comm`` and returned."""
        if self.nodes is not None:
            self.comm = self.nodes.data_plane(n_total, d)
        return self.comm

    def chain_kw(self, n_total: int, d: int, dynamic: bool = False) -> dict:
        """Keyword arguments (``comm``, ``engine_opts``) that put a chain-family solve (chain_admm,
        dynamic_group_admm, static_group_admm, ...) on its persistent kernel across GPUs: an xGMI fabric
        (D-GADMM: a ring of 8 table slots) with the data plane as the agreed fallback. One rank / CPU ranks:
        the session comm."""
        if self.nodes is None:
            return {"comm": self.comm}
        from ..parallel.comm import RankInfo
        plane = self.ensure_plane(n_total, d)
        if getattr(self, "backend", "auto") == "torch":  # the torch loops run over the data plane
            return {"comm": plane}
        fab = self.nodes.xgmi(n_total, d, 8 if dynamic else 1)
        if fab is None:
            return {"comm": plane}
        return {"comm": RankInfo(self.rank, self.world), "engine_opts": {"fabric": fab, "fallback_comm": plane}}

    def star_kw(self, n_total: int, d: int) -> dict:
        """``comm`` / ``engine_opts`` of the star comparator: its persistent kernel over an xGMI fabric
        (d <= 64), the data plane's reduce / broadcast otherwise."""
        if self.nodes is None:
            return {"comm": self.comm}
        plane = self.ensure_plane(n_total, d)
        fab = self.nodes.xgmi(n_total, d, 1) if d <= 64 else None
        return {"comm": plane, "engine_opts": {"fabric": fab} if fab is not None else {}}

    def close(self):
        if self.nodes is not None:
            self.nodes.close()


def make_session(device: str = "auto", fabric: str = "auto", timeout_s: float = 20.0) -> Session:
    from ..parallel.launch import setup_rank
    from ..parallel.node import NodeFabrics, session_plan, share_requested

    if device == "auto":
        device = "cuda" if torch.cuda.is_available() else "cpu"
    if device == "cuda":
        rank, world, local_rank, dev, comm = setup_rank("node")
        if world > 1:
            share = share_requested()
            plan = session_plan("cuda", world, fabric, share)
            nodes = NodeFabrics(rank, world, dev, plan, fabric, share, timeout_s=timeout_s)
            return Session(rank, world, dev, None, nodes=nodes)
        return Session(rank, world, dev, comm)
    rank, world, local_rank, dev, comm = setup_rank("gloo")
    return Session(rank, world, dev, comm)


def full_dataset(cfg: ExperimentConfig) -> ShardedDataset:
    if cfg.data == "linear_synthetic":
        return linear_synthetic(cfg.num_workers, seed=cfg.seed)
    if cfg.data == "logistic_synthetic":
        return logistic_synthetic(cfg.num_workers, seed=cfg.seed)
    if cfg.data in ("bodyfat", "derm"):
        if cfg.data_dir:
            from ..data.matfile import load_uci_dir

            X, y = load_uci_dir(cfg.data_dir)
            Xt, yt = torch.from_numpy(X), torch.from_numpy(y)
            if cfg.data == "bodyfat":
                return from_stacked(Xt, yt, cfg.rows_per_worker, name="bodyfat")
            return split_workers(Xt, yt, cfg.num_workers, name="derm")
        # real-shaped synthetic stand-in (the UCI files are not shipped with the reference)
        if cfg.data == "bodyfat":
            n = cfg.total_rows // cfg.rows_per_worker
            return gaussian_regression(n, cfg.rows_per_worker, cfg.dim, seed=cfg.seed, labels="linear")
        per = cfg.total_rows // cfg.num_workers
        return gaussian_regression(cfg.num_workers, per, cfg.dim, seed=cfg.seed, labels="logistic")
    if cfg.data == "gaussian":
        return gaussian_regression(cfg.num_workers, cfg.rows_per_worker, cfg.dim, seed=cfg.seed,
                                   labels="logistic" if cfg.model == "logistic" else "linear")
    raise ValueError("unknown data %r" % cfg.data)


class Problem:
    """This rank's slice of an experiment: local shards, model, the global optimum."""

    def __init__(self, cfg: ExperimentConfig, sess: Session, ds: Optional[ShardedDataset] = None):
        ds = ds if ds is not None else full_dataset(cfg)
        self.cfg = cfg
        self.n_total = ds.num_workers
        self.placement = Placement.contiguous(self.n_total, sess.world)
        self.local_ids = self.placement.local_workers(sess.rank)
        loc = ds.subset(self.local_ids).to(sess.device)
        self.model = make_model(cfg.model, loc.X.contiguous(), loc.y.contiguous(), lam=cfg.lam)
        self.dataset_meta = dict(ds.meta, name=ds.name, N=ds.num_workers, m=ds.rows_per_worker, d=ds.dim)
        self.d = int(ds.dim)
        comm = sess.ensure_plane(self.n_total, self.d)  # GPU ranks: the data plane of this experiment
        self.obj0 = self.model.optimum(comm if sess.world > 1 else None, n_total=self.n_total)


def parse_args(entry: str, argv=None):
    ap = argparse.ArgumentParser(prog="python -m gadmm_amd %s" % entry,
                                 description="Reference entry point %s on the MI355X framework" % entry)
    ap.add_argument("--device", default="auto", choices=["auto", "cpu", "cuda"])
    ap.add_argument("--cpu-ranks", type=int, default=0, help="spawn N gloo ranks on this host (CPU plumbing)")
    ap.add_argument("--out", default=None, help="output directory (default runs/<entry>)")
    ap.add_argument("--quick", action="store_true", help="reduced iteration budgets (smoke runs)")
    ap.add_argument("--set", nargs="*", default=[], metavar="KEY=VALUE", help="override preset fields")
    ap.add_argument("--no-baselines", action="store_true")
    ap.add_argument("--no-plot", action="store_true")
    ap.add_argument("--tol", type=float, default=None, help="override the stopping gap (reference: 1e-4)")
    ap.add_argument("--backend", default="auto", choices=["auto", "torch", "native"])
    ap.add_argument("--checkpoint", default=None, help="write per-worker checkpoints of the last GADMM run here")
    ap.add_argument("--fabric", default="auto", choices=["auto", "xgmi", "ipc", "rccl"],
                    help="several GPU ranks: auto/xgmi = the persistent kernels over xGMI fabrics with the IPC "
                         "transport as data plane; ipc = graph engines over the IPC transport only; rccl = "
                         "graph engines over RCCL (opt-in, watchdog-bounded, falls back to IPC)")
    ap.add_argument("--timeout", type=float, default=20.0, help="multi-GPU hand-off deadline in seconds")
    a = ap.parse_args(argv)
    cfg = get_preset(entry)
    if a.quick:
        cfg = cfg.quick()
    cfg = parse_overrides(cfg, a.set)  # explicit --set values win over the --quick budgets
    if a.no_baselines:
        cfg = cfg.override(run_baselines=False, run_dualavg=False)
    if a.tol is not None:
        cfg = cfg.override(acc=a.tol)
    return a, cfg


def run_entry(entry: str, body, argv=None) -> Dict:
    """Parse args, launch (optionally spawning gloo ranks), run ``body(cfg, sess, args) -> dict``."""
    args, cfg = parse_args(entry, argv)
    if args.cpu_ranks and args.cpu_ranks > 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        from ..parallel.launch import spawn

        outs = spawn(_spawned, args.cpu_ranks, entry, body, argv_without_ranks(argv))
        return outs[0]
    sess = make_session(args.device, args.fabric, args.timeout)
    try:
        return _run(entry, body, cfg, sess, args)
    finally:
        sess.close()


def argv_without_ranks(argv):
    import sys

    argv = list(sys.argv[2:] if argv is None else argv)
    out, skip = [], False
    for i, a in enumerate(argv):
        if skip:
            skip = False
            continue
        if a == "--cpu-ranks":
            skip = True
            continue
        if a.startswith("--cpu-ranks="):
            continue
        out.append(a)
    return out + ["--device", "cpu"]


def _spawned(rank, world, entry, body, argv):
    from ..parallel.comm import TorchDistComm

    args, cfg = parse_args(entry, argv)
    sess = Session(rank, world, torch.device("cpu"), TorchDistComm())
    return _run(entry, body, cfg, sess, args)


def _run(entry, body, cfg, sess, args) -> Dict:
    out_dir = args.out or os.path.join("runs", entry)
    writer = RunWriter(out_dir, sess.rank)
    sess.backend = args.backend
    t0 = time.perf_counter()
    sess.log("[%s] device=%s ranks=%d share=%s  (reference: %s)" % (
        entry, sess.device, sess.world, getattr(sess.nodes, "share", False), cfg.reference))
    res = body(cfg, sess, args, writer)
    if sess.nodes is not None:
        res["node_planes"] = [{"what": w, **{k: v for k, v in e.items()}} for w, e in sess.nodes.events]
    res["wall_s"] = time.perf_counter() - t0
    dim = (res.get("dataset") or {}).get("d")
    for k, r in res.get("runs", {}).items():
        r.extra.setdefault("dim", dim)
        writer.add(k, r)
    summary = writer.close({"entry": entry, "config": cfg.__dict__, "device": str(sess.device), "ranks": sess.world,
                            **{k: v for k, v in res.items() if k not in ("runs", "figure_groups")}})
    if sess.is_root and not args.no_plot:
        for title, group in res.get("figure_groups", {}).items():
            plot_three_panel(group, os.path.join(out_dir, _fname(title) + ".png"), title=title)
    if sess.is_root:
        for k, r in res.get("runs", {}).items():
            s = r.summary()
            print("  %-34s iters=%-7s converged=%-5s gap=%-10.3g wall=%.3fms comm_units=%s bytes=%s engine=%s "
                  "transport=%s" % (
                      k, s["iters"], s["converged"], s["final_loss"] if s["final_loss"] is not None else float("nan"),
                      1e3 * s["wall_s"], s["comm_units"], s["bytes_total"], s.get("engine", "torch"),
                      s.get("transport", _transport_of(sess))), flush=True)
        print("[%s] summary -> %s" % (entry, summary), flush=True)
    res["summary_path"] = summary
    res.pop("figure_groups", None)
    return {k: v for k, v in res.items() if k != "runs"} | {"runs": {k: r.summary() for k, r in res.get("runs", {}).items()}}


def _transport_of(sess) -> str:
    if sess.world <= 1:
        return "local"
    return str(getattr(sess.comm, "backend", "?"))


def _fname(s: str) -> str:
    return "".join(c if c.isalnum() or c in "-_" else "_" for c in s)


# ----------------------------------------------------------------------------------- building blocks
def attach_modelled_clock(result, model, rho: float, sess: Session):
    """Give ``result`` the reference's modelled clock (``2 * toc`` per iteration, toc = worker 1's
    local solve measured on this device; utils/timing.py). Worker 1 lives on rank 0: its toc is
    broadcast so every rank reports the same curve."""
    from ..utils.timing import modelled_time, reference_local_solve_s

    toc = reference_local_solve_s(model, rho) if sess.rank == 0 else 0.0
    if sess.world > 1:
        t = torch.tensor([toc], dtype=torch.float64, device=sess.device if sess.device.type == "cuda" else "cpu")
        sess.comm.broadcast(t, 0)
        toc = float(t.item())
    result.model_time = modelled_time(toc, len(result.obj))
    result.extra["model_toc_s"] = toc
    return result


def gadmm_solve(prob: Problem, sess: Session, rho: float, acc: float, max_iter: int, backend: str = "auto",
                name: str = "GADMM", local_solver: Optional[str] = None, need_state: bool = False):
    """One GADMM solve of the experiment on its engine. Several GPU ranks: closed-form linear solves on the
    headline's data-local blocked kernel over xGMI (engine/multigpu.node_chain_admm), the logistic local
    solvers on their persistent kernels over an xGMI fabric (``sess.chain_kw``); one rank / CPU ranks:
    ``chain_admm`` with the session comm. ``need_state``: the result must carry (theta, mu) for a
    checkpoint (the per-worker kernels return it, the blocked kernel does not)."""
    from ..algorithms import chain_admm

    cfg = prob.cfg
    solver = local_solver or ("closed" if cfg.model == "linear" else "gd")
    if sess.multi_gpu and backend != "torch":
        if solver == "closed" and not need_state:
            from ..engine.multigpu import node_chain_admm
            return node_chain_admm(prob.model, prob.local_ids, prob.n_total, prob.placement, sess.rank, sess.world,
                                   sess.device, rho, prob.obj0, acc, max_iter, fabric=sess.nodes.fabric_req,
                                   share=sess.nodes.share, plane=sess.ensure_plane(prob.n_total, prob.d),
                                   timeout_s=sess.nodes.timeout_s, name=name)
        kw = sess.chain_kw(prob.n_total, prob.d)
    else:
        kw = {"comm": sess.comm}
    return chain_admm(prob.model, prob.local_ids, prob.n_total, rho, prob.obj0, acc, max_iter,
                      placement=prob.placement, local_solver=solver, step=cfg.gd_step, max_inner=cfg.max_inner,
                      backend=backend, name=name, **kw)


def gadmm_sweep(prob: Problem, sess: Session, backend: str = "auto", state_rho: Optional[float] = None
                ) -> Dict[str, object]:
    """The reference's rho sweep (LinearRegression_Synthetic.m:78-94, LogisticRegression_Synthetic.m:88-100):
    one GADMM solve per rho on its engine (``gadmm_solve``); ``state_rho``: that run keeps its state for
    a checkpoint."""
    from ..utils.timing import roctx_range

    cfg = prob.cfg
    out = {}
    for rho in cfg.rhos:
        with roctx_range("gadmm_sweep rho=%g" % rho):
            r = gadmm_solve(prob, sess, rho, cfg.acc, cfg.gadmm_iters, backend, name="GADMM(rho=%g)" % rho,
                            need_state=(state_rho is not None and rho == state_rho))
        r.extra.pop("engine_obj", None)
        out["GADMM_rho%g" % rho] = attach_modelled_clock(r, prob.model, rho, sess)
    if cfg.model == "logistic":
        for rho in cfg.exact_rhos:  # exact local solves (D2 semantics), to the tighter exact_acc gap
            with roctx_range("gadmm_exact rho=%g" % rho):
                r = gadmm_solve(prob, sess, rho, cfg.exact_acc, cfg.exact_iters, backend,
                                name="GADMM-exact(rho=%g)" % rho, local_solver="newton")
            r.extra.pop("engine_obj", None)
            out["GADMM_exact_rho%g" % rho] = attach_modelled_clock(r, prob.model, rho, sess)
    return out


def baselines(prob: Problem, sess: Session) -> Dict[str, object]:
    from ..algorithms import gd_dgd_lag, dual_averaging

    cfg = prob.cfg
    out: Dict[str, object] = {}
    stepsize = None
    if cfg.run_baselines:
        b = gd_dgd_lag(prob.model, prob.local_ids, prob.n_total, cfg.baseline_iters,
                       prob.obj0 if cfg.model == "linear" else None, comm=sess.comm, placement=prob.placement,
                       accuracy=cfg.acc)
        stepsize = b["stepsize"]
        for k in ("GD", "DGD", "LAG-PS", "LAG-WK", "cIAG", "R-IAG"):
            if k in b:
                out[k] = b[k]
        if cfg.model == "logistic":
            # GD_DGD_LAG_logistic returns obj1 = last GD objective as the reference optimum
            out["_obj0_gd"] = b["obj0"]
    if cfg.run_dualavg:
        if stepsize is None:
            from ..algorithms import global_constants

            stepsize = global_constants(prob.model, sess.comm)["stepsize"]
        out["DualAvg"] = dual_averaging(prob.model, prob.local_ids, prob.n_total, stepsize, prob.obj0, cfg.acc,
                                        cfg.dualavg_iters or cfg.baseline_iters, comm=sess.comm,
                                        placement=prob.placement)
    return out


def maybe_checkpoint(args, sess: Session, prob: Problem, result, rho: float, name: str):
    """Write per-worker checkpoints of a chain-ADMM result (torch backend state)."""
    if not args.checkpoint:
        return None
    from ..utils.checkpoint import save_checkpoint

    st = result.extra.get("state")
    if st is None:
        return None
    theta, mu, nxt = st
    save_checkpoint(args.checkpoint, sess.rank, prob.local_ids, theta, mu, nxt, list(range(prob.n_total)),
                    {"algorithm": name, "rho": rho, "obj0": prob.obj0, "entry": prob.cfg.name})
    return args.checkpoint
