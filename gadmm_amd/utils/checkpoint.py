"""Per-worker model/dual checkpoints (BASELINE.json: "the same per-worker model/dual checkpoint
layout"; SURVEY.md §5 Checkpoint/resume).

The reference's state is the workspace matrices ``out`` (theta, d x N) and ``lambda`` (duals,
d x N; edge duals for GADMM ``group_ADMM_closedForm.m:6-7``, per-worker aggregated duals for
D-GADMM ``dynamic_group_ADMM_closedForm.m:8-10``). Here every logical worker owns one shard file:

    <dir>/manifest.json                 written by rank 0: algorithm, N, d, rho, next iteration,
                                        chain path, placement, targets, schedule seed ...
    <dir>/worker_00017.safetensors      theta (d,), mu (d,)  [+ lambda_edge (d,) when complete],
                                        metadata: worker id, chain position, next iteration

Every rank writes only its own workers, so a checkpoint of the 10M x 10k config is a parallel write
of 80 KB per worker. Resume: each rank reads its workers' theta/mu and the theta of their chain
neighbours (ghost rows) and continues bit-exactly (tests/test_checkpoint.py).
The per-worker dual ``mu_n = lambda_n - lambda_{n-1}`` converts to the reference's edge duals by a
prefix sum along the chain (``edge_duals``).
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

try:  # safetensors executes nothing on load
    from safetensors.torch import load_file as _st_load, save_file as _st_save
except Exception:  # pragma: no cover
    _st_load = _st_save = None

FORMAT = "gadmm-amd-worker-shards/1"


def _shard_path(directory: str, worker: int) -> str:
    return os.path.join(directory, "worker_%05d.safetensors" % worker)


def save_checkpoint(directory: str, rank: int, local_ids: Sequence[int], theta_table: torch.Tensor,
                    mu_local: torch.Tensor, next_iter: int, path: Sequence[int], manifest: Optional[Dict] = None
                    ) -> List[str]:
    """Write this rank's worker shards (and the manifest on rank 0). ``theta_table``: (N, d) with the
    local rows authoritative; ``mu_local``: (n_loc, d) in ``local_ids`` order."""
    os.makedirs(directory, exist_ok=True)
    pos = {int(w): p for p, w in enumerate(path)}
    written = []
    th = theta_table.detach().to("cpu", torch.float64)
    mu = mu_local.detach().to("cpu", torch.float64)
    for i, w in enumerate(local_ids):
        w = int(w)
        tensors = {"theta": th[w].contiguous().clone(), "mu": mu[i].contiguous().clone()}
        meta = {"format": FORMAT, "worker": str(w), "chain_pos": str(pos.get(w, -1)), "next_iter": str(int(next_iter))}
        p = _shard_path(directory, w)
        tmp = p + ".tmp"
        if _st_save is not None:
            _st_save(tensors, tmp, metadata=meta)
        else:  # pragma: no cover
            torch.save({"tensors": tensors, "meta": meta}, tmp)
        os.replace(tmp, p)
        written.append(p)
    if rank == 0:
        man = dict(manifest or {})
        man.update({"format": FORMAT, "next_iter": int(next_iter), "path": [int(w) for w in path],
                    "n_workers": int(theta_table.shape[0]), "dim": int(theta_table.shape[1])})
        tmp = os.path.join(directory, "manifest.json.tmp")
        with open(tmp, "w") as f:
            json.dump(man, f, indent=1, default=_json_default)
        os.replace(tmp, os.path.join(directory, "manifest.json"))
    return written


def _json_default(o):
    if isinstance(o, (np.integer,)):
        return int(o)
    if isinstance(o, (np.floating,)):
        return float(o)
    if isinstance(o, np.ndarray):
        return o.tolist()
    return str(o)


def read_manifest(directory: str) -> Dict:
    with open(os.path.join(directory, "manifest.json")) as f:
        return json.load(f)


def load_worker(directory: str, worker: int) -> Tuple[torch.Tensor, torch.Tensor, Dict[str, str]]:
    p = _shard_path(directory, worker)
    if _st_load is not None:
        from safetensors import safe_open

        with safe_open(p, framework="pt") as f:
            meta = f.metadata() or {}
        t = _st_load(p)
        return t["theta"], t["mu"], meta
    obj = torch.load(p, weights_only=True)  # pragma: no cover
    return obj["tensors"]["theta"], obj["tensors"]["mu"], obj["meta"]


def load_checkpoint(directory: str, local_ids: Sequence[int], device=None):
    """Returns ``(theta_table, mu_local, next_iter, path, manifest)`` for a rank owning
    ``local_ids``. The theta table holds every worker's theta (local rows + ghost rows)."""
    man = read_manifest(directory)
    N, d = int(man["n_workers"]), int(man["dim"])
    theta = torch.zeros((N, d), dtype=torch.float64)
    for w in range(N):
        p = _shard_path(directory, w)
        if os.path.exists(p):
            theta[w] = load_worker(directory, w)[0]
    mu = torch.zeros((len(local_ids), d), dtype=torch.float64)
    for i, w in enumerate(local_ids):
        th, m, meta = load_worker(directory, int(w))
        if int(meta.get("next_iter", man["next_iter"])) != int(man["next_iter"]):
            raise ValueError("inconsistent checkpoint: worker %d at a different iteration" % w)
        mu[i] = m
    if device is not None:
        theta, mu = theta.to(device), mu.to(device)
    return theta, mu, int(man["next_iter"]), [int(w) for w in man["path"]], man


def edge_duals(mu_by_worker: np.ndarray, path: Sequence[int]) -> np.ndarray:
    """Reference edge duals ``lambda(:, p)`` for chain edge p = (path[p], path[p+1]) from the
    per-worker duals: ``lambda_p = sum_{k <= p} mu_{path[k]}`` (inverse of mu_n = lambda_n - lambda_{n-1})."""
    mu = np.asarray(mu_by_worker)
    ordered = mu[list(path)]
    lam = np.cumsum(ordered, axis=0)
    return lam[:-1]
