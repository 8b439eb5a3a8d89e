"""Synthetic data builders for the reference experiments.

Every builder returns a :class:`~gadmm_amd.data.sharding.ShardedDataset` in float64: ``N`` shards
``(X_n, y_n)`` of identical shape ``m x d`` (the reference always uses equal-size contiguous row
blocks, ``group_ADMM_closedForm.m:30-34``).

Constructions (reference semantics, re-derived, not transliterated):

* ``linear_synthetic``: ``X_n = 1.3**(n-1) q_n q_n^T + I_50`` with ``q_n`` the n-th column of an
  orthogonal 50x50 ``Q`` and the same label vector ``y`` on every worker
  (``LinearRegression_Synthetic.m:21-37``; ``Dynamic_LinearRegression_Synthetic.m:17-37`` uses
  N = 50 with the same design).
* ``logistic_synthetic``: same with growth factor 1 (``LogisticRegression_Synthetic.m:21-35``).
  The reference ships exactly this dataset as ``inputData.mat``; when the fixture
  is present its rank-1 blocks ``P_n = X_n - I`` and labels are used, so results are comparable
  with the golden numbers in BASELINE.md.
* ``real_shaped``: Gaussian rows for the 10M x 10k "LinearRegression_Real-shaped" config, generated
  shard-by-shard (optionally directly on the device that will own the shard).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from .sharding import ShardedDataset
from .matfile import load_input_data

_FIXTURE_CANDIDATES = (
    os.path.join(os.path.dirname(__file__), "..", "..", "fixtures", "inputData.mat"),
    "/root/reference/inputData.mat",
)


def fixture_path() -> Optional[str]:
    for p in _FIXTURE_CANDIDATES:
        p = os.path.abspath(p)
        if os.path.exists(p):
            return p
    return None


@dataclass
class RankOneBasis:
    """Orthonormal rank-one projectors ``P_n = q_n q_n^T`` and the shared label vector."""

    P: np.ndarray  # (K, d, d) float64
    y: np.ndarray  # (m,) float64
    source: str


def rank_one_basis(num_workers: int, dim: int = 50, seed: int = 0,
                   use_fixture: bool = True) -> RankOneBasis:
    """Return ``num_workers`` projectors.

    With the reference fixture present (and ``num_workers <= 24``, ``dim == 50``) the projectors are
    read off ``inputData.mat`` (``P_n = X_n - I``), otherwise ``Q`` comes from the QR factorisation
    of a seeded Gaussian matrix, exactly as the reference builds it (``qr(randn(...))``).
    Labels: the fixture's block-0 labels, or seeded +-1.
    """
    path = fixture_path() if use_fixture else None
    rng = np.random.default_rng(seed)
    if path is not None and dim == 50:
        X, y = load_input_data(path)
        blocks = X.reshape(-1, 50, 50)
        y0 = y[:50].astype(np.float64)
        P_fix = blocks - np.eye(50)[None]
        if num_workers <= P_fix.shape[0]:
            return RankOneBasis(P=P_fix[:num_workers].copy(), y=y0, source="inputData.mat")
        # More workers than the fixture holds (e.g. N = 50 in the dynamic experiment): complete the
        # fixture's 24 orthonormal directions to a full basis of R^50.
        q = np.stack([_top_eigvec(p) for p in P_fix], axis=1)  # (50, 24)
        comp = rng.standard_normal((50, 50 - q.shape[1]))
        comp -= q @ (q.T @ comp)
        qc, _ = np.linalg.qr(comp)
        Q = np.concatenate([q, qc], axis=1)
        if num_workers > Q.shape[1]:
            raise ValueError("at most %d orthonormal directions in R^50" % Q.shape[1])
        P = np.einsum("in,jn->nij", Q[:, :num_workers], Q[:, :num_workers])
        P[: P_fix.shape[0]] = P_fix
        return RankOneBasis(P=P, y=y0, source="inputData.mat+completed")
    if num_workers > dim:
        raise ValueError("need num_workers <= dim orthonormal directions")
    Q, _ = np.linalg.qr(rng.standard_normal((dim, dim)))
    P = np.einsum("in,jn->nij", Q[:, :num_workers], Q[:, :num_workers])
    y = np.where(rng.random(dim) < 0.5, -1.0, 1.0)
    return RankOneBasis(P=P, y=y, source="seeded-qr(seed=%d)" % seed)


def _top_eigvec(P: np.ndarray) -> np.ndarray:
    w, V = np.linalg.eigh(P)
    return V[:, -1]


def _rank_one_dataset(num_workers: int, growth: float, seed: int, use_fixture: bool,
                      name: str, worker_ids=None) -> ShardedDataset:
    basis = rank_one_basis(num_workers, 50, seed=seed, use_fixture=use_fixture)
    d = basis.P.shape[-1]
    eye = np.eye(d)
    ids = list(range(num_workers)) if worker_ids is None else [int(w) for w in worker_ids]
    X = np.stack([growth ** n * basis.P[n] + eye for n in ids])
    y = np.broadcast_to(basis.y, (len(ids), basis.y.shape[0])).copy()
    return ShardedDataset(X=torch.from_numpy(X), y=torch.from_numpy(y), name=name,
                          meta={"source": basis.source, "growth": growth, "worker_ids": ids,
                                "num_workers_total": num_workers})


def linear_synthetic(num_workers: int = 24, seed: int = 0, use_fixture: bool = True,
                     worker_ids=None) -> ShardedDataset:
    """E1/E5/E7 design: ``X_n = 1.3^(n-1) q_n q_n^T + I`` (LinearRegression_Synthetic.m:32).
    ``worker_ids``: build only these workers' shards (a rank materialises nothing else)."""
    return _rank_one_dataset(num_workers, 1.3, seed, use_fixture, "linear_synthetic", worker_ids)


def logistic_synthetic(num_workers: int = 24, seed: int = 0, use_fixture: bool = True,
                       worker_ids=None) -> ShardedDataset:
    """E3 design: ``X_n = q_n q_n^T + I`` with +-1 labels (LogisticRegression_Synthetic.m:31-35)."""
    return _rank_one_dataset(num_workers, 1.0, seed, use_fixture, "logistic_synthetic", worker_ids)


def gaussian_regression(num_workers: int, rows_per_worker: int, dim: int, seed: int = 0,
                        noise: float = 0.1, labels: str = "linear",
                        device: Optional[torch.device] = None,
                        worker_ids: Optional[list] = None) -> ShardedDataset:
    """Real-shaped synthetic shards (Body-Fat / Derm / 10M x 10k shapes).

    Shard ``n`` is generated from its own seed ``(seed, n)`` so every rank can build exactly its own
    workers' shards, on its own device, without materialising anyone else's (the 10M x 10k config
    holds ~100 GB of float64 per MI355X). ``labels='linear'`` gives ``y = X theta* + noise``,
    ``labels='logistic'`` gives ``y = sign(X theta* + noise)``.
    """
    device = torch.device("cpu") if device is None else torch.device(device)
    ids = list(range(num_workers)) if worker_ids is None else list(worker_ids)
    g0 = torch.Generator(device="cpu").manual_seed(seed)
    theta_star = torch.randn(dim, generator=g0, dtype=torch.float64) / max(1.0, dim ** 0.5)
    theta_star = theta_star.to(device)
    Xs, ys = [], []
    for n in ids:
        gen = torch.Generator(device=device).manual_seed(seed * 1000003 + n + 1)
        Xn = torch.randn(rows_per_worker, dim, generator=gen, dtype=torch.float64, device=device)
        eps = torch.randn(rows_per_worker, generator=gen, dtype=torch.float64, device=device)
        yn = Xn @ theta_star + noise * eps
        if labels == "logistic":
            yn = torch.where(yn >= 0, torch.ones_like(yn), -torch.ones_like(yn))
        Xs.append(Xn)
        ys.append(yn)
    return ShardedDataset(X=torch.stack(Xs), y=torch.stack(ys), name="gaussian_%s" % labels,
                          meta={"seed": seed, "noise": noise, "worker_ids": ids,
                                "num_workers_total": num_workers})
