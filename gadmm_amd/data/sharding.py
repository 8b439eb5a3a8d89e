"""Sharded dataset container: worker ``n`` owns rows ``[n*m, (n+1)*m)`` of the stacked data.

Reference layout: ``X_fede``/``y_fede`` are the row-stacked shards and worker ``ii`` reads rows
``(ii-1)*s2+1 : ii*s2`` (``group_ADMM_closedForm.m:30-34``; ``LinearRegression_Real.m:33-39``).
Here the shards are kept as one ``(N, m, d)`` tensor so batched kernels see a single base pointer
with a fixed worker stride.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Any

import torch


@dataclass
class ShardedDataset:
    X: torch.Tensor  # (N, m, d) float64
    y: torch.Tensor  # (N, m)    float64
    name: str = "dataset"
    meta: Dict[str, Any] = field(default_factory=dict)

    def __post_init__(self):
        if self.X.dim() != 3 or self.y.dim() != 2:
            raise ValueError("expected X (N,m,d) and y (N,m)")
        if self.X.shape[:2] != self.y.shape:
            raise ValueError("X and y shard shapes disagree: %s vs %s" % (tuple(self.X.shape), tuple(self.y.shape)))
        self.X = self.X.to(torch.float64)
        self.y = self.y.to(torch.float64)

    @property
    def num_workers(self) -> int:
        return self.X.shape[0]

    @property
    def rows_per_worker(self) -> int:
        return self.X.shape[1]

    @property
    def dim(self) -> int:
        return self.X.shape[2]

    def stacked(self):
        """Row-stacked ``(X_fede, y_fede)`` as in the reference scripts."""
        N, m, d = self.X.shape
        return self.X.reshape(N * m, d), self.y.reshape(N * m)

    def subset(self, workers) -> "ShardedDataset":
        idx = torch.as_tensor(list(workers), dtype=torch.long, device=self.X.device)
        return ShardedDataset(X=self.X.index_select(0, idx), y=self.y.index_select(0, idx),
                              name=self.name, meta=dict(self.meta, workers=list(workers)))

    def to(self, device) -> "ShardedDataset":
        return ShardedDataset(X=self.X.to(device), y=self.y.to(device), name=self.name, meta=dict(self.meta))

    def numpy(self):
        return self.X.cpu().numpy(), self.y.cpu().numpy()


def from_stacked(X_fede: torch.Tensor, y_fede: torch.Tensor, rows_per_worker: int,
                 name: str = "stacked") -> ShardedDataset:
    """Split row-stacked data into ``floor(n / rows_per_worker)`` equal shards (the remainder rows
    are dropped, like ``LinearRegression_Real.m:13-18`` which uses ``floor(total/25)`` workers)."""
    X_fede = torch.as_tensor(X_fede, dtype=torch.float64)
    y_fede = torch.as_tensor(y_fede, dtype=torch.float64).reshape(-1)
    n = X_fede.shape[0] // rows_per_worker
    X = X_fede[: n * rows_per_worker].reshape(n, rows_per_worker, X_fede.shape[1])
    y = y_fede[: n * rows_per_worker].reshape(n, rows_per_worker)
    return ShardedDataset(X=X.contiguous(), y=y.contiguous(), name=name)


def split_workers(X_fede: torch.Tensor, y_fede: torch.Tensor, num_workers: int,
                  name: str = "stacked") -> ShardedDataset:
    """``per_split = floor(n / N)`` contiguous shards (``LogisticRegression_real.m:17-34``)."""
    per = X_fede.shape[0] // num_workers
    return from_stacked(X_fede[: per * num_workers], y_fede[: per * num_workers], per, name=name)
