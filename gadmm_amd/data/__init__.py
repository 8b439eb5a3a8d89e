from .sharding import ShardedDataset, from_stacked, split_workers
from .synthetic import linear_synthetic, logistic_synthetic, gaussian_regression, rank_one_basis, fixture_path

__all__ = ["ShardedDataset", "from_stacked", "split_workers", "linear_synthetic",
           "logistic_synthetic", "gaussian_regression", "rank_one_basis", "fixture_path"]
