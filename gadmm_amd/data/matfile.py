"""Safe loaders for the reference's data files.

* ``inputData.mat`` (MAT v5, MACI64): read with ``scipy.io.loadmat`` which parses the MAT v5
  container and never executes anything from the file.
* ``dataNN/data.txt`` + ``dataNN/y.txt`` (the reference's external UCI datasets, not shipped,
  ``LinearRegression_Synthetic.m:6-11``): whitespace-separated numeric text, loaded with
  ``numpy.loadtxt`` when the user provides them.
"""
from __future__ import annotations

import os
from typing import Tuple

import numpy as np


def load_input_data(path: str) -> Tuple[np.ndarray, np.ndarray]:
    import scipy.io as sio

    d = sio.loadmat(path)
    X = np.asarray(d["X_fede"], dtype=np.float64)
    y = np.asarray(d["y_fede"]).astype(np.float64).reshape(-1)
    return X, y


def load_optimal_sol(path: str):
    import scipy.io as sio

    d = sio.loadmat(path)
    return float(np.asarray(d["obj0"]).reshape(-1)[0]), np.asarray(d["opt_obj"], dtype=np.float64).reshape(-1)


def load_uci_dir(root: str) -> Tuple[np.ndarray, np.ndarray]:
    """Load ``root/data.txt`` and ``root/y.txt`` (reference dataset layout)."""
    X = np.loadtxt(os.path.join(root, "data.txt"), dtype=np.float64, ndmin=2)
    y = np.loadtxt(os.path.join(root, "y.txt"), dtype=np.float64).reshape(-1)
    return X, y
