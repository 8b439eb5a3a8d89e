"""Where the large-d native LAG (first_order_big.hip) and the torch loop part ways at d = 300 (VERDICT r04
weak #5): per-iteration upload counts of both, the first differing iteration, and the torch run's closest
trigger decision (relative margin). A margin far above rounding with different counts = a bug, not a tie."""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from gadmm_amd.data import gaussian_regression  # noqa: E402
from gadmm_amd.models import LinearRegression  # noqa: E402
from gadmm_amd.algorithms import lag, global_constants  # noqa: E402

dev = torch.device("cuda", 0)
for seed in (11, 12):
    ds = gaussian_regression(4, 600, 300, seed=seed, labels="linear", device=dev)
    m = LinearRegression(ds.X, ds.y)
    c = global_constants(m)
    s, obj0, hmax = c["stepsize"], m.optimum(), m.hmax()
    for v in ("PS", "WK"):
        a = lag(m, list(range(4)), 4, 300, obj0, s, hmax, v)
        b = lag(m, list(range(4)), 4, 300, obj0, s, hmax, v, backend="torch")
        ua, ub = np.diff(np.concatenate([[0.0], a.comm_units])), np.diff(np.concatenate([[0.0], b.comm_units]))
        diff = np.nonzero(np.abs(a.obj - b.obj) > 1e-9 * np.abs(b.obj))[0]
        first = int(diff[0]) + 1 if len(diff) else None
        print("seed %d LAG-%s engine=%s uploads native=%s torch=%s torch_margin=%.3e first_obj_diff_iter=%s"
              % (seed, v, a.extra.get("engine"), a.extra.get("uploads"), b.extra.get("uploads"),
                 b.extra["trigger_margin"], first), flush=True)
        if first is not None:
            lo = max(0, first - 4)
            print("  units/iter native", ua[lo:first + 2].tolist(), "torch", ub[lo:first + 2].tolist(), flush=True)
            print("  obj native", a.obj[lo:first + 2].tolist(), flush=True)
            print("  obj torch ", b.obj[lo:first + 2].tolist(), flush=True)
