"""Large-d SPD inverse (kernel K2 for d > 128): ms per inverse of (A + s I), A = X^T X / m + I.
Usage: python tools/bigd_inverse_bench.py [d ...]  (prints one JSON line per d and path)"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.ops import linalg  # noqa: E402

dev = torch.device("cuda", 0)
dims = [int(a) for a in sys.argv[1:]] or [1024, 4096, 10000]
for d in dims:
    g = torch.Generator(device=dev).manual_seed(d)
    X = torch.randn((2 * d, d), dtype=torch.float64, device=dev, generator=g)
    A = (X.T @ X / (2 * d)).unsqueeze(0).contiguous()
    shifts = torch.tensor([[0.5]], dtype=torch.float64, device=dev)
    paths = [("torch-rocsolver", lambda: linalg.spd_inverse_torch(A, shifts))]
    if hasattr(linalg, "spd_inverse_blocked"):
        paths.append(("native-blocked", lambda: linalg.spd_inverse_blocked(A, shifts)))
    ref = None
    for name, fn in paths:
        out = fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        M = A[0] + 0.5 * torch.eye(d, dtype=torch.float64, device=dev)
        resid = float((M @ out[0, 0] - torch.eye(d, dtype=torch.float64, device=dev)).abs().max())
        diff = float((out - ref).abs().max() / ref.abs().max()) if ref is not None else 0.0
        ref = out if ref is None else ref
        print(json.dumps({"d": d, "path": name, "ms": round(min(ts), 3), "ms_all": [round(t, 3) for t in ts],
                          "nominal_tflops": round(d ** 3 / (min(ts) * 1e-3) / 1e12, 2),
                          "max_abs_residual_MinvM_minus_I": resid, "rel_diff_vs_first": diff}), flush=True)
    del X, A
    torch.cuda.empty_cache()
