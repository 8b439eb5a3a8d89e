"""GPU time of the per-solve cached inverses (K2) at the headline shape: 24 workers x 2 shifts of
50 x 50 SPD matrices, gadmm_spd_inverse_small_f64, register kernel vs the LDS kernel (GADMM_INV_REG=0) and
against torch's f64 inverse. Usage: python tools/inverse_bench.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.ops.linalg import spd_inverse, spd_inverse_torch  # noqa: E402

dev = torch.device("cuda", 0)
REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 200
g = torch.Generator(device="cpu").manual_seed(3)
X = torch.randn((24, 200, 50), generator=g, dtype=torch.float64)
A = (X.transpose(1, 2) @ X).to(dev)
shifts = torch.tensor([[3.0, 6.0]] * 24, dtype=torch.float64, device=dev)
ref = spd_inverse_torch(A, shifts)
out = torch.empty_like(ref)
st = torch.zeros((1,), dtype=torch.int32, device=dev)


def timed(fn):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / REPS


for nw in ("8", "0"):
    os.environ["GADMM_INV_REG"] = nw
    us = timed(lambda: spd_inverse(A, shifts, out=out, check_status=False, status=st))
    err = float(((out - ref).abs().max() / ref.abs().max()).item())
    print("GADMM_INV_REG=%-2s %7.2f us per call (24 x 2 inverses), max rel err vs torch %.1e" % (nw, us, err), flush=True)
os.environ.pop("GADMM_INV_REG")
print("torch.linalg.inv        %7.2f us" % timed(lambda: spd_inverse_torch(A, shifts)), flush=True)
