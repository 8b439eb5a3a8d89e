"""Small SPD inverse (spd_inverse_reg64_kernel) on the headline's 24 shifted Grams (d = 50): prints us per
batched call (hip events) and writes the result to argv[1] (.pt) for a bitwise A/B between builds
(GADMM_NATIVE_LIB). python tools/inv_small_ab.py OUT.pt"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from gadmm_amd.data import linear_synthetic
from gadmm_amd.models import LinearRegression
from gadmm_amd.ops.linalg import spd_inverse


def main():
    dev = torch.device("cuda", 0)
    ds = linear_synthetic(24)
    m = LinearRegression(ds.X.to(dev).contiguous(), ds.y.to(dev).contiguous())
    sh = torch.tensor([[3.0, 6.0]] * 24, dtype=torch.float64)
    out = spd_inverse(m.A, sh)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        for _ in range(20):
            spd_inverse(m.A, sh, out=out)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / 20)
    ref = torch.linalg.inv(m.A.unsqueeze(1) + sh.to(dev).view(24, 2, 1, 1) * torch.eye(50, dtype=torch.float64,
                                                                                         device=dev))
    err = float(((out - ref).abs().max() / ref.abs().max()))
    print("spd_inverse 24 x 2 (d = 50): %.1f us per call, max rel err vs torch %.2e" % (best, err), flush=True)
    torch.save(out.cpu(), sys.argv[1])


if __name__ == "__main__":
    main()
