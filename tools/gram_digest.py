"""Digest of the Gram kernel's output on fixed seeded shards (compare runs under different kernel
switches, e.g. GADMM_GRAM_OZAKI=0 / 1 or GADMM_GRAM_INT8=crt / digits): python tools/gram_digest.py"""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.ops import linalg  # noqa: E402

dev = torch.device("cuda", 0)
for (N, m, d) in ((2, 1500, 1100), (1, 40000, 260), (2, 4096, 2100)):
    g = torch.Generator(device=dev).manual_seed(N * 7 + d)
    X = torch.randn(N, m, d, dtype=torch.float64, device=dev, generator=g)
    y = torch.randn(N, m, dtype=torch.float64, device=dev, generator=g)
    A, b, yy = linalg.gram(X, y)
    h = hashlib.sha256()
    for t in (A, b, yy):
        h.update(t.cpu().numpy().tobytes())
    print("gram %dx%dx%d sha256 %s" % (N, m, d, h.hexdigest()[:32]), flush=True)
