"""One Gram (SYRK) of a (1, M, D) shard, twice, for counter collection: python tools/gram_once.py M D"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gadmm_amd.ops import linalg
M = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
D = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(1, M, D, dtype=torch.float64, device=dev, generator=g)
y = torch.randn(1, M, dtype=torch.float64, device=dev, generator=g)
for _ in range(2):
    linalg.gram(X, y)
torch.cuda.synchronize()
print("ok")
