"""One CRT Gram (after a warm-up) of an N x m x d shard for rocprofv3 kernel traces."""
import sys
import torch
sys.path.insert(0, ".")
from gadmm_amd.ops import linalg
N, m, d = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1x625000x10000").split("x"))
which = sys.argv[2] if len(sys.argv) > 2 else "crt"
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(0)
X = torch.randn((N, m, d), dtype=torch.float64, device=dev, generator=g)
y = torch.randn((N, m), dtype=torch.float64, device=dev, generator=g)
fn = linalg.gram_crt if which == "crt" else linalg.gram_ozaki
for _ in range(2):
    fn(X, y)
torch.cuda.synchronize()
print("done", flush=True)
