"""Time the batched SPD inverse of the E1 set-up (24 workers, d = 50, 2 shifts) with the current
library (or GADMM_NATIVE_LIB): python tools/inv_time.py"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gadmm_amd.ops import native
lib = native.require()
dev = torch.device("cuda", 0)
N, d, nvar = 24, 50, 2
X = torch.randn(N, 3 * d, d, dtype=torch.float64, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
A = (X.transpose(1, 2) @ X).contiguous()
sh = torch.tensor([[3.0, 6.0]] * N, dtype=torch.float64, device=dev)
o = torch.empty(N, nvar, d, d, dtype=torch.float64, device=dev)
st = torch.zeros(1, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream().cuda_stream
for _ in range(5):
    lib.gadmm_spd_inverse_small_f64(A.data_ptr(), sh.data_ptr(), N, d, nvar, o.data_ptr(), st.data_ptr(), s)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(100):
    lib.gadmm_spd_inverse_small_f64(A.data_ptr(), sh.data_ptr(), N, d, nvar, o.data_ptr(), st.data_ptr(), s)
e1.record()
torch.cuda.synchronize()
print("spd_inverse (24 x 2 x 50^2): %.1f us per call; checksum %.17g" % (e0.elapsed_time(e1) * 10, float(o.sum())))
