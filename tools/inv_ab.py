"""A/B of the batched SPD inverse: the 64-wide kernel must reproduce the general one bit for bit.
    python tools/inv_ab.py"""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gadmm_amd.ops import native
lib = native.require()
dev = torch.device("cuda", 0)
for d, N, nvar in ((50, 24, 2), (14, 10, 2), (34, 10, 1), (64, 8, 3), (7, 3, 1)):
    X = torch.randn(N, 3 * d, d, dtype=torch.float64, device=dev)
    A = (X.transpose(1, 2) @ X).contiguous()
    sh = torch.rand(N, nvar, dtype=torch.float64, device=dev) * 3 + 0.1
    outs = []
    for env in ("1", "0"):
        os.environ["GADMM_GJ64"] = env
        o = torch.empty(N, nvar, d, d, dtype=torch.float64, device=dev)
        st = torch.zeros(1, dtype=torch.int32, device=dev)
        native.check(lib.gadmm_spd_inverse_small_f64(A.data_ptr(), sh.data_ptr(), N, d, nvar, o.data_ptr(),
                                                     st.data_ptr(), torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        outs.append(o)
    ref = torch.linalg.inv(A[:, None] + sh[..., None, None] * torch.eye(d, dtype=torch.float64, device=dev))
    err = ((outs[0] - ref).abs().max() / ref.abs().max()).item()
    print("d=%d N=%d nvar=%d rel err vs torch %.2e bit-identical to the general kernel: %s"
          % (d, N, nvar, err, bool(torch.equal(outs[0], outs[1]))))
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    lib.gadmm_spd_inverse_small_f64(A.data_ptr(), sh.data_ptr(), N, d, nvar, o.data_ptr(), st.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
print("us per call (last shape)", (time.perf_counter() - t0) / 20 * 1e6)
