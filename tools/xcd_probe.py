"""A/B of XCD packing in the temporally blocked kernel (E1 headline, one GPU): GADMM_XCD = 0 (default
grid), 1 (working blocks dealt onto one XCD), 2 (also plain-store publishes after the in-kernel
placement check). Interleaved solves; prints per-mode median wall time, iterations, whether theta is
bit-identical to mode 0, and the XCC_IDs the blocks posted (mode 2). argv[1] = coherence for a
D-GADMM (one-launch dynamic) run instead of the static chain (0 = static)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gadmm_amd.data import linear_synthetic
from gadmm_amd.engine.chain_engine import NativeChainEngine
from gadmm_amd.parallel import topology as T
from gadmm_amd.oracle.reference import opt_linear

dev = torch.device("cuda", 0)
N = int(os.environ.get("XP_N", "24"))
ds = linear_synthetic(N)
Xf, yf = ds.stacked()
obj0 = opt_linear(Xf.numpy(), yf.numpy())
COH = int(sys.argv[1]) if len(sys.argv) > 1 else 0
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 15
eng = NativeChainEngine(ds.X.to(dev), ds.y.to(dev), list(range(N)), N, "linear", rho=1.0, obj0=obj0, tol=1e-4,
                        max_iter=3000)
if COH:
    p0, c0, _ = T.find_path(N, np.random.default_rng(5))
    s = T.PathSchedule(N, p0, c0, COH, seed=99)
    rech = [it for it in range(2, 3001) if T.rechain_iteration(it, COH)]
    pre = s.prefetch(len(rech))
    epochs = [(1, list(p0))] + [(it, pc[0]) for it, pc in zip(rech, pre)]
    eng.set_path(p0, T.Placement.contiguous(N, 1), 0)
else:
    epochs = None
    eng.set_path(list(range(N)), T.Placement.contiguous(N, 1), 0)


def solve(mode):
    os.environ["GADMM_XCD"] = str(mode)
    eng.reset()
    r = eng.run_persistent(epochs=epochs) if epochs is not None else eng.run_persistent()
    torch.cuda.synchronize()
    return r


out = {"coherence": COH, "n": N}
times = {m: [] for m in (0, 1, 2)}
ref = None
for m in (0, 1, 2):
    solve(m)  # warm-up
for rep in range(REPS):
    for m in (0, 1, 2):
        r = solve(m)
        times[m].append(r.wall_ms)
        th = eng.theta.detach().clone() if hasattr(eng, "theta") else None
        if m == 0 and ref is None:
            ref = (r.iters, th)
        out.setdefault("iters_%d" % m, r.iters)
        if th is not None and ref[1] is not None:
            out["bitident_%d" % m] = bool(out.get("bitident_%d" % m, True) and torch.equal(th, ref[1]))
        if m == 2 and rep == 0:
            tab = eng._xchk.view(-1, 4).cpu().numpy().astype(np.uint32)
            ids = []
            for g in tab:
                if g[0] != 0x5a5a0001:
                    break
                ids.append(float(np.array([(int(g[3]) << 32) | int(g[1])], dtype=np.uint64).view(np.float64)[0]))
            out["xcc_ids_mode2"] = ids
for m in (0, 1, 2):
    out["ms_median_%d" % m] = float(np.median(times[m]))
    out["ms_min_%d" % m] = float(np.min(times[m]))
out["kernel"] = eng.last_kernel
print(json.dumps(out))
