"""Where a D-GADMM solve's wall time goes on the host: stamps at the solve start, at the persistent
kernel launch call, after the launch returns, after the stream sync, and at the solve end (the launch
entry points are wrapped on the ctypes library). Median over 40 solves of the bench config.
Usage: python tools/dgadmm_stage_times.py [coherence]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gadmm_amd.data import linear_synthetic  # noqa: E402
from gadmm_amd.models import LinearRegression  # noqa: E402
from gadmm_amd.algorithms import dynamic_group_admm  # noqa: E402
from gadmm_amd.parallel import topology as T  # noqa: E402
from gadmm_amd.oracle.reference import opt_linear  # noqa: E402
from gadmm_amd.ops import native  # noqa: E402

dev = torch.device("cuda", 0)
ds = linear_synthetic(24)
Xf, yf = ds.stacked()
obj0 = opt_linear(Xf.numpy(), yf.numpy())
m = LinearRegression(ds.X.to(dev).contiguous(), ds.y.to(dev).contiguous())
p0, c0, _ = T.find_path(24, np.random.default_rng(5))
COH = int(sys.argv[1]) if len(sys.argv) > 1 else 10
lib = native.require()
stamps = {}


def _wrap(orig):
    def wrapped(*a):
        stamps["launch"] = time.perf_counter()
        rc = orig(*a)
        stamps["launched"] = time.perf_counter()
        return rc
    return wrapped


# both D-GADMM kernels: the per-worker one and the blocked dynamic mode (GADMM_BLOCKED_DYN=1)
lib.gadmm_chain_persistent_launch = _wrap(lib.gadmm_chain_persistent_launch)
lib.gadmm_chain_blocked_launch = _wrap(lib.gadmm_chain_blocked_launch)
orig_sync = torch.cuda.Stream.synchronize


def sync(self):
    orig_sync(self)
    stamps["synced"] = time.perf_counter()


torch.cuda.Stream.synchronize = sync
acc = {}


def timed(name, fn):
    def w(*a, **k):
        t = time.perf_counter()
        r = fn(*a, **k)
        acc[name] = acc.get(name, 0.0) + time.perf_counter() - t
        return r
    return w


# pieces of the pre-launch path, summed per solve
T.PathSchedule.prefetch_arrays = timed("draws", T.PathSchedule.prefetch_arrays)
T.PathSchedule.__init__ = timed("schedule", T.PathSchedule.__init__)
lib.gadmm_epoch_tables = timed("epoch_tables", lib.gadmm_epoch_tables)
torch.cuda.synchronize = timed("device_sync", torch.cuda.synchronize)
from gadmm_amd.engine import chain_engine as CE  # noqa: E402
CE.NativeChainEngine.reset = timed("reset", CE.NativeChainEngine.reset)
CE.NativeChainEngine.set_path = timed("set_path", CE.NativeChainEngine.set_path)
CE.NativeChainEngine.dynamic_eligible = timed("eligible", CE.NativeChainEngine.dynamic_eligible)
CE.NativeChainEngine.traces = timed("traces", CE.NativeChainEngine.traces)


def solve():
    return dynamic_group_admm(m, 1.0, obj0, 1e-4, 3000, p0, c0, COH, seed=99, n_total=24, local_ids=list(range(24)),
                              engine_opts={"state": False, "residual": False})


for _ in range(3):
    solve()
torch.cuda.synchronize()
rows = []
acc.clear()
for _ in range(40):
    t0 = time.perf_counter()
    r = solve()
    t1 = time.perf_counter()
    rows.append([stamps["launch"] - t0, stamps["launched"] - stamps["launch"], stamps["synced"] - stamps["launched"],
                 t1 - stamps["synced"], t1 - t0])
a = np.median(np.asarray(rows), axis=0) * 1e6
print("coherence %d, %d iterations, engine %s" % (COH, r.iters, r.extra.get("engine")))
print("median us: before launch %.1f | launch call %.1f | kernel + sync %.1f | after sync %.1f | total %.1f"
      % tuple(a))
print("per solve, us: " + ", ".join("%s %.1f" % (k, v / 40 * 1e6) for k, v in sorted(acc.items())))
