"""On-device tests (MI355X): HIP kernels vs fp64 torch references, engine paths vs the reference
iteration counts, RCCL communicator and graph capture, bench/smoke entry points."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _poison_lds():
    """Every GPU test starts with NaN-filled LDS on every CU (csrc/kernels/debug_poison.hip), so a
    kernel that reads padding it never wrote fails here deterministically instead of depending on
    which kernel ran before it."""
    if torch.cuda.is_available():
        from gadmm_amd.ops import native
        native.poison_lds()
    yield


def _rel(a, b):
    return float((a.double().cpu() - b.double().cpu()).abs().max() / max(b.double().abs().max().item(), 1e-300))


@pytest.mark.parametrize("N,m,d", [(24, 50, 50), (5, 25, 14), (3, 36, 34), (2, 5000, 70), (2, 300, 200),
                                   (1, 40000, 20), (1, 1500, 1100), (2, 700, 2100)])
def test_gram_kernel_matches_torch(N, m, d):
    from gadmm_amd.ops import linalg
    g = torch.Generator().manual_seed(N * 1000 + d)
    X = torch.randn(N, m, d, dtype=torch.float64, generator=g)
    y = torch.randn(N, m, dtype=torch.float64, generator=g)
    A, b, yy = linalg.gram(X.to(DEV), y.to(DEV))
    A0, b0, yy0 = linalg.gram_torch(X, y)
    assert _rel(A, A0) < 1e-13 and _rel(b, b0) < 1e-13 and _rel(yy, yy0) < 1e-13
    assert torch.equal(A.cpu(), A.cpu().transpose(1, 2))  # exactly symmetric


def test_gram_kernel_asymmetric_identity_check():
    """A = I-style check with asymmetric data (catches row/col swaps in the MFMA C/D map)."""
    from gadmm_amd.ops import linalg
    X = torch.zeros(1, 64, 20, dtype=torch.float64)
    for i in range(20):
        X[0, i, i] = 1.0
        X[0, 20 + i, (i * 7) % 20] = float(i + 1)
    y = torch.arange(64, dtype=torch.float64).unsqueeze(0)
    A, b, yy = linalg.gram(X.to(DEV), y.to(DEV))
    A0, b0, yy0 = linalg.gram_torch(X, y)
    assert torch.equal(A.cpu(), A0) and torch.equal(b.cpu(), b0) and torch.equal(yy.cpu(), yy0)


@pytest.mark.parametrize("d", [14, 34, 50, 100, 128])
def test_spd_inverse_kernel(d):
    from gadmm_amd.ops import linalg
    g = torch.Generator().manual_seed(d)
    Z = torch.randn(6, 2 * d, d, dtype=torch.float64, generator=g)
    A = torch.bmm(Z.transpose(1, 2), Z)
    sh = torch.tensor([0.5, 3.0, 6.0], dtype=torch.float64)
    inv = linalg.spd_inverse(A.to(DEV), sh.to(DEV))
    ref = linalg.spd_inverse_torch(A, sh.unsqueeze(0).expand(6, 3))
    assert _rel(inv, ref) < 1e-11


@pytest.mark.parametrize("rows,cols", [(50, 50), (14, 14), (34, 36), (64, 64), (5, 61), (63, 3)])
def test_quad_gemv_matches_torch(rows, cols):
    """The split-column register GEMV (csrc/include/quad_gemv.h) == the fp64 torch product (its
    bit-identity with the other engines' summation order is checked through the engine traces)."""
    from gadmm_amd.ops import native
    lib = native.require()
    g = torch.Generator().manual_seed(rows * 100 + cols)
    M = torch.randn(7, rows, cols, dtype=torch.float64, generator=g)
    x = torch.randn(7, cols, dtype=torch.float64, generator=g)
    Md, xd = M.to(DEV), x.to(DEV)
    y = torch.empty(7, rows, dtype=torch.float64, device=DEV)
    native.check(lib.gadmm_quad_gemv_test(Md.data_ptr(), xd.data_ptr(), y.data_ptr(), 7, rows, cols,
                                          torch.cuda.current_stream().cuda_stream), "quad_gemv_test")
    ref = torch.einsum("brc,bc->br", M, x)
    assert _rel(y.cpu(), ref) < 1e-14


@pytest.mark.parametrize("d", [7, 50, 64])
def test_spd_inverse_gj64_bit_identical(d, monkeypatch):
    """The 64-wide Gauss-Jordan kernels (d <= 64: register rows, and the LDS variant) reproduce the
    general kernel bit for bit."""
    from gadmm_amd.ops import linalg
    g = torch.Generator().manual_seed(100 + d)
    Z = torch.randn(5, 2 * d, d, dtype=torch.float64, generator=g)
    A = torch.bmm(Z.transpose(1, 2), Z).to(DEV)
    sh = torch.tensor([0.3, 2.0], dtype=torch.float64, device=DEV)
    fast = linalg.spd_inverse(A, sh)             # register-row kernel (default for d <= 64)
    monkeypatch.setenv("GADMM_INV_REG", "0")
    lds64 = linalg.spd_inverse(A, sh)            # the LDS 64-wide kernel
    monkeypatch.setenv("GADMM_GJ64", "0")
    general = linalg.spd_inverse(A, sh)
    assert torch.equal(fast, general) and torch.equal(lds64, general)


def _engine(ds, rho, obj0, tol, **kw):
    from gadmm_amd.engine.chain_engine import NativeChainEngine
    from gadmm_amd.parallel.topology import Placement
    n = ds.num_workers
    eng = NativeChainEngine(ds.X.to(DEV), ds.y.to(DEV), list(range(n)), n, kw.pop("model", "linear"), rho=rho,
                            obj0=obj0, tol=tol, max_iter=kw.pop("max_iter", 3000), **kw)
    eng.set_path(list(range(n)), Placement.contiguous(n, 1), 0)
    eng.reset()
    return eng


@pytest.mark.parametrize("rho,it8", [(3.0, 1373), (5.0, 758), (7.0, 428)])
def test_engine_graph_and_persistent_iterations(lin24, lin_obj0, rho, it8):
    from gadmm_amd.oracle import reference as R
    eng = _engine(lin24, rho, lin_obj0, 1e-8)
    r = eng.run()
    assert r.done == 1 and r.iters == it8 and eng.graph_ok()
    tr = eng.objective_trace(r.iters).copy()
    X, y = lin24.numpy()
    o = R.gadmm_linear(X, y, rho, 50, lin_obj0, 1e-30)
    assert np.allclose(tr[:50], o.obj, rtol=1e-11)
    eng.reset()
    rp = eng.run_persistent()
    assert rp.done == 1 and rp.iters == it8
    assert np.array_equal(eng.objective_trace(it8), tr)  # persistent == graph path, bit for bit
    eng.reset()
    re = eng.run(use_graph=False)
    assert re.iters == it8


@pytest.mark.parametrize("pw,k,L", [(1, 2, 0), (2, 3, 0), (2, 2, 0), (2, 1, 0), (2, 3, 2), (1, 1, 3)])
def test_blocked_layouts_bit_identical(lin24, lin_obj0, pw, k, L, monkeypatch):
    """Both wave layouts of the temporally blocked kernel (pw = 1: one position per wave, 12 waves;
    pw = 2: a head + tail pair per wave, 8 waves) at several (k, L) reproduce the graph path's
    objective trace bit for bit and stop at the reference iteration."""
    monkeypatch.setenv("GADMM_BLOCK_PW", str(pw))
    monkeypatch.setenv("GADMM_BLOCK_K", str(k))
    if L:
        monkeypatch.setenv("GADMM_BLOCK_L", str(L))
    eng = _engine(lin24, 5.0, lin_obj0, 1e-8)
    r = eng.run()
    assert r.done == 1 and r.iters == 758
    tr = eng.objective_trace(758).copy()
    plan = eng.blocked_plan()
    assert plan is not None and plan[0] == k and plan[3] == pw and (not L or plan[1] == L)
    eng.reset()
    rp = eng.run_persistent()
    assert eng.last_kernel.startswith("blocked(") and ("pw=%d" % pw) in eng.last_kernel
    assert rp.done == 1 and rp.iters == 758
    assert np.array_equal(eng.objective_trace(758), tr)


def test_engine_monitor_path_with_rccl_one_rank(lin24, lin_obj0):
    """Multi-rank stop protocol (partial-objective ring, RCCL all-reduce, monitor kernel) on one GPU."""
    import torch.distributed as dist
    from gadmm_amd.parallel.comm import RcclComm
    from gadmm_amd.parallel.launch import free_port
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=0, world_size=1, init_method="tcp://127.0.0.1:%d" % free_port())
    comm = RcclComm(DEV)
    eng = _engine(lin24, 5.0, lin_obj0, 1e-8, comm=comm, force_monitor=True, block=16)
    r = eng.run()
    assert r.done == 1 and r.iters == 758
    assert r.iterations_launched >= 758 and r.iterations_launched - 758 < 3 * 16
    assert eng.graph_ok()  # RCCL all-reduce captured into the hipGraph
    # RCCL ops: all-reduce / broadcast / self send-recv
    t = torch.arange(8, dtype=torch.float64, device=DEV)
    comm.allreduce_sum(t)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), torch.arange(8, dtype=torch.float64))
    src = torch.randn(5, dtype=torch.float64, device=DEV)
    dst = torch.zeros(5, dtype=torch.float64, device=DEV)
    comm._raw([(0, 1, src), (0, 0, dst)])
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    assert comm.alive
    eng.close()
    comm.close()


_RCCL_WATCHDOG_SCRIPT = r'''
import time, torch, torch.distributed as dist
from gadmm_amd.parallel.comm import RcclComm
from gadmm_amd.parallel.launch import free_port
from gadmm_amd.ops import native
dist.init_process_group("gloo", rank=0, world_size=1, init_method="tcp://127.0.0.1:%d" % free_port())
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
c = RcclComm(dev, timeout_s=3.0)
t = torch.arange(1000, dtype=torch.float64, device=dev)
c.allreduce_sum(t)
print("SUM", float(t.sum()), flush=True)
st = torch.cuda.current_stream(dev).cuda_stream
t0 = time.time()
try:
    # a stalled peer, bounded: the stream stays busy for 4 s, the watchdog's deadline is 1 s
    native.check(native.require().gadmm_debug_busy_wait(4.0, st), "busy_wait")
    c.wait(timeout_s=1.0)
    print("NO_HANG", flush=True)
except native.RcclDead as e:
    print("WATCHDOG %.2f" % (time.time() - t0), flush=True)
print("ALIVE", c.alive, flush=True)
try:
    c.allreduce_sum(t)
    print("USED_AFTER_ABORT", flush=True)
except native.RcclDead:
    print("REFUSED", flush=True)
c.close()
torch.cuda.synchronize()
print("CLEAN_EXIT", flush=True)
'''


def test_rccl_watchdog_aborts_a_stalled_wait():
    """RCCL has no deadline of its own (VERDICT r04 missing #1): a host wait on a stream that does not
    finish (a stalled peer; here a bounded 4 s busy kernel, the deadline 1 s) ends at the watchdog's
    deadline -- the communicator is aborted (ncclCommAbort), the stream drains, native.RcclDead is raised
    (the caller falls back), and the dead communicator refuses further calls. The communicator itself is
    non-blocking (its set-up and the all-reduce before run through the deadline-bounded settle). Run in
    a child process so that a watchdog that failed could only hang the child (killed at 90 s). (A lone
    RCCL receive cannot stand in for the stalled peer on one rank: RCCL rejects it as invalid usage.)"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", _RCCL_WATCHDOG_SCRIPT], cwd=root, capture_output=True, text=True,
                       timeout=90, env=dict(os.environ, PYTHONPATH=root))
    out = p.stdout
    assert p.returncode == 0 and "CLEAN_EXIT" in out, (p.returncode, out[-2000:], p.stderr[-3000:])
    assert "SUM 499500.0" in out and "NO_HANG" not in out
    secs = float(out.split("WATCHDOG ")[1].split()[0])
    assert 3.5 <= secs <= 15.0, out  # the 1 s deadline, then the drain of the 4 s kernel
    assert "ALIVE False" in out and "REFUSED" in out


def test_graph_engine_rccl_deadline_aborts_and_raises(lin24, lin_obj0):
    """The chain engine's bounded host waits (chain_engine.cpp): with an RCCL data plane and a deadline
    shorter than one replay, the run returns GADMM_ENGINE_TIMEOUT (native.NativeTimeout) after aborting
    the communicator, instead of blocking in hipEventSynchronize."""
    import torch.distributed as dist
    from gadmm_amd.ops import native
    from gadmm_amd.parallel.comm import RcclComm
    from gadmm_amd.parallel.launch import free_port
    if not dist.is_initialized():
        dist.init_process_group("gloo", rank=0, world_size=1, init_method="tcp://127.0.0.1:%d" % free_port())
    comm = RcclComm(DEV)
    eng = _engine(lin24, 5.0, lin_obj0, 1e-8, comm=comm, force_monitor=True, block=16)
    assert eng.run().iters == 758  # the normal deadline (60 s): converges
    eng.reset()
    comm.timeout_s = 1e-6
    with pytest.raises(native.NativeTimeout):
        eng.run()
    assert not comm.alive
    torch.cuda.synchronize()
    eng.close()
    comm.close()


def test_engine_logistic(log24, log_obj0):
    eng = _engine(log24, 2e-4, log_obj0, 1e-4, model="logistic", lam=1e-5, step=2.2, max_inner=100, inner_tol=1e-4,
                  max_iter=400, block=8)
    r = eng.run()
    assert r.iters == 53
    eng.reset()
    eng.set_targets(log_obj0, 1e-4)
    assert eng.run(use_graph=False).iters == 53


@pytest.mark.parametrize("chord,persistent", [(0.0, False), (0.02, False), (0.1, False), (0.0, True), (0.02, True),
                                              (0.1, True), (0.3, True), (None, True)])
def test_logistic_newton_kernel_matches_torch(log24, log_obj0, chord, persistent):
    """Exact local solves on the device vs the torch Newton path on the same device: the
    1e-8 gap at the same iteration and objective traces equal to ~1e-12. persistent = False: the graph
    engine's phase kernels (chain_newton.hip: MFMA Hessian, in-place block Gauss-Jordan inverse);
    persistent = True: ONE launch (chain_persistent_newton.hip: a solver wave runs the chord steps, a
    4-wave crew rebuilds the inverse Hessian at the worker's previous iterate off the critical path).
    chord = 0: a fresh inverse every Newton step; chord > 0: the inverse is reused while steps contract
    by that factor."""
    import time
    from gadmm_amd.models import LogisticRegression
    from gadmm_amd.algorithms.gadmm import group_admm_logistic_exact
    m = LogisticRegression(log24.X.to(DEV), log24.y.to(DEV), lam=1e-5)
    a = group_admm_logistic_exact(m, 1e-3, log_obj0, 1e-8, 1000,
                                  engine_opts={"chord": chord, "cache": False, "persistent": persistent}
                                  if chord is not None else {"cache": False, "persistent": persistent})
    assert a.extra["backend"] == "native" and a.extra["solver"] == "newton"
    assert (a.extra["engine"] == "persistent") == persistent, a.extra["engine"]
    eng = a.extra["engine_obj"]
    used = eng.inner_iters.cpu().numpy()
    assert 1 <= used.min() and used.max() < 50  # Newton converged inside its cap on every worker
    t0 = time.perf_counter()
    b = group_admm_logistic_exact(m, 1e-3, log_obj0, 1e-8, 1000, backend="torch")
    t_torch = time.perf_counter() - t0
    assert b.extra["backend"] == "torch"
    assert a.iters == b.iters == 424 and a.converged and b.converged
    np.testing.assert_allclose(a.obj, b.obj, rtol=1e-12, atol=0)
    # the effective chord is recorded: the engine default (0.02 graph / 0.3 persistent) when none is given
    assert a.extra["chord"] == (chord if chord is not None else (0.3 if persistent else 0.02))
    assert a.extra["obj_mode"] == "exact"
    print("newton(chord=%s, persistent=%s): native %.1f ms, torch %.1f ms, %d iterations"
          % (chord, persistent, a.wall_s * 1e3, t_torch * 1e3, a.iters))


@pytest.mark.parametrize("rec,knobs", [("0", {}), ("1", {"GADMM_NEWTON_RLAG": "1", "GADMM_NEWTON_BG": "1"}),
                                       ("1", {"GADMM_NEWTON_URGENT_NS": "1"})])
def test_newton_persistent_variants_match_torch(log24, log_obj0, rec, knobs, monkeypatch):
    """Both persistent exact-logistic kernels stay exact: the round-4 one-wave solver kernel
    (GADMM_NEWTON_REC=0) and the four-wave pipeline under other refresh schedules (lag 1 / threshold 1,
    urgent refreshes by Newton-Schulz) -- the schedule changes which inverse a chord step uses, never the
    fixed point: 424 iterations and the torch trace to 1e-12."""
    from gadmm_amd.models import LogisticRegression
    from gadmm_amd.algorithms.gadmm import group_admm_logistic_exact
    monkeypatch.setenv("GADMM_NEWTON_REC", rec)
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    m = LogisticRegression(log24.X.to(DEV), log24.y.to(DEV), lam=1e-5)
    a = group_admm_logistic_exact(m, 1e-3, log_obj0, 1e-8, 1000, engine_opts={"cache": False, "persistent": True})
    assert a.extra["engine"] == "persistent", a.extra["engine"]
    b = group_admm_logistic_exact(m, 1e-3, log_obj0, 1e-8, 1000, backend="torch")
    assert a.iters == b.iters == 424 and a.converged
    np.testing.assert_allclose(a.obj, b.obj, rtol=1e-12, atol=0)


def test_lds_poison_lands():
    """The poison kernel really leaves NaN patterns in LDS: a probe kernel that reads LDS it never
    wrote finds them (otherwise the autouse poison fixture would be vacuous)."""
    from gadmm_amd.ops import native
    lib = native.require()
    native.poison_lds()
    blocks, words = 64, 2048
    out = torch.zeros(blocks, words, dtype=torch.int64, device=DEV)
    native.check(lib.gadmm_lds_probe(out.data_ptr(), blocks, words, native.stream_handle()), "lds_probe")
    hi = (out.cpu() >> 32) & 0xffffffff
    frac = float((hi == 0x7ff8dead).double().mean())
    assert frac > 0.99, frac


@pytest.mark.parametrize("d,m", [(50, 50), (3, 7), (34, 36)])
def test_newton_after_lds_poison(d, m):
    """chain_newton.hip read the gradient's padding slots d..63 (never written)
    and multiplied them by the inverse's exact-zero identity padding: 0 * NaN = NaN at iteration 1
    whenever the previous kernel on the CU had left a NaN there. With NaN-filled LDS before EVERY
    launch of the solve the kernel must still match the torch Newton path."""
    from gadmm_amd.ops import native
    from gadmm_amd.models import LogisticRegression
    from gadmm_amd.algorithms import chain_admm
    n = 4
    g = torch.Generator().manual_seed(7 * d + m)
    X = torch.randn(n, m, d, dtype=torch.float64, generator=g) / np.sqrt(d)
    y = torch.where(torch.randn(n, m, dtype=torch.float64, generator=g) > 0, 1.0, -1.0).to(torch.float64)
    mod = LogisticRegression(X.to(DEV), y.to(DEV), lam=1e-3)
    native.poison_lds()
    a = chain_admm(mod, list(range(n)), n, 0.05, 0.0, 1e-300, 6, local_solver="newton",
                   engine_opts={"chord": 0.0, "cache": False})
    b = chain_admm(mod, list(range(n)), n, 0.05, 0.0, 1e-300, 6, local_solver="newton", backend="torch")
    assert a.extra["backend"] == "native" and a.iters == b.iters == 6
    assert np.isfinite(a.obj).all()
    np.testing.assert_allclose(a.obj, b.obj, rtol=1e-12, atol=0)


@pytest.mark.parametrize("n,m,d", [(5, 36, 34), (4, 25, 14), (3, 64, 64), (6, 7, 3)])
def test_logistic_newton_kernel_odd_shapes(n, m, d):
    """Newton local-solve kernel at the real-shaped (Derm 36 x 34, Body-Fat-like 25 x 14) and edge
    shapes (d = m = 64: full register rows; d = 3: one padded pivot block) vs the torch Newton path:
    30 GADMM iterations, objective traces equal to ~1e-12."""
    from gadmm_amd.models import LogisticRegression
    from gadmm_amd.algorithms import chain_admm
    g = torch.Generator().manual_seed(n * 100 + d)
    X = torch.randn(n, m, d, dtype=torch.float64, generator=g) / np.sqrt(d)
    y = torch.where(torch.randn(n, m, dtype=torch.float64, generator=g) > 0, 1.0, -1.0).to(torch.float64)
    mod = LogisticRegression(X.to(DEV), y.to(DEV), lam=1e-3)
    a = chain_admm(mod, list(range(n)), n, 0.05, 0.0, 1e-300, 30, local_solver="newton")
    b = chain_admm(mod, list(range(n)), n, 0.05, 0.0, 1e-300, 30, local_solver="newton", backend="torch")
    assert a.extra["backend"] == "native" and a.iters == b.iters == 30
    np.testing.assert_allclose(a.obj, b.obj, rtol=1e-12, atol=0)


def test_logistic_register_kernel_trace_matches_torch(log24, log_obj0):
    """chain_phase_logistic_quad (shard + transpose in VGPRs) follows the torch inexact-GD path
    (logReg_GD.m semantics) iteration by iteration, not only in the final count."""
    import numpy as np
    from gadmm_amd.models import LogisticRegression
    from gadmm_amd.algorithms import chain_admm
    eng = _engine(log24, 2e-4, log_obj0, 1e-4, model="logistic", lam=1e-5, step=2.2, max_inner=100, inner_tol=1e-4,
                  max_iter=400, block=8)
    r = eng.run()
    tr = eng.objective_trace(r.iters)
    m = LogisticRegression(log24.X, log24.y, lam=1e-5)
    t = chain_admm(m, list(range(24)), 24, 2e-4, log_obj0, 1e-4, 400, local_solver="gd", step=2.2, max_inner=100,
                   inner_tol=1e-4, backend="torch")
    assert r.iters == t.iters == 53
    assert np.allclose(tr, t.obj, rtol=1e-11, atol=0)


def test_chain_admm_auto_native_matches_torch(lin24, lin_obj0):
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import chain_admm, dynamic_group_admm
    from gadmm_amd.parallel import topology as T
    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    r = chain_admm(m, list(range(24)), 24, 7.0, lin_obj0, 1e-8, 3000)
    assert r.extra["backend"] == "native" and r.extra["engine"] == "persistent" and r.iters == 428
    # D-GADMM epochs on the native engine vs the torch path (same seeded chain sequence)
    rng = np.random.default_rng(3)
    p0, c0, _ = T.find_path(24, rng)
    rn = dynamic_group_admm(m, 1.0, lin_obj0, 1e-4, 1500, p0, c0, 10, seed=5)
    mc = LinearRegression(lin24.X, lin24.y)
    rt = dynamic_group_admm(mc, 1.0, lin_obj0, 1e-4, 1500, p0, c0, 10, seed=5, backend="torch")
    assert rn.extra["backend"] == "native" and rn.iters == rt.iters
    assert np.allclose(rn.obj, rt.obj, rtol=1e-9)
    assert np.allclose(rn.com_cost, rt.com_cost)


def test_baselines_run_on_device(lin24, lin_obj0):
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import gd_dgd_lag, dual_averaging, standard_admm, global_constants
    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    out = gd_dgd_lag(m, list(range(24)), 24, 200, lin_obj0)
    mc = LinearRegression(lin24.X, lin24.y)
    outc = gd_dgd_lag(mc, list(range(24)), 24, 200, lin_obj0)
    for k in ("GD", "DGD", "LAG-PS", "LAG-WK", "cIAG"):
        assert np.allclose(out[k].obj, outc[k].obj, rtol=1e-9), k
    assert standard_admm(m, list(range(24)), 24, 1.0, lin_obj0, 1e-4, 1000).iters == 348
    c = global_constants(m)
    assert dual_averaging(m, list(range(24)), 24, c["stepsize"], lin_obj0, 1e-4, 50).iters == 50


@pytest.mark.parametrize("kind", ["linear", "logistic"])
def test_first_order_engine_matches_torch(kind, lin24, log24, lin_obj0, log_obj0):
    """Persistent first-order kernel (one launch per run) vs the torch implementations on the same
    device: objective traces, LAG upload counts, dual averaging (Gauss-Seidel and Jacobi)."""
    from gadmm_amd.models import LinearRegression, LogisticRegression
    from gadmm_amd.algorithms import gd_dgd_lag, dual_averaging, global_constants

    ds, obj0 = (lin24, lin_obj0) if kind == "linear" else (log24, log_obj0)
    m = (LinearRegression if kind == "linear" else LogisticRegression)(ds.X.to(DEV), ds.y.to(DEV),
                                                                      **({} if kind == "linear" else {"lam": 1e-5}))
    ids = list(range(24))
    iters = 1500
    nat = gd_dgd_lag(m, ids, 24, iters, obj0 if kind == "linear" else None, accuracy=1e-4, backend="native")
    ref = gd_dgd_lag(m, ids, 24, iters, obj0 if kind == "linear" else None, accuracy=1e-4, backend="torch")
    for k in ("GD", "DGD", "LAG-PS", "LAG-WK", "cIAG", "R-IAG"):
        assert nat[k].extra.get("engine") == "native-persistent", k
        assert len(nat[k].obj) == len(ref[k].obj), k
        assert np.allclose(nat[k].obj, ref[k].obj, rtol=1e-9, atol=1e-12), k
        assert np.array_equal(nat[k].comm_units, ref[k].comm_units), k
    for k in ("LAG-PS", "LAG-WK"):
        assert nat[k].extra["uploads"] == ref[k].extra["uploads"], k
    step = global_constants(m)["stepsize"]
    for jac in (False, True):
        a = dual_averaging(m, ids, 24, step, obj0, 1e-4, 800, jacobi=jac, backend="native")
        b = dual_averaging(m, ids, 24, step, obj0, 1e-4, 800, jacobi=jac, backend="torch")
        assert a.extra["engine"] == "native-persistent"
        assert len(a.obj) == len(b.obj) and np.allclose(a.obj, b.obj, rtol=1e-9, atol=1e-12), jac


def test_first_order_engine_golden(lin24, lin_obj0):
    """BASELINE.md golden numbers at the reference budget (60,000 iterations), on the native engine:
    GD 53,891; LAG-PS 52,890 (342,113 uploads); LAG-WK 44,368 (58,186 uploads)."""
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import gradient_descent, lag, global_constants

    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    s = global_constants(m)["stepsize"]
    ids = list(range(24))
    gd = gradient_descent(m, ids, 24, 60000, lin_obj0, s, backend="native")
    assert gd.first_below(1e-4) == 53891
    ps = lag(m, ids, 24, 60000, lin_obj0, s, m.hmax(), "PS", backend="native")
    assert ps.first_below(1e-4) == 52890 and ps.extra["uploads"] == 342113
    wk = lag(m, ids, 24, 60000, lin_obj0, s, m.hmax(), "WK", backend="native")
    assert wk.first_below(1e-4) == 44368 and wk.extra["uploads"] == 58186
    assert gd.wall_s < 5.0  # one launch, microseconds per iteration


def test_bench_json_contract():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "3", "--warmup", "1"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    j = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in j
    assert j["iterations_match_reference"] is True and j["value"] < 1.13


def test_graft_smoke():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as ge
    ge.smoke()


@pytest.mark.parametrize("d,obj_mode", [(512, "exact"), (1001, "exact"), (640, "identity"), (384, "auto")])
def test_large_d_engine_matches_torch(d, obj_mode):
    """Large-d phase kernels (d > 256; the inverses streamed as block-packed lower triangles, the
    symmetric GEMV of sym_gemv.h) vs the batched torch path (full inverses) on the same device: the
    same iteration count, traces to 1e-10."""
    from gadmm_amd.data import gaussian_regression
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import chain_admm
    from gadmm_amd.engine.chain_engine import NativeChainEngine
    from gadmm_amd.parallel.topology import Placement
    ds = gaussian_regression(4, 3 * d, d, seed=d, device=DEV)
    m = LinearRegression(ds.X, ds.y)
    obj0 = m.optimum()
    rho = 0.5 * 3 * d
    ref = chain_admm(m, list(range(4)), 4, rho, obj0, 1e-9 * abs(obj0), 400, backend="torch")
    eng = NativeChainEngine(ds.X, ds.y, list(range(4)), 4, "linear", rho=rho, obj0=obj0, tol=1e-9 * abs(obj0),
                            max_iter=400, precomputed=(m.A, m.b, m.yy), obj_mode=obj_mode)
    eng.set_path(list(range(4)), Placement.contiguous(4, 1), 0)
    eng.reset()
    r = eng.run()
    assert eng.obj_mode_name == ("identity" if obj_mode == "auto" else obj_mode)  # auto: identity at d > 256
    assert r.done == 1 and r.iters == ref.iters, (r.iters, ref.iters)
    n = r.iters - 1
    tr = eng.objective_trace(n)
    assert np.allclose(tr, ref.obj[:n], rtol=1e-10)
    th = eng.local_theta().cpu()
    x = m.optimum_point().cpu()
    assert float((th - x).abs().max()) < 1e-6 * float(x.abs().max())


@pytest.mark.parametrize("rows", [20000, 330])
def test_large_d_optimum_solve_paths(rows, monkeypatch):
    """The large-d oracle solve on the device (models/linear.py:_spd_solve, d > 256): CG for a
    well-conditioned Gram (rows >> d), the native Gauss-Jordan inverse when CG does not reach its
    residual (rows ~ d), both against torch's LU to 1e-10, and repeat calls bit-identical."""
    from gadmm_amd.models.linear import _spd_solve, _cg_solve
    d = 300
    g = torch.Generator(device="cpu").manual_seed(3)
    X = torch.randn(rows, d, dtype=torch.float64, generator=g).to(DEV)
    M = X.T @ X
    b = torch.randn(d, dtype=torch.float64, generator=g).to(DEV)
    ref = torch.linalg.solve(M, b)
    cg = _cg_solve(M, b)
    assert (cg is not None) == (rows > 10 * d)
    x1, x2 = _spd_solve(M, b), _spd_solve(M, b)
    assert torch.equal(x1, x2)
    assert float((x1 - ref).abs().max() / ref.abs().max()) < 1e-10
    monkeypatch.setenv("GADMM_OPT_CG", "0")  # the Gauss-Jordan path alone
    xg = _spd_solve(M, b)
    assert float((xg - ref).abs().max() / ref.abs().max()) < 1e-10


@pytest.mark.parametrize("d,db", [(50, 52), (30, 32)])
def test_quad_pad_image_native_matches_torch(d, db):
    """The D-GADMM lane-major inverse image rebuilt in place by the native gather (gadmm_pad_image_f64)
    == the torch-built image, bit for bit."""
    from gadmm_amd.engine.chain_engine import quad_pad_image
    M = torch.randn(6, d, d, dtype=torch.float64, device=DEV)
    ref = quad_pad_image(M.cpu(), db).to(DEV)  # the torch gather (CUDA inputs always take the native one)
    out = torch.full_like(ref, float("nan"))
    got = quad_pad_image(M, db, out=out)
    auto = quad_pad_image(M, db)  # no ``out``: allocated, same native gather
    torch.cuda.synchronize()
    assert got.data_ptr() == out.data_ptr() and torch.equal(got, ref) and torch.equal(auto, ref)


@pytest.mark.parametrize("d", [300, 301])
def test_resid_sq_matches_torch(d):
    """The optimum oracle's residual pass at d > 256 (models/linear.py:_resid_sq, one native pass over
    the shard) == torch's ||X x - y||^2 to 1e-12, bit-identical on repeat calls (even and odd d)."""
    from gadmm_amd.models.linear import _resid_sq
    g = torch.Generator(device="cpu").manual_seed(5)
    X = torch.randn(2, 3000, d, dtype=torch.float64, generator=g).to(DEV)
    y = torch.randn(2, 3000, dtype=torch.float64, generator=g).to(DEV)
    x = torch.randn(d, dtype=torch.float64, generator=g).to(DEV)
    ref = float(((torch.matmul(X, x) - y) ** 2).sum())
    a, b = _resid_sq(X, y, x), _resid_sq(X, y, x)
    assert torch.equal(a, b)
    assert abs(float(a) - ref) <= 1e-12 * ref


@pytest.mark.parametrize("d", [129, 300, 1001, 2048])
def test_sym_pack_roundtrip(d):
    """sym_pack (csrc/kernels/chain_big.hip): the block-packed lower triangle of a symmetric matrix holds
    exactly its lower half (diagonal blocks mirrored), padding zero; unpacking gives the matrix back."""
    import torch
    from gadmm_amd.ops.linalg import sym_pack, sym_unpack_torch
    g = torch.Generator(device="cpu").manual_seed(d)
    M = torch.randn(2, d, d, generator=g, dtype=torch.float64)
    low = torch.tril(M)
    S = low + torch.tril(M, -1).transpose(1, 2)  # the symmetric matrix of M's lower half
    P = sym_pack(M.to(DEV)).cpu()
    assert torch.equal(sym_unpack_torch(P, d), S)
    nb = (d + 127) // 128
    assert P.shape == (2, nb * (nb + 1) // 2 * 128 * 128)


def _xgmi_rank(rank, world, rho, tol):
    import torch
    from gadmm_amd.data import linear_synthetic
    from gadmm_amd.oracle.reference import opt_linear
    from gadmm_amd.engine.chain_engine import NativeChainEngine
    from gadmm_amd.parallel.comm import RankInfo
    from gadmm_amd.parallel.topology import Placement
    from gadmm_amd.parallel.xgmi import XgmiFabric
    dev = torch.device("cuda", 0)  # both ranks share the single GPU of the test box
    torch.cuda.set_device(dev)
    ds = linear_synthetic(24)
    Xf, yf = ds.stacked()
    obj0 = opt_linear(Xf.numpy(), yf.numpy())
    pl = Placement.contiguous(24, world)
    loc = pl.local_workers(rank)
    eng = NativeChainEngine(ds.X[loc].to(dev), ds.y[loc].to(dev), loc, 24, "linear", rho=rho, obj0=obj0, tol=tol,
                            max_iter=3000, comm=RankInfo(rank, world))
    eng.set_path(list(range(24)), pl, rank)
    fab = XgmiFabric(24, 50, 8, rank, world, dev)
    out = []
    for rep in range(3):  # repeated solves: epoch-salted tags, no buffer re-zeroing
        eng.reset()
        r = eng.run_persistent(fabric=fab, timeout_s=20.0)
        out.append((r.iters, r.done))
    tr = eng.objective_trace(out[-1][0]).tolist() if rank == 0 else None
    th = eng.local_theta().cpu().numpy()
    fab.close()
    eng.close()
    return {"runs": out, "trace": tr, "theta": th, "local": loc}


def test_xgmi_fabric_two_processes_one_gpu(lin24, lin_obj0):
    """The multi-GPU device-initiated protocol (IPC fine-grained granule tables, remote pushes,
    rank-0 monitor, decision fan-out) with two processes sharing one MI355X."""
    from gadmm_amd.parallel.launch import spawn
    from gadmm_amd.algorithms import chain_admm
    from gadmm_amd.models import LinearRegression
    res = spawn(_xgmi_rank, 2, 3.0, 1e-8, timeout=300)
    for r in res:
        assert all(it == 1373 and done == 1 for it, done in r["runs"])
    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    single = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 3000)
    assert np.array_equal(np.asarray(res[0]["trace"]), single.obj)  # bit-identical to the 1-GPU persistent run


@pytest.mark.parametrize("coh,blocked", [(10, "1"), (1, "1"), (10, "0"), (1, "0"), (3, "1")])
def test_dgadmm_persistent_dynamic_matches_epoch_path(lin24, lin_obj0, coh, blocked, monkeypatch):
    """D-GADMM in one persistent launch (per-epoch chains in device tables) == the epoch-by-epoch
    engine: same iterations, bit-identical objective trace, same communication-energy trace, and the
    schedule left in the same state. coh = 1 re-chains every iteration: a head's pending-dual flush
    reads its OLD tails' theta while they may already run ahead (the ring-slotted theta table)."""
    import numpy as np
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import dynamic_group_admm
    from gadmm_amd.parallel import topology as T

    monkeypatch.setenv("GADMM_BLOCKED_DYN", blocked)  # 1: the blocked kernel's dynamic mode, 0: per-worker
    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    p0, c0, _ = T.find_path(24, np.random.default_rng(5))
    a = dynamic_group_admm(m, 1.0, lin_obj0, 1e-4, 3000, p0, c0, coh, seed=99)
    kern = a.extra["engine_obj"].last_kernel
    assert kern.startswith("blocked-dyn(") if blocked == "1" else kern == "per-worker", kern
    b = dynamic_group_admm(m, 1.0, lin_obj0, 1e-4, 3000, p0, c0, coh, seed=99, engine_opts={"persistent": False})
    assert a.extra["engine"] == "persistent-dynamic" and b.extra["engine"] == "epochs"
    assert a.iters == b.iters and a.converged
    assert np.array_equal(a.obj, b.obj)
    assert np.allclose(a.com_cost, b.com_cost, rtol=1e-14)


@pytest.mark.parametrize("n", [2, 3, 5])
def test_dgadmm_blocked_dynamic_small_chains_idle_decision_wave(n, monkeypatch):
    """in the blocked kernel's dynamic mode a short chain leaves idle waves
    (u >= nv), and the stop-decision poll may run on one. Idle waves follow the same barrier schedule
    as the active ones, re-chain barriers included, so they must read the same staged epoch starts;
    with unstaged starts an idle decision wave drifted one barrier per re-chain and the launch hung
    (done = 4). Coherence 3 re-chains often: == the epoch-by-epoch engine, bit for bit."""
    import numpy as np
    from gadmm_amd.data import linear_synthetic
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.oracle.reference import opt_linear
    from gadmm_amd.algorithms import dynamic_group_admm
    from gadmm_amd.parallel import topology as T

    monkeypatch.setenv("GADMM_BLOCKED_DYN", "1")
    ds = linear_synthetic(n)
    Xf, yf = ds.stacked()
    obj0 = opt_linear(Xf.numpy(), yf.numpy())
    m = LinearRegression(ds.X.to(DEV), ds.y.to(DEV))
    p0, c0, _ = T.find_path(n, np.random.default_rng(5))
    a = dynamic_group_admm(m, 1.0, obj0, 1e-4, 2000, p0, c0, 3, seed=99)
    assert a.extra["engine_obj"].last_kernel.startswith("blocked-dyn("), a.extra["engine_obj"].last_kernel
    b = dynamic_group_admm(m, 1.0, obj0, 1e-4, 2000, p0, c0, 3, seed=99, engine_opts={"persistent": False})
    assert a.extra["engine"] == "persistent-dynamic" and b.extra["engine"] == "epochs"
    assert a.iters == b.iters and a.converged == b.converged
    assert np.array_equal(a.obj, b.obj)


def _blocked_xgmi_rank(rank, world, rho, tol):
    import torch
    from gadmm_amd.data import linear_synthetic
    from gadmm_amd.oracle.reference import opt_linear
    from gadmm_amd.engine.blocked_xgmi import BlockedXgmiEngine
    from gadmm_amd.parallel.topology import Placement
    dev = torch.device("cuda", 0)  # all ranks share the single GPU of the test box
    torch.cuda.set_device(dev)
    ds = linear_synthetic(24)
    Xf, yf = ds.stacked()
    obj0 = opt_linear(Xf.numpy(), yf.numpy())
    pl = Placement.contiguous(24, world)
    eng = BlockedXgmiEngine(ds.X, ds.y, 24, pl, rank, rho, obj0, tol, 3000, dev)
    out = []
    for rep in range(3):  # repeated solves: epoch-salted tags, no buffer re-zeroing
        eng.refresh()
        it, done, ms = eng.run(timeout_s=20.0)
        out.append((it, done))
    tr = eng.objective_trace(out[-1][0]).tolist() if rank == 0 else None
    kern = eng.last_kernel
    eng.close()
    return {"runs": out, "trace": tr, "kernel": kern}


@pytest.mark.parametrize("world,pw", [(2, 1), (2, 2), (4, 1), (4, 2)])
def test_blocked_xgmi_processes_one_gpu(world, pw, lin24, lin_obj0, monkeypatch):
    """Temporally blocked kernel across ranks (segments + halos, (theta, mu) pushed into the peers'
    IPC exchange tables once per k iterations, objective waves -> rank 0 monitor -> decision fan-out),
    rehearsed with several processes sharing one MI355X: exact iteration count and an objective trace
    bit-identical to the single-GPU run."""
    from gadmm_amd.parallel.launch import spawn
    from gadmm_amd.algorithms import chain_admm
    from gadmm_amd.models import LinearRegression
    monkeypatch.setenv("GADMM_BLOCK_PW", str(pw))  # inherited by the spawned ranks
    res = spawn(_blocked_xgmi_rank, world, 3.0, 1e-8, timeout=300)
    for r in res:
        assert all(it == 1373 and done == 1 for it, done in r["runs"]), r
        assert ("pw=%d" % pw) in r["kernel"]
    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    single = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 3000)
    assert np.array_equal(np.asarray(res[0]["trace"]), single.obj)


@pytest.mark.parametrize("name", ["LinearRegression_Synthetic", "LogisticRegression_Synthetic",
                                  "Dynamic_LinearRegression_Synthetic", "LinearRegression_gadmm_vs_admm"])
def test_entry_points_on_gpu(name, tmp_path):
    """The reference entry scripts end to end on the MI355X (reduced budgets): native engines for
    GADMM / D-GADMM and the persistent first-order engine for the baselines."""
    from gadmm_amd import entry
    argv = ["--quick", "--device", "cuda", "--out", str(tmp_path), "--no-plot"]
    if name.startswith("Dynamic"):
        argv += ["--set", "gadmm_iters=400", "coherences=1,10", "n_pregen_paths=60"]
    out = entry.get(name).main(argv)
    assert out["runs"], out
    for k, r in out["runs"].items():
        assert r["iters"] > 0, (k, r)
    assert os.path.exists(out["summary_path"])


def test_native_entry_measured_clock(tmp_path):
    """E1 on the native engine: the JSONL wall clock is the device's per-iteration decision stamp
    (non-uniform, increasing), next to the reference's modelled 2*toc clock; the figure is written."""
    import json
    from gadmm_amd import entry
    out = entry.get("LinearRegression_Synthetic").main(["--quick", "--device", "cuda", "--out", str(tmp_path),
                                                        "--no-baselines", "--set", "rhos=3", "acc=1e-8", "gadmm_iters=3000"])
    assert out["runs"]["GADMM_rho3"]["iters"] == 1373 and out["runs"]["GADMM_rho3"]["backend"] == "native"
    rows = [json.loads(l) for l in open(os.path.join(tmp_path, "GADMM_rho3.jsonl"))]
    wall = np.asarray([r["wall_s"] for r in rows])
    assert len(wall) == 1373 and np.all(np.diff(wall) >= 0) and wall[-1] > 0
    steps = np.diff(wall)
    assert steps.std() > 0  # measured, not an interpolated ramp
    assert wall[-1] < 0.1  # the whole solve is milliseconds on the device
    mc = np.asarray([r["model_clock_s"] for r in rows])
    assert mc[0] == 0 and np.all(np.diff(mc) > 0)
    assert [f for f in os.listdir(tmp_path) if f.endswith(".png")]


def test_native_run_checkpoint_resumes_in_torch_path(lin24, lin_obj0, tmp_path):
    """A GPU (native persistent) solve leaves a resumable state: per-worker checkpoint written from
    it, reloaded, and continued in the torch path reproduces a continuous torch run's objective."""
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import chain_admm
    from gadmm_amd.utils.checkpoint import save_checkpoint, load_checkpoint
    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    a = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-4, 3000)
    assert a.extra["backend"] == "native" and a.iters == 784
    theta, mu, nxt = a.extra["state"]
    save_checkpoint(str(tmp_path), 0, list(range(24)), theta, mu, nxt, list(range(24)), {"rho": 3.0})
    th2, mu2, nxt2, path2, man = load_checkpoint(str(tmp_path), list(range(24)))
    assert nxt2 == nxt and path2 == list(range(24))
    b = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-30, nxt + 49, backend="torch",
                   state=(th2, mu2, nxt2))
    ref = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-30, nxt + 49, backend="torch")
    assert len(b.obj) == 50
    assert np.allclose(b.obj, ref.obj[nxt - 1:nxt + 49], rtol=1e-10)


@pytest.mark.parametrize("persistent", [True, False])
def test_native_resume_continues_native_run(lin24, lin_obj0, tmp_path, persistent):
    """Checkpoint -> native resume: a native solve's state (per-worker checkpoint files) reloaded and
    continued on the native engine (persistent kernel from start_iter, or the graph engine)
    reproduces the uninterrupted native run's objective trace."""
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import chain_admm
    from gadmm_amd.utils.checkpoint import save_checkpoint, load_checkpoint
    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    opts = {"persistent": persistent}
    a = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-4, 3000, engine_opts=opts)
    assert a.extra["backend"] == "native" and a.iters == 784
    theta, mu, nxt = a.extra["state"]
    save_checkpoint(str(tmp_path), 0, list(range(24)), theta, mu, nxt, list(range(24)), {"rho": 3.0})
    th2, mu2, nxt2, _, _ = load_checkpoint(str(tmp_path), list(range(24)))
    b = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 3000, state=(th2, mu2, nxt2), engine_opts=opts)
    ref = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 3000, engine_opts=opts)
    assert b.extra["backend"] == "native", b.extra
    assert b.iters == ref.iters == 1373
    assert len(b.obj) == 1373 - nxt + 1 and len(b.primal_res) == len(b.obj)
    assert np.allclose(b.obj, ref.obj[nxt - 1:], rtol=1e-12, atol=0)
    assert np.allclose(b.primal_res, ref.primal_res[nxt - 1:], rtol=1e-9, atol=1e-20)


def test_native_resume_logistic_inner_gd(log24, log_obj0):
    """Native resume of the persistent logistic (inner GD) kernel: a solve stopped at a looser gap,
    continued from its state to the reference 1e-4 gap, follows the uninterrupted native solve
    (53 iterations, the reference count)."""
    from gadmm_amd.models import LogisticRegression
    from gadmm_amd.algorithms import chain_admm
    m = LogisticRegression(log24.X.to(DEV), log24.y.to(DEV), lam=1e-5)
    kw = dict(local_solver="gd", step=2.2, max_inner=100, inner_tol=1e-4)
    a = chain_admm(m, list(range(24)), 24, 2e-4, log_obj0, 1e-2, 400, **kw)
    assert a.extra["backend"] == "native" and a.converged and a.iters < 53
    th, mu, nxt = a.extra["state"]
    b = chain_admm(m, list(range(24)), 24, 2e-4, log_obj0, 1e-4, 400, state=(th, mu, nxt), **kw)
    ref = chain_admm(m, list(range(24)), 24, 2e-4, log_obj0, 1e-4, 400, **kw)
    assert b.extra["backend"] == "native" and b.extra["engine"] == "persistent", b.extra
    assert b.iters == ref.iters == 53 and len(b.obj) == 53 - nxt + 1
    assert np.allclose(b.obj, ref.obj[nxt - 1:], rtol=1e-12, atol=0)


def test_native_elastic_matches_torch_path(lin24, lin_obj0):
    """Elastic recovery on the native engine (workers 5 then 17, 18 fail; the survivors' chain
    resumes natively) follows the torch path's elastic run and reaches the survivors' optimum."""
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import chain_admm
    fail = {60: [5], 150: [17, 18]}
    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    nat = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 5000, failures=fail)
    tor = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 5000, failures=fail, backend="torch")
    assert nat.extra["backend"] == "native" and nat.extra["engine"] == "elastic", nat.extra
    segs = nat.extra["segments"]
    assert [(s["first"], s["last"], s["workers"]) for s in segs] == [(1, 59, 24), (60, 149, 23), (150, nat.iters, 21)]
    assert nat.converged and tor.converged and nat.iters == tor.iters
    assert len(nat.obj) == nat.iters
    assert np.allclose(nat.obj, tor.obj, rtol=1e-10, atol=0)
    assert abs(nat.obj[-1] - nat.extra["obj0_final"]) < 1e-8
    alive = [w for w in range(24) if w not in (5, 17, 18)]
    assert np.allclose(nat.extra["state"][0].cpu().numpy()[alive], tor.extra["state"][0].cpu().numpy()[alive],
                       rtol=1e-7, atol=1e-9)


@pytest.mark.parametrize("fail", [{1: [0]}, {3000: [3]}, {40: [23], 41: [22]}])
def test_native_elastic_edge_cases(lin24, lin_obj0, fail):
    """Native elastic recovery at the edges: a failure before the first iteration (the survivors
    start from scratch), one after convergence (never reached: one plain segment) and failures on
    consecutive iterations at the chain's end (a one-iteration segment in between)."""
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import chain_admm
    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    nat = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 5000, failures=fail)
    tor = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 5000, failures=fail, backend="torch")
    assert nat.extra["backend"] == "native" and nat.extra["engine"] == "elastic", nat.extra
    assert nat.converged and tor.converged and nat.iters == tor.iters and len(nat.obj) == nat.iters
    assert np.allclose(nat.obj, tor.obj, rtol=1e-10, atol=0)
    segs = nat.extra["segments"]
    assert segs[0]["first"] == 1 and segs[-1]["last"] == nat.iters
    assert all(b["first"] == a["last"] + 1 for a, b in zip(segs, segs[1:]))


@pytest.mark.parametrize("M,N,K", [(100, 70, 33), (256, 192, 128), (1, 5, 3), (130, 1, 64)])
def test_gemm_f64_mfma_matches_torch(M, N, K):
    """The f64-MFMA tile GEMM of the blocked inverse (spd_inverse_blocked.hip) vs torch fp64."""
    from gadmm_amd.ops.linalg import gemm_f64
    g = torch.Generator().manual_seed(M * 1000 + N + K)
    A = torch.randn(M, K, dtype=torch.float64, generator=g)
    B = torch.randn(K, N, dtype=torch.float64, generator=g)
    C = gemm_f64(A.to(DEV), B.to(DEV)).cpu()
    ref = A @ B
    assert torch.allclose(C, ref, rtol=1e-13, atol=1e-13 * float(ref.abs().max()))


@pytest.mark.parametrize("d", [129, 200, 300, 520])
def test_spd_inverse_blocked_matches_fp64_reference(d):
    """K2 for d > 128: blocked Gauss-Jordan with MFMA rank-128 updates (last block partial for d not a
    multiple of 128) vs the fp64 Cholesky inverse, 2 workers x 2 shifts."""
    from gadmm_amd.ops.linalg import spd_inverse_blocked, spd_inverse_torch
    g = torch.Generator().manual_seed(d)
    X = torch.randn(2, 2 * d, d, dtype=torch.float64, generator=g)
    A = torch.bmm(X.transpose(1, 2), X) / (2 * d)
    shifts = torch.tensor([[0.3, 0.6], [0.1, 1.0]], dtype=torch.float64)
    out = spd_inverse_blocked(A.to(DEV), shifts).cpu()
    ref = spd_inverse_torch(A, shifts)
    assert torch.allclose(out, ref, rtol=1e-11, atol=1e-11 * float(ref.abs().max()))
    assert torch.equal(out, out.transpose(-1, -2))
    eye = torch.eye(d, dtype=torch.float64)
    for n in range(2):
        for v in range(2):
            M = A[n] + shifts[n, v] * eye
            assert float((M @ out[n, v] - eye).abs().max()) < 1e-11


@pytest.mark.parametrize("mode", ["blocked", "per-worker", "graph"])
def test_native_primal_residual_matches_torch(lin24, lin_obj0, mode, monkeypatch):
    """K4 on the device: the tails of every native engine (temporally blocked / per-worker persistent
    kernel, graph-replayed phases) emit ||th_l - th||^2 + ||th - th_r||^2; the per-iteration sum over
    chain edges equals the torch path's primal residual trace."""
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import chain_admm
    if mode == "per-worker":
        monkeypatch.setenv("GADMM_BLOCKED", "0")
    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    opts = {"cache": False, "persistent": mode != "graph"}
    a = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 3000, engine_opts=opts)
    assert a.extra["backend"] == "native" and a.iters == 1373
    assert (a.extra["engine"] == "graph") == (mode == "graph")
    b = chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 3000, backend="torch")
    assert a.primal_res is not None and len(a.primal_res) == 1373
    np.testing.assert_allclose(a.primal_res, b.primal_res[:1373], rtol=1e-6, atol=1e-12 * float(b.primal_res.max()))


def test_native_primal_residual_large_d():
    """K4 from chain_big_post (d > 256, row-blocked phases) vs the torch path."""
    from gadmm_amd.data import gaussian_regression
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import chain_admm
    ds = gaussian_regression(4, 400, 300, seed=3, labels="linear")
    m = LinearRegression(ds.X.to(DEV), ds.y.to(DEV))
    mc = LinearRegression(ds.X, ds.y)
    obj0 = mc.optimum()
    a = chain_admm(m, list(range(4)), 4, 50.0, obj0, 1e-300, 40, engine_opts={"cache": False})
    b = chain_admm(mc, list(range(4)), 4, 50.0, obj0, 1e-300, 40)
    assert a.extra["backend"] == "native" and a.iters == b.iters == 40
    np.testing.assert_allclose(a.primal_res, b.primal_res, rtol=1e-8)


@pytest.mark.parametrize("zrec", ["0", "1"])
def test_logistic_persistent_kernel_matches_graph_engine(log24, log_obj0, zrec, monkeypatch):
    """Inner-GD logistic GADMM in ONE launch (chain_persistent_logistic.hip) at the reference's 53
    iterations (BASELINE configs[2]). zrec = "0": one resident wave per worker (shard in VGPRs, granule
    hand-offs) == the graph-replayed phase kernels bit for bit. zrec = "1" (the default): the margins
    z = X x carried by a recursion on a second wave (z' = z - step (-K s + lam z + X sh), K = X X^T), so
    each inner step's dependent chain holds one GEMV; s differs from X x in rounding only: the trace
    equals the graph engine's and torch's to 1e-12."""
    from gadmm_amd.models import LogisticRegression
    from gadmm_amd.algorithms import chain_admm
    monkeypatch.setenv("GADMM_LOGISTIC_ZREC", zrec)
    m = LogisticRegression(log24.X.to(DEV), log24.y.to(DEV), lam=1e-5)
    kw = dict(local_solver="gd", step=2.2)
    a = chain_admm(m, list(range(24)), 24, 2e-4, log_obj0, 1e-4, 400, engine_opts={"cache": False}, **kw)
    b = chain_admm(m, list(range(24)), 24, 2e-4, log_obj0, 1e-4, 400,
                   engine_opts={"cache": False, "persistent": False, "block": 8}, **kw)
    assert a.extra["engine"] == "persistent" and b.extra["engine"] == "graph"
    assert a.iters == b.iters == 53 and a.converged
    if zrec == "0":
        assert np.array_equal(a.obj, b.obj)
        np.testing.assert_allclose(a.primal_res, b.primal_res, rtol=0, atol=0)
    else:
        np.testing.assert_allclose(a.obj, b.obj, rtol=1e-12, atol=0)
        np.testing.assert_allclose(a.primal_res, b.primal_res, rtol=1e-8, atol=1e-20)
    t = chain_admm(m, list(range(24)), 24, 2e-4, log_obj0, 1e-4, 400, backend="torch", **kw)
    np.testing.assert_allclose(a.obj, t.obj[:53], rtol=1e-12)
    assert np.all(np.diff(a.time_trace) >= 0) and a.time_trace[-1] > 0


@pytest.mark.parametrize("coherence,chunk,blocked", [(10, 4, "0"), (1, 16, "0"), (10, 4, "1"), (1, 16, "1"),
                                                     (3, 5, "1")])
def test_dgadmm_epoch_chunks_bit_identical(lin24, lin_obj0, coherence, chunk, blocked, monkeypatch):
    """D-GADMM in chunks of persistent launches (hard stop before the chunk's last+1 epoch, then a
    continuation with the same tag salt that flushes the pending head duals with the old chain) ==
    one launch holding every epoch == the epoch-by-epoch graph engine: iterations, objective trace and
    energy trace bit for bit; only the chains the solve reaches are drawn. blocked = "1": the
    blocked kernel's dynamic mode (its monitor, objective and worker waves stop at the hard stop)."""
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import dynamic_group_admm
    from gadmm_amd.parallel import topology as T
    monkeypatch.setenv("GADMM_BLOCKED_DYN", blocked)
    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    p0, c0, _ = T.find_path(24, np.random.default_rng(5))
    run = lambda **o: dynamic_group_admm(m, 1.0, lin_obj0, 1e-4, 3000, p0, c0, coherence, seed=99,
                                         engine_opts=dict(cache=False, **o))
    a = run(epoch_chunk=chunk)
    kern = a.extra["engine_obj"].last_kernel
    assert kern.startswith("blocked-dyn(") if blocked == "1" else kern == "per-worker", kern
    b = run(epoch_chunk=100000)
    e = run(persistent=False)
    assert a.extra["engine"] == b.extra["engine"] == "persistent-dynamic" and e.extra["engine"] == "epochs"
    assert a.iters == b.iters == e.iters and a.converged
    assert a.iters > chunk * coherence  # several launches were chained
    assert np.array_equal(a.obj, b.obj) and np.array_equal(a.obj, e.obj)
    assert np.array_equal(a.com_cost, b.com_cost)


def _xcc_ids(xchk):
    """XCC_IDs the blocks of the last XCD-packed launch posted (placement-check granules: the launch's
    own tag, PersistArgs::xtag, high bit set; granules past its blocks hold older launches' tags)."""
    g = xchk.view(-1, 4).cpu().numpy().astype(np.int64) & 0xffffffff
    tag = int(g[0][0])
    ids = []
    for t, lo, t2, hi in g:
        if not (tag & 0x80000000) or t != tag or t2 != t:
            break
        ids.append(float(np.array([(int(hi) << 32) | int(lo)], dtype=np.uint64).view(np.float64)[0]))
    return ids


def test_xcd_packing_bit_identical(lin24, lin_obj0, log24, log_obj0, monkeypatch):
    """XCD packing (PersistArgs::xcd = 2, the default: working workgroups dealt onto one XCD, plain
    L2-resident granule stores once every block reported the same XCC_ID) == the plain grid
    (GADMM_XCD=0) bit for bit in every persistent kernel family: blocked chain, per-worker D-GADMM,
    persistent logistic, star ADMM, first-order engine. The placement check itself must pass (all
    blocks on one XCD), or the fast path would silently not run."""
    from gadmm_amd.models import LinearRegression, LogisticRegression
    from gadmm_amd.algorithms import chain_admm, dynamic_group_admm, standard_admm, gradient_descent, \
        global_constants
    from gadmm_amd.engine.chain_engine import NativeChainEngine
    from gadmm_amd.parallel import topology as T
    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    ml = LogisticRegression(log24.X.to(DEV), log24.y.to(DEV), lam=1e-5)
    p0, c0, _ = T.find_path(24, np.random.default_rng(5))
    step = global_constants(m)["stepsize"]
    runs = {
        "blocked": lambda: chain_admm(m, list(range(24)), 24, 3.0, lin_obj0, 1e-8, 3000,
                                      engine_opts={"cache": False}),
        "dgadmm": lambda: dynamic_group_admm(m, 1.0, lin_obj0, 1e-4, 3000, p0, c0, 1, seed=99,
                                             engine_opts={"cache": False}),
        "logistic": lambda: chain_admm(ml, list(range(24)), 24, 2e-4, log_obj0, 1e-4, 400, local_solver="gd",
                                       step=2.2, engine_opts={"cache": False}),
        "star": lambda: standard_admm(m, list(range(24)), 24, 1.0, lin_obj0, 1e-4, 1000),
        "fo": lambda: gradient_descent(m, list(range(24)), 24, 3000, lin_obj0, step, backend="native"),
    }
    for name, fn in runs.items():
        monkeypatch.setenv("GADMM_XCD", "0")
        a = fn()
        monkeypatch.setenv("GADMM_XCD", "2")
        b = fn()
        assert a.iters == b.iters, name
        assert np.array_equal(np.asarray(a.obj), np.asarray(b.obj)), name
    monkeypatch.delenv("GADMM_XCD")
    eng = NativeChainEngine(lin24.X.to(DEV), lin24.y.to(DEV), list(range(24)), 24, "linear", rho=3.0,
                            obj0=lin_obj0, tol=1e-8, max_iter=3000)
    eng.set_path(list(range(24)), T.Placement.contiguous(24, 1), 0)
    r = eng.run_persistent()
    ids = _xcc_ids(eng._xchk)
    k, L, W, _pw = eng.blocked_plan()
    nblocks = W + (24 + 11) // 12 + 1  # worker + objective workgroups + the monitor
    assert r.done == 1 and len(ids) == nblocks and len(set(ids)) == 1, (r.done, ids)


@pytest.mark.parametrize("n,m,d", [(4, 400, 200), (3, 700, 300), (2, 300, 70)])
def test_star_big_native_matches_torch(n, m, d):
    """Large-d star ADMM (csrc/kernels/star_big.hip: cached-inverse streaming GEMVs, device stop rule,
    blocks of iterations without a host sync) == the torch star path (standared_ADMM.m semantics): the
    same stop iteration and objective traces to ~1e-10; identity and exact objective modes agree."""
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import standard_admm
    g = torch.Generator().manual_seed(n * 1000 + d)
    X = torch.randn(n, m, d, dtype=torch.float64, generator=g)
    y = torch.randn(n, m, dtype=torch.float64, generator=g)
    mod = LinearRegression(X.to(DEV), y.to(DEV))
    obj0 = mod.optimum()
    rho = 0.5 * m
    a = standard_admm(mod, list(range(n)), n, rho, obj0, 1e-8 * abs(obj0), 400)
    assert a.extra["backend"] == "native" and a.extra["engine"].startswith("star-big")
    b = standard_admm(mod, list(range(n)), n, rho, obj0, 1e-8 * abs(obj0), 400, backend="torch")
    assert a.iters == b.iters and a.converged == b.converged
    np.testing.assert_allclose(a.obj, b.obj, rtol=1e-10, atol=0)
    c = standard_admm(mod, list(range(n)), n, rho, obj0, 1e-8 * abs(obj0), 400,
                      engine_opts={"exact_objective": True})
    assert c.iters == a.iters and c.extra["engine"] == "star-big(exact objective)"
    np.testing.assert_allclose(c.obj, a.obj, rtol=1e-9, atol=0)
    assert np.all(np.diff(a.time_trace) >= 0) and a.time_trace[-1] > 0  # measured device clock
    a2 = standard_admm(mod, list(range(n)), n, rho, obj0, 1e-8 * abs(obj0), 400)  # cached engine
    assert a2.iters == a.iters and np.array_equal(a2.obj, a.obj)


# ------------------------------------------------------------------------------------------------
# Large-d first-order comparators (d > 128: first_order_big.hip; VERDICT r03 missing #4)
def _fo_big_problem(n=4, m=600, d=300):
    import torch
    from gadmm_amd.data import gaussian_regression
    from gadmm_amd.models import LinearRegression
    ds = gaussian_regression(n, m, d, seed=11, labels="linear", device=DEV)
    return LinearRegression(ds.X, ds.y)


@pytest.mark.parametrize("alg", ["GD", "DGD", "LAG-PS", "LAG-WK", "cIAG", "R-IAG", "DualAvg", "DualAvg-J"])
def test_first_order_big_matches_torch(alg):
    """GD / DGD / LAG-PS / LAG-WK / cyclic and randomized IAG / dual averaging (Gauss-Seidel and Jacobi) at
    d = 300 on the stream-ordered large-d engine (packed Grams, symmetric GEMV, device stop rule) == the
    torch loop: objective traces to 1e-9, LAG upload counts exact. LAG's triggers are comparisons, so the
    test first checks that the run has no near-tie (the torch loop's closest decision is > 1e-7 relative
    away from its threshold): round 4 dropped LAG here as "near-ties", but the divergence was a bug --
    the LAG step history summed only the first 128 coordinates of |th^k - th^{k-1}|^2 at d > 128
    (tools/lag_diverge.py: margins ~1e-4, profiles/r05_a)."""
    from gadmm_amd.algorithms import gradient_descent, decentralized_gd, lag, iag, dual_averaging, global_constants
    m = _fo_big_problem()
    ids, n, iters = list(range(4)), 4, 300
    c = global_constants(m)
    s, obj0 = c["stepsize"], m.optimum()
    hmax = m.hmax()

    def run(backend):
        if alg == "GD":
            return gradient_descent(m, ids, n, iters, obj0, s, backend=backend)
        if alg == "DGD":
            return decentralized_gd(m, ids, n, iters, obj0, s, backend=backend)
        if alg.startswith("LAG"):
            return lag(m, ids, n, iters, obj0, s, hmax, alg[4:], backend=backend)
        if alg.endswith("IAG"):
            return iag(m, ids, n, iters, obj0, s, "cyclic" if alg == "cIAG" else "random", hmax, backend=backend)
        return dual_averaging(m, ids, n, s, obj0, 1e-12, iters, jacobi=alg.endswith("-J"), backend=backend)

    a, b = run("auto"), run("torch")
    assert a.extra.get("engine") == "native-big", a.extra.get("engine")
    assert len(a.obj) == len(b.obj) == iters
    if alg.startswith("LAG"):
        assert b.extra["trigger_margin"] > 1e-7, b.extra["trigger_margin"]  # no decision at rounding level
        assert a.extra["uploads"] == b.extra["uploads"] and np.array_equal(a.comm_units, b.comm_units)
    np.testing.assert_allclose(a.obj, b.obj, rtol=1e-9, atol=0)
    assert np.all(np.diff(a.time_trace) >= 0)


def test_first_order_big_lag_goldens(lin24, lin_obj0):
    """The large-d engine's GD / LAG-PS / LAG-WK logic on the reference problem (run directly at d = 50):
    the BASELINE.md goldens over the reference budget of 60,000 iterations -- GD first below 1e-4 at
    53,891; LAG-PS 52,890 with 342,113 uploads; LAG-WK 44,368 with 58,186 uploads."""
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import global_constants
    from gadmm_amd.engine.first_order_big import FirstOrderBigEngine
    m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
    s = global_constants(m)["stepsize"]
    hsq = m.hmax() ** 2
    eng = FirstOrderBigEngine(m, n_total=24)
    N = 24

    def first(o):
        hit = np.nonzero(np.abs(o["obj"] - lin_obj0) < 1e-4)[0]
        return int(hit[0]) + 1 if len(hit) else None

    gd = eng.run("GD", 60000, s, lin_obj0, None, True, block=256)
    assert gd["engine"] == "native-big" and first(gd) == 53891
    ps = eng.run("LAG-PS", 60000, s, lin_obj0, None, True, thrd=10.0 / (s ** 2 * N ** 2) / 10, hsq=hsq, block=256)
    assert first(ps) == 52890 and int(ps["uploads"]) == 342113, (first(ps), ps["uploads"])
    wk = eng.run("LAG-WK", 60000, s, lin_obj0, None, True, thrd=1.0 / (s ** 2 * N ** 2) / 10, hsq=hsq, block=256)
    assert first(wk) == 44368 and int(wk["uploads"]) == 58186, (first(wk), wk["uploads"])


def test_first_order_big_stops_on_device():
    """A tolerance stop on the device: the large-d GD stops at the same iteration as the torch loop."""
    from gadmm_amd.algorithms import iag, global_constants
    m = _fo_big_problem()
    c = global_constants(m)
    obj0 = m.optimum()
    ref = iag(m, list(range(4)), 4, 400, obj0, c["stepsize"], "cyclic", None, tol=1e-2 * abs(obj0), backend="torch")
    a = iag(m, list(range(4)), 4, 400, obj0, c["stepsize"], "cyclic", None, tol=1e-2 * abs(obj0))
    assert ref.converged and a.converged and a.iters == ref.iters


@pytest.mark.parametrize("N,m,d", [(2, 5000, 300), (1, 20000, 97), (1, 9000, 1000)])
def test_gram_ozaki_matches_f64(N, m, d):
    """The int8-MFMA Ozaki Gram (gram_ozaki.hip: 7 round-to-nearest digits per value, exact int32 digit-pair
    products, f64 recombination) equals an f64 reference (torch's bmm): every entry within 1e-14 of
    sqrt(A_aa A_bb), b and y'y likewise; chunk boundaries (8192 samples) and padded columns included;
    deterministic; both GEMM variants bit-identical."""
    from gadmm_amd.ops.linalg import gram, gram_ozaki
    g = torch.Generator(device=DEV)
    g.manual_seed(N * 1000 + d)
    X = torch.randn((N, m, d), dtype=torch.float64, device=DEV, generator=g) * 3.0
    X[:, :, 0] *= 1e-3  # columns of different scales: per-column exponents
    y = torch.randn((N, m), dtype=torch.float64, device=DEV, generator=g)
    A, b, yy = gram_ozaki(X, y)
    Ar = torch.bmm(X.transpose(1, 2), X)
    br = torch.bmm(X.transpose(1, 2), y.unsqueeze(-1)).squeeze(-1)
    yr = (y * y).sum(1)
    sc = torch.sqrt(torch.diagonal(Ar, dim1=1, dim2=2))
    assert torch.equal(A, A.transpose(1, 2))
    ea = float(((A - Ar).abs() / (sc.unsqueeze(2) * sc.unsqueeze(1))).max())
    eb = float(((b - br).abs() / (sc * yr.sqrt().unsqueeze(1))).max())
    ey = float(((yy - yr).abs() / yr).max())
    A64, _, _ = gram(X, y)
    e64 = float(((A64 - Ar).abs() / (sc.unsqueeze(2) * sc.unsqueeze(1))).max())
    assert ea < 1e-14 and eb < 1e-14 and ey < 1e-14, (ea, eb, ey, e64)
    A2, _, _ = gram_ozaki(X, y)
    assert torch.equal(A, A2)  # deterministic


def _strict_err(A, Ar, eps=1e-12, rows=None):
    """Entrywise error relative to |A_ab| + eps sqrt(A_aa A_bb): an outlier that
    dominates a diagonal cannot hide the loss on the entries it does not touch. ``rows``: only those rows."""
    sc = torch.sqrt(torch.diagonal(Ar, dim1=1, dim2=2).clamp_min(0))
    den = Ar.abs() + eps * sc.unsqueeze(2) * sc.unsqueeze(1)
    e = (A - Ar).abs() / den.clamp_min(1e-300)
    if rows is not None:
        e = e[:, rows]
    return float(e.max())


def _ref_gram(X, y, chunk: int = 1024):
    """A more accurate f64 reference than one long GEMM (whose own error at m = 70000 is ~3e-14 of
    sqrt(A_aa A_bb)): torch GEMMs over chunks of ``chunk`` rows, summed with Kahan compensation. Returned
    on the CPU."""
    N, m, d = X.shape
    Xa = torch.cat([X, y.unsqueeze(-1)], dim=2)
    S = torch.zeros((N, d + 1, d + 1), dtype=torch.float64, device=X.device)
    c = torch.zeros_like(S)
    for i0 in range(0, m, chunk):
        blk = Xa[:, i0:i0 + chunk]
        t = torch.bmm(blk.transpose(1, 2), blk) - c
        s2 = S + t
        c = (s2 - S) - t
        S = s2
    S = S.cpu()
    return S[:, :d, :d].contiguous(), S[:, :d, d].contiguous()


@pytest.mark.parametrize("scheme", ["crt", "digits"])
@pytest.mark.parametrize("case", ["outlier_row", "lognormal"])
def test_gram_ozaki_range_gate_hard_columns(case, scheme, monkeypatch):
    """Within-column dynamic range: a column whose maximum is one row 1e6 times the
    rest (that row zero elsewhere, so the entries A_0b are NOT dominated by it), or lognormal columns. The
    digits keep 49 bits relative to the column maximum, so the raw Ozaki Gram loses ~20 bits on A_0b; the
    gate (linalg.OZ_MAX_RANGE on max colmax / rms) sends these shards to the f64-MFMA kernel."""
    from gadmm_amd.ops import linalg
    g = torch.Generator(device=DEV)
    g.manual_seed(7)
    N, m, d = 1, 20000, 300
    X = torch.randn((N, m, d), dtype=torch.float64, device=DEV, generator=g)
    if case == "outlier_row":
        X[:, 1234, :] = 0.0
        X[:, 1234, 0] = 1e6
    else:
        X = torch.exp(1.5 * X)  # heavy-tailed positive columns
    y = torch.randn((N, m), dtype=torch.float64, device=DEV, generator=g)
    Ar, br = _ref_gram(X, y)
    raw = linalg.gram_crt if scheme == "crt" else linalg.gram_ozaki
    Araw, _, _, rng = raw(X, y, with_range=True)
    assert float(rng.max()) > linalg.OZ_MAX_RANGE, float(rng.max())
    monkeypatch.setenv("GADMM_GRAM_OZAKI", "1")  # d > 256: the auto rule would not try int8 at m = 20000
    monkeypatch.setenv("GADMM_GRAM_INT8", scheme)
    A, b, yy = linalg.gram(X, y)
    path = linalg.LAST_GRAM["path"]
    assert path.startswith("f64-mfma (%s-int8 range gate" % ("crt" if scheme == "crt" else "ozaki")), path
    A64 = linalg._gram_f64(X, y, None, None)[0]
    assert torch.equal(A, A64)  # the gate's fallback IS the f64 kernel
    rows = [0] if case == "outlier_row" else None
    e_gate, e_raw = _strict_err(A.cpu(), Ar, rows=rows), _strict_err(Araw.cpu(), Ar, rows=rows)
    print("case %s: range %.3g, strict error gated %.3g raw ozaki %.3g" % (case, float(rng.max()), e_gate, e_raw))
    assert e_gate < 1e-10, e_gate
    if case == "outlier_row":
        assert e_raw > 10 * e_gate  # the loss the gate exists for


@pytest.mark.parametrize("scheme", ["crt", "digits"])
def test_gram_ozaki_auto_shape_matches_f64(scheme, monkeypatch):
    """the auto-selected shape (d >= 3072, m >= 65536: several 8192-sample chunks) through
    ``gram`` itself, Gaussian columns plus one Laplace (heavier-tailed) column: the range gate keeps the
    Ozaki path, every entry within 1e-14 of sqrt(A_aa A_bb) of the CPU f64 reference."""
    from gadmm_amd.ops import linalg
    g = torch.Generator(device=DEV)
    g.manual_seed(11)
    N, m, d = 1, 70000, 3072
    X = torch.randn((N, m, d), dtype=torch.float64, device=DEV, generator=g)
    u = torch.rand((N, m), dtype=torch.float64, device=DEV, generator=g) - 0.5
    X[:, :, 5] = -torch.sign(u) * torch.log1p(-2 * u.abs())  # Laplace column
    y = torch.randn((N, m), dtype=torch.float64, device=DEV, generator=g)
    monkeypatch.setenv("GADMM_GRAM_INT8", scheme)
    A, b, yy = linalg.gram(X, y)
    assert linalg.LAST_GRAM["path"] == ("crt-int8" if scheme == "crt" else "ozaki-int8"), linalg.LAST_GRAM
    Ar, br = _ref_gram(X, y)
    sc = torch.sqrt(torch.diagonal(Ar, dim1=1, dim2=2))
    ea = float(((A.cpu() - Ar).abs() / (sc.unsqueeze(2) * sc.unsqueeze(1))).max())
    eb = float(((b.cpu() - br).abs() / (sc * yy.cpu().sqrt().unsqueeze(1))).max())
    A64, b64, _ = linalg._gram_f64(X, y, None, None)
    e64 = float(((A64.cpu() - Ar).abs() / (sc.unsqueeze(2) * sc.unsqueeze(1))).max())
    print("auto shape: %s %.3g, f64-mfma %.3g (of sqrt(A_aa A_bb))" % (scheme, ea, e64))
    assert ea < 1e-14 and eb < 1e-14, (ea, eb, e64)


def test_gram_ozaki_gadmm_iterations_match_f64(monkeypatch):
    """End to end: GADMM on a real-shaped problem (2 workers x 20000 x 300, one Laplace column) to a 1e-8
    relative gap takes the same number of iterations with either int8 Gram (forced) as with the f64 one."""
    from gadmm_amd.models import LinearRegression
    from gadmm_amd.algorithms import chain_admm
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    X = torch.randn((2, 20000, 300), dtype=torch.float64, device=DEV, generator=g)
    u = torch.rand((2, 20000), dtype=torch.float64, device=DEV, generator=g) - 0.5
    X[:, :, 7] = -torch.sign(u) * torch.log1p(-2 * u.abs())
    th = torch.randn((300,), dtype=torch.float64, device=DEV, generator=g)
    y = X @ th + 0.1 * torch.randn((2, 20000), dtype=torch.float64, device=DEV, generator=g)
    its = {}
    for mode, scheme in (("1", "crt"), ("1", "digits"), ("0", "crt")):
        monkeypatch.setenv("GADMM_GRAM_OZAKI", mode)
        monkeypatch.setenv("GADMM_GRAM_INT8", scheme)
        m = LinearRegression(X, y)
        obj0 = m.optimum()
        r = chain_admm(m, [0, 1], 2, 10000.0, obj0, 1e-8 * abs(obj0), 2000, engine_opts={"cache": False})
        assert r.converged
        its[(mode, scheme)] = r.iters
    assert len(set(its.values())) == 1, its


@pytest.mark.parametrize("kind", ["linear", "logistic", "newton"])
def test_persistent_state_at_stop_equals_graph(lin24, lin_obj0, log24, log_obj0, kind):
    """the persistent kernels learn the stop decision `lag` iterations late; the
    state a solve returns (checkpoints, resume) is nevertheless the state after the STOPPING iteration,
    equal to the graph engine's: same next_iter = iters + 1 and the same (theta, mu)."""
    from gadmm_amd.models import LinearRegression, LogisticRegression
    from gadmm_amd.algorithms import chain_admm
    if kind == "linear":
        m = LinearRegression(lin24.X.to(DEV), lin24.y.to(DEV))
        args, kw, expect = (3.0, lin_obj0, 1e-4, 3000), {}, 784
    elif kind == "logistic":
        m = LogisticRegression(log24.X.to(DEV), log24.y.to(DEV), lam=1e-5)
        args, kw, expect = (2e-4, log_obj0, 1e-4, 400), dict(local_solver="gd", step=2.2), 53
    else:
        m = LogisticRegression(log24.X.to(DEV), log24.y.to(DEV), lam=1e-5)
        args, kw, expect = (1e-3, log_obj0, 1e-8, 2000), dict(local_solver="newton"), 424
    a = chain_admm(m, list(range(24)), 24, *args, engine_opts={"cache": False}, **kw)
    b = chain_admm(m, list(range(24)), 24, *args, engine_opts={"cache": False, "persistent": False}, **kw)
    assert a.extra["engine"] == "persistent" and b.extra["engine"] in ("graph", "eager")
    assert a.iters == b.iters == expect
    (ta, ma, na), (tb, mb, nb) = a.extra["state"], b.extra["state"]
    assert na == nb == expect + 1, (na, nb, a.extra.get("state_from"))
    assert torch.equal(ta, tb) and torch.equal(ma, mb)


@pytest.mark.parametrize("kernel", ["logistic", "newton"])
def test_postfence_stress(log24, log_obj0, kernel, monkeypatch):
    """the fence-free LDS ring posts (chain_persistent_logistic.hip zr_post,
    chain_persistent_newton.hip lds_post) rely on a wave's LDS operations being performed in order, which
    gfx950 provides (persist_device.h: GADMM_LDS_IN_ORDER). Stress: many back-to-back solves with the
    fence-free posts and with the fenced ones (GADMM_*_POSTFENCE=1) give ONE bit-identical objective trace
    and primal residual -- a post seen before its ring data would change a margin or a chord step."""
    from gadmm_amd.models import LogisticRegression
    from gadmm_amd.algorithms import chain_admm
    m = LogisticRegression(log24.X.to(DEV), log24.y.to(DEV), lam=1e-5)
    if kernel == "logistic":
        env, reps, expect = "GADMM_LOGISTIC_POSTFENCE", 16, 53
        kw = dict(local_solver="gd", step=2.2)
        rho, tol, it = 2e-4, 1e-4, 400
    else:
        env, reps, expect = "GADMM_NEWTON_POSTFENCE", 8, 424
        kw = dict(local_solver="newton")
        rho, tol, it = 1e-3, 1e-8, 2000
    traces = {}
    for fenced in ("0", "1"):
        monkeypatch.setenv(env, fenced)
        for _ in range(reps):
            r = chain_admm(m, list(range(24)), 24, rho, log_obj0, tol, it,
                           engine_opts={"cache": False, "state": False}, **kw)
            assert r.extra["engine"] == "persistent" and r.iters == expect and r.converged
            key = (r.obj.tobytes(), r.primal_res.tobytes() if r.primal_res is not None else b"")
            traces[key] = traces.get(key, 0) + 1
    assert len(traces) == 1, "%d distinct traces over %d solves" % (len(traces), 2 * reps)


@pytest.mark.parametrize("persistent", [True, False])
def test_newton_chord_safety_net_e4_shape(log24, log_obj0, persistent):
    """Chord-Newton reuses a worker's inverse Hessian across ADMM iterations; on the derm-shaped E4 problem
    (LogisticRegression_Real stand-in: N = 10, d = 34, m = 35, rho = 0.02) a stale inverse sends the first
    chord steps so far off that local solves hit the 50-step cap unconverged. The kernels count such solves
    (ChainCtl::inner_fail) and the solve is re-run with exact Newton: the trace then follows torch's exact
    prox (group_ADMM_logistic.m:26-49) -- and the E3 problem, where chord steps converge, never re-runs."""
    from gadmm_amd.config import get_preset
    from gadmm_amd.entry.common import full_dataset
    from gadmm_amd.models import LogisticRegression
    from gadmm_amd.algorithms import chain_admm
    cfg = get_preset("LogisticRegression_Real")
    ds = full_dataset(cfg)
    m = LogisticRegression(ds.X.to(DEV).contiguous(), ds.y.to(DEV).contiguous(), lam=cfg.lam)
    n = ds.num_workers
    obj0 = m.optimum(None, n_total=n)
    opts = {"cache": False, "persistent": persistent}
    a = chain_admm(m, list(range(n)), n, 0.02, obj0, 1e-8, 60, local_solver="newton", engine_opts=opts)
    t = chain_admm(m, list(range(n)), n, 0.02, obj0, 1e-8, 60, local_solver="newton", backend="torch")
    assert "chord_fallback" in a.extra, a.extra
    np.testing.assert_allclose(a.obj, t.obj, rtol=1e-10, atol=0)
    e3 = LogisticRegression(log24.X.to(DEV), log24.y.to(DEV), lam=1e-5)
    b = chain_admm(e3, list(range(24)), 24, 1e-3, log_obj0, 1e-8, 2000, local_solver="newton", engine_opts=opts)
    assert b.iters == 424 and "chord_fallback" not in b.extra


@pytest.mark.parametrize("N,m,d", [(2, 5000, 300), (1, 20000, 97), (1, 9000, 1000), (1, 70000, 600)])
def test_gram_crt_matches_f64(N, m, d):
    """The CRT int8 Gram (gram_crt.hip: 49-bit integer images, 16 modular int8 GEMMs with exact int32 sums,
    Garner reconstruction): every entry within 1e-14 of sqrt(A_aa A_bb) of the Kahan-chunked f64 reference
    (chunk boundaries at 32768 samples and padded 256-feature tiles included), b and y'y likewise, exactly
    symmetric, deterministic; the range statistic equals the digit kernel's."""
    from gadmm_amd.ops.linalg import gram_crt, gram_ozaki
    g = torch.Generator(device=DEV)
    g.manual_seed(N * 1000 + d)
    X = torch.randn((N, m, d), dtype=torch.float64, device=DEV, generator=g) * 3.0
    X[:, :, 0] *= 1e-3
    y = torch.randn((N, m), dtype=torch.float64, device=DEV, generator=g)
    A, b, yy, rng = gram_crt(X, y, with_range=True)
    Ar, br = _ref_gram(X, y)
    sc = torch.sqrt(torch.diagonal(Ar, dim1=1, dim2=2))
    assert torch.equal(A, A.transpose(1, 2))
    ea = float(((A.cpu() - Ar).abs() / (sc.unsqueeze(2) * sc.unsqueeze(1))).max())
    eb = float(((b.cpu() - br).abs() / (sc * yy.cpu().sqrt().unsqueeze(1))).max())
    yr = (y.cpu() * y.cpu()).sum(1)
    ey = float(((yy.cpu() - yr).abs() / yr).max())
    Ao, _, _, rng_o = gram_ozaki(X, y, with_range=True)
    eo = float(((Ao.cpu() - Ar).abs() / (sc.unsqueeze(2) * sc.unsqueeze(1))).max())
    print("crt %.3g, digits %.3g (of sqrt(A_aa A_bb)); range %.4g / %.4g" % (ea, eo, float(rng.max()), float(rng_o.max())))
    assert ea < 1e-14 and eb < 1e-14 and ey < 1e-14, (ea, eb, ey, eo)
    assert torch.allclose(rng, rng_o, rtol=1e-12)
    A2 = gram_crt(X, y)[0]
    assert torch.equal(A, A2)


def test_readback_kernel_copies_exactly():
    """csrc/kernels/readback.hip: the persistent engines' result block goes to the pinned host buffer by
    a kernel (then a system-scope release) instead of an SDMA copy; the host sees every word right
    after the stream sync, for the full block, the 32-byte control block, and a non-16-byte size (the
    copy-engine fallback)."""
    from gadmm_amd.ops import native
    lib = native.load()
    s = torch.cuda.Stream(DEV)
    # (doubles, doubles copied): kernel path, control block, copy-engine fallback (odd size), a prefix
    for n, k in ((8 + 2 * 3001, 8 + 2 * 3001), (4, 4), (4097, 4097), (64, 32)):
        src = torch.randn((n,), dtype=torch.float64, device=DEV)
        torch.cuda.synchronize()
        host = torch.full((n,), float("nan"), dtype=torch.float64, pin_memory=True)
        nb = k * 8
        native.check(lib.gadmm_readback_d2h(host.data_ptr(), src.data_ptr(), nb, s.cuda_stream), "readback")
        s.synchronize()
        assert torch.equal(host[:k], src[:k].cpu()), n
        if k < n:
            assert torch.isnan(host[k:]).all()
