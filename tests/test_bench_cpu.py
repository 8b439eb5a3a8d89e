"""bench.py's CPU plumbing config (BASELINE.json configs[0]): GADMM over 2 gloo ranks, launched the
way the driver launches bench.py (torch.distributed.run, 127.0.0.1), one JSON line from rank 0."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_cpu_gloo_two_ranks():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29577", os.path.join(ROOT, "bench.py"),
           "--config", "cpu_gloo", "--steps", "1", "--warmup", "0", "--tol", "1e-4"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["iterations_to_tol"] == 784 and r["cpu_ranks"] == 2 and r["n_gpus"] == 0
    assert r["theta_payload_bytes_per_solve"] == 2 * 50 * 8 * 784  # one rank boundary, both directions
    assert r["value"] > 0 and r["unit"] == "s"


def test_expected_iteration_table_matches_reference_semantics():
    """Every bench config's correctness gate (benchmarks.EXPECTED_OTHER / EXPECTED_ITERS_1E8) equals the
    reference-semantics count for the bench's exact problem and seeds."""
    from gadmm_amd import benchmarks as B
    from gadmm_amd.data import linear_synthetic
    from gadmm_amd.oracle import reference as R

    for key, want in B.EXPECTED_OTHER.items():
        cfg, n = key[0], key[1]
        coh = key[2] if len(key) > 2 else 10
        assert B.reference_expected(cfg, n, coh) == want, key
        assert B.expected_for(cfg, n, coh) == want
    for (n, rho), want in B.EXPECTED_ITERS_1E8.items():
        ds = linear_synthetic(n)
        X, y = ds.X.numpy(), ds.y.numpy()
        obj0 = R.opt_linear(X.reshape(-1, X.shape[2]), y.reshape(-1))
        assert R.gadmm_linear(X, y, rho, 3000, obj0, 1e-8).iters == want, (n, rho)
