"""A/B of Gram kernel variants (env-selected) in interleaved child processes on one GPU.

    python tools/gram_ab.py [M D]"""
import os, sys, time, subprocess, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    import torch
    from gadmm_amd.ops import linalg
    M, D = int(sys.argv[2]), int(sys.argv[3])
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(1, M, D, dtype=torch.float64, device=dev, generator=g)
    y = torch.randn(1, M, dtype=torch.float64, device=dev, generator=g)
    ts = []
    for rep in range(5):
        torch.cuda.synchronize(); t0 = time.perf_counter(); linalg.gram(X, y); torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    fl = M * (D + 1) * (D + 2)
    out = {"tflops": fl / min(ts) / 1e12}
    if os.environ.get("GRAM_AB_LIB"):
        Xa = torch.cat([X[0], y[0, :, None]], 1)
        tl = []
        for rep in range(3):
            torch.cuda.synchronize(); t0 = time.perf_counter(); Xa.T @ Xa; torch.cuda.synchronize()
            tl.append(time.perf_counter() - t0)
        out["rocblas_dgemm_syrk_equiv_tflops"] = fl / min(tl) / 1e12
    print(json.dumps(out))
    sys.exit(0)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
D = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
for rnd in range(2):
    for name, env in (("nt256", {"GADMM_GRAM_NT": "256"}), ("nt512", {"GADMM_GRAM_NT": "512"})):
        out = subprocess.run([sys.executable, __file__, "child", str(M), str(D)], capture_output=True, text=True,
                             env=dict(os.environ, **env))
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(rnd, name, line[-1] if line else out.stderr[-500:], flush=True)
