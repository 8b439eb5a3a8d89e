#!/bin/bash
# round 4: native residual pass of the large-d optimum -- tests, timing, determinism, real10m
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu.py -k "resid_sq or optimum_solve or large_d_engine" > $O/t.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/optimum_timing.py 2 625000 10000 > $O/opt.log 2>&1 || exit $?
timeout -k 10 150 python -u tools/ipc_optimum_stress.py 2 3 > $O/s2.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_multirank.py -k "large_d" > $O/tm.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config real10m --steps 1 --warmup 0 > $O/real10m.log 2>&1
