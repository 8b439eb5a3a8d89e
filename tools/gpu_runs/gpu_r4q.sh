#!/bin/bash
# round 4: GEMV broadcast / accumulator probe; CG large-d optimum (test, multi-rank determinism, real10m)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4q; mkdir -p $O /tmp/p
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -I csrc/include -o /tmp/p/probe tools/gemv_bcast_probe.hip 2>/dev/null || exit 1
timeout -k 10 60 /tmp/p/probe 100000 > $O/probe.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu.py -k "optimum_solve or large_d_engine" > $O/t.log 2>&1 || exit $?
timeout -k 10 150 python -u tools/ipc_optimum_stress.py 2 3 > $O/s2.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_multirank.py -k "large_d" > $O/tm.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config real10m --steps 1 --warmup 0 > $O/real10m.log 2>&1
