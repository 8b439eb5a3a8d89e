#!/bin/bash
# round 4: multi-rank large-d test, optimum stress with rocSOLVER forced (A/B of the determinism fix),
# real10m / star / dgadmm benches without the profiler
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multirank.py -k "large_d or first_order_big" > $O/t.log 2>&1 || exit $?
GADMM_OPT_SOLVER=rocsolver timeout -k 10 150 python -u tools/ipc_optimum_stress.py 2 3 > $O/s2_rocsolver.log 2>&1 || exit $?
GADMM_OPT_SOLVER=rocsolver timeout -k 10 150 python -u tools/ipc_optimum_stress.py 1 3 > $O/s1_rocsolver.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config real10m --steps 1 --warmup 0 > $O/real10m.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config star --steps 10 --warmup 2 > $O/star.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config dgadmm --steps 10 --warmup 2 > $O/dg.log 2>&1
