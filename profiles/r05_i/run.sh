#!/bin/bash
# round 5, session i: D-GADMM host path -- first launch's greedy chains on the native host worker
# (overlapping refresh / reset), fused epoch-table staging -- tests, host stamps, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5i}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py \
  -k "dgadmm or dynamic or blocked or refresh or quad_pad or elastic or resume" > $O/t_gpu.log 2>&1 || exit $?
timeout -k 10 300 python tools/dgadmm_host_stamps.py 10 40 refresh > $O/dg_stamps.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --config dgadmm --steps 20 --warmup 3 > $O/dg_$i.log 2>&1 || exit $?
done
