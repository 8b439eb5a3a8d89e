#!/bin/bash
# round 4: two large-d inverses in flight on two streams -- tests, real10m benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4aa; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu.py -k "inverse or large_d or sym_pack or star_big or optimum_solve or first_order_big" > $O/t.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_multirank.py -k "large_d" > $O/tm.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config real10m --steps 1 --warmup 0 > $O/real10m.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config real10m --steps 1 --warmup 0 > $O/real10m_b.log 2>&1
