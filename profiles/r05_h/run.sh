#!/bin/bash
# round 5, session h: Ozaki Gram with the 64-tile / 2-waves-per-SIMD GEMM (no spills) -- correctness, time, kernel split
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5h; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu.py -k "gram_ozaki" \
  > $O/t_oz.log 2>&1 || exit $?
timeout -k 10 200 python tools/gram_ozaki_bench.py 2 20000 2048 3 > $O/bench_2048.log 2>&1 || exit $?
timeout -k 10 400 python tools/gram_ozaki_bench.py 1 312500 10000 2 > $O/bench_10k.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o oz -- python3 tools/gram_ozaki_bench.py 1 100000 4096 2 \
  > $O/prof.log 2>&1 || exit $?
