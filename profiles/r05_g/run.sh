#!/bin/bash
# round 5, session g: the int8 Ozaki Gram -- correctness, then time vs the f64-MFMA Gram
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5g; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu.py -k "gram_ozaki" \
  > $O/t_oz.log 2>&1 || exit $?
timeout -k 10 200 python tools/gram_ozaki_bench.py 2 20000 2048 3 > $O/bench_2048.log 2>&1 || exit $?
timeout -k 10 400 python tools/gram_ozaki_bench.py 1 312500 10000 2 > $O/bench_10k.log 2>&1 || exit $?
