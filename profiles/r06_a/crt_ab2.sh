#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/crt7; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "gram_crt" > $O/test.log 2>&1 || exit $?
for cfg in 2x4 2x3 4x2; do
  GADMM_CRT_STAGES=$cfg timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "gram_crt_matches and 70000" > $O/test_$cfg.log 2>&1 || exit $?
  GADMM_CRT_STAGES=$cfg timeout -k 10 200 python -u tools/gram_crt_bench.py 1x625000x10000 > $O/bench_$cfg.log 2>&1 || exit $?
done
