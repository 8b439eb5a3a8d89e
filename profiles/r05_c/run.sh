#!/bin/bash
# round 5, session c: the four-wave (sample-class split) logistic persistent kernel -- correctness
# (bit-identical to the graph engine / one-wave kernel, multi-rank fabric) and A/B timing; D-GADMM host stamps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py -k "logistic" \
  > $O/t_gpu.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multirank.py \
  -k "logistic" > $O/t_mr.log 2>&1 || exit $?
for i in 1 2; do
  GADMM_LOGISTIC_SPLIT=0 timeout -k 10 200 python bench.py --config logistic --steps 10 --warmup 2 > $O/logistic_one_$i.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --config logistic --steps 10 --warmup 2 > $O/logistic_split_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python tools/dgadmm_host_stamps.py 10 40 refresh > $O/dg_stamps.log 2>&1 || exit $?
