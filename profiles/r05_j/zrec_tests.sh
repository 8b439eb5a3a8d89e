#!/bin/bash
# round 5, session j3: the margins-recursion logistic kernel as the default -- logistic GPU tests, the
# multi-rank logistic tests, benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5jt}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu.py \
  -k "logistic or resume or entry" > $O/t_gpu.log 2>&1
r1=$?
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_multirank.py \
  -k "logistic" > $O/t_mr.log 2>&1
r2=$?
for i in 1 2; do
  timeout -k 10 200 python bench.py --config logistic --steps 20 --warmup 3 > $O/lg_$i.log 2>&1 || exit $?
  GADMM_LOGISTIC_ZREC=0 timeout -k 10 200 python bench.py --config logistic --steps 20 --warmup 3 > $O/lg_onewave_$i.log 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --config logistic --workers 8 --steps 20 --warmup 3 > $O/lg_w8.log 2>&1 || exit $?
exit $((r1 + r2))
