#!/bin/bash
# round 5, session j4: the margins wave's sigmoid by an Estrin-form exp and rcp + Newton (GADMM_LOGISTIC_FASTSIGM=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5jf}; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python bench.py --config logistic --steps 20 --warmup 3 > $O/lg_$i.log 2>&1 || exit $?
  GADMM_LOGISTIC_FASTSIGM=1 timeout -k 10 200 python bench.py --config logistic --steps 20 --warmup 3 > $O/lg_fast_$i.log 2>&1 || exit $?
done
GADMM_LOGISTIC_FASTSIGM=1 timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu.py \
  -k "logistic_persistent_kernel" > $O/t.log 2>&1
exit 0
