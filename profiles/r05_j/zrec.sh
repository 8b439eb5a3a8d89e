#!/bin/bash
# round 5, session j2: logistic inner GD with the margins recursion on a second wave (GADMM_LOGISTIC_ZREC=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5jz}; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python bench.py --config logistic --steps 10 --warmup 2 > $O/lg_base_$i.log 2>&1 || exit $?
  GADMM_LOGISTIC_ZREC=1 timeout -k 10 200 python bench.py --config logistic --steps 10 --warmup 2 > $O/lg_zrec_$i.log 2>&1 || exit $?
done
GADMM_LOGISTIC_ZREC=1 timeout -k 10 200 python bench.py --config logistic --workers 8 --steps 10 --warmup 2 > $O/lg_zrec_w8.log 2>&1 || exit $?
GADMM_LOGISTIC_ZREC=1 timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu.py \
  -k "logistic and not newton" > $O/t_logistic.log 2>&1
exit 0
