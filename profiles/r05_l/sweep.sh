#!/bin/bash
# refresh lag x background-refresh threshold of the Newton pipeline kernel (logistic_exact bench)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5ls}; mkdir -p $O
for cfg in ${CFGS:-2,1 3,1 2,2 3,2 2,3 3,3 4,2 4,3}; do
  rl=${cfg%,*}; bg=${cfg#*,}
  GADMM_NEWTON_RLAG=$rl GADMM_NEWTON_BG=$bg timeout -k 10 120 python bench.py --config logistic_exact --steps 20 --warmup 3 > $O/rl${rl}_bg${bg}.log 2>&1 || exit $?
done
GADMM_NEWTON_REC=0 timeout -k 10 120 python bench.py --config logistic_exact --steps 20 --warmup 3 > $O/one.log 2>&1 || exit $?
for cfg in ${UCFGS:-}; do
  rl=${cfg%,*}; bg=${cfg#*,}
  GADMM_NEWTON_URGENT_NS=1 GADMM_NEWTON_RLAG=$rl GADMM_NEWTON_BG=$bg timeout -k 10 120 python bench.py --config logistic_exact --steps 20 --warmup 3 > $O/u_rl${rl}_bg${bg}.log 2>&1 || exit $?
done
