#!/bin/bash
# round 5, session j: exact-logistic Newton warm start extrapolated from the last two own iterates
# (GADMM_NEWTON_EXTRAP=1) -- A/B on one box, then the Newton tests with it on
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5j}; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python bench.py --config logistic_exact --steps 10 --warmup 2 > $O/lx_base_$i.log 2>&1 || exit $?
  GADMM_NEWTON_EXTRAP=1 timeout -k 10 200 python bench.py --config logistic_exact --steps 10 --warmup 2 > $O/lx_extrap_$i.log 2>&1 || exit $?
done
GADMM_NEWTON_EXTRAP=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py \
  -k "newton" > $O/t_newton.log 2>&1 || exit $?
