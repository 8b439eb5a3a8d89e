#!/bin/bash
# round 5, session j7: the exact-logistic chord steps' sigmoid by inv1pexp_fast (GADMM_NEWTON_FASTSIGM) -- A/B, tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5j7}; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python bench.py --config logistic_exact --steps 10 --warmup 2 > $O/lx_fast_$i.log 2>&1 || exit $?
  GADMM_NEWTON_FASTSIGM=0 timeout -k 10 200 python bench.py --config logistic_exact --steps 10 --warmup 2 > $O/lx_libm_$i.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu.py -k "newton" > $O/t.log 2>&1
exit 0
