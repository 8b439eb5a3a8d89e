#!/bin/bash
# logistic inner GD: A (in ab_libs/libA.so) vs B (in-tree build), alternating, same box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-logiab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "logistic" > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
  GADMM_NATIVE_LIB=$PWD/ab_libs/libA.so timeout -k 10 200 python -u bench.py --config logistic --steps 20 --warmup 3 > $O/A_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --config logistic --steps 20 --warmup 3 > $O/B_$i.log 2>&1 || exit $?
  GADMM_NATIVE_LIB=$PWD/ab_libs/libA.so timeout -k 10 200 python -u bench.py --config logistic --workers 8 --steps 10 --warmup 2 > $O/A8_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --config logistic --workers 8 --steps 10 --warmup 2 > $O/B8_$i.log 2>&1 || exit $?
done
