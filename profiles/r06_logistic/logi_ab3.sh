#!/bin/bash
# logistic inner GD ring depth / check interval: B 16/8, E 16/4, F 32/8 (ab_libs/lib{B,E,F}.so), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-logiab3}; mkdir -p $O
for i in 1 2; do
  for v in B E F; do
    GADMM_NATIVE_LIB=$PWD/ab_libs/lib$v.so timeout -k 10 200 python -u bench.py --config logistic --steps 20 --warmup 3 > $O/${v}_$i.log 2>&1 || exit $?
  done
done
