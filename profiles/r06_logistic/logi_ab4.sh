#!/bin/bash
# logistic inner GD ring depth: G 64/8 vs H 128/8 + an early-end check every 8 steps (ab_libs/lib{G,H}.so), interleaved, 24 and 8 workers
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-logiab4}; mkdir -p $O
for i in 1 2; do
  for v in G H; do
    GADMM_NATIVE_LIB=$PWD/ab_libs/lib$v.so timeout -k 10 200 python -u bench.py --config logistic --steps 20 --warmup 3 > $O/${v}_$i.log 2>&1 || exit $?
    GADMM_NATIVE_LIB=$PWD/ab_libs/lib$v.so timeout -k 10 200 python -u bench.py --config logistic --workers 8 --steps 10 --warmup 2 > $O/${v}8_$i.log 2>&1 || exit $?
  done
done
