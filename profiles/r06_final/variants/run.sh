#!/bin/bash
# the bench's other shapes on the final tree: D-GADMM re-chaining every iteration (configs[3] literally),
# and the 8-worker variants of each config (BASELINE configs[1] / [2])
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6var}; mkdir -p $O
for i in 1 2; do timeout -k 10 200 python -u bench.py --config dgadmm --coherence 1 --steps 20 --warmup 3 > $O/dg_coh1_$i.log 2>&1 || exit $?; done
timeout -k 10 200 python -u bench.py --workers 8 --steps 50 --warmup 5 > $O/e1_w8.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --config dgadmm --workers 8 --steps 20 --warmup 3 > $O/dg_w8.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --config logistic --workers 8 --steps 10 --warmup 2 > $O/lg_w8.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --config logistic_exact --workers 8 --steps 10 --warmup 2 > $O/lx_w8.log 2>&1 || exit $?
