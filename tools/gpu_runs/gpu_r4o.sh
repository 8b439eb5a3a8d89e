#!/bin/bash
# round 4: Gram A/B -- MFMA section at wave priority 1 (GADMM_GRAM_PRIO=1) vs default, same box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 120 python -u tools/gram_bench.py 2 312500 10000 > $O/warm.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/gram_bench.py 2 312500 10000 > $O/g0.log 2>&1 || exit $?
GADMM_GRAM_PRIO=1 timeout -k 10 120 python -u tools/gram_bench.py 2 312500 10000 > $O/gp.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/gram_bench.py 2 312500 10000 > $O/g0b.log 2>&1 || exit $?
GADMM_GRAM_PRIO=1 timeout -k 10 120 python -u tools/gram_bench.py 2 312500 10000 > $O/gpb.log 2>&1
