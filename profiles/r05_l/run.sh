#!/bin/bash
# round 5, session l: the four-wave Newton pipeline (chain_persistent_newton_rec_kernel) vs the one-wave
# kernel: logistic_exact bench alternating, then the in-kernel timelines of both
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5l}; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python bench.py --config logistic_exact --steps 20 --warmup 3 > $O/rec_$rep.log 2>&1 || exit $?
  GADMM_NEWTON_REC=0 timeout -k 10 120 python bench.py --config logistic_exact --steps 20 --warmup 3 > $O/one_$rep.log 2>&1 || exit $?
done
timeout -k 10 120 python tools/newton_persist_tl.py --chord 0.3 > $O/tl_rec.log 2>&1 || exit $?
GADMM_NEWTON_REC=0 timeout -k 10 120 python tools/newton_persist_tl.py --chord 0.3 > $O/tl_one.log 2>&1 || exit $?
