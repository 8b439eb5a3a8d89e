#!/bin/bash
# round 5, session i (A/B): D-GADMM with / without the early asynchronous chain draw, one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5iab}; mkdir -p $O
timeout -k 10 300 python tools/dgadmm_host_stamps.py 10 40 refresh > $O/dg_stamps.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python bench.py --config dgadmm --steps 20 --warmup 3 > $O/dg_early_$i.log 2>&1 || exit $?
  GADMM_DGADMM_EARLY=0 timeout -k 10 200 python bench.py --config dgadmm --steps 20 --warmup 3 > $O/dg_sync_$i.log 2>&1 || exit $?
done
