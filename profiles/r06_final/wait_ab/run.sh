#!/bin/bash
# host wake-up after the solve: HIP's default wait (active for ROC_ACTIVE_WAIT_TIMEOUT, then the
# interrupt) vs a long active wait, E1 and D-GADMM benches alternating on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-waitab}; mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 python -u bench.py > $O/e1_def_$i.log 2>&1 || exit $?
  ROC_ACTIVE_WAIT_TIMEOUT=100000 timeout -k 10 120 python -u bench.py > $O/e1_spin_$i.log 2>&1 || exit $?
  timeout -k 10 120 python -u bench.py --config dgadmm --steps 20 --warmup 3 > $O/dg_def_$i.log 2>&1 || exit $?
  ROC_ACTIVE_WAIT_TIMEOUT=100000 timeout -k 10 120 python -u bench.py --config dgadmm --steps 20 --warmup 3 > $O/dg_spin_$i.log 2>&1 || exit $?
done
ROC_ACTIVE_WAIT_TIMEOUT=100000 timeout -k 10 200 python -u tools/dgadmm_host_stamps.py 10 60 refresh > $O/stamps_spin.log 2>&1 || exit $?
