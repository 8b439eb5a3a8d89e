#!/bin/bash
# round 4: the reference experiments end to end on one GPU (entry points), after this round's changes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4v; mkdir -p $O
export MPLBACKEND=Agg
timeout -k 10 200 python -u -m gadmm_amd LinearRegression_Synthetic --out /tmp/r4v/e1 --no-plot > $O/e1.log 2>&1 || exit $?
timeout -k 10 200 python -u -m gadmm_amd LogisticRegression_Synthetic --out /tmp/r4v/e3 --no-plot > $O/e3.log 2>&1 || exit $?
timeout -k 10 200 python -u -m gadmm_amd Dynamic_LinearRegression_Synthetic --out /tmp/r4v/e5 --no-plot > $O/e5.log 2>&1 || exit $?
timeout -k 10 200 python -u -m gadmm_amd LinearRegression_gadmm_vs_admm --out /tmp/r4v/e7 --no-plot > $O/e7.log 2>&1 || exit $?
timeout -k 10 300 python -u -m gadmm_amd LinearRegression_RealShaped --out /tmp/r4v/real --no-plot --set dim=2048 rows_per_worker=200000 > $O/real.log 2>&1
