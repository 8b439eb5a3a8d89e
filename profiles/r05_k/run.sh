#!/bin/bash
# round 5, session k: host stamps of the headline (E1) solve on one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5k}; mkdir -p $O
timeout -k 10 300 python tools/e1_host_stamps.py 60 > $O/e1_stamps.log 2>&1 || exit $?
