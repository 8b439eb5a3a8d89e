#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 200 python -u tools/ipc_optimum_stress.py 2 3 > $O/s2.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/ipc_optimum_stress.py 4 3 > $O/s4.log 2>&1 || exit $?
