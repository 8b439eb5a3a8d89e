#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-probe}; mkdir -p $O
timeout -k 10 200 python -u tools/readback_probe.py 24 > $O/gd.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/readback_probe.py 12 newton > $O/newton.log 2>&1 || exit $?
