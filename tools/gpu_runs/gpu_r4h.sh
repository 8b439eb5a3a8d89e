#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4h
timeout -k 10 120 python -u tools/symv_lab.py 10000 20 > gpurun_out/r4h/lab.log 2>&1 || exit $?
bash tools/gpu_runs/gpu_r4g.sh || exit $?
bash tools/gpu_runs/gpu_r4d.sh
