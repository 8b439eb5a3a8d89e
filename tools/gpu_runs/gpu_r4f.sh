#!/bin/bash
# round 4: the 4-rank large-d test on the current library, then the rocprofv3 statistics (gpu_r4d.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_multirank.py -k "large_d" > $O/large_d.log 2>&1 || exit $?
bash tools/gpu_runs/gpu_r4d.sh
