#!/bin/bash
# round 4: the rest of the GPU suite (from the stalled-peer test on) + smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py tests/test_native_selftest.py -m gpu -v --timeout 300 --timeout-method thread > $O/t2.log 2>&1
rc=$?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
exit $rc
