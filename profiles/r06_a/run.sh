#!/bin/bash
# round 6: the new GPU tests (post-fence stress, state at the stop, Ozaki range gate) and the entry points
# across ranks sharing the GPU (profiles/r06_entries/run.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6a}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "postfence or persistent_state or gram_ozaki or register_kernel" > $O/tests.log 2>&1 || exit $?
bash profiles/r06_entries/run.sh ${1:-r6a}/entries
