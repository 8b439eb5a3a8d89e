#!/bin/bash
# headline (E1) bench under a kernel + copy trace: the GPU timeline of each step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-e1trace}; mkdir -p $O
timeout -k 10 200 python -u tools/e1_host_stamps.py > $O/e1_stamps.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/$O/bench.log 2>&1
