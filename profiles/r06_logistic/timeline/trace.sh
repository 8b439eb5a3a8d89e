#!/bin/bash
# logistic bench (E3) under a kernel + copy trace: the GPU timeline of one solve
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-logtrace}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config logistic --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/$O/bench.log 2>&1
