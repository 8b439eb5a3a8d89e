#!/bin/bash
# D-GADMM bench under a kernel + copy trace: the GPU timeline of each solve (refresh, pad image,
# epoch-table copy, blocked kernel, read-back) and the gaps between them
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-dgtrace}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config dgadmm --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/$O/bench.log 2>&1
