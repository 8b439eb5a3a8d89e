#!/bin/bash
# CRT GEMM job order A/B: per-XCD contiguous runs (xcd) vs node-wide super-blocks (node, default)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/crt10; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "gram_crt_matches" > $O/test.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gram_crt_bench.py 2x625000x10000 1x131072x4096 > $O/bench_node.log 2>&1 || exit $?
GADMM_CRT_ORDER=xcd timeout -k 10 300 python -u tools/gram_crt_bench.py 2x625000x10000 1x131072x4096 > $O/bench_xcd.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gram_crt_bench.py 2x625000x10000 > $O/bench_node2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pb -o pb -- python3 tools/gram_crt_once.py 1x131072x10000 crt > $O/pb.log 2>&1 || exit $?
