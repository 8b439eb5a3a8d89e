#!/bin/bash
# CRT Gram with the integer slicer: GPU tests, A/B bench, slice/GEMM kernel durations (slicing serialized)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/crt9; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "gram_crt or gram_ozaki" > $O/test.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gram_crt_bench.py 1x625000x10000 2x625000x10000 1x131072x4096 1x65536x3072 > $O/bench.log 2>&1 || exit $?
GADMM_CRT_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/se -o se -- python3 tools/gram_crt_once.py 1x262144x10000 crt > $O/se.log 2>&1 || exit $?
