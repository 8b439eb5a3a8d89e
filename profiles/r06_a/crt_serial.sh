#!/bin/bash
# CRT Gram: slicing overlapped on a side stream vs serialized on the GEMM stream (kernel durations)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/crt8; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ov -o ov -- python3 tools/gram_crt_once.py 1x262144x10000 crt > $O/ov.log 2>&1 || exit $?
GADMM_CRT_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/se -o se -- python3 tools/gram_crt_once.py 1x262144x10000 crt > $O/se.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/gram_crt_bench.py 1x625000x10000 > $O/bench_ov.log 2>&1 || exit $?
GADMM_CRT_SERIAL=1 timeout -k 10 200 python -u tools/gram_crt_bench.py 1x625000x10000 > $O/bench_se.log 2>&1 || exit $?
