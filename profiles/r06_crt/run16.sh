#!/bin/bash
# CRT on 16 moduli <= 234: GPU tests of both int8 schemes, A/B bench, real10m
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6crt16}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "gram" > $O/test.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gram_crt_bench.py 2x625000x10000 1x131072x4096 1x65536x1024 > $O/bench.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config real10m --steps 3 --warmup 1 > $O/real10m.log 2>&1 || exit $?
