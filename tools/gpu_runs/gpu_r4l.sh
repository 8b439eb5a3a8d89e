#!/bin/bash
# round 4: Gram A/B on one box, real10m shape -- register-staged with the clamped boundary tiles
# pipelined (default), the build before that (ab/lib_noclamp.so), LDS-DMA 2-stage (GADMM_GRAM_GLDS=2) and
# 3-stage (=1) rings; then the Gram tests on the default and the 2-stage kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 120 python -u tools/gram_bench.py 2 312500 10000 > $O/g0.log 2>&1 || exit $?
GADMM_NATIVE_LIB=$PWD/gadmm_amd/_native/ab/lib_noclamp.so timeout -k 10 120 python -u tools/gram_bench.py 2 312500 10000 > $O/gprev.log 2>&1 || exit $?
GADMM_GRAM_GLDS=2 timeout -k 10 120 python -u tools/gram_bench.py 2 312500 10000 > $O/g2.log 2>&1 || exit $?
GADMM_GRAM_GLDS=1 timeout -k 10 120 python -u tools/gram_bench.py 2 312500 10000 > $O/g1.log 2>&1 || exit $?
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py -k gram > $O/t0.log 2>&1 || exit $?
GADMM_GRAM_GLDS=2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py -k gram > $O/t2.log 2>&1
