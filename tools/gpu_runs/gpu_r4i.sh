#!/bin/bash
# round 4: fused symmetric-GEMV reduce (large-d chain / star / first-order), pipelined boundary Gram
# tiles (A/B against the build without), the optimum stress at 1 and 2 ranks, real10m under rocprofv3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu.py -k "gram or large_d or sym_pack or star_big or first_order_big or primal_residual_large" > $O/t.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/gram_bench.py 2 312500 10000 > $O/gram_new.log 2>&1 || exit $?
GADMM_NATIVE_LIB=$PWD/gadmm_amd/_native/ab/lib_noclamp.so timeout -k 10 120 python -u tools/gram_bench.py 2 312500 10000 > $O/gram_old.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/symv_lab.py 10000 20 > $O/lab.log 2>&1 || exit $?
timeout -k 10 150 python -u tools/ipc_optimum_stress.py 1 3 > $O/s1.log 2>&1 || exit $?
timeout -k 10 150 python -u tools/ipc_optimum_stress.py 2 3 > $O/s2.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/real -o real -- python3 bench.py --config real10m --steps 1 --warmup 0 > $O/real.log 2>&1
