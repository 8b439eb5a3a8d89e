#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5pm; mkdir -p $O
GADMM_OZ_GEMM=2 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM -d $O/a -o a -- python3 tools/gram_ozaki_bench.py 1 100000 4096 1 > $O/a.log 2>&1 || exit $?
GADMM_OZ_GEMM=2 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TA_BUSY_avr TA_TA_BUSY_sum -d $O/b -o b -- python3 tools/gram_ozaki_bench.py 1 100000 4096 1 > $O/b.log 2>&1
exit 0
