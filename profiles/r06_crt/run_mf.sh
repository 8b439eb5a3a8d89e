#!/bin/bash
# CRT GEMM MFMA shape A/B: v_mfma_i32_32x32x32_i8 (default) vs v_mfma_i32_16x16x64_i8
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6mf; mkdir -p $O
GADMM_CRT_MFMA=16 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "gram_crt or gram_ozaki" > $O/test16.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "gram_crt_matches" > $O/test32.log 2>&1 || exit $?
for mf in 32 16 32 16; do
  GADMM_CRT_MFMA=$mf timeout -k 10 300 python -u tools/gram_crt_bench.py 2x625000x10000 1x131072x4096 > $O/bench_$mf.log 2>&1 || exit $?
  cat $O/bench_$mf.log >> $O/bench_all_$mf.log
done
GADMM_CRT_MFMA=16 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/pa -o pa -- python3 tools/gram_crt_once.py 1x131072x10000 crt > $O/pa.log 2>&1 || exit $?
GADMM_CRT_MFMA=16 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pb -o pb -- python3 tools/gram_crt_once.py 1x131072x10000 crt > $O/pb.log 2>&1 || exit $?
