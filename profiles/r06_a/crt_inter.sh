#!/bin/bash
# CRT GEMM with DMA pieces and fragment reads interleaved between the MFMAs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/crt11; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "gram_crt or gram_ozaki" > $O/test.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gram_crt_bench.py 2x625000x10000 1x131072x4096 > $O/bench.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/pa -o pa -- python3 tools/gram_crt_once.py 1x131072x10000 crt > $O/pa.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pb -o pb -- python3 tools/gram_crt_once.py 1x131072x10000 crt > $O/pb.log 2>&1 || exit $?
