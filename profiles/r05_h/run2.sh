#!/bin/bash
# round 5, session h2+ (arg: output name): Ozaki GEMM iterations -- correctness, time, PMC stall split
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5h2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu.py -k "gram_ozaki" \
  > $O/t_oz.log 2>&1 || exit $?
timeout -k 10 400 python tools/gram_ozaki_bench.py 1 312500 10000 2 > $O/bench_10k.log 2>&1 || exit $?
timeout -k 10 200 python tools/gram_ozaki_bench.py 1 100000 4096 2 > $O/bench_4096.log 2>&1 || exit $?
GADMM_OZ_GEMM=2 timeout -k 10 400 python tools/gram_ozaki_bench.py 1 312500 10000 2 > $O/bench2_10k.log 2>&1 || exit $?
GADMM_OZ_GEMM=2 timeout -k 10 200 python tools/gram_ozaki_bench.py 1 100000 4096 2 > $O/bench2_4096.log 2>&1 || exit $?
GADMM_OZ_GEMM=3 timeout -k 10 400 python tools/gram_ozaki_bench.py 1 312500 10000 2 > $O/bench3_10k.log 2>&1 || exit $?
GADMM_OZ_GEMM=3 timeout -k 10 200 python tools/gram_ozaki_bench.py 1 100000 4096 2 > $O/bench3_4096.log 2>&1 || exit $?
GADMM_OZ_GEMM=2 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d $O/pmc -o pmc -- \
  python3 tools/gram_ozaki_bench.py 1 100000 4096 1 > $O/pmc.log 2>&1 || exit $?
