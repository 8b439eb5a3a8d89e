#!/bin/bash
# rocprofv3 evidence for the exact-logistic pipeline kernel: kernel statistics of the logistic_exact
# bench (pipeline and one-wave kernels), then one PMC pass per kernel (SQ counters only). CSV output;
# only the statistics / counter files are kept (the merge-back limit is 64 MiB)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5lprof}; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rec -o rec -- python3 bench.py --config logistic_exact --steps 10 --warmup 2 > $O/rec.log 2>&1 || exit $?
GADMM_NEWTON_REC=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/one -o one -- python3 bench.py --config logistic_exact --steps 10 --warmup 2 > $O/one.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_VMEM -d $O/pmc_rec -o pmc -- python3 bench.py --config logistic_exact --steps 3 --warmup 1 > $O/pmc_rec.log 2>&1 || exit $?
GADMM_NEWTON_REC=0 timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_VMEM -d $O/pmc_one -o pmc -- python3 bench.py --config logistic_exact --steps 3 --warmup 1 > $O/pmc_one.log 2>&1
find $O -name "*.db" -delete
find $O -name "*kernel_trace.csv" -size +2M -delete
du -sh $O
exit 0
