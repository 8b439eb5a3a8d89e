set -o pipefail
R=$PWD
mkdir -p gpurun_out/prof_gram
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc MfmaUtil FETCH_SIZE TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/prof_gram -o p1 -- python $R/tools/gram_once.py 131072 8192 > $R/gpurun_out/prof_gram/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc LdsBankConflict VmemLatency MemUnitStalled OccupancyPercent -d $R/gpurun_out/prof_gram -o p2 -- python $R/tools/gram_once.py 131072 8192 > $R/gpurun_out/prof_gram/p2.log 2>&1
echo rc=$?
