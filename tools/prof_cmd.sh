# rocprofv3 summaries of the headline bench (blocked persistent kernel) and the large-d engine path.
set -o pipefail
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_e1b -o e1 -- python $R/bench.py --steps 5 --warmup 1 > $R/gpurun_out/prof_e1b.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fo -o fo -- python $R/tools/fo_bench.py > $R/gpurun_out/prof_fo.log 2>&1
echo rc=$?
