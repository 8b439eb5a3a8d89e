set -o pipefail
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_e1 -o e1 -- python $R/bench.py --steps 5 --warmup 1 > $R/gpurun_out/prof_e1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bigd -o bigd -- python $R/tools/prof_bigd.py > $R/gpurun_out/prof_bigd.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES -d $R/gpurun_out/prof_bigd_pmc -o pmc -- python $R/tools/prof_bigd.py > $R/gpurun_out/prof_bigd_pmc.log 2>&1
echo rc=$?
