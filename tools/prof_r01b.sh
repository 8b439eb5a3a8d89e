# rocprofv3 kernel summaries of the round-1 (second session) kernels: E1 headline (blocked, quad
# GEMV), E3 logistic (register inner GD), D-GADMM one launch; plus a PMC pass on the E1 kernel.
set -o pipefail
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_e1q -o e1 -- python $R/bench.py --steps 5 --warmup 1 > $R/gpurun_out/prof_e1q.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_logq -o lg -- python $R/bench.py --config logistic --steps 3 --warmup 1 > $R/gpurun_out/prof_logq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_dgq -o dg -- python $R/bench.py --config dgadmm --steps 3 --warmup 1 > $R/gpurun_out/prof_dgq.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc_e1q -o pmc -- python $R/bench.py --steps 2 --warmup 0 > $R/gpurun_out/pmc_e1q.log 2>&1
echo rc=$?
