set -o pipefail
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_lr -o reg -- python $R/tools/logistic_inner.py > $R/gpurun_out/prof_lr_reg.log 2>&1 && \
GADMM_LOGISTIC_LDS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_lr -o lds -- python $R/tools/logistic_inner.py > $R/gpurun_out/prof_lr_lds.log 2>&1
echo rc=$?
