set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/gpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 -u $GRAFT_REPO_ROOT/tools/gram_bench.py 1 262144 8192 > $O/plain.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o g -- python3 $GRAFT_REPO_ROOT/tools/gram_bench.py 1 262144 8192 > $O/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/p2 -o g -- python3 $GRAFT_REPO_ROOT/tools/gram_bench.py 1 262144 8192 > $O/p2.log 2>&1
