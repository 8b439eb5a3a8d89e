# Round 3: where the f64 Gram (gram_aug_kernel<128,512>) loses its MFMA cycles: one stall-breakdown
# PMC pass (--kernel-trace only, 8 SQ counters) on a 262144 x 8192 shard.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_gpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d $O/p1 -o g -- python3 $GRAFT_REPO_ROOT/tools/gram_once.py 262144 8192 > $O/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_MFMA_MOPS_F64 --output-format csv -d $O/p2 -o g -- python3 $GRAFT_REPO_ROOT/tools/gram_once.py 262144 8192 > $O/p2.log 2>&1
