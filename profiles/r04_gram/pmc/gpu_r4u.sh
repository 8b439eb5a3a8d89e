#!/bin/bash
# round 4: PMC pass of the Gram (same counters and shape as round 3's gpu_r3_gram_pmc.sh)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r4u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d $O/p1 -o g -- python3 $GRAFT_REPO_ROOT/tools/gram_once.py 262144 8192 > $O/p1.log 2>&1
