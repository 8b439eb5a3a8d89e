# PMC pass over the headline solve (blocked persistent kernel): instruction mix and LDS conflicts
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/e1pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o e1 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $O/p1.log 2>&1
