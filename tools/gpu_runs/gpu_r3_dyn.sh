# Round 3: D-GADMM kernel cost per re-chain -- blocked dynamic mode (GADMM_BLOCKED_DYN=1) vs the
# per-worker kernel at coherence 10 / 30 / 100, kernel durations from rocprofv3.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_dyn
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in 10 30 100; do
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pw$c -o k -- python3 $GRAFT_REPO_ROOT/bench.py --config dgadmm --coherence $c --steps 10 --warmup 2 > $O/pw$c.log 2>&1 || exit $?
  GADMM_BLOCKED_DYN=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/blk$c -o k -- python3 $GRAFT_REPO_ROOT/bench.py --config dgadmm --coherence $c --steps 10 --warmup 2 > $O/blk$c.log 2>&1 || exit $?
done
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 -u tools/dyn_timeline.py 10 > $O/dyn_tl10.log 2>&1 || exit $?
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/logi_pmc -o k -- python3 $GRAFT_REPO_ROOT/bench.py --config logistic --steps 3 --warmup 1 > $O/logi_pmc.log 2>&1 || exit $?
