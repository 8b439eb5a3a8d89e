# Round 3, session 2: headline A/B on one box, the session-start tree (ab_old/) vs the current tree.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s2v
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step new1 120 python3 -u bench.py --steps 20 --warmup 3
(cd ab_old && timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 3 > $O/old1.log 2>&1); echo "old1 rc=$?" >> $O/rc.txt
step new2 120 python3 -u bench.py --steps 20 --warmup 3
(cd ab_old && timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 3 > $O/old2.log 2>&1); echo "old2 rc=$?" >> $O/rc.txt
step dgnew 120 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
(cd ab_old && GADMM_BLOCKED_DYN=0 timeout -k 10 120 python3 -u bench.py --config dgadmm --steps 20 --warmup 3 > $O/dgold.log 2>&1); echo "dgold rc=$?" >> $O/rc.txt
