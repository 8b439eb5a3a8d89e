# Round 3: rocprofv3 kernel breakdown of real10m (configs[4]) and the headline, plus the headline
# kernel's in-kernel timeline.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/real10m -o k -- python3 $GRAFT_REPO_ROOT/bench.py --config real10m --steps 1 --warmup 1 > $O/real10m.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/e1 -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 > $O/e1.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 -u tools/blocked_timeline.py 300 > $O/e1_timeline.log 2>&1 || exit $?
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 200 python3 -u tools/dl_timeline.py 200 > $O/dl_timeline.log 2>&1 || exit $?
