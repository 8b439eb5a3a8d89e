set -o pipefail
O=gpurun_out/prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof/e1 -o e1 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof/e1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof/dg -o dg -- python3 $GRAFT_REPO_ROOT/bench.py --config dgadmm --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof/dg.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof/star -o star -- python3 $GRAFT_REPO_ROOT/bench.py --config star --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof/star.log 2>&1
