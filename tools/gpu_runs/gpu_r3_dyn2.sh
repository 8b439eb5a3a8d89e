# Round 3: blocked D-GADMM kernel with the padded-inverse re-chain reload -- bit-identity tests, then
# kernel time by coherence (blocked vs per-worker) and the bench.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_dyn2
mkdir -p $O
cd $GRAFT_REPO_ROOT
. tools/gpu_runs/gpu_step.sh
step tests 300 python3 -u -m pytest tests/test_gpu.py -v -k "dgadmm_persistent_dynamic or dynamic or xcd" --timeout 150 --timeout-method thread
grep -q " passed" $O/tests.log && ! grep -qE "[0-9]+ failed" $O/tests.log || exit 1
cd /tmp && export TMPDIR=/tmp
for c in 10 100; do
  GADMM_BLOCKED_DYN=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/blk$c -o k -- python3 $GRAFT_REPO_ROOT/bench.py --config dgadmm --coherence $c --steps 10 --warmup 2 > $O/blk$c.log 2>&1 || exit $?
done
cd $GRAFT_REPO_ROOT
GADMM_BLOCKED_DYN=1 step bench_blk 120 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
step bench_pw 120 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
GADMM_BLOCKED_DYN=1 step bench_blk_c1 120 python3 -u bench.py --config dgadmm --coherence 1 --steps 20 --warmup 3
