# Round 3: blocked D-GADMM with epoch chunks (hard stop + continuation) -- bit-identity, then timing.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_dyn3
mkdir -p $O
cd $GRAFT_REPO_ROOT
. tools/gpu_runs/gpu_step.sh
step tests 300 python3 -u -m pytest tests/test_gpu.py -v -k "dgadmm or dynamic or xcd" --timeout 150 --timeout-method thread
grep -q " passed" $O/tests.log && ! grep -qE "[0-9]+ failed" $O/tests.log || exit 1
for r in 1 2; do
  GADMM_BLOCKED_DYN=1 step bench_blk_$r 120 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
  step bench_pw_$r 120 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
done
GADMM_BLOCKED_DYN=1 step bench_blk_c1 120 python3 -u bench.py --config dgadmm --coherence 1 --steps 20 --warmup 3
step bench_pw_c1 120 python3 -u bench.py --config dgadmm --coherence 1 --steps 20 --warmup 3
GADMM_BLOCKED_DYN=1 step stage 120 python3 -u tools/dgadmm_stage_times.py 10
