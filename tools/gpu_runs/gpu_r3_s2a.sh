# Round 3, session 2: re-validate HEAD (native epoch/flush table builder) on a fresh box:
# the full GPU tier, smoke, the headline, and D-GADMM in both kernel modes.
set -o pipefail
O=gpurun_out/r3_s2a
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step tier 1000 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 120 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step e1 120 python3 -u bench.py --steps 20 --warmup 3
step dg 150 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
GADMM_BLOCKED_DYN=1 step dg_blk 150 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
step pw 150 python3 -u tools/dgadmm_stage_times.py 10
GADMM_BLOCKED_DYN=1 step blk 150 python3 -u tools/dgadmm_stage_times.py 10
