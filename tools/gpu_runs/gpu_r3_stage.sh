# Round 3: D-GADMM host / kernel stage times, per-worker vs blocked dynamic mode.
set -o pipefail
O=gpurun_out/r3_stage
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step pw 150 python3 -u tools/dgadmm_stage_times.py 10
GADMM_BLOCKED_DYN=1 step blk 150 python3 -u tools/dgadmm_stage_times.py 10
step pw_b 150 python3 -u tools/dgadmm_stage_times.py 10
GADMM_BLOCKED_DYN=1 step blk_b 150 python3 -u tools/dgadmm_stage_times.py 10
