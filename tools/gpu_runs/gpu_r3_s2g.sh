# Round 3, session 2: D-GADMM host path after the re-chain change (blocked dynamic mode default).
set -o pipefail
O=gpurun_out/r3_s2g
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step pyprof 200 python3 -u tools/dgadmm_pyprof.py 10
step stage 150 python3 -u tools/dgadmm_stage_times.py 10
