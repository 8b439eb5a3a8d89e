# Round 3, session 2: D-GADMM host clock at coherence 1, blocked vs per-worker kernel.
set -o pipefail
O=gpurun_out/r3_s2p
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
GADMM_BLOCKED_DYN=1 step blk 150 python3 -u tools/dgadmm_host_stamps.py 1 30
GADMM_BLOCKED_DYN=0 step pw 150 python3 -u tools/dgadmm_host_stamps.py 1 30
