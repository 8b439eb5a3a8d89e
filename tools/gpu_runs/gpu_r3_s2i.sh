# Round 3, session 2: D-GADMM host clock between labelled points of the solve path.
set -o pipefail
O=gpurun_out/r3_s2i
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step stamps 150 python3 -u tools/dgadmm_host_stamps.py 10 40
