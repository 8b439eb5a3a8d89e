# Round 3, session 2: data-local 2-rank kernel, normal vs free-running (no stop-rule pipeline).
set -o pipefail
O=gpurun_out/r3_s2f
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step free 200 python3 -u tools/dl_free.py 300
