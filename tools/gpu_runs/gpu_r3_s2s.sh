# Round 3, session 2: waves per matrix of the register-row Gauss-Jordan inverse (E1 set-up), A/B.
set -o pipefail
O=gpurun_out/r3_s2s
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
for W in 8 4 16; do
  GADMM_INV_REG=$W step inv$W 60 python3 -u tools/inv_time.py
done
step inv8b 60 python3 -u tools/inv_time.py
