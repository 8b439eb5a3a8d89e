# Round 3, session 2: stop-decision lag A/B on the one-GPU headline and D-GADMM (persistent kernels).
set -o pipefail
O=gpurun_out/r3_s2q
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
for L in 8 16 6 12; do
  GADMM_PERSIST_LAG=$L step e1_lag$L 120 python3 -u bench.py --steps 20 --warmup 3
done
for L in 8 16; do
  GADMM_PERSIST_LAG=$L step dg_lag$L 120 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
done
step e1_lag8b 120 python3 -u bench.py --steps 20 --warmup 3
