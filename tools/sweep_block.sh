# Sweep of the temporally blocked kernel's (k, L) on the E1 headline (one GPU call, same box).
set -o pipefail
for kl in "2 4" "2 3" "2 2" "1 8" "1 6" "1 4" "2 4"; do
  set -- $kl
  GADMM_BLOCK_K=$1 GADMM_BLOCK_L=$2 timeout -k 10 100 python bench.py --steps 50 > gpurun_out/sw_$1_$2.log 2>&1 || exit 1
  echo "k=$1 L=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw_$1_$2.log) $(grep -o '"kernel": "[^"]*"' gpurun_out/sw_$1_$2.log)"
done
