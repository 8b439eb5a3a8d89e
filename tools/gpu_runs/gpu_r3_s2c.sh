# Round 3, session 2: blocked D-GADMM re-chain (LDS-staged epoch tables, lane-major inverse image,
# reloads only on solving positions): tests, device pace, bench, and an owned-run length sweep.
set -o pipefail
O=gpurun_out/r3_s2c
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step tests 400 python3 -u -m pytest tests/test_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "dgadmm or dynamic or blocked"
GADMM_BLOCKED_DYN=1 step pace_blk 150 python3 -u tools/dgadmm_pace.py 10 20
GADMM_BLOCKED_DYN=1 step dg_blk 150 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
step dg_pw 150 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
for L in 2 3 4; do
  GADMM_BLOCK_L=$L GADMM_BLOCKED_DYN=1 step pace_L$L 150 python3 -u tools/dgadmm_pace.py 10 20
done
GADMM_BLOCKED_DYN=1 step pace_blk1 150 python3 -u tools/dgadmm_pace.py 1 10
