#!/bin/bash
# does rank 0's one-GPU calibration disturb the tournament? share 2 / 4 with it off and on
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6calab}; mkdir -p $O
for n in 2 4; do
  for c in 0 1; do
    GADMM_TOURNAMENT_CALIBRATE=$c GADMM_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port 297$c$n bench.py --gpus $n --steps 20 --warmup 3 > $O/share${n}_c$c.log 2>&1 || exit $?
  done
done
