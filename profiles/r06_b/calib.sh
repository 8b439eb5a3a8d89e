#!/bin/bash
# tournament cost model with rank 0's one-GPU calibration: 2 / 4 ranks sharing one GPU, plus N = 1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6calib}; mkdir -p $O
timeout -k 10 120 python bench.py > $O/e1.log 2>&1 || exit $?
for n in 2 4; do
  GADMM_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2971$n bench.py --gpus $n --steps 20 --warmup 3 > $O/share$n.log 2>&1 || exit $?
done
