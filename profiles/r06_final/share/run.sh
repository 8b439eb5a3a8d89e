#!/bin/bash
# the driver's multi-rank bench command with 2 / 4 / 8 ranks sharing one GPU (GADMM_BENCH_SHARE_GPU=1)
# on the final tree: tournament, timed loop, calibration, JSON line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6share}; mkdir -p $O
for n in 2 4 8; do
  GADMM_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2981$n bench.py --gpus $n --steps 10 --warmup 2 > $O/share$n.log 2>&1 || exit $?
done
