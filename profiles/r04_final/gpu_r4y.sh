#!/bin/bash
# round 4, final: the multi-rank headline rehearsal (ranks sharing the GPU) at 2 / 4 / 8 ranks
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4y; mkdir -p $O
for n in 2 4 8; do
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2954$n bench.py --gpus $n --steps 20 --warmup 3 > $O/e1_$n.log 2>&1 || exit $?
done
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29552 bench.py --gpus 2 --config real10m --rows 100000 --dim 2048 --steps 1 --warmup 0 > $O/real_2.log 2>&1
