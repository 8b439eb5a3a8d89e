#!/bin/bash
# round 4: large-d (configs[4]) across ranks sharing the GPU: IPC star collectives + chain_big graph engine
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_multirank.py -k large_d > $O/t.log 2>&1 || exit $?
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config real10m --rows 100000 --dim 2048 --steps 1 --warmup 1 > $O/bench2.log 2>&1
