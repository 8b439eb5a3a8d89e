#!/bin/bash
# round 4: IPC collective check at 2/4 ranks, LAG goldens on the large-d engine, remaining benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 200 python -u tools/ipc_coll_check.py 2 > $O/coll2.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/ipc_coll_check.py 4 > $O/coll4.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu.py -k "first_order_big" > $O/t1.log 2>&1
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --steps 20 --warmup 3 > $O/e1_8.log 2>&1 || exit $?
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29536 bench.py --gpus 4 --steps 20 --warmup 3 > $O/e1_4.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --steps 20 --warmup 3 > $O/e1_1.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config dgadmm --steps 10 --warmup 2 > $O/dg.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config star --steps 10 --warmup 2 > $O/star.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config real10m --steps 1 --warmup 0 > $O/real10m.log 2>&1
