#!/bin/bash
# round 5, session b: large-d LAG fix + multi-rank LAG / dual averaging / goldens; every bench config with
# its pinned expected count; the multi-rank headline rehearsal (tournament with the k sweep) at 2 / 4 / 8
# ranks and the configs[1] literal (--workers 8) at 2 / 4 / 8 ranks.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 300 python -u tools/lag_diverge.py > $O/lag_diverge.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py -k "first_order_big" \
  > $O/t_gpu.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_gpu_multirank.py \
  -k "first_order_big" > $O/t_mr.log 2>&1 || exit $?
for c in dgadmm star logistic logistic_exact; do
  timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 > $O/$c.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --config $c --workers 8 --steps 10 --warmup 2 > $O/${c}_w8.log 2>&1 || exit $?
done
for n in 2 4 8; do
  GADMM_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2957$n bench.py --gpus $n --steps 20 --warmup 3 > $O/e1_share$n.log 2>&1 || exit $?
  GADMM_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2958$n bench.py --gpus $n --workers 8 --steps 20 --warmup 3 \
    > $O/w8_share$n.log 2>&1 || exit $?
done
