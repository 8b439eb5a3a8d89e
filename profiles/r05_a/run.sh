#!/bin/bash
# round 5, session a: the new data-plane pieces (RCCL watchdog, distributed-CG optimum, tournament
# with the replicated-halo k sweep and graph candidates), then the full-d real10m share rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 300 python -u tools/lag_diverge.py > $O/lag_diverge.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py \
  -k "rccl or spd_inverse_blocked or large_d_optimum or first_order_big or bench_json or graft_smoke or gemm_f64" \
  > $O/t_gpu.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_multirank.py \
  -k "large_d_gadmm_and_star or bench_tournament or timed_loop_stall or first_order_big" > $O/t_mr.log 2>&1 || exit $?
timeout -k 10 120 python bench.py > $O/e1.log 2>&1 || exit $?
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --config real10m --rows 40000 --dim 10000 \
  --steps 1 --warmup 0 > $O/real_s2.log 2>&1 || exit $?
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 4 --config real10m --rows 40000 --dim 10000 \
  --steps 1 --warmup 0 > $O/real_s4.log 2>&1 || exit $?
