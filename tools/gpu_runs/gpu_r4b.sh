#!/bin/bash
# round 4: packed symv, configs[4] across ranks, hosted halo at 2 ranks, bench tournament / hop probe / fallback,
# large-d first-order engine, branch-free Gram prefetch (A/B vs the previous build)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu.py -k "gram or sym_pack or large_d_engine or star_big or idle_decision or newton_kernel_matches or first_order_big" > $O/t1.log 2>&1
timeout -k 10 300 python -u tools/gram_bench.py 2 312500 10000 > $O/gram_new.log 2>&1 || exit $?
GADMM_NATIVE_LIB=$PWD/gadmm_amd/_native/ab/lib_prev.so timeout -k 10 300 python -u tools/gram_bench.py 2 312500 10000 > $O/gram_old.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_multirank.py -k "large_d or bench_ or epoch_wrap or data_local_xgmi or first_order_big" > $O/t.log 2>&1
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config real10m --rows 100000 --dim 2048 --steps 1 --warmup 1 > $O/real2.log 2>&1 || exit $?
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --steps 20 --warmup 3 > $O/e1_2.log 2>&1 || exit $?
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --steps 20 --warmup 3 > $O/e1_8.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config dgadmm --steps 10 --warmup 2 > $O/dg.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config star --steps 10 --warmup 2 > $O/star.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config real10m --steps 1 --warmup 0 > $O/real10m.log 2>&1
