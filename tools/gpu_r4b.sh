#!/bin/bash
# round 4: configs[4] across ranks + bench tournament / hop probe / timed-loop fallback (ranks sharing the GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_multirank.py -k "large_d or bench_ or epoch_wrap" tests/test_gpu.py::test_dgadmm_blocked_dynamic_small_chains_idle_decision_wave tests/test_gpu.py::test_logistic_newton_kernel_matches_torch > $O/t.log 2>&1
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config real10m --rows 100000 --dim 2048 --steps 1 --warmup 1 > $O/real2.log 2>&1 || exit $?
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --steps 20 --warmup 3 > $O/e1_8.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config dgadmm --steps 10 --warmup 2 > $O/dg.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config star --steps 10 --warmup 2 > $O/star.log 2>&1
