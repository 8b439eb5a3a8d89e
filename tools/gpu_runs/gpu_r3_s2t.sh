# Round 3, session 2: the multi-rank data-local tests after factoring the halo plan (blocked_xgmi.py).
set -o pipefail
O=gpurun_out/r3_s2t
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step mr 600 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu -v --timeout 300 --timeout-method thread -x -k "data_local or stalled"
GADMM_BENCH_SHARE_GPU=1 step share4 200 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29784 bench.py --gpus 4 --steps 10 --warmup 2
