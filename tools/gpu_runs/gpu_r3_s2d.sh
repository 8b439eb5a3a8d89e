# Round 3, session 2: the data-local one-position halo mode (2 / 4 / 8 ranks sharing the GPU):
# multi-rank tests, then share-mode benches with and without the halo.
set -o pipefail
O=gpurun_out/r3_s2d
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step mr 600 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu -v --timeout 300 --timeout-method thread -x -k "data_local or stalled"
for N in 2 4 8; do
  GADMM_BENCH_SHARE_GPU=1 step halo$N 200 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29720 + N)) bench.py --gpus $N --steps 10 --warmup 2
  GADMM_DL_HALO=0 GADMM_BENCH_SHARE_GPU=1 step nohalo$N 200 python3 -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29730 + N)) bench.py --gpus $N --steps 10 --warmup 2
done
