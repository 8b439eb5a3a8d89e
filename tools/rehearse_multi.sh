# Multi-rank rehearsal of bench.py on ONE GPU (ranks share cuda:0; xGMI fabric via IPC on the same device)
set -o pipefail
mkdir -p gpurun_out
for N in 2 4 8; do
  GADMM_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py --gpus $N --steps 10 --warmup 2 \
    > gpurun_out/rehearse_$N.json 2> gpurun_out/rehearse_$N.err || exit 1
done
echo done
