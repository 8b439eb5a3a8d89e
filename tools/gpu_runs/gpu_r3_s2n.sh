# Round 3, session 2: stop-decision lag A/B for the data-local multi-rank kernel (ranks sharing the GPU).
set -o pipefail
O=gpurun_out/r3_s2n
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
for N in 2 4; do
  for L in 8 16 4; do
    GADMM_DL_LAG=$L GADMM_BENCH_SHARE_GPU=1 step s${N}_lag$L 200 python3 -u -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29760 + N + L)) bench.py --gpus $N --steps 10 --warmup 2
  done
done
