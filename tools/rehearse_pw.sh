# Multi-rank rehearsal (ranks share cuda:0) of the two blocked wave layouts: pw=1 (k=2) vs pw=2 (k=3)
set -o pipefail
mkdir -p gpurun_out
for N in 2 4; do
  for PW in 1 2; do
    GADMM_BLOCK_PW=$PW GADMM_BENCH_SHARE_GPU=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29600 + 10 * N + PW)) bench.py --gpus $N \
      --steps 20 --warmup 2 > gpurun_out/rehearse_${N}_pw$PW.json 2> gpurun_out/rehearse_${N}_pw$PW.err || exit 1
  done
done
echo done
