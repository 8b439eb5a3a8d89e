set -o pipefail
O=gpurun_out/share
mkdir -p $O
for n in 2 4 8; do
  GADMM_BENCH_SHARE_GPU=1 timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 5 --warmup 2 > $O/share$n.json 2> $O/share$n.err || exit 1
done
for n in 2 4; do
  GADMM_BENCH_SHARE_GPU=1 timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29700 + n)) bench.py --gpus $n --steps 5 --warmup 2 --config dgadmm > $O/share_dg$n.json 2> $O/share_dg$n.err || exit 1
done
