set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/ -m gpu -q --timeout 170 --timeout-method thread > $O/gpu_tier.log 2>&1 && \
timeout -k 10 150 python3 -u bench.py --steps 20 --warmup 3 > $O/bench1.json 2> $O/bench1.err && \
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
for c in logistic logistic_exact dgadmm star; do
  timeout -k 10 300 python3 -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || exit 1
done && \
timeout -k 10 150 python3 -u bench.py --workers 8 > $O/bench_w8.json 2> $O/bench_w8.err && \
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 300 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench_share2.json 2> $O/bench_share2.err
