set -o pipefail
mkdir -p gpurun_out/r2d
O=gpurun_out/r2d
timeout -k 10 300 python -u -m pytest "tests/test_gpu_multirank.py::test_dgadmm_multirank_matches_one_gpu" -v --timeout 170 --timeout-method thread > $O/mr_dg.log 2>&1 && \
for c in star dgadmm logistic logistic_exact; do timeout -k 10 200 python -u bench.py --config $c --steps 5 --warmup 2 > $O/bc_$c.json 2> $O/bc_$c.err || exit 1; done && \
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > $O/b2.json 2> $O/b2.err && \
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --workers 8 --steps 5 --warmup 1 > $O/b4w8.json 2> $O/b4w8.err && \
for c in star dgadmm; do GADMM_BENCH_SHARE_GPU=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --config $c --steps 5 --warmup 1 > $O/b2_$c.json 2> $O/b2_$c.err || exit 1; done
