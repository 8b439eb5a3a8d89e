set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python -u bench.py --steps 10 --warmup 2 > gpurun_out/b1.json 2> gpurun_out/b1.err && \
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/b2.json 2> gpurun_out/b2.err && \
timeout -k 10 1200 python -u -m pytest tests/test_gpu_multirank.py -v --timeout 300 --timeout-method thread > gpurun_out/mr.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/g1.log 2>&1
