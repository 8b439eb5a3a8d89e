set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -v --timeout 300 --timeout-method thread > gpurun_out/mr2.log 2>&1 ; echo "rc=$?" >> gpurun_out/mr2.log
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/g1.log 2>&1 ; echo "rc=$?" >> gpurun_out/g1.log
for c in star dgadmm logistic logistic_exact; do timeout -k 10 200 python -u bench.py --config $c --steps 5 --warmup 2 > gpurun_out/bc_$c.json 2> gpurun_out/bc_$c.err || break; done
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --workers 8 --steps 5 --warmup 1 > gpurun_out/b4w8.json 2> gpurun_out/b4w8.err
