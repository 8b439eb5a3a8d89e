# Round 3: barrier-free streaming Gram (GADMM_GRAM_KERNEL=streamP) vs the LDS-staged kernel.
set -o pipefail
O=gpurun_out/r3_gram2
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
GADMM_GRAM_KERNEL=stream2 step test_s2 200 python3 -u -m pytest tests/test_gpu.py -v -k "gram" --timeout 150 --timeout-method thread
GADMM_GRAM_KERNEL=stream3 step test_s3 200 python3 -u -m pytest tests/test_gpu.py -v -k "gram" --timeout 150 --timeout-method thread
step lds 300 python3 -u tools/gram_bench.py 2 625000 10000
GADMM_GRAM_KERNEL=stream2 step s2 300 python3 -u tools/gram_bench.py 2 625000 10000
GADMM_GRAM_KERNEL=stream3 step s3 300 python3 -u tools/gram_bench.py 2 625000 10000
GADMM_GRAM_KERNEL=stream2 step s2_small 300 python3 -u tools/gram_bench.py 1 262144 8192
step lds_small 300 python3 -u tools/gram_bench.py 1 262144 8192
