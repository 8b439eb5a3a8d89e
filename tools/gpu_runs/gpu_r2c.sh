set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -q --timeout 170 --timeout-method thread > gpurun_out/g1.log 2>&1 && \
timeout -k 10 1200 python -u -m pytest tests/test_gpu_multirank.py -v --timeout 170 --timeout-method thread > gpurun_out/mr.log 2>&1
