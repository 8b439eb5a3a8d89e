set -o pipefail
mkdir -p gpurun_out/r2e
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -q --timeout 170 --timeout-method thread > gpurun_out/r2e/g1.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config star --steps 5 --warmup 2 > gpurun_out/r2e/bc_star.json 2> gpurun_out/r2e/bc_star.err
