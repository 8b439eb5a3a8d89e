set -o pipefail
O=gpurun_out/r2j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -q -x --timeout 170 --timeout-method thread > $O/g1.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py -v -x --timeout 170 --timeout-method thread > $O/mr.log 2>&1 && \
timeout -k 10 150 python -u bench.py --steps 20 --warmup 3 > $O/b1.json 2> $O/b1.err
