set -o pipefail
O=gpurun_out/r2m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -v -k "star" --timeout 170 --timeout-method thread > $O/mr_star.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config star --steps 10 --warmup 2 > $O/bc_star.json 2> $O/bc_star.err
