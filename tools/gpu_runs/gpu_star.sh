set -o pipefail
O=gpurun_out/star2
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_multirank.py -k "star or baselines or xcd or std_admm" > $O/tests.log 2>&1 && \
timeout -k 10 300 python3 -u tools/star_sweep.py > $O/star.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --config star > $O/bench_star.json 2> $O/bench_star.err
