set -o pipefail
O=gpurun_out/skip2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_multirank.py -k "blocked or dgadmm or xcd or residual or engine_graph or smoke or bench_json or entry" > $O/tests.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 200 python3 -u bench.py --workers 8 > $O/w8.json 2> $O/w8.err && \
timeout -k 10 200 python3 -u tools/blocked_timeline.py 300 > $O/tl.json 2> $O/tl.err
