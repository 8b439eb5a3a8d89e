set -o pipefail
O=gpurun_out/ring
mkdir -p $O
timeout -k 10 200 python3 -u bench.py --steps 30 > $O/bench.json 2> $O/bench.err && \
timeout -k 10 200 python3 -u tools/blocked_timeline.py 300 > $O/tl.json 2> $O/tl.err && \
GADMM_BLK_DBG=32 timeout -k 10 200 python3 -u tools/blocked_timeline.py 300 > $O/tl_w8.json 2> $O/tl_w8.err && \
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu.py -k "blocked or dgadmm or xcd or residual or engine_graph" > $O/tests.log 2>&1
