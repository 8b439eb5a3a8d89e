set -o pipefail
O=gpurun_out/xcd
mkdir -p $O
timeout -k 10 240 python3 -u tools/xcd_probe.py 0 15 > $O/static.json 2> $O/static.err && \
timeout -k 10 240 python3 -u tools/xcd_probe.py 1 10 > $O/dyn1.json 2> $O/dyn1.err && \
timeout -k 10 240 python3 -u tools/xcd_probe.py 10 10 > $O/dyn10.json 2> $O/dyn10.err && \
GADMM_XCD=0 timeout -k 10 300 python3 -u bench.py > $O/bench_x0.json 2> $O/bench_x0.err && \
timeout -k 10 300 python3 -u bench.py > $O/bench_x2.json 2> $O/bench_x2.err && \
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests > $O/tests_gpu.log 2>&1
