set -o pipefail
O=gpurun_out/dyn2
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_multirank.py -k "dgadmm or dynamic or xcd or checkpoint" > $O/tests.log 2>&1 && \
timeout -k 10 240 python3 -u tools/xcd_probe.py 1 8 > $O/dyn1.json 2> $O/dyn1.err && \
timeout -k 10 240 python3 -u tools/xcd_probe.py 10 8 > $O/dyn10.json 2> $O/dyn10.err && \
timeout -k 10 300 python3 -u bench.py --config dgadmm > $O/bench10.json 2> $O/bench10.err && \
timeout -k 10 300 python3 -u bench.py --config dgadmm --coherence 1 > $O/bench1.json 2> $O/bench1.err
