set -o pipefail
O=gpurun_out/startrim
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_multirank.py -x -q --timeout 170 --timeout-method thread -k "star or dgadmm or dynamic or trace or clock or persistent" > $O/tests.log 2>&1 && \
timeout -k 10 150 python3 -u bench.py --config star > $O/star.json 2> $O/star.err && \
timeout -k 10 150 python3 -u bench.py --config dgadmm > $O/dg.json 2> $O/dg.err && \
timeout -k 10 150 python3 -u bench.py > $O/e1.json 2> $O/e1.err
