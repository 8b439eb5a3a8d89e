set -o pipefail
O=gpurun_out/dghint
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_multirank.py -k "dgadmm or dynamic or checkpoint" > $O/tests.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --config dgadmm > $O/b10.json 2> $O/b10.err && \
timeout -k 10 300 python3 -u bench.py --config dgadmm --coherence 1 > $O/b1.json 2> $O/b1.err && \
timeout -k 10 300 python3 -u bench.py --config dgadmm > $O/b10b.json 2> $O/b10b.err
