set -o pipefail
O=gpurun_out/skip
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_multirank.py -k "blocked or dgadmm or xcd or residual or engine_graph or smoke or bench_json" > $O/tests.log 2>&1 && \
timeout -k 10 200 python3 -u bench.py --steps 30 > $O/bench.json 2> $O/bench.err && \
GADMM_BLOCK_L=2 timeout -k 10 200 python3 -u bench.py --steps 30 > $O/bench_L2.json 2> $O/bench_L2.err && \
GADMM_BLOCK_K=1 timeout -k 10 200 python3 -u bench.py --steps 30 > $O/bench_k1.json 2> $O/bench_k1.err && \
GADMM_NATIVE_LIB=$PWD/build/ab/libold.so timeout -k 10 200 python3 -u bench.py --steps 30 > $O/bench_old.json 2> $O/bench_old.err && \
timeout -k 10 200 python3 -u bench.py --steps 30 > $O/bench2.json 2> $O/bench2.err
