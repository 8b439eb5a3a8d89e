set -o pipefail
O=gpurun_out/gram_ab
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu tests/test_gpu.py -k "gram" > $O/tests.log 2>&1 && \
GADMM_NATIVE_LIB=$PWD/build/ab/libold.so timeout -k 10 200 python3 -u tools/gram_bench.py 1 262144 8192 > $O/old.log 2>&1 && \
timeout -k 10 200 python3 -u tools/gram_bench.py 1 262144 8192 > $O/new.log 2>&1 && \
GADMM_NATIVE_LIB=$PWD/build/ab/libold.so timeout -k 10 200 python3 -u tools/gram_bench.py 2 312500 10000 > $O/old10k.log 2>&1 && \
timeout -k 10 200 python3 -u tools/gram_bench.py 2 312500 10000 > $O/new10k.log 2>&1
