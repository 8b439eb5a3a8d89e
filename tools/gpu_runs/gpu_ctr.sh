set -o pipefail
O=gpurun_out/ctr
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_multirank.py -k "blocked or dgadmm or xcd or residual or engine_graph" > $O/tests.log 2>&1 && \
for r in 1 2; do
  GADMM_NATIVE_LIB=$PWD/build/ab/libold.so timeout -k 10 200 python3 -u bench.py --steps 30 > $O/old_$r.json 2> $O/old_$r.err && \
  timeout -k 10 200 python3 -u bench.py --steps 30 > $O/new_$r.json 2> $O/new_$r.err || exit 1
done
