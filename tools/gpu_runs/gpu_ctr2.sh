set -o pipefail
O=gpurun_out/ctr2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_multirank.py -k "persistent or dgadmm or xcd or residual or engine_graph or xgmi or stall or resid" > $O/tests.log 2>&1 && \
for r in 1 2; do
  GADMM_NATIVE_LIB=$PWD/build/ab/libold.so timeout -k 10 240 python3 -u tools/xcd_probe.py 1 8 > $O/old1_$r.json 2>> $O/err.log && \
  timeout -k 10 240 python3 -u tools/xcd_probe.py 1 8 > $O/new1_$r.json 2>> $O/err.log && \
  GADMM_NATIVE_LIB=$PWD/build/ab/libold.so timeout -k 10 240 python3 -u tools/xcd_probe.py 10 8 > $O/old10_$r.json 2>> $O/err.log && \
  timeout -k 10 240 python3 -u tools/xcd_probe.py 10 8 > $O/new10_$r.json 2>> $O/err.log || exit 1
done
