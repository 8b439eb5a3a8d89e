set -o pipefail
O=gpurun_out/aq
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_multirank.py -k "persistent or dgadmm or xcd or residual or engine_graph or xgmi or stall" > $O/tests.log 2>&1 && \
for r in 1 2; do
  GADMM_NATIVE_LIB=$PWD/build/ab/libold.so timeout -k 10 240 python3 -u tools/xcd_probe.py 1 8 > $O/old1_$r.json 2>> $O/err.log && \
  timeout -k 10 240 python3 -u tools/xcd_probe.py 1 8 > $O/new1_$r.json 2>> $O/err.log && \
  GADMM_NATIVE_LIB=$PWD/build/ab/libold.so timeout -k 10 240 python3 -u tools/xcd_probe.py 10 8 > $O/old10_$r.json 2>> $O/err.log && \
  timeout -k 10 240 python3 -u tools/xcd_probe.py 10 8 > $O/new10_$r.json 2>> $O/err.log && \
  GADMM_BLOCKED=0 GADMM_NATIVE_LIB=$PWD/build/ab/libold.so timeout -k 10 200 python3 -u bench.py --steps 20 > $O/oldpw_$r.json 2>> $O/err.log && \
  GADMM_BLOCKED=0 timeout -k 10 200 python3 -u bench.py --steps 20 > $O/newpw_$r.json 2>> $O/err.log || exit 1
done
