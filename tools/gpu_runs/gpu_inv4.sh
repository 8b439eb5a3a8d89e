set -o pipefail
O=gpurun_out/inv4
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu.py -k "spd_inverse or engine_graph" > $O/tests.log 2>&1 && \
for r in 1 2; do
GADMM_NATIVE_LIB=$PWD/build/ab/libold.so timeout -k 10 120 python3 -u tools/inv_time.py >> $O/inv_old.log 2>&1 && \
timeout -k 10 120 python3 -u tools/inv_time.py >> $O/inv_new.log 2>&1 || exit 1
done
