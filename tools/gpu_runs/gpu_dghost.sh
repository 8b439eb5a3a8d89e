set -o pipefail
O=gpurun_out/dghost
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu tests/test_gpu.py -k "engine_graph or blocked_layouts or measured_clock or dgadmm" > $O/tests.log 2>&1 && \
timeout -k 10 300 python3 -u tools/dgadmm_host_profile.py 10 > $O/prof10.log 2>&1
