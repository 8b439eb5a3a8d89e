set -o pipefail
O=gpurun_out/resume
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "resume or elastic or checkpoint" > $O/tests.log 2>&1
