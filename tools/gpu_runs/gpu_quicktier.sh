set -o pipefail
O=gpurun_out/quick
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -q --timeout 170 --timeout-method thread > $O/gpu_tier.log 2>&1 && \
timeout -k 10 120 python3 -u bench.py --config dgadmm > $O/dg.json 2>/dev/null && \
timeout -k 10 120 python3 -u bench.py > $O/e1.json 2>/dev/null
