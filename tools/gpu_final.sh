set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 170 --timeout-method thread > $O/gpu_tier.log 2>&1 && \
timeout -k 10 150 python -u bench.py --steps 20 --warmup 3 > $O/bench1.json 2> $O/bench1.err && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
