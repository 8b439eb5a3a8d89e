set -o pipefail
O=gpurun_out/r2f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -v -k "newton or measured_clock or entry" --timeout 170 --timeout-method thread > $O/g_newton.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config logistic_exact --steps 5 --warmup 2 > $O/bc_logistic_exact.json 2> $O/bc_logistic_exact.err && \
timeout -k 10 300 python -u tools/newton_stats.py > $O/newton_stats.log 2>&1
