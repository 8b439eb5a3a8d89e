set -o pipefail
O=gpurun_out/r2q
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -q -k "dgadmm or clock or chain_admm or residual" --timeout 170 --timeout-method thread > $O/g.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config dgadmm --coherence 1 --steps 10 --warmup 2 > $O/bc_dg_c1.json 2> $O/bc_dg_c1.err && \
timeout -k 10 200 python -u bench.py --config dgadmm --steps 10 --warmup 2 > $O/bc_dg.json 2> $O/bc_dg.err && \
timeout -k 10 200 python -u bench.py --config logistic --steps 10 --warmup 2 > $O/bc_log.json 2> $O/bc_log.err && \
timeout -k 10 200 python -u bench.py --config logistic_exact --steps 5 --warmup 2 > $O/bc_logx.json 2> $O/bc_logx.err
