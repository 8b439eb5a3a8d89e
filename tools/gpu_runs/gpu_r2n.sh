set -o pipefail
O=gpurun_out/r2n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -v -k "dgadmm" --timeout 170 --timeout-method thread > $O/g_dg.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -v -k "dgadmm" --timeout 170 --timeout-method thread > $O/mr_dg.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config dgadmm --steps 10 --warmup 2 > $O/bc_dgadmm.json 2> $O/bc_dgadmm.err
