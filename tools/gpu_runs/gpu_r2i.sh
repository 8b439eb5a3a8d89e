set -o pipefail
O=gpurun_out/r2i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -v -k "gemm_f64 or spd_inverse_blocked" --timeout 170 --timeout-method thread > $O/g_k2.log 2>&1 && \
timeout -k 10 300 python -u tools/bigd_inverse_bench.py 1024 4096 10000 > $O/bigd_inverse.jsonl 2> $O/bigd_inverse.err && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o inv10k -- python -u tools/bigd_inverse_bench.py 10000 > $O/inv10k.jsonl 2> $O/inv10k.err
