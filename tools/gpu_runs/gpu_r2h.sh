set -o pipefail
O=gpurun_out/r2h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -v -k "gemm_f64 or spd_inverse_blocked or newton_kernel_matches" --timeout 170 --timeout-method thread > $O/g_k2.log 2>&1 && \
timeout -k 10 300 python -u tools/bigd_inverse_bench.py > $O/bigd_inverse.jsonl 2> $O/bigd_inverse.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o real10m -- python -u bench.py --config real10m --steps 1 --warmup 1 > $O/real10m.json 2> $O/real10m.err
