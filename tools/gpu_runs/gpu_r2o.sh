set -o pipefail
O=gpurun_out/r2o
mkdir -p $O
timeout -k 10 200 python -u bench.py --config dgadmm --coherence 1 --steps 10 --warmup 2 > $O/bc_dg_c1.json 2> $O/bc_dg_c1.err && \
timeout -k 10 200 python -u bench.py --config dgadmm --coherence 1 --workers 8 --steps 10 --warmup 2 > $O/bc_dg_c1_w8.json 2> $O/bc_dg_c1_w8.err && \
timeout -k 10 200 python -u bench.py --workers 8 --steps 20 --warmup 3 > $O/b1_w8.json 2> $O/b1_w8.err
