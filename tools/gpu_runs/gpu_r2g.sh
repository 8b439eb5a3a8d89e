set -o pipefail
O=gpurun_out/r2g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bigd_inverse_bench.py > $O/bigd_inverse.jsonl 2> $O/bigd_inverse.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o real10m -- python -u bench.py --config real10m --steps 1 --warmup 0 > $O/real10m.json 2> $O/real10m.err
