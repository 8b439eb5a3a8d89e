set -o pipefail
O=gpurun_out/r2l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o real10m -- python -u bench.py --config real10m --steps 1 --warmup 1 > $O/real10m.json 2> $O/real10m.err && \
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --config logistic --steps 5 --warmup 1 > $O/b2_logistic.json 2> $O/b2_logistic.err
