# Round 3, session 2: checkpoint of the final tree -- full GPU tier, smoke, every bench config, and the
# multi-rank rehearsal (ranks sharing the GPU).
set -o pipefail
O=gpurun_out/r3_s2m
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step tier 1000 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 120 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step e1 120 python3 -u bench.py --steps 20 --warmup 3
for c in logistic logistic_exact dgadmm star; do
  step $c 150 python3 -u bench.py --config $c --steps 10 --warmup 2
done
step w8 120 python3 -u bench.py --workers 8 --steps 20 --warmup 3
step real10m 400 python3 -u bench.py --config real10m --steps 1 --warmup 1
for N in 2 4 8; do
  GADMM_BENCH_SHARE_GPU=1 step share$N 200 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29750 + N)) bench.py --gpus $N --steps 10 --warmup 2
done
