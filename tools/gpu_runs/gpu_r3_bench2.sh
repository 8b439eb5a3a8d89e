# Round 3: every bench config on one MI355X, plus the share-mode multi-rank rehearsals.
set -o pipefail
O=gpurun_out/r3_bench2
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step selftest 200 python3 -u -m pytest tests/test_native_selftest.py -v -m gpu --timeout 150 --timeout-method thread
step e1 120 python3 -u bench.py
step e1_20 120 python3 -u bench.py --steps 20 --warmup 3
for c in logistic logistic_exact dgadmm star; do
  step $c 150 python3 -u bench.py --config $c --steps 10 --warmup 2
done
step w8 120 python3 -u bench.py --workers 8 --steps 20 --warmup 3
step real10m 400 python3 -u bench.py --config real10m --steps 1 --warmup 1
for N in 2 4 8; do
  GADMM_BENCH_SHARE_GPU=1 step share$N 200 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29700 + N)) bench.py --gpus $N --steps 10 --warmup 2
done
