# Round 3: pipelined hand-off polls (persist_device.h pipe_poll) -- correctness first (the chain
# kernels' GPU tests, bit-identity across engines / ranks), then old/new library A/B on one box.
set -o pipefail
O=gpurun_out/r3_pipe
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step tests 600 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_multirank.py -x -v --timeout 170 --timeout-method thread \
  -k "persistent or blocked or dgadmm or dynamic or data_local or stalled or xgmi or newton or headline or xcd"
grep -q "passed" $O/tests.log && ! grep -qE "[0-9]+ failed" $O/tests.log || exit 1
OLD=$PWD/build/libgadmm_native_prepipe.so
for r in 1 2; do
  GADMM_NATIVE_LIB=$OLD step e1_old_$r 120 python3 -u bench.py --steps 20 --warmup 3
  step e1_new_$r 120 python3 -u bench.py --steps 20 --warmup 3
  GADMM_NATIVE_LIB=$OLD step dg_old_$r 120 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
  step dg_new_$r 120 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
  GADMM_BENCH_SHARE_GPU=1 GADMM_NATIVE_LIB=$OLD step dl2_old_$r 200 python3 -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29620 + r)) bench.py --gpus 2 --steps 10 --warmup 2
  GADMM_BENCH_SHARE_GPU=1 step dl2_new_$r 200 python3 -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29630 + r)) bench.py --gpus 2 --steps 10 --warmup 2
done
