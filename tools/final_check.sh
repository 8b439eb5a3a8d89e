# Round-end rehearsal on one GPU: the GPU test suite, smoke(), the headline bench, the other configs,
# and the 2/4-rank rehearsal of the multi-GPU path (ranks share cuda:0). Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu.py > gpurun_out/fc_tests.log 2>&1 || { tail -5 gpurun_out/fc_tests.log; exit 1; }
tail -1 gpurun_out/fc_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fc_smoke.log 2>&1 || { tail -5 gpurun_out/fc_smoke.log; exit 1; }
tail -1 gpurun_out/fc_smoke.log
timeout -k 10 120 python bench.py > gpurun_out/fc_bench.json 2> gpurun_out/fc_bench.err || exit 1
cut -c1-400 gpurun_out/fc_bench.json
for c in logistic logistic_exact dgadmm; do
  timeout -k 10 120 python bench.py --config $c --steps 10 --warmup 2 > gpurun_out/fc_$c.json 2> gpurun_out/fc_$c.err || exit 1
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fc_$c.json) $(grep -o '"iterations_to_tol": [0-9]*' gpurun_out/fc_$c.json)"
done
for N in 2 4; do
  GADMM_BENCH_SHARE_GPU=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29700 + N)) bench.py --gpus $N --steps 10 --warmup 2 \
    > gpurun_out/fc_rehearse_$N.json 2> gpurun_out/fc_rehearse_$N.err || exit 1
  echo "rehearsal N=$N $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fc_rehearse_$N.json) $(grep -o '"iterations_to_tol": [0-9]*' gpurun_out/fc_rehearse_$N.json) $(grep -o '"kernel": "[^"]*"' gpurun_out/fc_rehearse_$N.json)"
done
