# Round 3, session 2: where a D-GADMM solve's time goes (device pace per epoch offset, host cProfile,
# kernel + copy trace of the blocked dynamic mode), and the replicated-halo engine in share mode.
set -o pipefail
O=gpurun_out/r3_s2b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
. tools/gpu_runs/gpu_step.sh
step pace_pw 150 python3 -u tools/dgadmm_pace.py 10 20
GADMM_BLOCKED_DYN=1 step pace_blk 150 python3 -u tools/dgadmm_pace.py 10 20
GADMM_BLOCKED_DYN=1 step pace_blk100 150 python3 -u tools/dgadmm_pace.py 100 10
GADMM_BLOCKED_DYN=1 step pyprof_blk 200 python3 -u tools/dgadmm_pyprof.py 10
GADMM_BLOCKED_DYN=1 step trace_blk 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d $O/trace_blk -o run -- python3 -u bench.py --config dgadmm --steps 10 --warmup 2
for N in 2 4; do
  GADMM_BENCH_SHARE_GPU=1 step rh$N 200 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29710 + N)) bench.py --gpus $N --steps 10 --warmup 2 --engine replicated-halo
done
