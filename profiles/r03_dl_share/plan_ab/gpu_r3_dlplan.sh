# Round 3: data-local plan A/B at 2 / 4 ranks sharing the GPU -- one workgroup per segment (default)
# vs the one-GPU blocked plan inside the segment (GADMM_DL_PLAN=blocked, L from GADMM_BLOCK_L).
set -o pipefail
O=gpurun_out/r3_dlplan
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
export GADMM_BENCH_SHARE_GPU=1
run() {  # name nranks [env...]
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 200 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29800 + RANDOM % 100)) bench.py --gpus $n --steps 10 --warmup 2 > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/rc.txt
  case $rc in 124|134|137|139) exit $rc ;; esac
}
run one2 2
run blk2_L1 2 GADMM_DL_PLAN=blocked GADMM_BLOCK_L=1
run blk2_L2 2 GADMM_DL_PLAN=blocked GADMM_BLOCK_L=2
run blk2_L4 2 GADMM_DL_PLAN=blocked GADMM_BLOCK_L=4
run one4 4
run blk4_L1 4 GADMM_DL_PLAN=blocked GADMM_BLOCK_L=1
run one2b 2
