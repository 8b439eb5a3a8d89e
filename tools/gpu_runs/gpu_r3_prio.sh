# Round 3: data-local boundary waves at raised issue priority (GADMM_DL_DBG=256) vs default, 2 / 4 ranks.
set -o pipefail
O=gpurun_out/r3_prio
mkdir -p $O
export GADMM_BENCH_SHARE_GPU=1
run() {
  local name=$1 n=$2; shift 2
  env "$@" timeout -k 10 200 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29800 + RANDOM % 100)) bench.py --gpus $n --steps 10 --warmup 2 > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/rc.txt
  case $rc in 124|134|137|139) exit $rc ;; esac
}
for r in 1 2; do
  run base2_$r 2
  run prio2_$r 2 GADMM_DL_DBG=256
done
run base4 4
run prio4 4 GADMM_DL_DBG=256
