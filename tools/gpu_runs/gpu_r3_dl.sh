# Round 3: data-local blocked multi-GPU kernel, rehearsed with ranks sharing the one GPU; plus the
# A/B evidence for the Newton NaN fix (pre-fix library under LDS poison must fail).
set -o pipefail
O=gpurun_out/r3_dl
mkdir -p $O
export GADMM_BENCH_SHARE_GPU=1
for w in 2 4 8; do
  timeout -k 10 200 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
    --master-port $((29600 + w)) bench.py --gpus $w --steps 10 --warmup 2 > $O/share$w.json 2> $O/share$w.err || exit $?
done
timeout -k 10 200 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 2 --engine per-worker > $O/share2_pw.json 2> $O/share2_pw.err || exit $?
unset GADMM_BENCH_SHARE_GPU
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_multirank.py -v -k "data_local or stalled" --timeout 170 --timeout-method thread > $O/mr.log 2>&1
echo "mr rc=$?" >> $O/rc.txt
GADMM_NATIVE_LIB=$PWD/gadmm_amd/_native_ab/libgadmm_oldnewton.so timeout -k 10 120 python3 -u -m pytest tests/test_gpu.py -v -k "newton_after_lds_poison" --timeout 100 --timeout-method thread > $O/oldnewton.log 2>&1
echo "oldnewton rc=$?" >> $O/rc.txt
