#!/bin/bash
# round 5 final: the whole GPU suite + smoke + headline, every bench config with its pinned count,
# real10m, and the multi-rank headline rehearsals (ranks sharing the one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5final}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/suite.log 2>&1
rc=$?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 120 python bench.py > $O/e1.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --steps 50 --warmup 5 > $O/e1_50.log 2>&1 || exit $?
for c in dgadmm star logistic logistic_exact; do
  timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 > $O/$c.log 2>&1 || exit $?
done
timeout -k 10 400 python -u bench.py --config real10m --steps 2 --warmup 1 > $O/real10m.log 2>&1 || exit $?
for n in 2 4; do
  GADMM_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2959$n bench.py --gpus $n --steps 20 --warmup 3 > $O/e1_share$n.log 2>&1 || exit $?
done
exit $rc
