#!/bin/bash
# round 6: the whole GPU suite, smoke, headline bench, and the 8-rank share rehearsal of the driver's
# SCALE run (tournament without RCCL)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6b2}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/suite.log 2>&1
rc=$?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 120 python bench.py > $O/e1.log 2>&1 || exit $?
GADMM_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29598 bench.py --gpus 8 --steps 20 --warmup 3 > $O/e1_share8.log 2>&1 || exit $?
exit $rc
