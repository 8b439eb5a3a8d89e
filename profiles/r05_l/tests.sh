#!/bin/bash
# the Newton / logistic GPU tests (single GPU and the multi-rank rehearsals) with the pipeline default,
# then the bench and the in-kernel timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5lt}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_multirank.py -v --timeout 200 --timeout-method thread -k "newton or logistic" > $O/tests.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --config logistic_exact --steps 20 --warmup 3 > $O/rec.log 2>&1 || exit $?
timeout -k 10 120 python tools/newton_persist_tl.py --chord 0.3 > $O/tl_rec.log 2>&1 || exit $?
