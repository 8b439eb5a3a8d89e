#!/bin/bash
# round 4, final: the whole GPU suite, smoke, and every bench config on one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4x; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 120 python bench.py > $O/e1_default.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --steps 20 --warmup 3 > $O/e1.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config dgadmm --steps 10 --warmup 2 > $O/dg.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config star --steps 10 --warmup 2 > $O/star.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config logistic --steps 10 --warmup 2 > $O/logistic.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --config logistic_exact --steps 10 --warmup 2 > $O/logistic_exact.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config real10m --steps 1 --warmup 0 > $O/real10m.log 2>&1 || exit $?
exit $rc
