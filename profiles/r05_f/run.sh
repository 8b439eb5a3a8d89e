#!/bin/bash
# round 5, session f: the whole GPU suite + smoke + headline, after the round's changes so far
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/suite.log 2>&1
rc=$?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 120 python bench.py > $O/e1.log 2>&1 || exit $?
exit $rc
