#!/bin/bash
# round 6 final tree: the whole GPU suite, smoke, every bench config at its reference count, and a
# rocprofv3 kernel summary of the headline step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6f}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/suite.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 120 python bench.py > $O/e1.log 2>&1 || exit $?
for c in dgadmm logistic logistic_exact star real10m; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 > $O/$c.log 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o e1 -- python3 bench.py --steps 50 --warmup 5 > $O/prof.log 2>&1 || exit $?
