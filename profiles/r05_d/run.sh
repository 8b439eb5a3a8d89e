#!/bin/bash
# round 5, session d: where the D-GADMM host time goes (cProfile + stamps), as the bench runs it
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5d; mkdir -p $O
timeout -k 10 300 python tools/dgadmm_pyprof.py 10 refresh > $O/pyprof.log 2>&1 || exit $?
