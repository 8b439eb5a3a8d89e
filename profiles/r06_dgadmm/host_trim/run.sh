#!/bin/bash
# PersistArgs template + traces() trim: the GPU suite, host stamps, D-GADMM and E1 benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-hosttrim}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/suite.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/dgadmm_host_stamps.py 10 60 refresh > $O/stamps.log 2>&1 || exit $?
for i in 1 2 3; do timeout -k 10 200 python -u bench.py --config dgadmm --steps 20 --warmup 3 > $O/dg_$i.log 2>&1 || exit $?; done
for i in 1 2; do timeout -k 10 200 python -u bench.py > $O/e1_$i.log 2>&1 || exit $?; done
