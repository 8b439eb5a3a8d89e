#!/bin/bash
# D-GADMM host path: refresh launched before the chain draw; host stamps, bench, tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6dg}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "dgadmm or dynamic or pad_image" > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/dgadmm_host_stamps.py 10 60 refresh > $O/stamps.log 2>&1 || exit $?
for i in 1 2 3; do timeout -k 10 200 python -u bench.py --config dgadmm --steps 20 --warmup 3 > $O/dg_$i.log 2>&1 || exit $?; done
timeout -k 10 200 python -u -m gadmm_amd LinearRegression_gadmm_vs_admm --quick --no-plot --out $O/e7 > $O/e7.log 2>&1 || exit $?
