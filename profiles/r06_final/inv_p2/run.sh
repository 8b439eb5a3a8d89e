#!/bin/bash
# two-pivot inverse kernel: bit-identity and numerics tests, the inverse micro-benchmark, the
# inverse-dependent GPU tests, then E1 / D-GADMM benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-invp2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "spd_inverse or inverse or smoke or dgadmm or blocked or persistent_state" > $O/tests.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/inverse_bench.py 300 > $O/inv.log 2>&1 || exit $?
for i in 1 2; do
  GADMM_INV_P2=0 timeout -k 10 120 python -u bench.py > $O/e1_p1_$i.log 2>&1 || exit $?
  timeout -k 10 120 python -u bench.py > $O/e1_p2_$i.log 2>&1 || exit $?
done
