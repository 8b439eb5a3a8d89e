#!/bin/bash
# D-GADMM re-chain image loads: A (ab_libs/libA.so: every image at the re-chain) vs B (in-tree:
# the variant under test), alternating, same box; D-GADMM / dynamic tests on B first
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-dgab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "dgadmm or dynamic or pad_image" > $O/tests.log 2>&1 || exit $?
for i in 1 2 3; do
  GADMM_NATIVE_LIB=$PWD/ab_libs/libA.so timeout -k 10 200 python -u bench.py --config dgadmm --steps 20 --warmup 3 > $O/A_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --config dgadmm --steps 20 --warmup 3 > $O/B_$i.log 2>&1 || exit $?
done
