#!/bin/bash
# round 4: the small-d set-up (Gram + inverses) in one native call per solve -- GPU tests, A/B benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4ae; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/t.log 2>&1 || exit $?
for r in 1 2; do
for cfg in e1 dgadmm star; do
timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 > $O/${cfg}_new_$r.log 2>&1 || exit $?
GADMM_NATIVE_LIB=$PWD/gadmm_amd/_native/ab/lib_head.so timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 > $O/${cfg}_old_$r.log 2>&1 || exit $?
done
done
