#!/bin/bash
# round 4: D-GADMM inverse image rebuilt in place (one native launch) -- tests, host stamps, A/B bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4ad; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu.py -k "quad_pad or dgadmm or dynamic or resid_sq" > $O/t.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/dgadmm_host_stamps.py 10 40 refresh > $O/stamps.log 2>&1 || exit $?
for r in 1 2; do
timeout -k 10 200 python bench.py --config dgadmm --steps 20 --warmup 3 > $O/dg_new_$r.log 2>&1 || exit $?
GADMM_NATIVE_LIB=$PWD/gadmm_amd/_native/ab/lib_head.so timeout -k 10 200 python bench.py --config dgadmm --steps 20 --warmup 3 > $O/dg_old_$r.log 2>&1 || exit $?
done
