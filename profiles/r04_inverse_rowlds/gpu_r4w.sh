#!/bin/bash
# round 4: small inverse with the pivot row through LDS -- A/B (timing, bits) and the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4w; mkdir -p $O
timeout -k 10 120 python -u tools/inv_small_ab.py /tmp/new.pt > $O/inv_new.log 2>&1 || exit $?
GADMM_NATIVE_LIB=$PWD/gadmm_amd/_native/ab/lib_before_inv.so timeout -k 10 120 python -u tools/inv_small_ab.py /tmp/old.pt > $O/inv_old.log 2>&1 || exit $?
python -c "import torch; a=torch.load('/tmp/new.pt'); b=torch.load('/tmp/old.pt'); print('bit-identical:', torch.equal(a,b))" > $O/bits.log 2>&1 || exit $?
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py -k "inverse or spd" > $O/t.log 2>&1 || exit $?
for r in 1 2; do
timeout -k 10 120 python bench.py --steps 20 --warmup 3 > $O/e1_new_$r.log 2>&1 || exit $?
GADMM_NATIVE_LIB=$PWD/gadmm_amd/_native/ab/lib_before_inv.so timeout -k 10 120 python bench.py --steps 20 --warmup 3 > $O/e1_old_$r.log 2>&1 || exit $?
done
