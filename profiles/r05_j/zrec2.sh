#!/bin/bash
# round 5, session j5: shorter margins chain (flag released behind the GEMV's reads, the z update's
# K-free part formed during the GEMV, one Newton step on v_rcp_f64) -- tests, benches, timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5j5}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu.py \
  -k "logistic_persistent_kernel or native_resume_logistic" > $O/t.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python bench.py --config logistic --steps 20 --warmup 3 > $O/lg_$i.log 2>&1 || exit $?
  GADMM_LOGISTIC_ZREC=0 timeout -k 10 200 python bench.py --config logistic --steps 20 --warmup 3 > $O/lg_onewave_$i.log 2>&1 || exit $?
done

