#!/bin/bash
# round 4: rocprofv3 kernel statistics of the headline, real10m (packed-inverse iterations, new Gram),
# D-GADMM and star, one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/e1 -o e1 -- python3 bench.py --steps 20 --warmup 3 > $O/e1.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/real -o real -- python3 bench.py --config real10m --steps 1 --warmup 0 > $O/real.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/dg -o dg -- python3 bench.py --config dgadmm --steps 10 --warmup 2 > $O/dg.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/star -o star -- python3 bench.py --config star --steps 10 --warmup 2 > $O/star.log 2>&1
