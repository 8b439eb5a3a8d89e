#!/bin/bash
# round 5, session h-real: real10m (1.25M x 10k f64 per GPU) with the f64-MFMA Gram vs the int8 Ozaki Gram
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5hr; mkdir -p $O
timeout -k 10 400 python -u bench.py --config real10m --steps 2 --warmup 1 > $O/real10m_f64.json 2> $O/real10m_f64.err || exit $?
GADMM_GRAM_OZAKI=1 timeout -k 10 400 python -u bench.py --config real10m --steps 2 --warmup 1 > $O/real10m_oz.json 2> $O/real10m_oz.err || exit $?
