#!/bin/bash
# result read-back by kernel, xchk memset dropped, inverse image built in the refresh: the GPU suite,
# D-GADMM and E1 benches, host stamps, and the kernel + copy trace of the D-GADMM bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6dg5}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/suite.log 2>&1 || exit $?
for i in 1 2 3; do timeout -k 10 200 python -u bench.py --config dgadmm --steps 20 --warmup 3 > $O/dg_$i.log 2>&1 || exit $?; done
for i in 1 2; do timeout -k 10 200 python -u bench.py > $O/e1_$i.log 2>&1 || exit $?; done
timeout -k 10 200 python -u tools/dgadmm_host_stamps.py 10 60 refresh > $O/stamps.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config dgadmm --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/$O/trace_bench.log 2>&1
