set -o pipefail
O=gpurun_out/dynblk2
mkdir -p $O
for c in 10 1; do
  timeout -k 10 150 python3 -u bench.py --config dgadmm --coherence $c > $O/pw_c$c.json 2> $O/pw_c$c.err || exit 1
  GADMM_BLOCKED_DYN=1 timeout -k 10 150 python3 -u bench.py --config dgadmm --coherence $c > $O/blk_c$c.json 2> $O/blk_c$c.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
GADMM_BLOCKED_DYN=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o blk -- python3 $GRAFT_REPO_ROOT/bench.py --config dgadmm --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
