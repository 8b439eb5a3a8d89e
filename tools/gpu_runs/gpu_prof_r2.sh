# rocprofv3 kernel statistics of every bench config at the round-2 head (one call, one box)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in e1 dgadmm star logistic logistic_exact; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$c -o $c -- \
    python3 $R/bench.py --config $c --steps 20 --warmup 3 > $O/$c.json 2> $O/$c.err || exit 1
done
echo done
