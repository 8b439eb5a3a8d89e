# Round 3, session 2: rocprofv3 kernel statistics of D-GADMM (blocked dynamic mode, coherence 10 and 1)
# and of the 4-rank halo rehearsal (ranks sharing the GPU).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3_s2r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dg10 -o k -- python3 $GRAFT_REPO_ROOT/bench.py --config dgadmm --steps 10 --warmup 2 > $O/dg10.log 2>&1 || exit $?
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dg1 -o k -- python3 $GRAFT_REPO_ROOT/bench.py --config dgadmm --coherence 1 --steps 10 --warmup 2 > $O/dg1.log 2>&1 || exit $?
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/e1 -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 > $O/e1.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/summarize_prof.py $O/dg10 $O/sum_dg10 && python3 tools/summarize_prof.py $O/dg1 $O/sum_dg1 && python3 tools/summarize_prof.py $O/e1 $O/sum_e1
