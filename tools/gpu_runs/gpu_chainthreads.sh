set -o pipefail
O=gpurun_out/chainthr
mkdir -p $O
for t in 1 2 4; do
  GADMM_CHAIN_THREADS=$t timeout -k 10 120 python3 -u tools/dgadmm_stage_times.py 1 > $O/c1_t$t.log 2>&1 || exit 1
  GADMM_CHAIN_THREADS=$t timeout -k 10 120 python3 -u tools/dgadmm_stage_times.py 10 > $O/c10_t$t.log 2>&1 || exit 1
done
