# the reference experiments end to end on the final tree (1x MI355X); run outputs stay on the box
# (JSONL traces of the 60,000-iteration baselines), logs and wall times come back
set -o pipefail
O=gpurun_out/entries
mkdir -p $O
for e in LinearRegression_Synthetic LogisticRegression_Synthetic Dynamic_LinearRegression_Synthetic LinearRegression_gadmm_vs_admm; do
  t0=$(date +%s%N)
  timeout -k 10 240 python3 -u -m gadmm_amd $e --no-plot --out /tmp/entries/$e > $O/$e.log 2>&1 || exit 1
  t1=$(date +%s%N)
  echo "$e: $(( (t1 - t0) / 1000000 )) ms wall incl. Python start-up" >> $O/walls.txt
done
