# Round 3: full GPU tier with LDS poisoning before every test, then the headline bench.
set -o pipefail
O=gpurun_out/r3_tier
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/ -m gpu -v --timeout 170 --timeout-method thread > $O/gpu_tier.log 2>&1
rc=$?
echo "tier rc=$rc" > $O/rc.txt
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 150 python3 -u bench.py --steps 20 --warmup 3 > $O/bench1.json 2> $O/bench1.err
