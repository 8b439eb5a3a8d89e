# Round 3, session 2: full GPU tier + every bench config after the D-GADMM re-chain, halo and
# read-back changes.
set -o pipefail
O=gpurun_out/r3_s2h
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step tier 1000 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 120 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step e1 120 python3 -u bench.py --steps 20 --warmup 3
for c in logistic logistic_exact dgadmm star; do
  step $c 150 python3 -u bench.py --config $c --steps 10 --warmup 2
done
step dg1 150 python3 -u bench.py --config dgadmm --coherence 1 --steps 10 --warmup 2
step w8 120 python3 -u bench.py --workers 8 --steps 20 --warmup 3
