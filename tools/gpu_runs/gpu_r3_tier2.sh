# Round 3: the full GPU tier (every -m gpu test, NaN-poisoned LDS before each) and smoke().
set -o pipefail
O=gpurun_out/r3_tier2
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step tier 1000 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 120 python3 -u -c "import __graft_entry__ as g; g.smoke()"
