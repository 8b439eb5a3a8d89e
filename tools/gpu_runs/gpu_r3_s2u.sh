# Round 3, session 2: D-GADMM after the host trims (set_path keys, re-chain count): tests + bench + stamps.
set -o pipefail
O=gpurun_out/r3_s2u
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step tests 400 python3 -u -m pytest tests/test_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "dgadmm or dynamic or elastic or resume"
step dg 150 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
step stamps 150 python3 -u tools/dgadmm_host_stamps.py 10 40
step dg_b 150 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
