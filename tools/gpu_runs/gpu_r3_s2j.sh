# Round 3, session 2: streamed D-GADMM epochs (blocked dynamic mode, GADMM_DYN_STREAM=1) + host trims.
set -o pipefail
O=gpurun_out/r3_s2j
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
GADMM_DYN_STREAM=1 step tests 400 python3 -u -m pytest tests/test_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "dgadmm or dynamic or blocked"
GADMM_DYN_STREAM=1 step stamps 150 python3 -u tools/dgadmm_host_stamps.py 10 40
GADMM_DYN_STREAM=0 step stamps_nostream 150 python3 -u tools/dgadmm_host_stamps.py 10 40
GADMM_DYN_STREAM=1 step dg 150 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
GADMM_DYN_STREAM=0 step dg_nostream 150 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
GADMM_DYN_STREAM=1 step dg_b 150 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
GADMM_DYN_STREAM=1 step pace 150 python3 -u tools/dgadmm_pace.py 10 20
