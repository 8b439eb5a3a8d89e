# Round 3, session 2: blocked D-GADMM objective waves indexed by worker (no Gram reload per re-chain).
set -o pipefail
O=gpurun_out/r3_s2o
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step tests 400 python3 -u -m pytest tests/test_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "dgadmm or dynamic or blocked"
step pace10 150 python3 -u tools/dgadmm_pace.py 10 20
GADMM_BLOCKED_DYN=1 step pace1 150 python3 -u tools/dgadmm_pace.py 1 10
GADMM_BLOCKED_DYN=1 step pace3 150 python3 -u tools/dgadmm_pace.py 3 10
step dg 150 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
GADMM_BLOCKED_DYN=1 step dg1_blk 150 python3 -u bench.py --config dgadmm --coherence 1 --steps 10 --warmup 2
step dg1 150 python3 -u bench.py --config dgadmm --coherence 1 --steps 10 --warmup 2
GADMM_BLOCKED_DYN=1 step dg3_blk 150 python3 -u bench.py --config dgadmm --coherence 3 --steps 10 --warmup 2
GADMM_BLOCKED_DYN=0 step dg3_pw 150 python3 -u bench.py --config dgadmm --coherence 3 --steps 10 --warmup 2
