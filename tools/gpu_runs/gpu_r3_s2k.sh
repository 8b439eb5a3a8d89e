# Round 3, session 2: the aborting streamed-epoch case alone, with HIP runtime error logging.
set -o pipefail
O=gpurun_out/r3_s2k
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
AMD_LOG_LEVEL=1 step one 150 python3 -u -m pytest tests/test_gpu.py -m gpu -v --timeout 100 --timeout-method thread -k "test_dgadmm_epoch_chunks_bit_identical and 1-16-1"
