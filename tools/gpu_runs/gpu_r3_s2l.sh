# Round 3, session 2: the LDS-DMA Gram kernel (GADMM_GRAM_GLDS=1) vs the register-staged one:
# numerics (fp64 torch), bit-identity digests, and throughput at the real10m shape.
set -o pipefail
O=gpurun_out/r3_s2l
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
GADMM_GRAM_GLDS=1 step test 200 python3 -u -m pytest tests/test_gpu.py -v -k "gram" --timeout 150 --timeout-method thread
step dig0 120 python3 -u tools/gram_digest.py
GADMM_GRAM_GLDS=1 step dig1 120 python3 -u tools/gram_digest.py
step base 300 python3 -u tools/gram_bench.py 2 625000 10000
GADMM_GRAM_GLDS=1 step glds 300 python3 -u tools/gram_bench.py 2 625000 10000
