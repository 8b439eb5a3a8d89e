# Round 3: Gram (K1) split-K round efficiency A/B at the real10m shape, plus the numerics test.
set -o pipefail
O=gpurun_out/r3_gram
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step test 200 python3 -u -m pytest tests/test_gpu.py -v -k "gram" --timeout 150 --timeout-method thread
GADMM_GRAM_EFF=0.9 step eff90 300 python3 -u tools/gram_bench.py 2 625000 10000
step eff97 300 python3 -u tools/gram_bench.py 2 625000 10000
GADMM_GRAM_EFF=0.9 GADMM_GRAM_ST=0 step eff90_st0 300 python3 -u tools/gram_bench.py 2 625000 10000
GADMM_GRAM_ST=0 step eff97_st0 300 python3 -u tools/gram_bench.py 2 625000 10000
