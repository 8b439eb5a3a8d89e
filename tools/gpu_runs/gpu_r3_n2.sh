set -o pipefail
O=gpurun_out/r3_n2
mkdir -p $O
. tools/gpu_runs/gpu_step.sh
step pingpong 60 build/pingpong
step newton_sweep 300 python3 -u tools/newton_persist_tl.py --sweep
step newton_tests 200 python3 -u -m pytest tests/test_gpu.py -v -k "newton" --timeout 120 --timeout-method thread
step bench_lx 200 python3 -u bench.py --config logistic_exact --steps 10 --warmup 2
step dg_x2 120 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
GADMM_XCD=1 step dg_x1 120 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
GADMM_XCD=0 step dg_x0 120 python3 -u bench.py --config dgadmm --steps 20 --warmup 3
step real10m_st8 400 python3 -u bench.py --config real10m --steps 1 --warmup 1
GADMM_GRAM_ST=0 step real10m_st0 400 python3 -u bench.py --config real10m --steps 1 --warmup 1
