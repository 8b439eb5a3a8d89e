set -o pipefail
O=gpurun_out/dgtrim
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_multirank.py -x -q --timeout 170 --timeout-method thread -k "dgadmm or dynamic or resume or elastic or trace or clock" > $O/tests.log 2>&1 && \
timeout -k 10 120 python3 -u tools/dgadmm_stage_times.py 10 > $O/stages.log 2>&1 && \
timeout -k 10 120 python3 -u tools/dgadmm_stage_times.py 1 >> $O/stages.log 2>&1 && \
timeout -k 10 150 python3 -u bench.py --config dgadmm > $O/bench_dg.json 2> $O/bench_dg.err && \
timeout -k 10 150 python3 -u bench.py > $O/bench_e1.json 2> $O/bench_e1.err
