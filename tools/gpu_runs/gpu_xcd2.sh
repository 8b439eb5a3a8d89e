set -o pipefail
O=gpurun_out/xcd2
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests/test_gpu.py -k "xcd or star or first_order or logistic_persistent or baselines" > $O/tests.log 2>&1 && \
for c in logistic star dgadmm; do
  GADMM_XCD=0 timeout -k 10 300 python3 -u bench.py --config $c > $O/bench_${c}_x0.json 2> $O/bench_${c}_x0.err && \
  timeout -k 10 300 python3 -u bench.py --config $c > $O/bench_${c}_x2.json 2> $O/bench_${c}_x2.err || exit 1
done
