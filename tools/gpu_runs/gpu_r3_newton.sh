set -o pipefail
O=gpurun_out/r3_newton
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -v -k "newton" --timeout 120 --timeout-method thread > $O/t.log 2>&1
echo "t rc=$?" >> $O/rc.txt
timeout -k 10 200 python3 -u bench.py --config logistic_exact --steps 5 --warmup 2 > $O/bench_le.json 2> $O/bench_le.err
echo "b rc=$?" >> $O/rc.txt
GADMM_NEWTON_PERSISTENT=0 timeout -k 10 200 python3 -u bench.py --config logistic_exact --steps 5 --warmup 2 > $O/bench_le_graph.json 2> $O/bench_le_graph.err
echo "bg rc=$?" >> $O/rc.txt
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_multirank.py -v -k "first_order_chain" --timeout 250 --timeout-method thread > $O/fomr.log 2>&1
echo "fomr rc=$?" >> $O/rc.txt
