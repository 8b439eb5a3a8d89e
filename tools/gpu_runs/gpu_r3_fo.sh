# Round 3: multi-rank first-order engine + single-GPU FO regression + data-local 8x8 fix
set -o pipefail
O=gpurun_out/r3_fo
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -v -k "first_order" --timeout 200 --timeout-method thread > $O/fo1.log 2>&1
echo "fo1 rc=$?" >> $O/rc.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multirank.py -v -k "first_order or 8-8" --timeout 500 --timeout-method thread > $O/fomr.log 2>&1
echo "fomr rc=$?" >> $O/rc.txt
