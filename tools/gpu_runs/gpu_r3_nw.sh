set -o pipefail
O=gpurun_out/r3_nw2
mkdir -p $O
timeout -k 10 500 python3 -u tools/newton_persist_tl.py --sweep > $O/newton_sweep.log 2>&1
echo "nw rc=$?" >> $O/rc.txt
timeout -k 10 100 python3 -u tools/newton_persist_tl.py --chord 0.1 --bg 1 > $O/newton_detail.log 2>&1
echo "nd rc=$?" >> $O/rc.txt
timeout -k 10 200 python3 -u -m pytest tests/test_gpu.py -v -k "newton" --timeout 120 --timeout-method thread > $O/t.log 2>&1
echo "t rc=$?" >> $O/rc.txt
timeout -k 10 120 python3 -u tools/dgadmm_pyprof.py > $O/dg_pyprof.log 2>&1
echo "dg rc=$?" >> $O/rc.txt
