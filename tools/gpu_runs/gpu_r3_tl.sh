set -o pipefail
O=gpurun_out/r3_tl
mkdir -p $O
timeout -k 10 300 python3 -u tools/newton_persist_tl.py --sweep > $O/newton_sweep.log 2>&1
echo "nw rc=$?" >> $O/rc.txt
timeout -k 10 200 python3 -u tools/dgadmm_stage_times.py 10 > $O/dg_stage10.log 2>&1
echo "dg rc=$?" >> $O/rc.txt
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_multirank.py -v -k "recovers_after" --timeout 250 --timeout-method thread > $O/ipc_recover.log 2>&1
echo "ipc rc=$?" >> $O/rc.txt
