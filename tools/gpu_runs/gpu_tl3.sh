set -o pipefail
O=gpurun_out/tl3
mkdir -p $O
timeout -k 10 200 python3 -u tools/blocked_timeline.py 300 > $O/tl.json 2> $O/tl.err && \
GADMM_BLK_DBG=32 timeout -k 10 200 python3 -u tools/blocked_timeline.py 300 > $O/tl_w8.json 2> $O/tl_w8.err
