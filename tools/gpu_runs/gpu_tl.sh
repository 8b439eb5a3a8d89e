set -o pipefail
O=gpurun_out/tl
mkdir -p $O
for w in 0 1 2 3 4 5; do
  GADMM_BLK_DBG=$((w * 16)) timeout -k 10 200 python3 -u tools/blocked_timeline.py 300 > $O/blk_w$w.json 2> $O/blk_w$w.err || exit 1
done
