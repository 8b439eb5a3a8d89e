set -o pipefail
O=gpurun_out/dynblk2
mkdir -p $O
timeout -k 10 240 python3 -u tools/xcd_probe.py 10 8 > $O/dyn10_pw.json 2> $O/err.log && \
GADMM_BLOCKED_DYN=1 timeout -k 10 240 python3 -u tools/xcd_probe.py 10 8 > $O/dyn10_blk.json 2>> $O/err.log && \
timeout -k 10 240 python3 -u tools/xcd_probe.py 1 8 > $O/dyn1_pw.json 2>> $O/err.log && \
GADMM_BLOCKED_DYN=1 timeout -k 10 240 python3 -u tools/xcd_probe.py 1 8 > $O/dyn1_blk.json 2>> $O/err.log
