set -o pipefail
O=gpurun_out/tl2
mkdir -p $O
timeout -k 10 300 python3 -u tools/star_sweep.py > $O/star.log 2>&1 && \
timeout -k 10 200 python3 -u tools/dyn_timeline.py 1 > $O/dyn1.json 2> $O/dyn1.err && \
timeout -k 10 200 python3 -u tools/dyn_timeline.py 10 > $O/dyn10.json 2> $O/dyn10.err
