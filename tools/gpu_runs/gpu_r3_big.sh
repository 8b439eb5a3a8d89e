set -o pipefail
O=gpurun_out/r3_big
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -v -k "star_big or large_d or star" --timeout 200 --timeout-method thread > $O/t.log 2>&1
echo "t rc=$?" >> $O/rc.txt
timeout -k 10 400 python3 -u bench.py --config real10m --steps 1 --warmup 1 > $O/real10m.json 2> $O/real10m.err
echo "b rc=$?" >> $O/rc.txt
