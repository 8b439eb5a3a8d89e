set -o pipefail
O=gpurun_out/lsweep
mkdir -p $O
for r in 1 2; do
for L in 1 2 3 4; do
  GADMM_BLOCK_L=$L timeout -k 10 200 python3 -u bench.py --steps 30 > $O/L${L}_$r.json 2> $O/L${L}_$r.err || exit 1
done
GADMM_BLOCK_K=1 GADMM_BLOCK_L=2 timeout -k 10 200 python3 -u bench.py --steps 30 > $O/k1L2_$r.json 2> $O/k1L2_$r.err || exit 1
GADMM_BLOCK_K=1 GADMM_BLOCK_L=4 timeout -k 10 200 python3 -u bench.py --steps 30 > $O/k1L4_$r.json 2> $O/k1L4_$r.err || exit 1
done
timeout -k 10 200 python3 -u bench.py --steps 30 --workers 8 > $O/w8.json 2> $O/w8.err
