set -o pipefail
O=gpurun_out/ab
mkdir -p $O
for r in 1 2; do
  GADMM_NATIVE_LIB=$PWD/build/ab/libold.so timeout -k 10 240 python3 -u tools/xcd_probe.py 1 8 > $O/old1_$r.json 2>> $O/err.log && \
  timeout -k 10 240 python3 -u tools/xcd_probe.py 1 8 > $O/new1_$r.json 2>> $O/err.log && \
  GADMM_NATIVE_LIB=$PWD/build/ab/libold.so timeout -k 10 240 python3 -u tools/xcd_probe.py 10 8 > $O/old10_$r.json 2>> $O/err.log && \
  timeout -k 10 240 python3 -u tools/xcd_probe.py 10 8 > $O/new10_$r.json 2>> $O/err.log || exit 1
done
