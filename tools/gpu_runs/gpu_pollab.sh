# A/B (same box): hand-off polls back to back (GADMM_POLL_SLEEP=0 build) vs the default pause
set -o pipefail
O=gpurun_out/pollab
mkdir -p $O
B=$PWD/build/ab/lib_sleep0.so
for pass in 1 2; do
  timeout -k 10 120 python3 -u bench.py > $O/e1_def_$pass.json 2>/dev/null || exit 1
  GADMM_NATIVE_LIB=$B timeout -k 10 120 python3 -u bench.py > $O/e1_s0_$pass.json 2>/dev/null || exit 1
  timeout -k 10 120 python3 -u bench.py --config dgadmm > $O/dg_def_$pass.json 2>/dev/null || exit 1
  GADMM_NATIVE_LIB=$B timeout -k 10 120 python3 -u bench.py --config dgadmm > $O/dg_s0_$pass.json 2>/dev/null || exit 1
  GADMM_BLOCKED=0 timeout -k 10 120 python3 -u bench.py > $O/pw_def_$pass.json 2>/dev/null || exit 1
  GADMM_BLOCKED=0 GADMM_NATIVE_LIB=$B timeout -k 10 120 python3 -u bench.py > $O/pw_s0_$pass.json 2>/dev/null || exit 1
  timeout -k 10 120 python3 -u bench.py --config star > $O/st_def_$pass.json 2>/dev/null || exit 1
  GADMM_NATIVE_LIB=$B timeout -k 10 120 python3 -u bench.py --config star > $O/st_s0_$pass.json 2>/dev/null || exit 1
done
