# A/B of the quad-GEMV transpose-reduce (permlane swaps, default) vs the LDS version
# (build/ab/libgadmm_native_ldsred.so), in one GPU call: E1 headline and the logistic inner-GD config.
set -o pipefail
mkdir -p gpurun_out
B=build/ab/libgadmm_native_ldsred.so
for rep in 1 2; do
  timeout -k 10 120 python bench.py --steps 50 > gpurun_out/ab_e1_perm_$rep.log 2>&1 || exit 1
  GADMM_NATIVE_LIB=$B timeout -k 10 120 python bench.py --steps 50 > gpurun_out/ab_e1_lds_$rep.log 2>&1 || exit 1
  timeout -k 10 120 python bench.py --config logistic --steps 10 --warmup 2 > gpurun_out/ab_log_perm_$rep.log 2>&1 || exit 1
  GADMM_NATIVE_LIB=$B timeout -k 10 120 python bench.py --config logistic --steps 10 --warmup 2 > gpurun_out/ab_log_lds_$rep.log 2>&1 || exit 1
done
for f in gpurun_out/ab_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"iterations_match_reference": [a-z]*' $f)"; done
