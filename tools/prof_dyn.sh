# Kernel time of the D-GADMM one-launch solve: blocked dynamic mode vs the per-worker kernel.
set -o pipefail
export TMPDIR=/tmp
for v in 1 0; do
  GADMM_BLOCKED_DYN=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dyn_$v -o run -- python bench.py --config dgadmm --steps 10 --warmup 2 > gpurun_out/prof_dyn_$v.log 2>&1 || exit 1
  echo "blocked_dyn=$v"; head -3 gpurun_out/prof_dyn_$v/run_kernel_stats.csv | cut -c1-140
done
