#!/bin/bash
# round 6: the reference entry points across ranks on the node engines: one GPU vs
# 2 / 4 ranks sharing the GPU (GADMM_SHARE_GPU=1), every run's engine / transport in its summary line;
# E1 also to the headline's 1e-8 gap (1373 iterations at rho = 3) for the per-solve time vs bench.py
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6entries}; mkdir -p $O
E="python -u -m gadmm_amd"
TR="python -u -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
Q="--quick --set gadmm_iters=1000 --no-plot"
H="--no-baselines --no-plot --tol 1e-8 --set gadmm_iters=2000 rhos=3,3"  # the second solve is warm
timeout -k 10 300 $E LinearRegression_Synthetic $Q --out $O/e1_1gpu > $O/e1_1gpu.log 2>&1 || exit $?
timeout -k 10 300 $E LinearRegression_Synthetic $H --out $O/e1h_1gpu > $O/e1h_1gpu.log 2>&1 || exit $?
for n in 2 4; do
  GADMM_SHARE_GPU=1 timeout -k 10 300 $TR --nproc-per-node $n --master-port 2961$n -m gadmm_amd \
    LinearRegression_Synthetic $Q --out $O/e1_share$n > $O/e1_share$n.log 2>&1 || exit $?
  GADMM_SHARE_GPU=1 timeout -k 10 300 $TR --nproc-per-node $n --master-port 2962$n -m gadmm_amd \
    LinearRegression_Synthetic $H --out $O/e1h_share$n > $O/e1h_share$n.log 2>&1 || exit $?
done
timeout -k 10 300 $E LinearRegression_gadmm_vs_admm --quick --no-plot --out $O/e7_1gpu > $O/e7_1gpu.log 2>&1 || exit $?
GADMM_SHARE_GPU=1 timeout -k 10 300 $TR --nproc-per-node 2 --master-port 29632 -m gadmm_amd \
  LinearRegression_gadmm_vs_admm --quick --no-plot --out $O/e7_share2 > $O/e7_share2.log 2>&1 || exit $?
timeout -k 10 300 $E LogisticRegression_Synthetic --quick --no-plot --out $O/e3_1gpu > $O/e3_1gpu.log 2>&1 || exit $?
GADMM_SHARE_GPU=1 timeout -k 10 300 $TR --nproc-per-node 2 --master-port 29642 -m gadmm_amd \
  LogisticRegression_Synthetic --quick --no-plot --out $O/e3_share2 > $O/e3_share2.log 2>&1 || exit $?
timeout -k 10 300 $E Dynamic_LinearRegression_Synthetic --quick --no-plot --out $O/e5_1gpu > $O/e5_1gpu.log 2>&1 || exit $?
GADMM_SHARE_GPU=1 timeout -k 10 300 $TR --nproc-per-node 2 --master-port 29652 -m gadmm_amd \
  Dynamic_LinearRegression_Synthetic --quick --no-plot --out $O/e5_share2 > $O/e5_share2.log 2>&1 || exit $?
GADMM_SHARE_GPU=1 timeout -k 10 300 $TR --nproc-per-node 2 --master-port 29662 -m gadmm_amd \
  LinearRegression_Real --quick --no-plot --out $O/e2_share2 > $O/e2_share2.log 2>&1 || exit $?
timeout -k 10 300 $E LogisticRegression_Real --quick --no-plot --out $O/e4_1gpu > $O/e4_1gpu.log 2>&1 || exit $?
GADMM_SHARE_GPU=1 timeout -k 10 300 $TR --nproc-per-node 2 --master-port 29672 -m gadmm_amd \
  LogisticRegression_Real --quick --no-plot --out $O/e4_share2 > $O/e4_share2.log 2>&1 || exit $?
GADMM_SHARE_GPU=1 timeout -k 10 300 $TR --nproc-per-node 2 --master-port 29682 -m gadmm_amd \
  Dynamic_LinearRegression_Real --quick --no-plot --out $O/e6_share2 > $O/e6_share2.log 2>&1 || exit $?
for n in 2 4; do
  GADMM_SHARE_GPU=1 timeout -k 10 300 $TR --nproc-per-node $n --master-port 2969$n bench.py --gpus $n --steps 20 \
    --warmup 3 > $O/bench_share$n.log 2>&1 || exit $?
done
