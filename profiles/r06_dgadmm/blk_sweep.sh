#!/bin/bash
# D-GADMM bench over the blocked kernel's segment length L and block depth k (GADMM_BLOCK_L / _K):
# a re-chain reloads the inverse image of every solving position of a workgroup (owned + halo), so
# longer segments reload fewer redundant images per owned position
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-blksweep}; mkdir -p $O
for i in 1 2; do
  for kl in "2 1" "2 2" "2 3" "2 4" "1 1" "1 2" "1 4" "1 8"; do
    set -- $kl
    GADMM_BLOCK_K=$1 GADMM_BLOCK_L=$2 timeout -k 10 120 python -u bench.py --config dgadmm --steps 20 --warmup 3 > $O/k$1_L$2_$i.log 2>&1 || exit $?
  done
done
