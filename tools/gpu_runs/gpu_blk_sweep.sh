set -o pipefail
O=gpurun_out/blk_sweep
mkdir -p $O
run() { # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --steps 30 > $O/$name.json 2> $O/$name.err || return 1
}
run default && run perworker GADMM_BLOCKED=0 && run k1 GADMM_BLOCK_K=1 && run k1L6 GADMM_BLOCK_K=1 GADMM_BLOCK_L=6 && \
run k1L4 GADMM_BLOCK_K=1 GADMM_BLOCK_L=4 && run k2L3 GADMM_BLOCK_K=2 GADMM_BLOCK_L=3 && run k2L2 GADMM_BLOCK_K=2 GADMM_BLOCK_L=2 && \
run pw2k3 GADMM_BLOCK_PW=2 && run pw2k2 GADMM_BLOCK_PW=2 GADMM_BLOCK_K=2 && run pw2k1 GADMM_BLOCK_PW=2 GADMM_BLOCK_K=1 && run default2
