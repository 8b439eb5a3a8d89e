# A/B of the register-row SPD inverse against the LDS kernel (GADMM_INV_REG=0),
# the bit-identity check against the general kernel, and the inverse GPU tests. Run on the GPU box.
set -o pipefail
for nw in 0 8; do
  GADMM_INV_REG=$nw timeout -k 10 100 python tools/inv_time.py || exit 1
done
timeout -k 10 100 python tools/inv_ab.py || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu.py -k "inverse" 2>&1 | tail -2
