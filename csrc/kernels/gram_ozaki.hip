// Augmented Gram (K1) on the INT8 matrix cores: the Ozaki scheme (error-free slicing of the f64
// operands into int8 digits, exact int32 MFMA products, f64 recombination).
//
// gfx950's f64 MFMA peaks at 78.6 TF/s; its int8 MFMA (v_mfma_i32_32x32x32_i8) runs 2x the bf16 rate,
// ~64x the f64 one. A Gram A = X^T X of a tall shard (X: m x D, the real-shaped config: 625k x 10001
// per worker) is therefore computed here as
//   x_ij = 2^{e_j} sum_{p=1..S} d_p(i, j) 2^{-7 p},     d_p in [-127, 127]  (digits of x / 2^{e_j})
//   A_ab = 2^{e_a + e_b} sum_{L=2}^{S+1} 2^{-7 L} sum_{p+q=L} sum_i d_p(i, a) d_q(i, b)
// where e_j is the column's exponent (|x_ij| < 2^{e_j}), the digits are the truncated base-128
// expansion (every digit has the sign of x), and the pairs with p + q > S + 1 are dropped (each below
// 2^{-7(S+2)} of the column scales: far under f64 rounding). Every inner sum is an EXACT int32 MFMA
// accumulation (|d_p d_q| < 2^14; a chunk of K samples with at most S pairs per level stays below
// 2^31 for K * S * 127^2 < 2^31, K = 8192 here), so the only roundings are the f64 recombination and
// the chunk sums -- the result is as accurate as the f64-MFMA Gram (whose K-sum rounds at every
// step) or better; the S-digit truncation of the inputs is 2^{-7S} of the column scale (S = 7: 2^-49).
//
// Kernels (host driver gadmm_gram_ozaki_f64 below, one chunk of KC samples at a time):
//   oz_colexp   column exponents of the augmented [X | y] over the whole shard (one pass)
//   oz_slice    digits of a chunk: S[p][kb][j][32] int8 -- slice p, 32-sample block kb, feature j,
//               the block's 32 samples contiguous, so one MFMA operand fragment is one 1 KB run
//   oz_gemm     lower-triangle tiles of 32 x 32 features per wave, all S(S+1)/2 digit pairs as int8
//               MFMAs into S level accumulators, flushed once per chunk into the f64 Gram
//   oz_finish   the f64 Gram -> A (full symmetric), b, y'y
#include <stdlib.h>
#include <string.h>
#include "gadmm_common.h"

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

namespace {

// One v_mfma_i32_32x32x32_i8 on raw per-lane fragments (layout probe for the tests: the lane maps of
// the A / B operands are established from exact integer data, tests/test_gpu.py).
__global__ void __launch_bounds__(64) mfma_i8_probe_kernel(const v4i* a, const v4i* b, int* d) {
  const int l = threadIdx.x;
  v16i c = {};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[l], b[l], c, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 16; ++r) d[l * 16 + r] = c[r];
}

}  // namespace

extern "C" {

int gadmm_mfma_i8_probe(const void* a_frag, const void* b_frag, int* d_out, hipStream_t st) {
  if (!a_frag || !b_frag || !d_out) {
    gadmm_set_error("mfma_i8_probe: null argument");
    return -1;
  }
  hipLaunchKernelGGL(mfma_i8_probe_kernel, dim3(1), dim3(64), 0, st, (const v4i*)a_frag, (const v4i*)b_frag, d_out);
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"
