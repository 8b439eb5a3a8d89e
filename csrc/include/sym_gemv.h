// Symmetric f64 GEMV over a block-packed lower triangle: the cached inverses of the large-d kernels
// (d > 256, BASELINE configs[4]: 10k x 10k = 800 MB full, 400 MB packed) -- chain_big.hip (GADMM
// phases) and star_big.hip (star ADMM). An iteration of those solvers is HBM-bound on streaming the
// inverses, so storing only the lower triangle halves the bytes per iteration.
//
// Layout: the d x d matrix is cut into B x B blocks (B = 128, zero padded to nb = ceil(d / B)); only
// blocks (I, J) with J <= I are stored, block b = I (I + 1) / 2 + J at offset b B^2, row-major inside
// the block; a diagonal block is stored full (symmetric, mirrored from its lower half).
//
// y = M r in two launches:
//   sym_part    one workgroup per stored block (nb (nb + 1) / 2 >> 256 of them at d = 10k): the
//               block's direct product  P[I][J] = M_IJ r_J  and, off the diagonal, its transposed one
//               P[J][I] = M_IJ^T r_I, from ONE read of the block (each wave: 32 block rows, a lane owns
//               two columns -- one 1-KiB contiguous load per row; the transposed sums accumulate in the
//               lane's registers, the direct ones are row sums across the wave, folded by a 5-stage
//               reduce-scatter of 32 rows over the 64 lanes: one shuffle per row instead of six)
//   sym_reduce  y[t B + k] = sum_s P[t][s][k] in a fixed order (reduce_row: RG groups of s per block row)
// Every partial has exactly one writer and the reduction order is fixed: deterministic.
#pragma once
#include "gadmm_common.h"

namespace symv {

typedef double dv2 __attribute__((ext_vector_type(2)));

constexpr int B = 128;   // block edge (a wave row = 64 lanes x 2 doubles)
constexpr int NT = 256;  // 4 waves x 32 block rows
constexpr int RW = 32;   // block rows per wave

__host__ __device__ __forceinline__ int nblk(int d) { return (d + B - 1) / B; }
__host__ __device__ __forceinline__ long nstored(int d) {
  const long n = nblk(d);
  return n * (n + 1) / 2;
}
// doubles of one packed matrix / of the partial table P [nb][nb][B] / of a zero-padded vector
__host__ __device__ __forceinline__ long packed_doubles(int d) { return nstored(d) * B * B; }
__host__ __device__ __forceinline__ long part_doubles(int d) { return (long)nblk(d) * nblk(d) * B; }
__host__ __device__ __forceinline__ long padded(int d) { return (long)nblk(d) * B; }

__device__ __forceinline__ void block_ij(int b, int& I, int& J) {
  int i = (int)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
  while ((long)(i + 1) * (i + 2) / 2 <= b) ++i;
  while ((long)i * (i + 1) / 2 > b) --i;
  I = i;
  J = b - i * (i + 1) / 2;
}

// Partials of y = M r for the stored block `b` of one matrix. `r` zero padded to padded(d).
__device__ __forceinline__ void part_block(const double* __restrict__ Mp, const double* __restrict__ r,
                                           double* __restrict__ P, int nb, int b, dv2 (*tl)[64]) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int I, J;
  block_ij(b, I, J);
  const dv2* rowp = reinterpret_cast<const dv2*>(Mp + (long)b * B * B + (long)w * RW * B) + lane;
  const dv2 rj = reinterpret_cast<const dv2*>(r + (long)J * B)[lane];
  const double* ri = r + (long)I * B + w * RW;  // wave-uniform: scalar loads
  double p[RW];
  double t0 = 0.0, t1 = 0.0;
#pragma unroll
  for (int c = 0; c < RW; c += 8) {
    dv2 m[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = __builtin_nontemporal_load(rowp + (c + k) * (B / 2));
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      p[c + k] = fma(m[k].x, rj.x, m[k].y * rj.y);
      const double rk = ri[c + k];
      t0 = fma(m[k].x, rk, t0);
      t1 = fma(m[k].y, rk, t1);
    }
  }
  // reduce-scatter of the 32 row partials over the 64 lanes: stage (mask m, n kept) halves the rows a
  // lane holds; afterwards lane l holds row l >> 1 summed over the lanes sharing its bit 0
#pragma unroll
  for (int n = 16, msk = 32; n >= 1; n >>= 1, msk >>= 1) {
    const bool hi = (lane & msk) != 0;
#pragma unroll
    for (int k = 0; k < n; ++k) {
      const double send = hi ? p[k] : p[k + n];
      const double keep = hi ? p[k + n] : p[k];
      p[k] = keep + __shfl_xor(send, msk, 64);
    }
  }
  const double v = p[0] + __shfl_xor(p[0], 1, 64);
  if ((lane & 1) == 0) P[((long)I * nb + J) * B + w * RW + (lane >> 1)] = v;
  if (I != J) {  // transposed product: the four waves' column sums, fixed order
    tl[w][lane] = dv2{t0, t1};
    __syncthreads();
    if (w == 0) {
      dv2 s = tl[0][lane];
#pragma unroll
      for (int q = 1; q < NT / 64; ++q) {
        s.x += tl[q][lane].x;
        s.y += tl[q][lane].y;
      }
      reinterpret_cast<dv2*>(P + ((long)J * nb + I) * B)[lane] = s;
    }
  }
}

// y[t B + k] (< d) = sum_s P[t][s][k] for one block row t, by a workgroup of RNT = RG x B threads:
// thread (g, k) sums the s of group g = [g S, (g + 1) S) (S = ceil(nb / RG), eight loads in flight at a
// time), then thread (0, k) adds the RG group sums in group order. Fixed order, so deterministic; the
// whole workgroup must call it (one barrier). Valid in the threads < B (k = threadIdx.x).
constexpr int RG = 8;
constexpr int RNT = RG * B;

__device__ __forceinline__ double reduce_row(const double* __restrict__ P, int nb, int t, double (*red)[B]) {
  const int k = threadIdx.x & (B - 1), g = threadIdx.x / B;
  const int per = (nb + RG - 1) / RG, s0 = g * per, s1 = s0 + per < nb ? s0 + per : nb;
  const double* q = P + (long)t * nb * B + k;
  double acc = 0.0;
  for (int s = s0; s < s1; s += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = s + u < s1 ? q[(long)(s + u) * B] : 0.0;
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  red[g][k] = acc;
  __syncthreads();
  double y = 0.0;
  if (g == 0) {
    y = red[0][k];
#pragma unroll
    for (int h = 1; h < RG; ++h) y += red[h][k];
  }
  return y;
}

}  // namespace symv
