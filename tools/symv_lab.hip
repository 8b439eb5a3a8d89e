// Symmetric-GEMV lab (sym_gemv.h variants, real10m iteration: 10k x 10k block-packed inverses).
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -I csrc/include tools/symv_lab.hip -o tools/libsymv_lab.so
// Driven by tools/symv_lab.py: times each variant with hip events and checks it against variant 0.
//   v0  sym_gemv.h as shipped (4 waves x 32 rows, one block per workgroup)
//   v1  v0 at >= 3 waves / SIMD (amdgpu_waves_per_eu)
//   v2  8 waves x 16 rows per block (512 threads)
//   v3  v0's body in a grid-stride loop over blocks (grid = k x 256 workgroups)
//   v4  4 waves x 32 rows, loads in two half-batches (16 rows in flight per wave)
//   v9  plain streaming read of the packed matrix (the bandwidth roof on this box)
#include "sym_gemv.h"
#include <hip/hip_runtime.h>

namespace {
using symv::dv2;
using symv::B;

template <int RW>
__device__ __forceinline__ double fold_rows(double (&p)[RW], int lane) {
  // reduce-scatter of RW row partials over 64 lanes, then fold the lanes that share a row
#pragma unroll
  for (int n = RW / 2, msk = 32; n >= 1; n >>= 1, msk >>= 1) {
    const bool hi = (lane & msk) != 0;
#pragma unroll
    for (int k = 0; k < n; ++k) {
      const double send = hi ? p[k] : p[k + n];
      const double keep = hi ? p[k + n] : p[k];
      p[k] = keep + __shfl_xor(send, msk, 64);
    }
  }
  double v = p[0];
#pragma unroll
  for (int msk = 32 / RW; msk >= 1; msk >>= 1) v += __shfl_xor(v, msk, 64);
  return v;  // lane l: row l / (64 / RW)
}

template <int WPB, int BATCH>
__device__ __forceinline__ void part_block_g(const double* __restrict__ Mp, const double* __restrict__ r,
                                             double* __restrict__ P, int nb, int b, dv2 (*tl)[64]) {
  constexpr int RW = B / WPB;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int I, J;
  symv::block_ij(b, I, J);
  const dv2* rowp = reinterpret_cast<const dv2*>(Mp + (long)b * B * B + (long)w * RW * B) + lane;
  const dv2 rj = reinterpret_cast<const dv2*>(r + (long)J * B)[lane];
  const double* ri = r + (long)I * B + w * RW;
  double p[RW];
  double t0 = 0.0, t1 = 0.0;
#pragma unroll
  for (int c = 0; c < RW; c += BATCH) {
    dv2 m[BATCH];
#pragma unroll
    for (int k = 0; k < BATCH; ++k) m[k] = __builtin_nontemporal_load(rowp + (c + k) * (B / 2));
#pragma unroll
    for (int k = 0; k < BATCH; ++k) {
      p[c + k] = fma(m[k].x, rj.x, m[k].y * rj.y);
      const double rk = ri[c + k];
      t0 = fma(m[k].x, rk, t0);
      t1 = fma(m[k].y, rk, t1);
    }
  }
  const double v = fold_rows<RW>(p, lane);
  constexpr int SH = 64 / RW;
  if ((lane % SH) == 0) P[((long)I * nb + J) * B + w * RW + lane / SH] = v;
  if (I != J) {
    tl[w][lane] = dv2{t0, t1};
    __syncthreads();
    if (w == 0) {
      dv2 s = tl[0][lane];
#pragma unroll
      for (int q = 1; q < WPB; ++q) {
        s.x += tl[q][lane].x;
        s.y += tl[q][lane].y;
      }
      reinterpret_cast<dv2*>(P + ((long)J * nb + I) * B)[lane] = s;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) v0_part(const double* Mp, const double* r, double* P, int nb) {
  __shared__ dv2 tl[4][64];
  symv::part_block(Mp, r, P, nb, blockIdx.x, tl);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 8)))
v1_part(const double* Mp, const double* r, double* P, int nb) {
  __shared__ dv2 tl[4][64];
  symv::part_block(Mp, r, P, nb, blockIdx.x, tl);
}
__global__ void __launch_bounds__(512) v2_part(const double* Mp, const double* r, double* P, int nb) {
  __shared__ dv2 tl[8][64];
  part_block_g<8, 8>(Mp, r, P, nb, blockIdx.x, tl);
}
__global__ void __launch_bounds__(256) v3_part(const double* Mp, const double* r, double* P, int nb, int nst) {
  __shared__ dv2 tl[4][64];
  for (int b = blockIdx.x; b < nst; b += gridDim.x) part_block_g<4, 8>(Mp, r, P, nb, b, tl);
}
__global__ void __launch_bounds__(256) v4_part(const double* Mp, const double* r, double* P, int nb) {
  __shared__ dv2 tl[4][64];
  part_block_g<4, 16>(Mp, r, P, nb, blockIdx.x, tl);
}
__global__ void __launch_bounds__(256) v9_read(const dv2* Mp, long n2, double* out) {
  double s = 0.0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256) {
    const dv2 v = __builtin_nontemporal_load(Mp + i);
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;  // keeps the loads alive
}
__global__ void __launch_bounds__(symv::RNT) reduce(const double* P, double* y, int nb, int d) {
  __shared__ double red[symv::RG][B];
  const int t = blockIdx.x, k = threadIdx.x;
  const double v = symv::reduce_row(P, nb, t, red);
  if (k < B && t * B + k < d) y[t * B + k] = v;
}

void launch(int v, const double* Mp, const double* r, double* P, double* y, int d, int grid_k, hipStream_t st) {
  const int nb = symv::nblk(d);
  const int nst = (int)symv::nstored(d);
  switch (v) {
    case 0: hipLaunchKernelGGL(v0_part, dim3(nst), dim3(256), 0, st, Mp, r, P, nb); break;
    case 1: hipLaunchKernelGGL(v1_part, dim3(nst), dim3(256), 0, st, Mp, r, P, nb); break;
    case 2: hipLaunchKernelGGL(v2_part, dim3(nst), dim3(512), 0, st, Mp, r, P, nb); break;
    case 3: hipLaunchKernelGGL(v3_part, dim3(grid_k * 256 < nst ? grid_k * 256 : nst), dim3(256), 0, st, Mp, r, P, nb,
                               nst); break;
    case 4: hipLaunchKernelGGL(v4_part, dim3(nst), dim3(256), 0, st, Mp, r, P, nb); break;
    case 9: hipLaunchKernelGGL(v9_read, dim3(grid_k * 256), dim3(256), 0, st, (const dv2*)Mp,
                               symv::packed_doubles(d) / 2, y); return;
    default: return;
  }
  hipLaunchKernelGGL(reduce, dim3(nb), dim3(symv::RNT), 0, st, P, y, nb, d);
}
}  // namespace

extern "C" {
// Mean microseconds per call over `reps` calls (after 2 untimed), part + reduce; -1 on error.
double symv_lab_time(int v, const double* Mp, const double* r, double* P, double* y, int d, int grid_k, int reps) {
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -1.0;
  for (int i = 0; i < 2; ++i) launch(v, Mp, r, P, y, d, grid_k, 0);
  hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) launch(v, Mp, r, P, y, d, grid_k, 0);
  hipEventRecord(e1, 0);
  if (hipEventSynchronize(e1) != hipSuccess) return -1.0;
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return hipGetLastError() == hipSuccess ? 1e3 * ms / reps : -1.0;
}
long symv_lab_packed_doubles(int d) { return symv::packed_doubles(d); }
long symv_lab_part_doubles(int d) { return symv::part_doubles(d); }
long symv_lab_padded(int d) { return symv::padded(d); }
}
