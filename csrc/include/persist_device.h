// Device helpers shared by the persistent (single-launch) kernels: data-is-flag granules
// (cdna_hip_programming.md §6 Guideline 16, R2), wall-clock deadlines, LDS-resident GEMV.
#pragma once
#include "gadmm_common.h"

// Pause between two polls of a hand-off spin (s_sleep units of 64 clocks; 0 = poll back to back).
#ifndef GADMM_POLL_SLEEP
#define GADMM_POLL_SLEEP 1
#endif
#define GADMM_POLL_PAUSE()                                              \
  do {                                                                  \
    if (GADMM_POLL_SLEEP > 0) __builtin_amdgcn_s_sleep(GADMM_POLL_SLEEP); \
  } while (0)
#include "gadmm_chain.h"
#include "quad_gemv.h"

// The fence-free LDS ring posts (chain_persistent_logistic.hip: zr_post, chain_persistent_newton.hip:
// lds_post) rely on one hardware property: the LDS instructions of ONE wave are performed in issue order
// (CDNA3 / CDNA4: the property every counted `s_waitcnt lgkmcnt(N)` on a wave's LDS traffic relies on,
// cdna_hip_programming.md §5). The HIP / LLVM memory model does not promise it, so it is enabled only
// for the architectures whose ISA documents it; any other target compiles the fenced (release) post.
// tests/test_gpu.py::test_postfence_stress checks the two posts give bit-identical traces on gfx950.
#if defined(__gfx950__) || defined(__gfx942__)
#define GADMM_LDS_IN_ORDER 1
#else
#define GADMM_LDS_IN_ORDER 0
#endif

namespace persist {


__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}

template <bool SYS>
__device__ __forceinline__ void store_granule(__amdgpu_buffer_rsrc_t rs, int byte_off, unsigned tag, double v) {
  const unsigned long long bits = __double_as_longlong(v);
  u32x4 g = {tag, (unsigned)(bits & 0xffffffffull), tag, (unsigned)(bits >> 32)};
  if (SYS) __builtin_amdgcn_raw_buffer_store_b128(g, rs, byte_off, 0, 17 /* sc0 sc1 */);
  else __builtin_amdgcn_raw_buffer_store_b128(g, rs, byte_off, 0, 16 /* sc1 */);
}

// Plain (write-back) granule store: the line stays in this XCD's L2, so a same-XCD `sc1` reader is
// served from L2 instead of re-fetching it across the fabric (MI355X_MICROARCH.md, price list:
// `sc1` stores DROP the line). Visible ONLY to readers on the same XCD: callers must have verified
// the placement of every reader (chain_blocked.hip: xcd_verdict).
__device__ __forceinline__ void store_granule_local(__amdgpu_buffer_rsrc_t rs, int byte_off, unsigned tag, double v) {
  const unsigned long long bits = __double_as_longlong(v);
  u32x4 g = {tag, (unsigned)(bits & 0xffffffffull), tag, (unsigned)(bits >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(g, rs, byte_off, 0, 0);
}

// store_granule, or (one GPU, placement verified: `local` wave-uniform) store_granule_local
template <bool SYS>
__device__ __forceinline__ void put_granule(bool local, __amdgpu_buffer_rsrc_t rs, int byte_off, unsigned tag, double v) {
  if (!SYS && local) store_granule_local(rs, byte_off, tag, v);
  else store_granule<SYS>(rs, byte_off, tag, v);
}

// This wave's XCD (0-7).
__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x;
}

template <bool SYS>
__device__ __forceinline__ bool load_granule(__amdgpu_buffer_rsrc_t rs, int byte_off, unsigned tag, double* v) {
  const u32x4 g = SYS ? __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 17)
                      : __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 16);
  *v = __longlong_as_double((long long)(((unsigned long long)g.w << 32) | g.y));
  return g.x == tag && g.z == tag;
}

template <bool SYS>
__device__ __forceinline__ u32x4 load_raw(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  return SYS ? __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 17)
             : __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 16);
}
__device__ __forceinline__ bool granule_ok(const u32x4& g, unsigned tag) { return g.x == tag && g.z == tag; }
__device__ __forceinline__ double granule_val(const u32x4& g) {
  return __longlong_as_double((long long)(((unsigned long long)g.w << 32) | g.y));
}

template <bool SYS>
__device__ __forceinline__ void store_dec(unsigned long long* p, unsigned long long v) {
  if (SYS) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool SYS>
__device__ __forceinline__ unsigned long long load_dec(unsigned long long* p) {
  if (SYS) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ unsigned make_tag(unsigned epoch, int it) { return (epoch << 20) | ((unsigned)it & 0xfffffu); }

// Every lane of wave 0 polls the granules of its elements of table row `row` until all carry `tag`.
template <int NC, bool SYS>
__device__ __forceinline__ bool wait_row(__amdgpu_buffer_rsrc_t rs, int row, int d, unsigned tag, double (&out)[NC],
                                         unsigned long long deadline) {
  const int lane = threadIdx.x & 63;
  for (;;) {
    bool ok = true;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      if (i < d) ok &= load_granule<SYS>(rs, (row * d + i) * 16, tag, &out[c]);
    }
    if (__all(ok)) return true;
    if (now_ticks() > deadline) return false;
    GADMM_POLL_PAUSE();
  }
}

// Poll up to two rows (row < 0: skipped) in ONE loop, so a worker waiting on both chain neighbours
// pays one round trip, not two. Rows may carry different tags. `stopw` (nullable) is a run-wide stop
// word: -1 abort, k > 0 stopped after iteration k (the wait is abandoned once it > k).
// Returns 1 ok, 0 deadline passed, -1 stopped. Wave-uniform.
template <int NC, bool SYS>
__device__ __forceinline__ int wait_pair(__amdgpu_buffer_rsrc_t rs, int d, int ra, unsigned ta, double (&va)[NC],
                                         int rb, unsigned tb, double (&vb)[NC], unsigned long long deadline,
                                         const int* stopw = nullptr, int it = 0) {
  const int lane = threadIdx.x & 63;
  for (int spin = 0;; ++spin) {
    bool ok = true;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      if (i < d) {
        if (ra >= 0) ok &= load_granule<SYS>(rs, (ra * d + i) * 16, ta, &va[c]);
        if (rb >= 0) ok &= load_granule<SYS>(rs, (rb * d + i) * 16, tb, &vb[c]);
      }
    }
    if (__all(ok)) return 1;
    if ((spin & 7) == 7) {
      if (stopw) {
        const int s = __hip_atomic_load(stopw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (s < 0 || (s > 0 && it > s)) return -1;
      }
      if (now_ticks() > deadline) return 0;
    }
    GADMM_POLL_PAUSE();
  }
}

// y[i] = sum_{j < rows} M[j][i] x[j] (M row-major, `cols` wide) with M and x in LDS; lanes own i,
// the block's NW waves split j. Every wave ends with the full y for its lanes' elements; the wave
// partials are combined in fixed order (deterministic, identical in every workgroup).
template <int NC>
__device__ __forceinline__ void gemv_t_lds(const double* M, const double* x, double (&y)[NC], double* red, int rows,
                                           int cols) {
  constexpr int NW = 4;
  const int d = cols;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = 0.0;
  // 4 rows of M per batch per wave: the 4 (x NC) LDS loads issue together, one wait per batch
  int j = w;
  for (; j + 3 * NW < rows; j += 4 * NW) {
    double mv[4][NC], xv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      xv[q] = x[j + q * NW];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int i = lane + 64 * c;
        mv[q][c] = i < d ? M[(j + q * NW) * d + i] : 0.0;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[c] = fma(mv[q][c], xv[q], acc[c]);
  }
  for (; j < rows; j += NW) {
    const double xj = x[j];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      if (i < d) acc[c] = fma(M[j * d + i], xj, acc[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) red[(w * NC + c) * 64 + lane] = acc[c];
  lds_barrier();
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    double s = 0.0;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) s += red[(ww * NC + c) * 64 + lane];
    y[c] = s;  // every wave holds the full result for its lanes' rows
  }
  lds_barrier();
}

// y = M x for symmetric M (d x d) in LDS.
template <int NC>
__device__ __forceinline__ void symv_lds(const double* M, const double* x, double (&y)[NC], double* red, int d) {
  gemv_t_lds<NC>(M, x, y, red, d, d);
}

constexpr int DREG = 64;  // register-resident variant: d <= 64, one wave per worker

// y_i = sum_j M[i][j] x_j with lane i holding row i of M in registers and x broadcast from LDS
// (zero-padded to DREG); four independent accumulators over j = k mod 4, combined ((a0 + a1) + a2) + a3:
// exactly the summation order of symv_lds / symv_cols (wave k of 4 sums rows j = k mod 4, partials
// added in wave order), so every engine produces bit-identical iterates (M is exactly symmetric).
template <int DB>
__device__ __forceinline__ double reg_gemv(const double (&Mr)[DB], const double* xv) {
  static_assert(DB % 4 == 0, "row length must be a multiple of 4");
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll
  for (int j = 0; j < DB; j += 4) {
    const double2 x01 = *reinterpret_cast<const double2*>(xv + j);
    const double2 x23 = *reinterpret_cast<const double2*>(xv + j + 2);
    a0 = fma(Mr[j], x01.x, a0);
    a1 = fma(Mr[j + 1], x01.y, a1);
    a2 = fma(Mr[j + 2], x23.x, a2);
    a3 = fma(Mr[j + 3], x23.y, a3);
  }
  return ((a0 + a1) + a2) + a3;
}

constexpr unsigned XTAG = 0x5a5a0001u;  // placement-check granule tag of launchers that zero xchk first

// XCD packing (PersistArgs::xcd): every working block posts its XCC_ID into xchk[bid] and waits for
// all nb; true iff they are all equal, i.e. every reader of every granule shares this block's L2.
// The verdict is identical in every block (same inputs); false on a deadline (the run then times
// out through its normal path, with sc1 stores). lds_flag: one int of LDS. tag: XTAG behind a memset
// of xchk, or the launch's own PersistArgs::xtag (no memset: earlier launches' granules never match).
__device__ __forceinline__ bool xcd_verdict(u32x4* xchk, int bid, int nb, unsigned long long deadline, int* lds_flag,
                                            unsigned tag = XTAG) {
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(xchk);
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < 64) {
    if (lane == 0) store_granule<false>(rs, bid * 16, tag, (double)xcc_id());
    bool ok = true, same = true;
    double first = -1.0;
    for (int i0 = 0; i0 < nb; i0 += 64) {
      const int i = i0 + lane;
      double x = 0.0;
      if (i < nb)
        for (int spin = 0;; ++spin) {
          if (load_granule<false>(rs, i * 16, tag, &x)) break;
          if ((spin & 7) == 7 && now_ticks() > deadline) {
            ok = false;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      if (i0 == 0) first = __shfl(x, 0, 64);  // block 0's XCD
      same &= i >= nb || x == first;
    }
    same = __all(ok && same);
    if (lane == 0) *lds_flag = same ? 1 : 0;
  }
  lds_barrier();
  return __builtin_amdgcn_readfirstlane(*lds_flag) != 0;
}

}  // namespace persist
using namespace persist;
