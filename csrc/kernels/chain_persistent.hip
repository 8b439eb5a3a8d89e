// Persistent single-launch GADMM (linear, closed form) for one MI355X: the whole solve in ONE kernel.
//
// Why: at the reference shapes (N = 24..50 workers, d = 50) an iteration is two dependent phases of
// ~1 us of arithmetic each; as separate launches every phase pays a kernel boundary and re-reads
// the worker's cached inverse and Gram from L2/MALL (profiles/r01_baseline_multikernel: 7.7 us per
// phase). Here each worker is one resident workgroup that keeps (A + c rho I)^{-1} and A in LDS for
// the entire solve; the only traffic per phase is the neighbours' theta (<= 2 x 400 B).
//
// Schedule == group_ADMM_closedForm.m / dynamic_group_ADMM_closedForm.m with a static chain:
//   head (even chain position) at iteration i: wait tails' theta^{i-1}; lazy dual update (the
//   reference's end-of-iteration dual, applied when both tails are known); solve; publish theta^i.
//   tail at iteration i: wait heads' theta^i; solve; publish theta^i; dual update.
//   every worker then publishes f_n(theta_n^i); the monitor workgroup sums them in worker order,
//   records the trace and posts the stop decision for iteration i (|obj - obj0| < tol).
//   A worker starts iteration i only after the decision of iteration i - LAG is known, so all
//   workers leave at the same iteration boundary; the reported iteration count is exact.
//
// Hand-offs use the data-is-flag granule form of cdna_hip_programming.md §6 Guideline 16 (R2): each
// double travels as one 16-byte {tag, lo, tag, hi} write-through (sc1) store; the consumer re-reads
// its 16-byte sc1 granule until both tags equal the expected iteration. No flags, no fences, no
// counters. Every spin is bounded by a wall-clock deadline (s_memrealtime); on timeout the kernel
// records done = 4 and every workgroup exits.
#include "gadmm_common.h"
#include "gadmm_chain.h"



namespace {

constexpr int NT = 256;
constexpr int NW = 4;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}

__device__ __forceinline__ void store_granule(__amdgpu_buffer_rsrc_t rs, int byte_off, unsigned tag, double v) {
  const unsigned long long bits = __double_as_longlong(v);
  u32x4 g = {tag, (unsigned)(bits & 0xffffffffull), tag, (unsigned)(bits >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(g, rs, byte_off, 0, 16 /* sc1 */);
}

__device__ __forceinline__ bool load_granule(__amdgpu_buffer_rsrc_t rs, int byte_off, unsigned tag, double* v) {
  const u32x4 g = __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 16 /* sc1 */);
  *v = __longlong_as_double((long long)(((unsigned long long)g.w << 32) | g.y));
  return g.x == tag && g.z == tag;
}

__device__ __forceinline__ unsigned long long now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

// Every lane of the block polls the granules of its elements of `src_row` until all carry `tag`.
template <int NC>
__device__ __forceinline__ bool wait_row(__amdgpu_buffer_rsrc_t rs, int row, int d, unsigned tag, double (&out)[NC],
                                         unsigned long long deadline, volatile int* abort_lds) {
  const int lane = threadIdx.x & 63;
  for (;;) {
    bool ok = true;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      if (i < d) ok &= load_granule(rs, (row * d + i) * 16, tag, &out[c]);
    }
    if (__all(ok)) return true;
    if (now_ticks() > deadline || *abort_lds) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

// y[i] = sum_j M[j][i] x[j] with M (symmetric) and x in LDS; lanes own i, waves split j.
template <int NC>
__device__ __forceinline__ void symv_lds(const double* M, const double* x, double (&y)[NC], double* red, int d) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = 0.0;
  // 4 rows of M per batch per wave: the 4 (x NC) LDS loads issue together, one wait per batch
  int j = w;
  for (; j + 3 * NW < d; j += 4 * NW) {
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
  for (; j < d; j += NW) {
    const double xj = x[j];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      if (i < d) acc[c] = fma(M[j * d + i], xj, acc[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) red[(w * NC + c) * 64 + lane] = acc[c];
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    double s = 0.0;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) s += red[(ww * NC + c) * 64 + lane];
    y[c] = s;  // every wave holds the full result for its lanes' rows
  }
  __syncthreads();
}

}  // namespace

template <int NC>
__global__ void __launch_bounds__(NT) chain_persistent_kernel(PersistArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int abort_lds;
  __shared__ int stop_lds;
  const int d = a.d, n = a.n;
  const int lane = threadIdx.x & 63;
  const bool w0 = threadIdx.x < 64;  // wave 0 owns the worker state; waves 1..3 help in the GEMVs
  const __amdgpu_buffer_rsrc_t rth = rsrc_of(a.thg);
  const __amdgpu_buffer_rsrc_t rob = rsrc_of(a.objg);
  const unsigned long long deadline = now_ticks() + (unsigned long long)a.timeout_ticks;
  if (threadIdx.x == 0) {
    abort_lds = 0;
    stop_lds = 0;
  }
  __syncthreads();

  if ((int)blockIdx.x == n) {
    // ---------------------------------------------------------------- monitor workgroup
    double* vals = lds;  // [n]
    for (int it = a.start_iter;; ++it) {
      const unsigned tag = (unsigned)it;
      const int slot = it % a.ring;
      if (w0) {
        for (int w = lane; w < n; w += 64) {
          double v = 0.0;
          for (;;) {
            if (load_granule(rob, (slot * n + w) * 16, tag, &v)) break;
            if (now_ticks() > deadline) {
              abort_lds = 1;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          vals[w] = v;
        }
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        unsigned code = 0;
        if (abort_lds) {
          code = 4;
        } else {
          double s = 0.0;
          for (int w = 0; w < n; ++w) s += vals[w];  // fixed order: deterministic, == multi-kernel path
          if (it - 1 < a.max_iter) a.trace[it - 1] = s;
          if (!(s == s) || isinf(s)) code = 3;
          else if (fabs(s - a.obj0) < a.tol) code = 1;
          else if (it >= a.max_iter) code = 2;
        }
        __hip_atomic_store(&a.decg[slot], ((unsigned long long)tag << 32) | code, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        if (code) {
          a.ctl->done = (int)code;
          a.ctl->conv_iter = it;
          a.ctl->iter = it + a.lag;
          a.ctl->pending = 1;
          a.ctl->monitored = it;
          stop_lds = 1;
        }
      }
      __syncthreads();
      if (stop_lds) return;
    }
  }

  // ------------------------------------------------------------------ worker workgroup
  const int pos = blockIdx.x;
  const int w = a.path[pos];
  const int left = pos > 0 ? a.path[pos - 1] : -1;
  const int right = pos < n - 1 ? a.path[pos + 1] : -1;
  const bool head = (pos % 2) == 0;
  const int deg = (left >= 0) + (right >= 0);
  const double rho = a.rho;
  const double crho = deg * rho;

  double* Ml = lds;                                            // d*d
  double* Al = lds + (long)d * d;                              // d*d (obj_mode 0)
  double* xv = lds + (long)(a.obj_mode == 0 ? 2 : 1) * d * d;  // [64*NC] rhs / theta staging
  double* red = xv + 64 * NC;                                  // [NW*NC*64]

  const double* Mg = a.Minv + ((long)w * a.nvar + a.deg_to_var[deg]) * (long)d * d;
  for (int e = threadIdx.x; e < d * d; e += NT) Ml[e] = Mg[e];
  if (a.obj_mode == 0) {
    const double* Ag = a.A + (long)w * d * d;
    for (int e = threadIdx.x; e < d * d; e += NT) Al[e] = Ag[e];
  }
  // worker state, meaningful in wave 0 (lane owns elements i = lane + 64c)
  double th[NC], mu[NC], bb[NC], tl[NC], tr[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = lane + 64 * c;
    const bool in = w0 && i < d;
    th[c] = in ? a.theta[(long)w * d + i] : 0.0;
    mu[c] = in ? a.mu[(long)w * d + i] : 0.0;
    bb[c] = in ? a.b[(long)w * d + i] : 0.0;
    tl[c] = (in && left >= 0) ? a.theta[(long)left * d + i] : 0.0;
    tr[c] = (in && right >= 0) ? a.theta[(long)right * d + i] : 0.0;
  }
  const double half_yy = 0.5 * a.yy[w];
  int pending = a.pending_in;
  __syncthreads();

  for (int it = a.start_iter;; ++it) {
    // -- stop rule: decision of iteration it - lag (all workers leave at the same boundary)
    if (it - a.start_iter >= a.lag) {
      const int j = it - a.lag;
      if (threadIdx.x == 0) {
        unsigned long long v;
        for (;;) {
          v = __hip_atomic_load(&a.decg[j % a.ring], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((unsigned)(v >> 32) == (unsigned)j) break;
          if (now_ticks() > deadline) {
            v = 4;
            abort_lds = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        stop_lds = ((unsigned)(v & 0xffffffffu)) != 0u;
      }
      __syncthreads();
      if (stop_lds) break;
    }
    if (it > a.max_iter + a.lag) break;

    // -- neighbours' theta and the rhs (wave 0)
    if (w0) {
      bool ok = true;
      if (head) {
        if (it > a.start_iter) {
          if (left >= 0) ok &= wait_row<NC>(rth, left, d, (unsigned)(it - 1), tl, deadline, &abort_lds);
          if (ok && right >= 0) ok &= wait_row<NC>(rth, right, d, (unsigned)(it - 1), tr, deadline, &abort_lds);
        }
        if (pending) {  // lazy end-of-iteration dual (reference order: -rho(th_l - th) then +rho(th - th_r))
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            double m = mu[c];
            if (left >= 0) m = m - rho * (tl[c] - th[c]);
            if (right >= 0) m = m + rho * (th[c] - tr[c]);
            mu[c] = m;
          }
        }
      } else {
        if (left >= 0) ok &= wait_row<NC>(rth, left, d, (unsigned)it, tl, deadline, &abort_lds);
        if (ok && right >= 0) ok &= wait_row<NC>(rth, right, d, (unsigned)it, tr, deadline, &abort_lds);
      }
      if (!ok && lane == 0) abort_lds = 1;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int i = lane + 64 * c;
        double r = bb[c] - mu[c];
        if (left >= 0) r = r + rho * tl[c];
        if (right >= 0) r = r + rho * tr[c];
        if (i < d) xv[i] = r;
      }
    }
    __syncthreads();
    if (abort_lds) break;

    // -- solve theta = (A + deg rho I)^{-1} r
    double tn[NC];
    symv_lds<NC>(Ml, xv, tn, red, d);
    double part = 0.0;
    if (w0) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {  // publish theta^it: one 16-B sc1 granule per element
        const int i = lane + 64 * c;
        if (i < d) store_granule(rth, (w * d + i) * 16, (unsigned)it, tn[c]);
      }
      if (!head) {  // tails: both neighbours are this iteration's heads -> dual update now
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          double m = mu[c];
          if (left >= 0) m = m - rho * (tl[c] - tn[c]);
          if (right >= 0) m = m + rho * (tn[c] - tr[c]);
          mu[c] = m;
        }
      } else {
        pending = 1;
      }
      if (a.obj_mode != 0) {  // A th = r - deg rho th  (xv still holds r)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int i = lane + 64 * c;
          if (i < d) part += (0.5 * (xv[i] - crho * tn[c]) - bb[c]) * tn[c];
        }
      }
    }
    if (a.obj_mode == 0) {  // exact: 1/2 th^T A th - b^T th + 1/2 y^T y
      __syncthreads();
      if (w0) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int i = lane + 64 * c;
          if (i < d) xv[i] = tn[c];
        }
      }
      __syncthreads();
      double q[NC];
      symv_lds<NC>(Al, xv, q, red, d);
      if (w0) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int i = lane + 64 * c;
          if (i < d) part += (0.5 * q[c] - bb[c]) * tn[c];
        }
      }
    }
    if (w0) {
      const double f = wave_sum_f64(part) + half_yy;
      if (lane == 0) store_granule(rob, ((it % a.ring) * n + w) * 16, (unsigned)it, f);
#pragma unroll
      for (int c = 0; c < NC; ++c) th[c] = tn[c];
    }
    __syncthreads();
  }

  // write back the final state (plain stores; visible to the host after the kernel)
  if (w0) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      if (i < d) {
        a.theta[(long)w * d + i] = th[c];
        a.mu[(long)w * d + i] = mu[c];
      }
    }
  }
  if (abort_lds && threadIdx.x == 0) a.ctl->done = 4;
}

extern "C" {

// LDS bytes the persistent kernel needs; 0 if the shape is not eligible.
long gadmm_chain_persistent_lds(int d, int obj_mode) {
  if (d > 128) return 0;
  const int nc = (d + 63) / 64;
  long doubles = (long)(obj_mode == 0 ? 2 : 1) * d * d + 64 * nc + NW * nc * 64 + NW + 16;
  long bytes = doubles * 8;
  if (bytes > 160 * 1024 - 64) return 0;
  return bytes;
}

int gadmm_chain_persistent_launch(const PersistArgs* args, hipStream_t st) {
  const PersistArgs& a = *args;
  const long lds = gadmm_chain_persistent_lds(a.d, a.obj_mode);
  if (lds == 0) {
    gadmm_set_error("persistent chain kernel: d=%d not eligible", a.d);
    return -1;
  }
  if (a.n + 1 > 256) {
    gadmm_set_error("persistent chain kernel: %d workers exceed one workgroup per CU", a.n);
    return -1;
  }
  if (a.ring <= a.lag + 1) {
    gadmm_set_error("persistent chain kernel: ring must exceed lag + 1");
    return -1;
  }
  const long monitor_lds = (long)a.n * 8;
  const size_t shm = (size_t)(lds > monitor_lds ? lds : monitor_lds);
  if (a.d <= 64) {
    if (shm > 65536)
      GADMM_CHECK(hipFuncSetAttribute((const void*)chain_persistent_kernel<1>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    hipLaunchKernelGGL(chain_persistent_kernel<1>, dim3(a.n + 1), dim3(NT), shm, st, a);
  } else {
    if (shm > 65536)
      GADMM_CHECK(hipFuncSetAttribute((const void*)chain_persistent_kernel<2>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    hipLaunchKernelGGL(chain_persistent_kernel<2>, dim3(a.n + 1), dim3(NT), shm, st, a);
  }
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"
