// Persistent first-order baseline engine: GD, DGD, LAG-PS, LAG-WK, cyclic / randomized IAG and dual
// averaging (linear and logistic) in ONE launch per run per GPU.
//
// Reference semantics: GD_DGD_LAG.m / GD_DGD_LAG_logistic.m (A10, A11), dual_averaging.m /
// dual_averaging_logisticReg.m (A8, A9), as implemented by gadmm_amd/algorithms/baselines.py and
// dual_averaging.py (the torch path, kept as the test oracle).
//
// Why one kernel: the reference runs these for 40k-500k iterations of d = 14..50 arithmetic; as
// torch ops each iteration is a dozen launches plus a host read of the objective (~100 us), as a
// persistent kernel it is one L2 (or xGMI) round trip (~2-4 us).
//
// Layout: workgroup b < n_local is worker w = w_lo + b and keeps its Gram (linear) or its shard X_n,
// y_n (logistic) in LDS for the whole run; workgroup n_local is the monitor (rank 0). Per iteration
// every worker evaluates grad f_n and f_n at its point and publishes what the algorithm uploads as
// 16-byte data-is-flag granules ({tag, lo, tag, hi}, tag = epoch:iteration; persist_device.h):
// * server algorithms (GD, LAG, IAG; GD_DGD_LAG.m:102,238,318,344,369): the server's table of the
//   latest upload of every worker is REPLICATED in every workgroup (LDS), and every workgroup applies
//   the server step itself, summing the table rows in one fixed order, so theta stays bit-identical
//   everywhere without a broadcast. Only real uploads move: GD every worker every iteration, IAG the
//   scheduled worker (the schedule is known everywhere), LAG-PS / LAG-WK the triggered workers,
//   announced by a one-granule upload flag per worker per iteration (conditional uploads,
//   GD_DGD_LAG.m:184-327). Across GPUs an upload goes to every rank's table (the replicated server).
// * DGD reads its chain neighbours' gradients (GD_DGD_LAG.m:155-171); dual averaging reads the left
//   neighbour's current-sweep Z and the right neighbour's previous-sweep Z (the Gauss-Seidel
//   wavefront of dual_averaging.m:44, a cross-rank pipeline across GPUs) or both previous (Jacobi).
//   Rows go to the chain neighbours' ranks.
// Row slots: a producer overwrites the slot of iteration it at it + slots. Two suffice where every
// reader reads every iteration (GD: all rows, LAG: all flags, DGD / dual averaging: the neighbours',
// whose next row needs this reader's): it + 2 needs data every reader of `it` publishes after its
// read. IAG moves one row per iteration and no lock-step, so its table has ring + 3 slots: writing
// iteration it + ring + 3 needs the monitor to have seen iteration it + 3 of every worker.
// The monitor sums f_n in worker order, records the objective / trigger / clock traces and posts
// the stop iteration (|obj - obj0| < tol) into every rank's stop word; workers leave once they see
// it. The objective ring has `ring` slots with back-pressure on the monitor's progress word. Every
// spin has a wall-clock deadline. SYS: several GPUs (system-scope granules in IPC fine-grained memory).
#include "gadmm_common.h"
#include "gadmm_fo.h"
#include "persist_device.h"
#include <hip/hip_runtime.h>

namespace {

constexpr int NT = 256;
constexpr int NWV = NT / 64;
constexpr int LAG_SLOT = 10;  // GD_DGD_LAG.m:18 triggerslot

__device__ __forceinline__ double softplus_f64(double t) {  // log(1 + exp(t)), stable
  return t > 30.0 ? t + log1p(exp(-t)) : log1p(exp(t));
}

// Run-wide words (this rank's copy): the monitor's progress and the stop iteration (0: running,
// k > 0: stopped after iteration k, -1: abort). One GPU: fields of FoCtl; several: fine-grained
// words the monitor pushes into every rank.
template <bool SYS>
__device__ __forceinline__ int load_word(const int* p) {
  return SYS ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
             : __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool SYS>
__device__ __forceinline__ void store_word(int* p, int v) {
  if (SYS) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool should_stop(int s, int it) { return s < 0 || (s > 0 && it > s); }

__host__ __device__ __forceinline__ bool is_server_alg(int alg) {
  return alg == FO_GD || alg == FO_LAG_PS || alg == FO_LAG_WK || alg == FO_IAG;
}

// LDS layout (doubles) shared by host sizing (gadmm_fo_lds) and the kernel. `cache`: the replicated
// server table (n rows of d, server algorithms only).
struct FoLds {
  int mat, xs, aux, red, wred, dl, cache, total;
  __host__ __device__ FoLds(int model, int alg, int n, int d, int m, int nc, int mc) {
    mat = 0;
    // linear: A | logistic: X (m x d) | X^T (d x m, when mc > 0) | y | s
    const int msz = model == FO_LINEAR ? d * d : m * d * (mc > 0 ? 2 : 1) + 2 * m;
    xs = (msz + 1) & ~1;
    aux = xs + 64 * nc;
    red = aux + 64 * nc;
    wred = red + NWV * nc * 64;
    dl = wred + 8;
    cache = dl + 16;
    total = cache + (is_server_alg(alg) ? n * d : 0);
  }
};

// f_n and grad f_n at the point held in LDS `xs` (and in registers `th`, lane element i = lane + 64c,
// identical in every wave). Results are identical in every wave. Contains __syncthreads.
template <int NC, int MC>
__device__ __forceinline__ double local_eval(const FoArgs& a, double* lds, const FoLds& L, const double (&th)[NC],
                                             const double (&bb)[NC], double half_yy, double (&g)[NC]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int d = a.d;
  double* red = lds + L.red;
  double* wred = lds + L.wred;
  if (a.model == FO_LINEAR) {
    double At[NC];
    gemv_t_lds<NC>(lds + L.mat, lds + L.xs, At, red, d, d);
    double p = 0.0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      g[c] = i < d ? At[c] - bb[c] + a.lam * th[c] : 0.0;
      if (i < d) p += 0.5 * th[c] * At[c] - bb[c] * th[c] + 0.5 * a.lam * th[c] * th[c];
    }
    return wave_sum_f64(p) + half_yy;
  }
  // logistic: z = X theta, s_j = y_j / (1 + exp(y_j z_j)), f = sum softplus(-y_j z_j), g = -X^T s
  const int m = a.m;
  const double* X = lds + L.mat;
  const double* Yl = X + (long)m * d * (MC > 0 ? 2 : 1);
  double* sv = const_cast<double*>(Yl) + m;
  if constexpr (MC > 0) {
    // z from the transposed copy: lanes own rows j, every wave holds z; no serial wave reductions
    double z[MC];
    gemv_t_lds<MC>(X + (long)m * d, lds + L.xs, z, red, d, m);
    double sp = 0.0;
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      const int j = lane + 64 * c;
      if (j < m) {
        const double yj = Yl[j];
        sp += softplus_f64(-yj * z[c]);
        if (wv == 0) sv[j] = yj / (1.0 + exp(yj * z[c]));
      }
    }
    sp = wave_sum_f64(sp);
    lds_barrier();
    double Xs[NC];
    gemv_t_lds<NC>(X, sv, Xs, red, m, d);
    double q = 0.0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      g[c] = i < d ? -Xs[c] + a.lam * th[c] : 0.0;
      if (i < d) q += th[c] * th[c];
    }
    return 0.5 * a.lam * wave_sum_f64(q) + sp;
  }
  double sp = 0.0;
  for (int j = wv; j < m; j += NWV) {  // m > 128: one wave per row
    double p = 0.0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      if (i < d) p = fma(X[j * d + i], th[c], p);
    }
    const double z = wave_sum_f64(p);
    const double yj = Yl[j];
    sp += softplus_f64(-yj * z);
    if (lane == 0) sv[j] = yj / (1.0 + exp(yj * z));
  }
  if (lane == 0) wred[wv] = sp;
  lds_barrier();
  double Xs[NC];
  gemv_t_lds<NC>(X, sv, Xs, red, m, d);
  double q = 0.0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = lane + 64 * c;
    g[c] = i < d ? -Xs[c] + a.lam * th[c] : 0.0;
    if (i < d) q += th[c] * th[c];
  }
  double f = 0.5 * a.lam * wave_sum_f64(q);
#pragma unroll
  for (int w = 0; w < NWV; ++w) f += wred[w];
  return f;
}

// Spin until every lane's granules of the rows rows[0..nrows) (wave-uniform) carry `tag`, then copy
// them into the LDS table `cache` (row-major, d wide). Returns 1 ok, 0 timeout, -1 the run stopped.
template <int NC, int RB, bool SYS>
__device__ __forceinline__ int fetch_rows(__amdgpu_buffer_rsrc_t rs, int slot_base, const int (&rows)[RB], int nrows,
                                          int d, unsigned tag, double* cache, unsigned long long deadline,
                                          const int* wstop, int it) {
  const int lane = threadIdx.x & 63;
  double v[RB][NC];
  for (int spin = 0;; ++spin) {
    bool ok = true;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      if (r < nrows) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int i = lane + 64 * c;
          if (i < d) ok &= load_granule<SYS>(rs, ((slot_base + rows[r]) * d + i) * 16, tag, &v[r][c]);
        }
      }
    }
    if (__all(ok)) break;
    if ((spin & 15) == 15) {
      if (should_stop(load_word<SYS>(wstop), it)) return -1;
      if (now_ticks() > deadline) return 0;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int r = 0; r < RB; ++r)
    if (r < nrows)
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int i = lane + 64 * c;
        if (i < d) cache[rows[r] * d + i] = v[r][c];
      }
  return 1;
}

// wait_pair (persist_device.h) with the stop word read at SYS scope
template <int NC, bool SYS>
__device__ __forceinline__ int wait_pair_fo(__amdgpu_buffer_rsrc_t rs, int d, int ra, unsigned ta, double (&va)[NC],
                                            int rb, unsigned tb, double (&vb)[NC], unsigned long long deadline,
                                            const int* wstop, int it) {
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
      if (should_stop(load_word<SYS>(wstop), it)) return -1;
      if (now_ticks() > deadline) return 0;
    }
    GADMM_POLL_PAUSE();
  }
}

template <bool SYS>
__device__ void fo_abort(const FoArgs& a) {
  a.ctl->status = 4;
  store_word<SYS>(a.wstop, -1);
  if (SYS && a.nranks > 1 && a.wpush)  // tell every rank (best effort: their own deadlines also fire)
    for (int r = 0; r < a.nranks; ++r)
      if (a.wpush[r]) store_word<true>(a.wpush[r] + 1, -1);
}

}  // namespace

template <int NC, int MC, bool SYS>
__global__ void __launch_bounds__(NT) fo_persistent_kernel(FoArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int flag_lds;
  const int n = a.n, d = a.d, nl = a.n_local;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const unsigned long long deadline = now_ticks() + (unsigned long long)a.timeout_ticks;
  const FoLds L(a.model, a.alg, n, d, a.m, NC, MC);
  const __amdgpu_buffer_rsrc_t rtab = rsrc_of(a.tab);
  const __amdgpu_buffer_rsrc_t rpart = rsrc_of(a.part);
  FoCtl* ctl = a.ctl;
  const bool multi = SYS && a.nranks > 1;
  const bool packed = !SYS && a.xcd > 0;    // XCD packing (FoArgs::xcd)
  if (packed && (blockIdx.x & 7u)) return;  // a spacer block: only b % 8 == 0 work (one XCD)
  const int bid = packed ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  bool local = false;  // publish with plain stores (every block verified on this XCD)
  if (!SYS && a.xcd > 1) local = xcd_verdict(a.xchk, bid, nl + (a.has_monitor ? 1 : 0), deadline, &flag_lds);

  if (a.has_monitor && bid == nl) {
    // ------------------------------------------------------------------ monitor (wave 0 only)
    if (wv != 0) return;
    double* vals = lds;  // [2 n]
    const unsigned long long t0 = now_ticks();
    double uploads = 0.0;
    auto post = [&](int off, int v) {  // progress (off 0) / stop (off 1) word of every rank
      if (multi) {
        for (int r = 0; r < a.nranks; ++r) store_word<true>(a.wpush[r] + off, v);
      } else {
        store_word<SYS>(off == 0 ? a.wmon : a.wstop, v);
      }
    };
    for (int it = 1; it <= a.max_iter; ++it) {
      const unsigned tag = make_tag(a.epoch, it);
      const int slot = it % a.ring;
      bool okall = true;
      for (int w = lane; w < n; w += 64) {
        double f = 0.0, cnt = 0.0;
        for (int spin = 0;; ++spin) {
          const bool ok = load_granule<SYS>(rpart, ((slot * n + w) * 2) * 16, tag, &f) &&
                          load_granule<SYS>(rpart, ((slot * n + w) * 2 + 1) * 16, tag, &cnt);
          if (ok) break;
          if ((spin & 15) == 15 && (now_ticks() > deadline || load_word<SYS>(a.wstop) < 0)) {
            okall = false;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        vals[2 * w] = f;
        vals[2 * w + 1] = cnt;
      }
      if (!__all(okall)) {
        if (lane == 0) {
          fo_abort<SYS>(a);
          ctl->iters = it - 1;
        }
        return;
      }
      int hit = 0;
      if (lane == 0) {
        double s = 0.0, c = 0.0;
        for (int w = 0; w < n; ++w) {  // worker order: deterministic
          s += vals[2 * w];
          c += vals[2 * w + 1];
        }
        uploads += c;
        a.obj_trace[it - 1] = s;
        a.cnt_trace[it - 1] = c;
        a.time_trace[it - 1] = (long long)(now_ticks() - t0);
        ctl->uploads = uploads;
        ctl->iters = it;
        hit = a.has_tol && fabs(s - a.obj0) < a.tol;
        if (hit) {
          ctl->status = 1;
          post(1, it);
        } else if (it == a.max_iter) {
          ctl->status = 2;
        }
        post(0, it);
      }
      if (__shfl(hit, 0, 64)) return;
    }
    return;
  }
  if (bid >= nl) return;

  // -------------------------------------------------------------------- worker workgroup
  const int li = bid, w = a.w_lo + bid;  // local slot, global worker id
  const bool w0 = wv == 0;
  double* xs = lds + L.xs;
  double* dl = lds + L.dl;
  double* cache = lds + L.cache;  // server algorithms: the replicated table of every worker's upload
  if (a.model == FO_LINEAR) {
    const double* Ag = a.A + (long)li * d * d;
    for (int e = threadIdx.x; e < d * d; e += NT) lds[L.mat + e] = Ag[e];
  } else {
    const int m = a.m;
    const double* Xg = a.X + (long)li * m * d;
    for (int e = threadIdx.x; e < m * d; e += NT) lds[L.mat + e] = Xg[e];
    const int yoff = m * d * (MC > 0 ? 2 : 1);
    for (int e = threadIdx.x; e < m; e += NT) lds[L.mat + yoff + e] = a.Y[(long)li * m + e];
    if (MC > 0)
      for (int e = threadIdx.x; e < m * d; e += NT) {  // X^T[i][j] = X[j][i]
        const int i = e / m, j = e % m;
        lds[L.mat + m * d + e] = Xg[(long)j * d + i];
      }
  }
  if (threadIdx.x < 16) dl[threadIdx.x] = 0.0;
  double bb[NC], th[NC], G[NC], aux[NC], g[NC];
  const bool linear = a.model == FO_LINEAR;
  const bool server = is_server_alg(a.alg);
  const bool lagalg = a.alg == FO_LAG_PS || a.alg == FO_LAG_WK;
  // GD_DGD_LAG.m:44-67: the server table / DGD gradients start as ones
  const double g_init = (a.alg == FO_DUALAVG || a.alg == FO_GD) ? 0.0 : (a.faithful || a.alg != FO_DGD ? 1.0 : 0.0);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = lane + 64 * c;
    bb[c] = (linear && i < d) ? a.b[(long)li * d + i] : 0.0;
    th[c] = 0.0;
    aux[c] = 0.0;  // LAG-PS theta_hat / dual averaging Z
    G[c] = i < d ? g_init : 0.0;
    if (i < d && w0) xs[i] = 0.0;
  }
  if (server)
    for (int e = threadIdx.x; e < n * d; e += NT) cache[e] = g_init;
  const double half_yy = linear ? 0.5 * a.yy[li] : 0.0;
  const double hsq = a.alg == FO_LAG_PS ? a.hsq[w] : 0.0;
  // ranks this worker's upload rows go to besides its own: every other rank (server algorithms), the
  // chain neighbours' ranks (DGD, dual averaging); up to 2 + a bitmask for the server case
  const int left_rank = (multi && w > 0) ? a.owner[w - 1] : a.my_rank;
  const int right_rank = (multi && w < n - 1) ? a.owner[w + 1] : a.my_rank;
  const int nb0 = left_rank != a.my_rank ? left_rank : -1;
  const int nb1 = (right_rank != a.my_rank && right_rank != nb0) ? right_rank : -1;
  double rows_pushed = 0.0, flags_pushed = 0.0;  // granule rows stored into OTHER ranks' tables
  // one upload row (granules of element i = lane + 64 c) into own + the readers' tables
  auto publish_row = [&](int gidx_row, unsigned tag, const double (&v)[NC]) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      if (i < d) put_granule<SYS>(local, rtab, (gidx_row * d + i) * 16, tag, v[c]);
    }
    if (!multi) return;
    for (int r = 0; r < a.nranks; ++r) {
      if (r == a.my_rank || !(server || r == nb0 || r == nb1)) continue;
      const __amdgpu_buffer_rsrc_t rr = rsrc_of(a.tab_push[r]);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int i = lane + 64 * c;
        if (i < d) store_granule<true>(rr, (gidx_row * d + i) * 16, tag, v[c]);
      }
      rows_pushed += 1.0;
    }
  };
  // LAG upload flag of iteration `tag` (slot): 1 = this worker's row changed (granule after the rows)
  auto publish_flag = [&](int slot, unsigned tag, double f) {
    const int off = (a.slots * n * d + slot * n + w) * 16;
    put_granule<SYS>(local, rtab, off, tag, f);
    if (!multi) return;
    for (int r = 0; r < a.nranks; ++r) {
      if (r == a.my_rank) continue;
      store_granule<true>(rsrc_of(a.tab_push[r]), off, tag, f);
      flags_pushed += 1.0;
    }
  };
  lds_barrier();
  double f = 0.0;
  if (a.alg == FO_DUALAVG) f = local_eval<NC, MC>(a, lds, L, th, bb, half_yy, g);  // grad at theta^0 = 0

  int mon_seen = 0;
  for (int it = 1; it <= a.max_iter; ++it) {
    // the stop word is loaded here and tested at the end of the iteration: its latency hides
    // behind the local evaluation (workers may run one iteration past the stop; the traces are the
    // monitor's, so results are unaffected)
    const int sw = threadIdx.x == 0 ? load_word<SYS>(a.wstop) : 0;
    const unsigned tag = make_tag(a.epoch, it);
    const int slot = it % a.slots;  // upload rows
    const int fslot = it & 1;       // LAG flags
    double cnt = 0.0;
    double pub[NC];
    bool upload = false;  // this worker's server-table row changes in this iteration
    if (a.alg != FO_DUALAVG) {
      f = local_eval<NC, MC>(a, lds, L, th, bb, half_yy, g);
      if (a.alg == FO_GD) {
        upload = true;
        if (it == 1 && a.faithful) {  // linear: ones; logistic: worker 1's gradient (GD_DGD_LAG_logistic.m:97)
#pragma unroll
          for (int c = 0; c < NC; ++c) pub[c] = w == 0 ? (linear ? (lane + 64 * c < d ? 1.0 : 0.0) : g[c]) : 0.0;
        } else {
#pragma unroll
          for (int c = 0; c < NC; ++c) pub[c] = g[c];
        }
      } else if (a.alg == FO_DGD) {
        if (it > 1 || !a.faithful)
#pragma unroll
          for (int c = 0; c < NC; ++c) G[c] = g[c];
#pragma unroll
        for (int c = 0; c < NC; ++c) pub[c] = G[c];
      } else if (a.alg == FO_IAG) {
        upload = it > 1 && a.sched[it - 1] == w;
        if (upload)
#pragma unroll
          for (int c = 0; c < NC; ++c) G[c] = g[c];
#pragma unroll
        for (int c = 0; c < NC; ++c) pub[c] = G[c];
      } else {  // LAG-PS / LAG-WK (GD_DGD_LAG.m:184-327)
        bool mask = false;
        if (it > LAG_SLOT) {
          double trig = 0.0;
          for (int k = 1; k <= LAG_SLOT; ++k) trig += dl[(it - k) % LAG_SLOT];  // newest first
          double dd = 0.0;
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            const double e = a.alg == FO_LAG_PS ? aux[c] - th[c] : g[c] - G[c];
            dd += e * e;
          }
          dd = wave_sum_f64(dd);
          mask = a.alg == FO_LAG_PS ? hsq * dd > a.thrd * trig : dd > a.thrd * trig;
        }
        const bool forced = a.alg == FO_LAG_PS && a.faithful && it > 1 && w == 0;  // quirk 4 (:204-209)
        upload = mask || forced;
        if (upload)
#pragma unroll
          for (int c = 0; c < NC; ++c) G[c] = g[c];
        if (mask && a.alg == FO_LAG_PS)
#pragma unroll
          for (int c = 0; c < NC; ++c) aux[c] = th[c];
        cnt = mask ? 1.0 : 0.0;
#pragma unroll
        for (int c = 0; c < NC; ++c) pub[c] = G[c];
      }
    } else {
      // dual averaging: mix neighbours' Z (no self weight), theta = -alpha Z (dual_averaging.m:34-44)
      bool has_l = w > 0, has_r = w < n - 1;
      double zl[NC], zr[NC];
      int ok = 1;
      if (w0) {
#pragma unroll
        for (int c = 0; c < NC; ++c) zl[c] = zr[c] = 0.0;
        const int lit = a.jacobi ? it - 1 : it;
        const int rl = (has_l && (!a.jacobi || it > 1)) ? ((lit % a.slots) * n) + w - 1 : -1;
        const int rr = (has_r && it > 1) ? (((it - 1) % a.slots) * n) + w + 1 : -1;
        ok = wait_pair_fo<NC, SYS>(rtab, d, rl, make_tag(a.epoch, lit), zl, rr, make_tag(a.epoch, it - 1), zr,
                                   deadline, a.wstop, it);
        if (lane == 0) flag_lds = ok;
      }
      lds_barrier();
      ok = flag_lds;
      if (ok != 1) {
        if (ok == 0 && threadIdx.x == 0) fo_abort<SYS>(a);
        break;
      }
      if (w0) {
        double zrow[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int i = lane + 64 * c;
          double z;
          if (!has_l && !has_r) z = g[c];
          else if (!has_l) z = zr[c] + g[c];
          else if (!has_r) z = zl[c] + g[c];
          else z = 0.5 * zr[c] + 0.5 * zl[c] + g[c];
          aux[c] = i < d ? z : 0.0;
          th[c] = i < d ? -a.step * z : 0.0;
          zrow[c] = aux[c];
          if (i < d) xs[i] = th[c];
        }
        publish_row(slot * n + w, tag, zrow);
      }
      lds_barrier();
      // every wave needs theta in registers for local_eval
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int i = lane + 64 * c;
        th[c] = i < d ? xs[i] : 0.0;
      }
      f = local_eval<NC, MC>(a, lds, L, th, bb, half_yy, g);
    }

    // ---- publish the upload (server algorithms: only a changed row, + the LAG flag; DGD: the
    // gradient row) and (f_n, count) to the monitor
    if (w0) {
      if (a.alg == FO_DGD || upload) publish_row(slot * n + w, tag, pub);
      if (lagalg) publish_flag(fslot, tag, upload ? 1.0 : 0.0);
      int ok = 1;
      if (mon_seen < it - a.ring) {  // back-pressure: slot it % ring must have been consumed by the monitor
        for (int spin = 0;; ++spin) {
          mon_seen = load_word<SYS>(a.wmon);
          if (mon_seen >= it - a.ring) break;
          if ((spin & 15) == 15) {
            if (should_stop(load_word<SYS>(a.wstop), it)) { ok = -1; break; }
            if (now_ticks() > deadline) { ok = 0; break; }
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      if (ok == 1 && lane == 0) {
        const int ps = it % a.ring;
        put_granule<SYS>(local, rpart, ((ps * n + w) * 2) * 16, tag, f);
        put_granule<SYS>(local, rpart, ((ps * n + w) * 2 + 1) * 16, tag, cnt);
      }
      if (lane == 0) flag_lds = ok;
    }
    lds_barrier();
    if (flag_lds != 1) {
      if (flag_lds == 0 && threadIdx.x == 0) fo_abort<SYS>(a);
      break;
    }
    if (a.alg != FO_DUALAVG) {
    // ---- consume: server step (replicated) or neighbour average (DGD)
    double S[NC];
    int ok = 1;
    if (server) {
      // wave wv owns table rows r = wv (mod NWV): it fetches the ones that changed in this iteration
      // (GD: all; IAG: the scheduled worker's; LAG: the flagged ones) into the LDS table, then sums
      // its rows in ascending order; the wave partials are combined in wave order (one fixed order)
      constexpr int RB = 8;
      const int nmine = (n - wv + NWV - 1) / NWV;  // rows wv, wv + NWV, ...
      unsigned long long chg = 0ull;               // bit j: row wv + NWV j changed (j < 64)
      if (a.alg == FO_GD) {
        chg = nmine >= 64 ? ~0ull : ((1ull << nmine) - 1ull);
      } else if (a.alg == FO_IAG) {
        const int s = it > 1 ? a.sched[it - 1] : -1;
        if (s >= 0 && s % NWV == wv) chg = 1ull << (s / NWV);
      } else {  // LAG: poll the flags of this wave's rows (lane j: row wv + NWV j)
        double fl = 0.0;
        bool okf = true;
        const int row = wv + NWV * lane;
        for (int spin = 0;; ++spin) {
          okf = lane >= nmine || load_granule<SYS>(rtab, (a.slots * n * d + fslot * n + row) * 16, tag, &fl);
          if (__all(okf)) break;
          if ((spin & 15) == 15) {
            if (should_stop(load_word<SYS>(a.wstop), it)) { ok = -1; break; }
            if (now_ticks() > deadline) { ok = 0; break; }
          }
          __builtin_amdgcn_s_sleep(1);
        }
        chg = __ballot(lane < nmine && fl != 0.0);
      }
      int rows[RB];
      int k = 0;
      for (int j = 0; j < 64 && ok == 1; ++j) {
        if (!((chg >> j) & 1ull)) continue;
        rows[k++] = wv + NWV * j;
        if (k == RB) {
          ok = fetch_rows<NC, RB, SYS>(rtab, slot * n, rows, k, d, tag, cache, deadline, a.wstop, it);
          k = 0;
        }
      }
      if (ok == 1 && k > 0) ok = fetch_rows<NC, RB, SYS>(rtab, slot * n, rows, k, d, tag, cache, deadline, a.wstop, it);
      double acc[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[c] = 0.0;
      for (int r = wv; r < n; r += NWV)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int i = lane + 64 * c;
          if (i < d) acc[c] += cache[r * d + i];
        }
      double* red = lds + L.red;
#pragma unroll
      for (int c = 0; c < NC; ++c) red[(wv * NC + c) * 64 + lane] = acc[c];
      if (lane == 0) lds[L.wred + wv] = (double)ok;
      lds_barrier();
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < NWV; ++q) s += red[(q * NC + c) * 64 + lane];  // fixed order
        S[c] = s;
      }
      for (int q = 0; q < NWV; ++q) ok = min(ok, (int)lds[L.wred + q]);
      lds_barrier();
    } else {  // DGD: average with the chain neighbours' gradients (GD_DGD_LAG.m:155-171)
      double gl[NC], gr[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) gl[c] = gr[c] = 0.0;
      ok = wait_pair_fo<NC, SYS>(rtab, d, w > 0 ? slot * n + w - 1 : -1, tag, gl, w < n - 1 ? slot * n + w + 1 : -1,
                                 tag, gr, deadline, a.wstop, it);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (n == 1) S[c] = G[c];
        else if (w == 0) S[c] = G[c] + gr[c];
        else if (w == n - 1) S[c] = G[c] + gl[c];
        else S[c] = G[c] + gr[c] + gl[c];
      }
      if (lane == 0) lds[L.wred + wv] = (double)ok;
      lds_barrier();
      for (int q = 0; q < NWV; ++q) ok = min(ok, (int)lds[L.wred + q]);
      lds_barrier();
    }
    if (ok != 1) {
      if (ok == 0 && threadIdx.x == 0) fo_abort<SYS>(a);
      break;
    }
    double coef = a.step;
    if (a.alg == FO_DGD && n > 1) coef = (w == 0 || w == n - 1) ? 0.5 * a.step : (1.0 / 3.0) * a.step;
    double dsq = 0.0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      const double nt = i < d ? th[c] - coef * S[c] : 0.0;
      const double e = nt - th[c];
      dsq += e * e;
      th[c] = nt;
    }
    if (lagalg) {
      dsq = wave_sum_f64(dsq);
      if (threadIdx.x == 0) dl[it % LAG_SLOT] = dsq;  // ||theta^it - theta^{it-1}||^2
    }
    if (w0)
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int i = lane + 64 * c;
        if (i < d) xs[i] = th[c];
      }
    }  // consume
    if (threadIdx.x == 0) flag_lds = should_stop(sw, it + 1);
    lds_barrier();
    if (flag_lds) break;
  }
  if (w0)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int i = lane + 64 * c;
      if (i < d) a.theta_out[(long)li * d + i] = th[c];
    }
  if (threadIdx.x == 0 && a.pushc) {
    a.pushc[2 * li] = rows_pushed;
    a.pushc[2 * li + 1] = flags_pushed;
  }
}

extern "C" int gadmm_xcd_pick(int want, int multi, int blocks, long cap_total, const void* xchk);  // chain_persistent.hip

extern "C" {

static int fo_mc(int model, int m) { return model == FO_LINEAR ? 0 : (m <= 64 ? 1 : (m <= 128 ? 2 : 0)); }

long gadmm_fo_lds(int model, int alg, int n, int d, int m) {
  const int nc = d <= 64 ? 1 : 2;
  const FoLds L(model, alg, n, d, m, nc, fo_mc(model, m));
  long b = (long)L.total * 8;
  if (b < 16L * n + 64) b = 16L * n + 64;  // the monitor stages 2 doubles per worker
  return b;
}

// Granules of a rank's upload table: [slots][n][d] rows + [2][n] LAG flags.
long gadmm_fo_tab_granules(int n, int d, int slots) { return (long)slots * n * d + 2L * n; }

int gadmm_fo_abi_layout(long long* out, int n) {
  long long v[] = {(long long)sizeof(FoCtl), (long long)sizeof(FoArgs), (long long)offsetof(FoArgs, step),
                   (long long)offsetof(FoArgs, timeout_ticks), (long long)offsetof(FoArgs, A),
                   (long long)offsetof(FoArgs, ctl), (long long)offsetof(FoArgs, xchk),
                   (long long)offsetof(FoArgs, nranks), (long long)offsetof(FoArgs, owner),
                   (long long)offsetof(FoArgs, pushc)};
  const int k = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < n && i < k; ++i) out[i] = v[i];
  return k;
}

// Launch one run (one rank's share of it). Returns 0, or a negative code when the configuration is
// outside the engine (d > 128, LDS overflow, the grid cannot be co-resident, a multi-rank field
// missing): the caller then uses the torch path.
int gadmm_fo_launch(const FoArgs* a, void* stream) {
  if (a->d < 1 || a->d > 128 || a->n < 1 || a->ring < 2 || a->max_iter >= (1 << 20)) return -2;
  if (a->n_local < 1 || a->w_lo < 0 || a->w_lo + a->n_local > a->n || !a->wmon || !a->wstop) return -2;
  if (a->slots < 2 || (a->alg == FO_IAG && a->slots < a->ring + 3)) return -2;
  const bool multi = a->nranks > 1;
  if (multi && (!a->owner || !a->tab_push || a->my_rank < 0 || a->my_rank >= a->nranks ||
                (a->has_monitor && !a->wpush)))
    return -2;
  if (!multi && (a->n_local != a->n || !a->has_monitor)) return -2;
  if (a->alg != FO_DUALAVG && a->alg != FO_DGD && a->n > 64 * NWV) return -2;  // the changed-row bitmask
  const long lds = gadmm_fo_lds(a->model, a->alg, a->n, a->d, a->m);
  if (lds > 160 * 1024 - 1024) return -3;
  const long ncu = gadmm_cu_count();
  if (ncu <= 0) return -4;
  int per_cu = 0;
  const int mc = fo_mc(a->model, a->m);
  const void* fns[2][2][3] = {
      {{(const void*)fo_persistent_kernel<1, 0, false>, (const void*)fo_persistent_kernel<1, 1, false>,
        (const void*)fo_persistent_kernel<1, 2, false>},
       {(const void*)fo_persistent_kernel<2, 0, false>, (const void*)fo_persistent_kernel<2, 1, false>,
        (const void*)fo_persistent_kernel<2, 2, false>}},
      {{(const void*)fo_persistent_kernel<1, 0, true>, (const void*)fo_persistent_kernel<1, 1, true>,
        (const void*)fo_persistent_kernel<1, 2, true>},
       {(const void*)fo_persistent_kernel<2, 0, true>, (const void*)fo_persistent_kernel<2, 1, true>,
        (const void*)fo_persistent_kernel<2, 2, true>}}};
  const int nci = a->d <= 64 ? 0 : 1;
  const void* fn = fns[multi ? 1 : 0][nci][mc];
  const int blocks = a->n_local + (a->has_monitor ? 1 : 0);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, NT, (size_t)lds) != hipSuccess) return -4;
  if ((long)per_cu * ncu < blocks) return -5;  // persistent: all must be resident
  if (lds > 65536 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -3;
  FoArgs ka = *a;
  ka.xcd = multi ? 0 : gadmm_xcd_pick(a->xcd, 0, blocks, (long)per_cu * ncu, a->xchk);
  if (ka.xcd > 1 && hipMemsetAsync(a->xchk, 0, (size_t)XCHK * 16, (hipStream_t)stream) != hipSuccess) return -1;
  void* args[] = {&ka};
  if (hipLaunchKernel(fn, dim3(ka.xcd > 0 ? 8 * blocks : blocks), dim3(NT), args, (size_t)lds, (hipStream_t)stream) !=
      hipSuccess)
    return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
