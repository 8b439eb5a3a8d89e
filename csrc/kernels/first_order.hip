// Persistent first-order baseline engine: GD, DGD, LAG-PS, LAG-WK, cyclic / randomized IAG and dual
// averaging (linear and logistic) in ONE launch per run.
//
// Reference semantics: GD_DGD_LAG.m / GD_DGD_LAG_logistic.m (A10, A11), dual_averaging.m /
// dual_averaging_logisticReg.m (A8, A9), as implemented by gadmm_amd/algorithms/baselines.py and
// dual_averaging.py, which stay the multi-rank path and the test oracle.
//
// Why one kernel: the reference runs these for 40k-500k iterations of d = 14..50 arithmetic; as
// torch ops each iteration is a dozen launches plus a host read of the objective (~100 us), as a
// persistent kernel it is one L2 round trip (~2-4 us).
//
// Layout: workgroup n < N is worker n and keeps its Gram (linear) or its shard X_n, y_n (logistic)
// in LDS for the whole run; workgroup N is the monitor. Per iteration every worker evaluates
// grad f_n and f_n at its point, publishes what the algorithm uploads as 16-byte data-is-flag
// granules ({tag, lo, tag, hi}, tag = epoch:iteration; persist_device.h), and publishes (f_n,
// trigger) to the monitor ring. Replicated-server algorithms (GD, LAG, IAG) read every worker's row
// and apply the server step themselves: every workgroup sums the rows in the same fixed order, so
// theta stays bit-identical across workgroups without a broadcast. DGD reads its chain neighbours'
// gradients; dual averaging reads the left neighbour's current-sweep Z and the right neighbour's
// previous-sweep Z (the Gauss-Seidel wavefront of dual_averaging.m:44) or both previous (Jacobi).
// Two table slots suffice: a producer can only overwrite slot it&1 at it+2, which needs data that
// every reader of `it` publishes after its read.
// The monitor sums f_n in worker order, records the objective / trigger / clock traces and posts
// the stop iteration (|obj - obj0| < tol); workers leave once they see it. The objective ring has
// `ring` slots with back-pressure on the monitor's progress. Every spin has a wall-clock deadline.
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

__device__ __forceinline__ int stop_word(const FoCtl* c) {
  return __hip_atomic_load(&c->stop_iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool should_stop(int s, int it) { return s < 0 || (s > 0 && it > s); }

// LDS layout (doubles) shared by host sizing (gadmm_fo_lds) and the kernel.
struct FoLds {
  int mat, xs, aux, red, wred, dl, total;
  __host__ __device__ FoLds(int model, int d, int m, int nc, int mc) {
    mat = 0;
    // linear: A | logistic: X (m x d) | X^T (d x m, when mc > 0) | y | s
    const int msz = model == FO_LINEAR ? d * d : m * d * (mc > 0 ? 2 : 1) + 2 * m;
    xs = (msz + 1) & ~1;
    aux = xs + 64 * nc;
    red = aux + 64 * nc;
    wred = red + NWV * nc * 64;
    dl = wred + 8;
    total = dl + 16;
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

// Spin until every lane's granules of `nrows` rows (row r = row0 + rstep * r) carry `tag`.
// Returns 1 ok, 0 timeout, -1 the run stopped. Wave-uniform.
template <int NC, int RB>
__device__ __forceinline__ int wait_rows(__amdgpu_buffer_rsrc_t rs, int row0, int rstep, int nrows, int d,
                                         unsigned tag, double (&v)[RB][NC], unsigned long long deadline,
                                         const FoCtl* ctl, int it) {
  const int lane = threadIdx.x & 63;
  for (int spin = 0;; ++spin) {
    bool ok = true;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      if (r < nrows) {
        const int row = row0 + rstep * r;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int i = lane + 64 * c;
          if (i < d) ok &= load_granule<false>(rs, (row * d + i) * 16, tag, &v[r][c]);
          else v[r][c] = 0.0;
        }
      }
    }
    if (__all(ok)) return 1;
    if ((spin & 15) == 15) {
      if (should_stop(stop_word(ctl), it)) return -1;
      if (now_ticks() > deadline) return 0;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ void fo_abort(FoCtl* ctl) {
  __hip_atomic_store(&ctl->status, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&ctl->stop_iter, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

template <int NC, int MC>
__global__ void __launch_bounds__(NT) fo_persistent_kernel(FoArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int flag_lds;
  const int n = a.n, d = a.d;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const unsigned long long deadline = now_ticks() + (unsigned long long)a.timeout_ticks;
  const FoLds L(a.model, d, a.m, NC, MC);
  const __amdgpu_buffer_rsrc_t rtab = rsrc_of(a.tab);
  const __amdgpu_buffer_rsrc_t rpart = rsrc_of(a.part);
  FoCtl* ctl = a.ctl;
  const bool packed = a.xcd > 0;            // XCD packing (FoArgs::xcd)
  if (packed && (blockIdx.x & 7u)) return;  // a spacer block: only b % 8 == 0 work (one XCD)
  const int bid = packed ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  bool local = false;  // publish with plain stores (every block verified on this XCD)
  if (a.xcd > 1) local = xcd_verdict(a.xchk, bid, n + 1, deadline, &flag_lds);

  if (bid == n) {
    // ------------------------------------------------------------------ monitor (wave 0 only)
    if (wv != 0) return;
    double* vals = lds;  // [2 n]
    const unsigned long long t0 = now_ticks();
    double uploads = 0.0;
    for (int it = 1; it <= a.max_iter; ++it) {
      const unsigned tag = make_tag(a.epoch, it);
      const int slot = it % a.ring;
      bool okall = true;
      for (int w = lane; w < n; w += 64) {
        double f = 0.0, cnt = 0.0;
        for (int spin = 0;; ++spin) {
          const bool ok = load_granule<false>(rpart, ((slot * n + w) * 2) * 16, tag, &f) &&
                          load_granule<false>(rpart, ((slot * n + w) * 2 + 1) * 16, tag, &cnt);
          if (ok) break;
          if ((spin & 15) == 15 && (now_ticks() > deadline || stop_word(ctl) < 0)) {
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
          fo_abort(ctl);
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
        __hip_atomic_store(&ctl->monitored, it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        hit = a.has_tol && fabs(s - a.obj0) < a.tol;
        if (hit) {
          ctl->status = 1;
          __hip_atomic_store(&ctl->stop_iter, it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (it == a.max_iter) {
          ctl->status = 2;
        }
      }
      if (__shfl(hit, 0, 64)) return;
    }
    return;
  }

  // -------------------------------------------------------------------- worker workgroup
  const int w = bid;
  const bool w0 = wv == 0;
  double* xs = lds + L.xs;
  double* dl = lds + L.dl;
  if (a.model == FO_LINEAR) {
    const double* Ag = a.A + (long)w * d * d;
    for (int e = threadIdx.x; e < d * d; e += NT) lds[L.mat + e] = Ag[e];
  } else {
    const int m = a.m;
    const double* Xg = a.X + (long)w * m * d;
    for (int e = threadIdx.x; e < m * d; e += NT) lds[L.mat + e] = Xg[e];
    const int yoff = m * d * (MC > 0 ? 2 : 1);
    for (int e = threadIdx.x; e < m; e += NT) lds[L.mat + yoff + e] = a.Y[(long)w * m + e];
    if (MC > 0)
      for (int e = threadIdx.x; e < m * d; e += NT) {  // X^T[i][j] = X[j][i]
        const int i = e / m, j = e % m;
        lds[L.mat + m * d + e] = Xg[(long)j * d + i];
      }
  }
  if (threadIdx.x < 16) dl[threadIdx.x] = 0.0;
  double bb[NC], th[NC], G[NC], aux[NC], g[NC];
  const bool linear = a.model == FO_LINEAR;
  const bool replicated = a.alg == FO_GD || a.alg == FO_LAG_PS || a.alg == FO_LAG_WK || a.alg == FO_IAG;
  // GD_DGD_LAG.m:44-67: the server table / DGD gradients start as ones
  const double g_init = (a.alg == FO_DUALAVG || a.alg == FO_GD) ? 0.0 : (a.faithful || a.alg != FO_DGD ? 1.0 : 0.0);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int i = lane + 64 * c;
    bb[c] = (linear && i < d) ? a.b[(long)w * d + i] : 0.0;
    th[c] = 0.0;
    aux[c] = 0.0;  // LAG-PS theta_hat / dual averaging Z
    G[c] = i < d ? g_init : 0.0;
    if (i < d && w0) xs[i] = 0.0;
  }
  const double half_yy = linear ? 0.5 * a.yy[w] : 0.0;
  const double hsq = a.alg == FO_LAG_PS ? a.hsq[w] : 0.0;
  lds_barrier();
  double f = 0.0;
  if (a.alg == FO_DUALAVG) f = local_eval<NC, MC>(a, lds, L, th, bb, half_yy, g);  // grad at theta^0 = 0

  int mon_seen = 0;
  for (int it = 1; it <= a.max_iter; ++it) {
    // the stop word is loaded here and tested at the end of the iteration: its L2 latency hides
    // behind the local evaluation (workers may run one iteration past the stop; the traces are the
    // monitor's, so results are unaffected)
    const int sw = threadIdx.x == 0 ? stop_word(ctl) : 0;
    const unsigned tag = make_tag(a.epoch, it);
    const int slot = it & 1;
    double cnt = 0.0;
    double pub[NC];
    if (a.alg != FO_DUALAVG) {
      f = local_eval<NC, MC>(a, lds, L, th, bb, half_yy, g);
      if (a.alg == FO_GD) {
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
        if (it > 1 && a.sched[it - 1] == w)
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
        if (mask || forced)
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
      double zl[1][NC], zr[1][NC];
      int ok = 1;
      if (w0) {
#pragma unroll
        for (int c = 0; c < NC; ++c) zl[0][c] = zr[0][c] = 0.0;
        const int lit = a.jacobi ? it - 1 : it;
        const int rl = (has_l && (!a.jacobi || it > 1)) ? ((lit & 1) * n) + w - 1 : -1;
        const int rr = (has_r && it > 1) ? (((it - 1) & 1) * n) + w + 1 : -1;
        ok = wait_pair<NC, false>(rtab, d, rl, make_tag(a.epoch, lit), zl[0], rr, make_tag(a.epoch, it - 1), zr[0],
                                  deadline, &ctl->stop_iter, it);
        if (lane == 0) flag_lds = ok;
      }
      lds_barrier();
      ok = flag_lds;
      if (ok != 1) {
        if (ok == 0 && threadIdx.x == 0) fo_abort(ctl);
        break;
      }
      if (w0) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int i = lane + 64 * c;
          double z;
          if (!has_l && !has_r) z = g[c];
          else if (!has_l) z = zr[0][c] + g[c];
          else if (!has_r) z = zl[0][c] + g[c];
          else z = 0.5 * zr[0][c] + 0.5 * zl[0][c] + g[c];
          aux[c] = i < d ? z : 0.0;
          th[c] = i < d ? -a.step * z : 0.0;
          if (i < d) {
            xs[i] = th[c];
            put_granule<false>(local, rtab, ((slot * n + w) * d + i) * 16, tag, z);
          }
        }
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

    // ---- publish the upload row (replicated / DGD) and (f_n, count) to the monitor
    if (w0) {
      if (a.alg != FO_DUALAVG) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int i = lane + 64 * c;
          if (i < d) put_granule<false>(local, rtab, ((slot * n + w) * d + i) * 16, tag, pub[c]);
        }
      }
      int ok = 1;
      if (mon_seen < it - a.ring) {  // back-pressure: slot it % ring must have been consumed by the monitor
        for (int spin = 0;; ++spin) {
          mon_seen = __hip_atomic_load(&ctl->monitored, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (mon_seen >= it - a.ring) break;
          if ((spin & 15) == 15) {
            if (should_stop(stop_word(ctl), it)) { ok = -1; break; }
            if (now_ticks() > deadline) { ok = 0; break; }
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      if (ok == 1 && lane == 0) {
        const int ps = it % a.ring;
        put_granule<false>(local, rpart, ((ps * n + w) * 2) * 16, tag, f);
        put_granule<false>(local, rpart, ((ps * n + w) * 2 + 1) * 16, tag, cnt);
      }
      if (lane == 0) flag_lds = ok;
    }
    lds_barrier();
    if (flag_lds != 1) {
      if (flag_lds == 0 && threadIdx.x == 0) fo_abort(ctl);
      break;
    }
    if (a.alg != FO_DUALAVG) {
    // ---- consume: server step (replicated) or neighbour average (DGD)
    double S[NC];
    int ok = 1;
    if (replicated) {
      constexpr int RB = 8;
      double acc[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[c] = 0.0;
      for (int base = wv; base < n && ok == 1; base += NWV * RB) {
        const int nr = min(RB, (n - base + NWV - 1) / NWV);
        double v[RB][NC];
        ok = wait_rows<NC, RB>(rtab, slot * n + base, NWV, nr, d, tag, v, deadline, ctl, it);
        if (ok == 1)
#pragma unroll
          for (int r = 0; r < RB; ++r)
            if (r < nr)
#pragma unroll
              for (int c = 0; c < NC; ++c) acc[c] += v[r][c];
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
      double gl[1][NC], gr[1][NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) gl[0][c] = gr[0][c] = 0.0;
      ok = wait_pair<NC, false>(rtab, d, w > 0 ? slot * n + w - 1 : -1, tag, gl[0], w < n - 1 ? slot * n + w + 1 : -1, tag,
                                gr[0], deadline, &ctl->stop_iter, it);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (n == 1) S[c] = G[c];
        else if (w == 0) S[c] = G[c] + gr[0][c];
        else if (w == n - 1) S[c] = G[c] + gl[0][c];
        else S[c] = G[c] + gr[0][c] + gl[0][c];
      }
      if (lane == 0) lds[L.wred + wv] = (double)ok;
      lds_barrier();
      for (int q = 0; q < NWV; ++q) ok = min(ok, (int)lds[L.wred + q]);
      lds_barrier();
    }
    if (ok != 1) {
      if (ok == 0 && threadIdx.x == 0) fo_abort(ctl);
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
    if (a.alg == FO_LAG_PS || a.alg == FO_LAG_WK) {
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
      if (i < d) a.theta_out[(long)w * d + i] = th[c];
    }
}

extern "C" int gadmm_xcd_pick(int want, int multi, int blocks, long cap_total, const void* xchk);  // chain_persistent.hip

extern "C" {

static int fo_mc(int model, int m) { return model == FO_LINEAR ? 0 : (m <= 64 ? 1 : (m <= 128 ? 2 : 0)); }

long gadmm_fo_lds(int model, int d, int m) {
  const int nc = d <= 64 ? 1 : 2;
  const FoLds L(model, d, m, nc, fo_mc(model, m));
  return (long)L.total * 8;
}

int gadmm_fo_abi_layout(long long* out, int n) {
  long long v[] = {(long long)sizeof(FoCtl), (long long)sizeof(FoArgs), (long long)offsetof(FoArgs, step),
                   (long long)offsetof(FoArgs, timeout_ticks), (long long)offsetof(FoArgs, A),
                   (long long)offsetof(FoArgs, ctl), (long long)offsetof(FoArgs, xchk)};
  const int k = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < n && i < k; ++i) out[i] = v[i];
  return k;
}

// Launch one run. Returns 0, or a negative code when the configuration is outside the engine
// (d > 128, LDS overflow, the grid cannot be co-resident): the caller then uses the torch path.
int gadmm_fo_launch(const FoArgs* a, void* stream) {
  if (a->d < 1 || a->d > 128 || a->n < 1 || a->ring < 2 || a->max_iter >= (1 << 20)) return -2;
  long lds = gadmm_fo_lds(a->model, a->d, a->m);
  if (lds < 16L * a->n + 64) lds = 16L * a->n + 64;  // the monitor stages 2 doubles per worker
  if (lds > 160 * 1024 - 1024) return -3;
  const long ncu = gadmm_cu_count();
  if (ncu <= 0) return -4;
  int per_cu = 0;
  const int mc = fo_mc(a->model, a->m);
  const void* fns[2][3] = {{(const void*)fo_persistent_kernel<1, 0>, (const void*)fo_persistent_kernel<1, 1>,
                            (const void*)fo_persistent_kernel<1, 2>},
                           {(const void*)fo_persistent_kernel<2, 0>, (const void*)fo_persistent_kernel<2, 1>,
                            (const void*)fo_persistent_kernel<2, 2>}};
  const int nci = a->d <= 64 ? 0 : 1;
  const void* fn = fns[nci][mc];
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, NT, (size_t)lds) != hipSuccess) return -4;
  if ((long)per_cu * ncu < a->n + 1) return -5;  // persistent: all must be resident
  FoArgs ka = *a;
  ka.xcd = gadmm_xcd_pick(a->xcd, 0, a->n + 1, (long)per_cu * ncu, a->xchk);
  if (ka.xcd > 1 && hipMemsetAsync(a->xchk, 0, (size_t)XCHK * 16, (hipStream_t)stream) != hipSuccess) return -1;
  void* args[] = {&ka};
  if (hipLaunchKernel(fn, dim3(ka.xcd > 0 ? 8 * (a->n + 1) : a->n + 1), dim3(NT), args, (size_t)lds, (hipStream_t)stream) !=
      hipSuccess)
    return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
