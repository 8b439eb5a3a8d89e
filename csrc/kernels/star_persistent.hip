// Persistent star (parameter-server) ADMM, closed form -- standared_ADMM.m in ONE
// launch per GPU, the comparator of LinearRegression_gadmm_vs_admm.m and BASELINE configs[4].
//
// Worker n-1 is the hub and also owns a shard. Per iteration i (standared_ADMM.m:17-88):
//   workers  theta_n = (A_n + rho I)^-1 (b_n - lam_n + rho theta_hub^{i-1})         (:42)
//   hub      theta_h = (A_h + (n-1) rho I)^-1 (b_h + sum lam_n + rho sum theta_n)   (:66-73)
//   duals    lam_n += rho (theta_n - theta_h)                                        (:84-88)
//   stop     |sum_n f_n(theta_n) - obj0| < tol                                       (:95-107)
// Roles are resident workgroups: a worker (one wave) keeps (A_n + rho I)^-1 and A_n in VGPRs (the
// quad layout of quad_gemv.h, d <= 64) and uploads theta_n (d doubles) as tagged 16-byte granules into
// the hub rank's table; the hub's helper waves poll those n-1 rows and sum them (fixed order: rows of
// each helper in row order, then the helpers' partials in wave order); its wave 0 solves and
// publishes theta_h into EVERY rank's table (the broadcast). A worker applies its dual update lazily
// at the start of the next iteration, when it reads theta_h^i anyway; the hub keeps its own copies
// of the n-1 duals (same arithmetic, bit-identical), so an upload is theta alone (the reference's
// "N-1 uploads + N-1 downloads" per iteration). Objectives go to the monitor as in
// chain_persistent.hip (stop decision of iteration i - lag gates iteration i: every wave leaves at
// the same boundary). Multi-GPU: the tables are IPC-mapped fine-grained buffers (parallel/xgmi.py),
// the granule stores travel over xGMI. Every spin has a deadline (done = 4).
// Table slots: a single row per worker suffices -- worker n writes theta_n^{i+1} only after it read
// theta_h^i, which the hub publishes only after it read every theta_n^i.
#include "gadmm_common.h"
#include "gadmm_chain.h"
#include "gadmm_star.h"
#include "persist_device.h"
#include <stdlib.h>
#include <cstddef>

constexpr int SB = 8;  // hub: upload rows polled per batch by each hub wave
// Waves per workgroup. The hub's HW - 1 helper waves poll its n - 1 upload rows (wave v: rows
// q = v - 1 mod HW - 1), sum their rows' duals and thetas and mirror the workers' dual steps; wave 0
// polls the stop decision, combines the partials, solves, broadcasts and evaluates the objective. One
// wave polling 23 rows spent ~2.5 us per spin on issue and serialised batches (hub ready 5.2 us after
// the last upload, profiles/r02_star). Worker and monitor workgroups use wave 0 only.
constexpr int HW = 4;

template <int QT, bool SYS>
__global__ void __launch_bounds__(64 * HW) star_persistent_kernel(StarArgs a) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int oc_lds[HW];               // hub: each wave's poll outcome
  __shared__ int stop_flag;                // hub: wave 0 saw a stop decision (helpers stop polling)
  __shared__ __attribute__((aligned(16))) double thh_lds[64];  // hub: theta_h^it for the helpers' dual steps
  __shared__ __attribute__((aligned(16))) double part_lds[(HW - 1) * 128];  // hub: helpers' (C1, term_1) partials
  const int d = a.d, n = a.n, hub = n - 1;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const bool in = lane < d;
  const __amdgpu_buffer_rsrc_t rth = rsrc_of(a.thg);
  const __amdgpu_buffer_rsrc_t rob = rsrc_of(a.objg);
  const unsigned long long deadline = now_ticks() + (unsigned long long)a.timeout_ticks;
  __shared__ int xcd_lds;
  const bool packed = !SYS && a.xcd > 0;   // XCD packing (StarArgs::xcd)
  if (packed && (blockIdx.x & 7u)) return;  // a spacer block: only b % 8 == 0 work (one XCD)
  const int bid = packed ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  if (threadIdx.x == 0) stop_flag = 0;
  bool local = false;  // publish with plain stores (every block verified on this XCD)
  if (!SYS && a.xcd > 1) local = xcd_verdict(a.xchk, bid, a.n_local + (a.has_monitor ? 1 : 0), deadline, &xcd_lds);
  lds_barrier();

  if (a.has_monitor && bid == a.n_local) {
    if (wv != 0) return;
    // ---- monitor: sum f_n in worker order, record, decide, fan the decision out
    double* vals = lds;
    for (int it = 1;; ++it) {
      const unsigned tag = make_tag(a.epoch, it);
      const int slot = it % a.ring;
      bool okall = true;
      for (int w = lane; w < n; w += 64) {
        double v = 0.0;
        for (int spin = 0;; ++spin) {
          if (load_granule<SYS>(rob, (slot * n + w) * 16, tag, &v)) break;
          if ((spin & 7) == 7 && now_ticks() > deadline) {
            okall = false;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        vals[w] = v;
      }
      const bool ok = __all(okall);
      unsigned code = 0;
      if (lane == 0) {
        if (!ok) {
          code = 4;
        } else {
          double s = 0.0;
          for (int w = 0; w < n; ++w) s += vals[w];
          if (it - 1 < a.max_iter) a.trace[it - 1] = s;
          if (!(s == s) || isinf(s)) code = 3;
          else if (fabs(s - a.obj0) < a.tol) code = 1;
          else if (it >= a.max_iter) code = 2;
          if (a.tstamp && it - 1 < a.max_iter) a.tstamp[it - 1] = (long long)now_ticks();
        }
        const unsigned long long dv = ((unsigned long long)tag << 32) | code;
        for (int r = 0; r < a.nranks; ++r) store_dec<SYS>(a.dec_push[r] + slot, dv);
        if (a.timeline && it - 1 < a.timeline_iters)
          a.timeline[((long)bid * a.timeline_iters + it - 1) * 4] = (long long)now_ticks();
      }
      if (__shfl((int)code, 0, 64)) return;
    }
  }

  // ---- worker / hub
  const int b = bid;
  const int w = a.gid[b];
  const bool is_hub = w == hub;
  if (!is_hub && wv != 0) return;
  double Mq[4][QT], Aq[4][QT];
  quad_load<QT>(Mq, a.Minv + (long)b * d * d, d, wv == 0);
  quad_load<QT>(Aq, a.A + (long)b * d * d, d, wv == 0);
  double* st = lds;  // QSTAGE doubles of quad-GEMV staging
  double* snap = lds + QSTAGE;  // hub: [n-1][64] this iteration's uploads, read once from the table
  double* lamS = snap + (n - 1) * 64;  // hub: [n-1][64] its copies of the workers' duals (LDS-resident)
  if (is_hub && in && wv > 0)  // helper wave v owns rows q = v - 1 mod (HW - 1)
    for (int q = wv - 1; q < hub; q += HW - 1) lamS[q * 64 + lane] = a.lam_hub[(long)q * d + lane];
  const double bb = in ? a.b[(long)b * d + lane] : 0.0;
  const double half_yy = 0.5 * a.yy[b];
  const double rho = a.rho;
  double th = 0.0, lam = 0.0, thh = 0.0;  // this lane's element of theta_n, lam_n, theta_hub^{i-1}
  // uploads go to the hub rank's table (own table when the hub is local); the hub row goes everywhere
  const __amdgpu_buffer_rsrc_t rup = rsrc_of(a.peer_thg[a.hub_rank]);
  int stop_code = 0, stop_iter = 0, abort = 0;
  int it = 1;
  long long* tlr = nullptr;  // this workgroup's timeline row of the current iteration (debug)
  for (;; ++it) {
    if (it > a.max_iter + a.lag) break;
    tlr = (a.timeline && wv == 0 && it - 1 < a.timeline_iters) ? a.timeline + ((long)b * a.timeline_iters + it - 1) * 4
                                                               : nullptr;
    if (tlr && lane == 0) tlr[0] = (long long)now_ticks();
    const bool check = it - 1 >= a.lag;
    const int jdec = it - a.lag;
    const unsigned tj = make_tag(a.epoch, jdec);
    bool decided = !check;
    unsigned long long dv = 0;
    int outcome = 0;  // 1 go, 2 stop, 3 timeout
    if (!is_hub) {
      // theta_hub^{it-1} (the broadcast) and the decision of it - lag, polled together
      const unsigned tp = make_tag(a.epoch, it - 1);
      double v = 0.0;
      for (int spin = 0;; ++spin) {
        bool ok = true;
        if (it > 1 && in) ok = load_granule<SYS>(rth, (hub * d + lane) * 16, tp, &v);
        if (!decided) {
          dv = __shfl(load_dec<SYS>(&a.decg[jdec % a.ring]), 0, 64);
          decided = (unsigned)(dv >> 32) == tj;
        }
        if (decided && (unsigned)(dv & 0xffffffffu) != 0u) { outcome = 2; break; }
        if (decided && __all(ok)) { outcome = 1; break; }
        if ((spin & 7) == 7 && now_ticks() > deadline) { outcome = 3; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      if (outcome != 1) {
        if (outcome == 2) { stop_code = (int)(unsigned)(dv & 0xffffffffu); stop_iter = jdec; }
        else abort = 1;
        break;
      }
      if (tlr && lane == 0) tlr[1] = (long long)now_ticks();
      if (it > 1) {
        lam = lam + rho * (th - v);  // lam_n += rho (theta_n^{it-1} - theta_h^{it-1})   (:84-88)
        thh = v;
      }
      const double r = in ? (bb - lam) + rho * thh : 0.0;  // H'Y - C1 + rho theta_h   (:42)
      th = quad_gemv<QT>(Mq, r, st);
      if (in) put_granule<SYS>(local, rup, (w * d + lane) * 16, make_tag(a.epoch, it), th);
      if (tlr && lane == 0) tlr[2] = (long long)now_ticks();
    } else {
      // every worker's theta^it (the uploads) and the decision of it - lag. Helper wave v >= 1 polls
      // rows q = v - 1 + (HW - 1) j (bit j of `got`: seen by this lane; a seen row cannot change
      // before the hub publishes), SB loads in flight before any is consumed, then sums its rows'
      // duals and thetas in row order; wave 0 polls the decision and raises stop_flag on a stop,
      // which ends the helpers' polls (the rows of it never come then).
      const unsigned tn = make_tag(a.epoch, it);
      if (wv > 0) {
        unsigned long long got = 0ull;
        for (int spin = 0;; ++spin) {
          bool ok = true;
          if (in) {
            for (int j0 = 0; wv - 1 + (HW - 1) * j0 < hub; j0 += SB) {
              u32x4 g[SB];
#pragma unroll
              for (int k = 0; k < SB; ++k) {
                const int j = j0 + k, q = wv - 1 + (HW - 1) * j;
                const bool want = q < hub && !((got >> j) & 1ull);
                g[k] = want ? load_raw<SYS>(rth, (q * d + lane) * 16) : u32x4{0u, 0u, 0u, 0u};
              }
#pragma unroll
              for (int k = 0; k < SB; ++k) {
                const int j = j0 + k, q = wv - 1 + (HW - 1) * j;
                if (q >= hub || ((got >> j) & 1ull)) continue;
                if (granule_ok(g[k], tn)) {
                  snap[q * 64 + lane] = granule_val(g[k]);  // this wave's row: it alone reads it back
                  got |= 1ull << j;
                } else {
                  ok = false;
                }
              }
            }
          }
          if (__all(ok)) { outcome = 1; break; }
          if (__hip_atomic_load(&stop_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;  // outcome 0
          if ((spin & 7) == 7 && now_ticks() > deadline) { outcome = 3; break; }
          __builtin_amdgcn_s_sleep(1);
        }
        if (outcome == 1 && in) {  // C1 / term_1 partials over this wave's rows (:66-71)
          double c1 = 0.0, s1 = 0.0;
          for (int q = wv - 1; q < hub; q += HW - 1) {
            c1 += lamS[q * 64 + lane];
            s1 += snap[q * 64 + lane];
          }
          part_lds[(wv - 1) * 128 + lane] = c1;
          part_lds[(wv - 1) * 128 + 64 + lane] = s1;
        }
      } else {
        for (int spin = 0;; ++spin) {
          if (!decided) {
            dv = __shfl(load_dec<SYS>(&a.decg[jdec % a.ring]), 0, 64);
            decided = (unsigned)(dv >> 32) == tj;
          }
          if (decided && (unsigned)(dv & 0xffffffffu) != 0u) {
            outcome = 2;
            if (lane == 0) __hip_atomic_store(&stop_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            break;
          }
          if (decided) { outcome = 1; break; }
          if ((spin & 7) == 7 && now_ticks() > deadline) { outcome = 3; break; }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (lane == 0) oc_lds[wv] = outcome;
      lds_barrier();  // the partials are in part_lds
      int oc = oc_lds[0];
      if (oc != 2)
        for (int v = 1; v < HW; ++v)
          if (oc_lds[v] == 3) oc = 3;
      if (oc != 1) {
        if (oc == 2) { stop_code = (int)(unsigned)(dv & 0xffffffffu); stop_iter = jdec; }
        else abort = 1;
        break;
      }
      if (tlr && lane == 0) tlr[1] = (long long)now_ticks();
      if (wv == 0) {
        double c1 = 0.0, s1 = 0.0;
        if (in)
          for (int v = 0; v < HW - 1; ++v) {
            c1 += part_lds[v * 128 + lane];
            s1 += part_lds[v * 128 + 64 + lane];
          }
        const double r = in ? (bb + c1) + rho * s1 : 0.0;
        thh = quad_gemv<QT>(Mq, r, st);
        th = thh;
        if (in) {
          const unsigned tg = make_tag(a.epoch, it);
          for (int rr = 0; rr < a.nranks; ++rr) put_granule<SYS>(local, rsrc_of(a.peer_thg[rr]), (hub * d + lane) * 16, tg, thh);
          if (tlr && lane == 0) tlr[2] = (long long)now_ticks();
        }
        thh_lds[lane] = thh;
      }
      lds_barrier();
      if (wv != 0) {
        // the workers' dual step, mirrored on the hub's copies (:84-88), each helper on its own rows
        // (from the LDS snapshot: once theta_h^it is out, worker q may already be overwriting its
        // table row with theta_q^{it+1})
        if (in) {
          const double th_h = thh_lds[lane];
          for (int q = wv - 1; q < hub; q += HW - 1)
            lamS[q * 64 + lane] = lamS[q * 64 + lane] + rho * (snap[q * 64 + lane] - th_h);
        }
        continue;  // helpers: next iteration (their loop state matches wave 0's)
      }
    }
    // f_n(theta_n^it) = 1/2 th' A th - b' th + 1/2 y'y  (the quadratic form of :95-101)
    const double q = quad_gemv<QT>(Aq, in ? th : 0.0, st);
    const double f = wave_sum_f64(in ? (0.5 * q - bb) * th : 0.0) + half_yy;
    if (lane == 0) put_granule<SYS>(local, rob, ((it % a.ring) * n + w) * 16, make_tag(a.epoch, it), f);
    if (tlr && lane == 0) tlr[3] = (long long)now_ticks();
  }
  if (in && wv == 0) {
    a.theta[(long)b * d + lane] = th;
    a.lam[(long)b * d + lane] = is_hub ? 0.0 : lam;
  }
  if (is_hub && in && wv > 0)  // each helper its own rows
    for (int q = wv - 1; q < hub; q += HW - 1) a.lam_hub[(long)q * d + lane] = lamS[q * 64 + lane];
  if (lane == 0 && wv == 0) {
    if (abort) a.ctl->done = 4;
    else if (b == 0 && stop_code) {
      a.ctl->done = stop_code;
      a.ctl->conv_iter = stop_iter;
      a.ctl->iter = it;
    }
  }
}

extern "C" long gadmm_resident_capacity(const void* fn, int threads, size_t shm);
extern "C" int gadmm_xcd_pick(int want, int multi, int blocks, long cap_total, const void* xchk);  // chain_persistent.hip

static const void* star_variant(const StarArgs& a) {
  if (a.d > 64) return nullptr;
  if (a.sys_scope) return a.d <= 52 ? (const void*)star_persistent_kernel<13, true> : (const void*)star_persistent_kernel<16, true>;
  return a.d <= 52 ? (const void*)star_persistent_kernel<13, false> : (const void*)star_persistent_kernel<16, false>;
}

// monitor: n doubles; worker/hub: quad-GEMV staging + the hub's [n-1][64] upload snapshot
static size_t star_shm(const StarArgs& a) {
  const size_t mon = (size_t)a.n * 8, wk = (size_t)(QSTAGE + 2 * (a.n - 1) * 64) * 8;
  return mon > wk ? mon : wk;
}

extern "C" {

int gadmm_star_abi_layout(long long* out, int n) {
  long long v[] = {(long long)sizeof(StarArgs), (long long)offsetof(StarArgs, rho), (long long)offsetof(StarArgs, gid),
                   (long long)offsetof(StarArgs, ctl), (long long)offsetof(StarArgs, xchk)};
  const int k = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; i < n && i < k; ++i) out[i] = v[i];
  return k;
}

// Workgroups the star kernel can keep resident (0: shape not eligible).
long gadmm_star_capacity(const StarArgs* args) {
  const void* fn = star_variant(*args);
  if (!fn) return 0;
  const size_t shm = star_shm(*args);
  if (shm > 160 * 1024) return 0;
  return gadmm_resident_capacity(fn, 64 * HW, shm);
}

int gadmm_star_launch(const StarArgs* args, hipStream_t st) {
  const StarArgs& a = *args;
  const void* fn = star_variant(a);
  if (!fn || a.n < 2 || a.n_local < 1 || !a.peer_thg || !a.gid || a.hub_rank < 0 || a.hub_rank >= a.nranks ||
      a.ring <= a.lag + 1 || a.max_iter + a.lag >= (1 << 20) || (a.has_monitor && !a.dec_push)) {
    gadmm_set_error("star kernel: unsupported configuration (d=%d n=%d)", a.d, a.n);
    return -1;
  }
  const size_t shm = star_shm(a);
  const int blocks = a.n_local + (a.has_monitor ? 1 : 0);
  const long cap = gadmm_resident_capacity(fn, 64 * HW, shm);
  if (blocks > cap) {
    gadmm_set_error("star kernel: %d workgroups but only %ld can be resident", blocks, cap);
    return -2;
  }
  if (shm > 65536) GADMM_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  StarArgs ka = a;
  ka.xcd = gadmm_xcd_pick(a.xcd, a.sys_scope || a.nranks > 1, blocks, cap, a.xchk);
  if (ka.xcd > 1) GADMM_CHECK(hipMemsetAsync(a.xchk, 0, (size_t)XCHK * 16, st));
  void* kargs[] = {&ka};
  GADMM_CHECK(hipLaunchKernel(fn, dim3(ka.xcd > 0 ? 8 * blocks : blocks), dim3(64 * HW), kargs, shm, st));
  GADMM_CHECK(hipGetLastError());
  return 0;
}

}  // extern "C"
