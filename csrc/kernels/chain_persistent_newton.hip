// Persistent single-launch GADMM with EXACT logistic local solves (the dead CVX variant
// group_ADMM_logistic.m:26-49): one kernel per GPU for the whole solve.
//
// The graph engine runs the exact solve as replayed phase kernels (chain_newton.hip: 512 threads per
// worker, an in-place Gauss-Jordan inverse of the Hessian on the critical path whenever a chord step
// contracts too slowly; ~864 launches per solve). Here every worker is ONE resident workgroup for the
// whole solve, and the two costs of that path leave the critical path:
//
//   wave 0 ("solver") keeps the shard X and X^T in VGPRs (split-column quad layout, quad_gemv.h) and
//   runs the chord-Newton steps of its active phase with no barrier at all:
//       z = X x,  s_i = y_i sigma(-y_i z_i),  g = -X^T s + (lam + deg rho) x + mu - rho (th_l + th_r),
//       dx = Hinv g,  x <- x - dx           until max|dx| < 1e-13 max(1, max|x|) (<= 50 steps)
//   waves 1-4 ("crew") build the inverse Hessian H(x_r)^{-1}, H = X^T diag(w) X + (lam + deg rho) I
//   (f64 MFMA Hessian, 4-wave in-place block Gauss-Jordan in registers, synchronised among themselves
//   through an LDS counter, never with wave 0) at the worker's own final iterate of its last active
//   phase, DURING the idle phase in which the other group solves. The next active phase starts from
//   that inverse (its own previous iterate: the chord Newton preconditioner is one iteration old).
//   A step that contracts by less than `chord` (|dx_k| > chord |dx_{k-1}|) asks the crew for an
//   urgent inverse at the current x, exactly like the graph kernel's chord rule.
// Which inverse each step uses is fixed by the iterates alone (the solver waits for the inverse it
// asked for), so the run is deterministic. The fixed point and the stopping rule are exact Newton's.
//
// Cross-worker protocol (heads / tails, lazy head dual, tagged theta granules, a monitor workgroup
// that sums f_n in worker order and posts the lagged stop decision into every rank's ring, deadlines
// on every spin, the xGMI fabric across GPUs): as chain_persistent_logistic.hip.
#include "gadmm_common.h"
#include "gadmm_chain.h"
#include "persist_device.h"
#include "chain_device.h"
#include "fast_sigm.h"
#include <cstddef>
#include <cstdlib>

struct LogiArgs {  // == chain_persistent_logistic.hip (one ABI for both persistent logistic kernels)
  const double* X;  // [n_local][m][d]
  const double* Y;  // [n_local][m]
  int m, max_inner;
  double lam, step, inner_tol;  // Newton: step = chord threshold (<= 0: a fresh inverse every step)
  int* inner_iters;             // [n_local] optional: Newton steps of the worker's last local solve
  double* scratch;              // pipeline kernel: [n_local][RSLOTS][4 QB] refresh images (P | B | XP | XB)
};

namespace {

// Wave layout: 6 waves, dealt round-robin to the CU's 4 SIMDs (wave w -> SIMD w % 4): wave 0 is the
// solver, wave 4 (its SIMD mate) leaves right after the set-up, so the solver's SIMD runs nothing
// else; waves 1, 2, 3, 5 are the crew (crew index 0..3). A crew wave on the solver's SIMD would take
// its f64 issue slots during every refresh (measured: 3.3 us per chord step with a 5-wave layout).
constexpr int NT = 384;
__device__ __forceinline__ int crew_index(int wid) { return wid == 5 ? 3 : wid - 1; }  // wid in {1,2,3,5}
constexpr int CREW = 4;
constexpr int NCW = 64 / CREW;  // Gauss-Jordan: columns per crew lane (j = cw + CREW c)
constexpr int NMAX = 50;      // Newton step cap (== models/logistic.py:newton_prox)
constexpr double NTOL = 1e-13;
constexpr int QT = 13;        // quad layout: d, m <= 52
constexpr int QB = 4 * 64 * (QT + (QT & 1));  // doubles of one quad-LDS inverse buffer
constexpr int HS = 65;        // LDS Hessian row stride

// LDS layout (doubles)
struct NLds {
  int xt, hs, qb0, qb1, qb2, wq, slab, stage, total;
  __host__ __device__ int buf(int r) const { return qb0 + (r % 3) * QB; }
  __host__ __device__ NLds(int m, int d) {
    (void)m;
    (void)d;
    xt = 0;                        // X^T in the quad-LDS layout: the solver's gradient GEMV and the
                                   // crew's Hessian operands (X itself stays in the solver's VGPRs)
    hs = xt + QB;                  // Hessian [64][HS]
    qb0 = ((hs + 64 * HS + 1) & ~1);
    qb1 = qb0 + QB;                // three inverse buffers (quad-LDS layout: quad_gemv_lds): the one in
    qb2 = qb1 + QB;                // use, a background refresh in progress, an urgent refresh
    wq = qb2 + QB;                 // [64] w_i = sigma (1 - sigma) at the refresh point
    slab = wq + 64;                // [2][4][64] Gauss-Jordan pivot-column slabs
    stage = slab + 512;            // [QSTAGE] solver quad GEMV staging
    total = stage + QSTAGE;
  }
};

struct NCtl {        // LDS words of the solver <-> crew protocol
  int req;           // last refresh requested (solver; -1: quit)
  int ready;         // last refresh completed (crew)
  int cnt;           // crew barrier counter
  int src;           // refresh mode: -1 Gauss-Jordan; r >= 0: one Newton-Schulz step from refresh r's inverse
  double shift;      // lam + deg rho of the requested refresh
  int quit;          // the solve is over: the crew leaves once it has served every request posted before
};

// LDS-only ordering: the fences name the "local" address space, so they wait for LDS operations only
// (lgkmcnt). A plain workgroup fence would also wait for this wave's outstanding GLOBAL stores
// (vmcnt) -- for the solver, the write-through theta granules it has just published (~1 us each).
__device__ __forceinline__ int lds_load_acq(const int* p) {
  const int v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  return v;
}
__device__ __forceinline__ void lds_store_rel(int* p, int v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// barrier among the 4 crew waves only (the solver wave never joins): an LDS arrival counter
__device__ __forceinline__ void crew_sync(int* cnt, int& gen) {
  gen += CREW;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < gen) __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ double wave_max_abs(double v) {
  v = fabs(v);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

__device__ __forceinline__ double rcp_nr(double v) {  // v_rcp_f64 + one Newton-Raphson step
  const double r = __builtin_amdgcn_rcp(v);
  return fma(r, fma(-v, r, 1.0), r);
}

// element (row, col) of a quad-LDS inverse buffer (quad_gemv_lds<QT> layout; columns >= 4 (QT + 1) are 0)
__device__ __forceinline__ int qidx(int row, int col) {
  const int r = row >> 4, iq = row & 15, c4 = col & 3, t = col >> 2;
  return ((t >> 1) * 4 + r) * 128 + 2 * (iq + 16 * c4) + (t & 1);
}
constexpr int QCOLS = 4 * (QT + (QT & 1));

// One refresh by the crew (crew index cw = 0..3): Hs = X^T diag(wq) X + shift I (MFMA), then the inverse
// into the quad-LDS buffer `qb`, either
//   src == nullptr: in-place block Gauss-Jordan in registers (exact), or
//   src != nullptr: ONE Newton-Schulz step from the inverse X0 in `src` (the one the solver uses):
//       X1 = X0 (2 I - H X0) = 2 X0 - X0 (H X0),   I - H X1 = (I - H X0)^2
//   two 64 x 64 x 64 f64 MFMA products, no pivot chain. X0 was exact for a nearby Hessian (the
//   worker's previous point), so its residual is small and squaring it gives a chord preconditioner
//   far better than the stale inverse, at a fraction of the Gauss-Jordan cost.
// Every LDS word read here is written first (padding included): the result never depends on stale LDS.
__device__ void crew_refresh(double* lds, const NLds& L, int m, int d, double shift, int cw, int* cnt, int& gen,
                             double* qb, long long* tl, const double* src) {
  const int lane = threadIdx.x & 63;
  const double* XT = lds + L.xt;  // X^T, quad-LDS layout: X[k][j] = XT[qidx(j, k)] (0 beyond d / m)
  double* Hs = lds + L.hs;
  const double* wq = lds + L.wq;
  {  // Hessian tiles (R, C = cw), R = 0..3: v_mfma_f64_16x16x4f64, K = samples in chunks of 4
    const int k4 = lane >> 4, c16 = lane & 15;
    f64x4 acc[4];
#pragma unroll
    for (int R = 0; R < 4; ++R) acc[R] = f64x4{0.0, 0.0, 0.0, 0.0};
    const int cc = 16 * cw + c16;
    for (int k0 = 0; k0 < m; k0 += 4) {
      const int kk = k0 + k4;
      const bool kin = kk < m;
      const double w = kin ? wq[kk] : 0.0;
      const double bv = kin ? XT[qidx(cc, kk)] : 0.0;
#pragma unroll
      for (int R = 0; R < 4; ++R) {
        const double av = kin ? w * XT[qidx(16 * R + c16, kk)] : 0.0;
        acc[R] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[R], 0, 0, 0);
      }
    }
#pragma unroll
    for (int R = 0; R < 4; ++R)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int row = 16 * R + k4 + 4 * reg, col = 16 * cw + c16;
        double v;
        if (row < d && col < d) v = acc[R][reg] + (row == col ? shift : 0.0);
        else v = row == col ? 1.0 : 0.0;  // identity padding
        Hs[row * HS + col] = v;
      }
  }
  crew_sync(cnt, gen);
  if (tl && cw == 0 && lane == 0) tl[1] = (long long)__builtin_amdgcn_s_memrealtime();
  if (src) {
    const int k4 = lane >> 4, c16 = lane & 15;
    const int cc = 16 * cw + c16;
    f64x4 acc[4];
    // T = H X0: tiles (R, C = cw); A[i][k] = H[16R + i][k], B[k][j] = X0[k][16 cw + j]
#pragma unroll
    for (int R = 0; R < 4; ++R) acc[R] = f64x4{0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < 64; k0 += 4) {
      const int kk = k0 + k4;
      const double bv = cc < QCOLS ? src[qidx(kk, cc)] : 0.0;
#pragma unroll
      for (int R = 0; R < 4; ++R) acc[R] = __builtin_amdgcn_mfma_f64_16x16x4f64(Hs[(16 * R + c16) * HS + kk], bv,
                                                                               acc[R], 0, 0, 0);
    }
    crew_sync(cnt, gen);  // every crew wave is done reading H: T goes where H was
#pragma unroll
    for (int R = 0; R < 4; ++R)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) Hs[(16 * R + k4 + 4 * reg) * HS + cc] = acc[R][reg];
    crew_sync(cnt, gen);
    // U = X0 T: A[i][k] = X0[16R + i][k], B[k][j] = T[k][16 cw + j]; X1 = 2 X0 - U
#pragma unroll
    for (int R = 0; R < 4; ++R) acc[R] = f64x4{0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < 64; k0 += 4) {
      const int kk = k0 + k4;
      const double bv = Hs[kk * HS + cc];
#pragma unroll
      for (int R = 0; R < 4; ++R) {
        const double av = kk < QCOLS ? src[qidx(16 * R + c16, kk)] : 0.0;
        acc[R] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[R], 0, 0, 0);
      }
    }
    if (tl && cw == 0 && lane == 0) tl[2] = (long long)__builtin_amdgcn_s_memrealtime();
    if (cc < QCOLS) {
#pragma unroll
      for (int R = 0; R < 4; ++R)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int row = 16 * R + k4 + 4 * reg;
          const int q = qidx(row, cc);
          qb[q] = (row < d && cc < d) ? 2.0 * src[q] - acc[R][reg] : 0.0;
        }
    }
    crew_sync(cnt, gen);
    return;
  }
  // in-place block Gauss-Jordan (SPD, no pivoting), 4 x 4 pivot blocks; lane i of crew wave cw keeps row
  // i's columns j = cw + 4c. Block K = p..p+3: P = A_KK, non-pivot rows L_i = A_iK P^-1, A_ij -= L_i A_Kj,
  // A_iK = -L_i; pivot rows A_Kj = P^-1 A_Kj, A_KK = P^-1. Only column K is published; the pivot rows
  // follow from the symmetric structure (processed / unprocessed cross blocks are antisymmetric), as in
  // chain_newton.hip.
  const int i = lane;
  double h[NCW];
#pragma unroll
  for (int c = 0; c < NCW; ++c) h[c] = Hs[i * HS + cw + CREW * c];
  const int nb = (d + 3) >> 2;
  double* slabs = lds + L.slab;
  for (int bb = 0; bb < nb; ++bb) {
    const int p = 4 * bb;
    double* slab = slabs + (bb & 1) * 256;  // [4][64]: column p + q of the current matrix
    {  // the block's column p + q is register c = p / 4 of crew wave q
      double hv = 0.0;
#pragma unroll
      for (int c = 0; c < NCW; ++c) hv = (c == bb) ? h[c] : hv;
      slab[cw * 64 + i] = hv;
    }
    crew_sync(cnt, gen);
    double P[4][4], Rr[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      Rr[q] = slab[q * 64 + i];
#pragma unroll
      for (int r = 0; r < 4; ++r) P[q][r] = slab[q * 64 + p + r];
    }
    const bool pivrow = (i >> 2) == bb;
    if (pivrow) {
#pragma unroll
      for (int q = 0; q < 4; ++q) Rr[q] = (q == (i & 3)) ? 1.0 : 0.0;
    }
    const double a00 = P[0][0], a01 = P[1][0], a11 = P[1][1];
    const double ia = rcp_nr(fma(a00, a11, -a01 * a01));
    const double A00 = a11 * ia, A01 = -a01 * ia, A11 = a00 * ia;
    const double b00 = P[2][0], b01 = P[3][0], b10 = P[2][1], b11 = P[3][1];
    const double w00 = fma(A00, b00, A01 * b10), w01 = fma(A00, b01, A01 * b11);
    const double w10 = fma(A01, b00, A11 * b10), w11 = fma(A01, b01, A11 * b11);
    const double s00 = P[2][2] - fma(b00, w00, b10 * w10);
    const double s01 = P[3][2] - fma(b00, w01, b10 * w11);
    const double s11 = P[3][3] - fma(b01, w01, b11 * w11);
    const double is = rcp_nr(fma(s00, s11, -s01 * s01));
    const double y0 = fma(A00, Rr[0], A01 * Rr[1]), y1 = fma(A01, Rr[0], A11 * Rr[1]);
    const double z2 = Rr[2] - fma(b00, y0, b10 * y1), z3 = Rr[3] - fma(b01, y0, b11 * y1);
    const double l2 = fma(s11, z2, -s01 * z3) * is, l3 = fma(s00, z3, -s01 * z2) * is;
    const double l0 = y0 - fma(w00, l2, w01 * l3), l1 = y1 - fma(w10, l2, w11 * l3);
    const double lw = cw == 0 ? l0 : (cw == 1 ? l1 : (cw == 2 ? l2 : l3));  // l[j - p] for j = p + cw
#pragma unroll
    for (int c = 0; c < NCW; ++c) {
      const int j = cw + CREW * c;
      const double tq = fma(l0, slab[j], fma(l1, slab[64 + j], fma(l2, slab[128 + j], l3 * slab[192 + j])));
      const bool inK = c == bb;
      const double sg = j < p ? -1.0 : 1.0;
      double v;
      if (inK) v = pivrow ? lw : -lw;
      else v = pivrow ? sg * tq : fma(-sg, tq, h[c]);
      h[c] = v;
    }
  }
  if (tl && cw == 0 && lane == 0) tl[2] = (long long)__builtin_amdgcn_s_memrealtime();
  // the inverse into the quad-LDS layout of quad_gemv_lds<QT>: element (row, col) at
  // ((t >> 1) * 4 + r) * 128 + 2 lq + (t & 1), row = iq + 16 r, col = c4 + 4 t, lq = iq + 16 c4; padding 0
  {
    const int r = i >> 4, iq = i & 15;
#pragma unroll
    for (int c = 0; c < NCW; ++c) {
      const int col = cw + CREW * c;
      const int t = col >> 2, c4 = col & 3;
      if (t < QT + (QT & 1)) {
        const double v = (i < d && col < d && t < QT) ? h[c] : 0.0;
        qb[((t >> 1) * 4 + r) * 128 + 2 * (iq + 16 * c4) + (t & 1)] = v;
      }
    }
  }
  crew_sync(cnt, gen);
}

}  // namespace

template <bool SYS>
__global__ void __launch_bounds__(NT) chain_persistent_newton_kernel(PersistArgs a, LogiArgs g) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ NCtl nc;
  const int d = a.d, n = a.n, m = g.m;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t rth = rsrc_of(a.thg);
  const __amdgpu_buffer_rsrc_t rob = rsrc_of(a.objg);
  const unsigned long long deadline = now_ticks() + (unsigned long long)a.timeout_ticks;
  const int bid = (int)blockIdx.x;
  const NLds L(m, d);

  if (a.has_monitor && bid == a.n_local) {
    // ---------------------------------------------------------------- monitor (wave 0)
    if (wid != 0) return;
    double* vals = lds;  // [n]
    for (int it = a.start_iter;; ++it) {
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
          for (int w = 0; w < n; ++w) s += vals[w];  // worker order
          if (it - 1 < a.max_iter) a.trace[it - 1] = s;
          if (!(s == s) || isinf(s)) code = 3;
          else if (fabs(s - a.obj0) < a.tol) code = 1;
          else if (it >= a.max_iter) code = 2;
          if (a.tstamp && it - 1 < a.max_iter) a.tstamp[it - 1] = (long long)now_ticks();
        }
        const unsigned long long dv = ((unsigned long long)tag << 32) | code;
        for (int r = 0; r < a.nranks; ++r) store_dec<SYS>(a.dec_push[r] + slot, dv);
      }
      if (__shfl((int)code, 0, 64)) return;
    }
  }
  if (bid >= a.n_local) return;

  // ------------------------------------------------------------------ worker workgroup
  const PhaseSlot sl = a.slots[bid];
  const int li = sl.li, w = sl.gid, left = sl.left, right = sl.right;
  const bool head = (a.pos[bid] % 2) == 0;
  const double rho = a.rho, lam = g.lam, chord = g.step;
  const double shift = lam + rho * (double)((left >= 0 ? 1 : 0) + (right >= 0 ? 1 : 0));
  const double* Xg = g.X + (long)li * m * d;
  // shared set-up: X^T into LDS in the quad-LDS layout (element (row j, col i) = X[i][j]), protocol words
  for (int e = threadIdx.x; e < QB; e += NT) {
    const int blk = e >> 7, within = e & 127;
    const int r = blk & 3, th = blk >> 2, lq = within >> 1, t = 2 * th + (within & 1);
    const int row = (lq & 15) + 16 * r, col = (lq >> 4) + 4 * t;  // row: feature j, col: sample i
    lds[L.xt + e] = (row < d && col < m && t < QT) ? Xg[(long)col * d + row] : 0.0;
  }
  if (threadIdx.x == 0) {
    nc.req = 0;
    nc.ready = -1;
    nc.cnt = 0;
    nc.src = -1;  // refresh 0: Gauss-Jordan
    nc.shift = shift;
    nc.quit = 0;
  }
  // refresh 0 is built at the worker's start point theta^{start - 1}: w_i = sigma(z_i)(1 - sigma(z_i)),
  // z_i = X_i theta (zeros on a fresh solve: w = 1/4)
  if (threadIdx.x < 64) {
    const int i = threadIdx.x;
    double wi = 0.0;
    if (i < m) {
      double z = 0.0;
      for (int j = 0; j < d; ++j) z = fma(Xg[(long)i * d + j], a.theta[(long)w * d + j], z);
      const double pz = 1.0 / (1.0 + exp(g.Y[(long)li * m + i] * z));
      wi = pz * (1.0 - pz);
    }
    lds[L.wq + i] = wi;
  }
  lds_barrier();  // the only workgroup-wide barrier: solver and crew run decoupled from here on

  if (wid == 4) return;  // keeps the solver's SIMD free
  if (wid > 0) {
    // ---------------------------------------------------------------- crew (waves 1, 2, 3, 5)
    const int cw = crew_index(wid);
    const int li_ = sl.li;
    int gen = 0, done_req = -1;
    for (;;) {
      // quit is read BEFORE req: a quit seen here was posted after every request (same wave, release),
      // so all four crew waves serve the same requests and leave together (none waits in crew_sync alone)
      int r;
      for (int spin = 0;; ++spin) {
        const int q = lds_load_acq(&nc.quit);
        r = lds_load_acq(&nc.req);
        if (r != done_req) break;
        if (q) return;
        if ((spin & 63) == 63 && now_ticks() > deadline + 100000000ull) return;  // solver gone (abort path)
        __builtin_amdgcn_s_sleep(1);
      }
      // instrumented runs (PersistArgs::timeline, [n_local][128][8] stamps): refreshes 0..63 in rows 0..63
      long long* tl = (a.timeline && r < 64) ? a.timeline + ((long)li_ * 128 + r) * 8 : nullptr;
      if (tl && cw == 0 && lane == 0) tl[0] = (long long)__builtin_amdgcn_s_memrealtime();
      const int srcr = nc.src;  // written before the request (release / acquire on nc.req)
      crew_refresh(lds, L, m, d, nc.shift, cw, &nc.cnt, gen, lds + L.buf(r), tl,
                   srcr >= 0 ? lds + L.buf(srcr) : nullptr);
      if (tl && cw == 0 && lane == 0) tl[3] = (long long)__builtin_amdgcn_s_memrealtime();
      if (cw == 0 && lane == 0) lds_store_rel(&nc.ready, r);
      done_req = r;
    }
  }

  // ------------------------------------------------------------------ solver (wave 0)
  double* st = lds + L.stage;
  // X in VGPRs (margins), X^T from LDS (gradient): both in registers would be 208 VGPRs and spill
  double Xq[4][QT];
  const double* XTl = lds + L.xt;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      const int qi = lane & 15, qc = lane >> 4;
      const int row = qi + 16 * r, col = qc + 4 * t;
      Xq[r][t] = (row < m && col < d) ? Xg[(long)row * d + col] : 0.0;
    }
  u32x4* const p0 = a.push ? a.push[2 * bid] : nullptr;
  u32x4* const p1 = a.push ? a.push[2 * bid + 1] : nullptr;
  const __amdgpu_buffer_rsrc_t rp0 = rsrc_of(p0 ? (const void*)p0 : (const void*)a.thg);
  const __amdgpu_buffer_rsrc_t rp1 = rsrc_of(p1 ? (const void*)p1 : (const void*)a.thg);
  const bool inj = lane < d, ini = lane < m;
  const double yv = ini ? g.Y[(long)li * m + lane] : 0.0;
  double th = inj ? a.theta[(long)w * d + lane] : 0.0;
  const bool fast_sig = (a.dbg & 32) == 0;
  double mu = inj ? a.mu[(long)li * d + lane] : 0.0;
  double tl = (inj && left >= 0) ? a.theta[(long)left * d + lane] : 0.0;
  double tr = (inj && right >= 0) ? a.theta[(long)right * d + lane] : 0.0;
  int pending = a.pending_in;
  int stop_code = 0, stop_iter = 0, abort = 0, used = 0, nfail = 0;
  // Inverse bookkeeping (refresh ids are consecutive; refresh r lives in buffer r % 3):
  //   cur   the inverse the chord steps use (refresh 0, at the start point, requested in the set-up)
  //   pend  a background refresh in progress (-1: none), requested at iteration pend_it at the
  //         worker's final iterate; adopted at the active phase of iteration pend_it + RLAG (waiting
  //         for it if the crew is not done), so the crew gets RLAG - 1 whole iterations of slack
  //   urgent refreshes (a step that contracts by less than `chord`) are waited for at once
  // Every choice depends on the iterates only: deterministic.
  constexpr int RLAG = 2;
  int cur = 0, pend = -1, pend_it = 0, next_id = 0;
  bool cur_fresh = true;  // `cur` was built at the start point of the next solve
  const int bg_steps = (g.max_inner >= 1 && g.max_inner < NMAX) ? g.max_inner : 1;
  const bool ns_bg = g.inner_tol >= 0.0;  // LogiArgs::inner_tol < 0: background refreshes by Gauss-Jordan
  auto wait_ready = [&](int r) -> bool {
    for (int spin = 0;; ++spin) {
      if (lds_load_acq(&nc.ready) >= r) return true;
      if ((spin & 63) == 63 && now_ticks() > deadline) return false;
      __builtin_amdgcn_s_sleep(1);
    }
  };
  auto post = [&](int r) { lds_store_rel(&nc.req, r); };

  int it = a.start_iter;
  for (;; ++it) {
    if (it > a.max_iter + a.lag) break;
    const bool check = it - a.start_iter >= a.lag;
    const int jdec = it - a.lag;
    const bool need_nb = head ? it > a.start_iter : true;
    const int jnb = head ? it - 1 : it;
    const unsigned tnb = make_tag(a.epoch, jnb), tj = make_tag(a.epoch, jdec);
    const int ra = need_nb ? left : -1, rb = need_nb ? right : -1;
    bool decided = !check;
    unsigned long long dv = 0;
    int outcome = 0;  // 1 go, 2 stop, 3 timeout
    for (int spin = 0;; ++spin) {
      bool nb = true;
      if (inj) {
        if (ra >= 0) nb &= load_granule<SYS>(rth, (ra * d + lane) * 16, tnb, &tl);
        if (rb >= 0) nb &= load_granule<SYS>(rth, (rb * d + lane) * 16, tnb, &tr);
      }
      if (!decided) {
        dv = __shfl(load_dec<SYS>(&a.decg[jdec % a.ring]), 0, 64);
        decided = (unsigned)(dv >> 32) == tj;
      }
      if (decided && (unsigned)(dv & 0xffffffffu) != 0u) { outcome = 2; break; }
      if (decided && __all(nb)) { outcome = 1; break; }
      if ((spin & 7) == 7 && now_ticks() > deadline) { outcome = 3; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (outcome != 1) {
      if (outcome == 2) {
        stop_code = (int)(unsigned)(dv & 0xffffffffu);
        stop_iter = jdec;
      } else {
        abort = 1;
      }
      break;
    }
    // -- lazy dual (heads); x-independent gradient part cv = mu - rho (th_l + th_r)
    double cv = 0.0, x = 0.0;
    if (inj) {
      double mm = mu;
      if (head && pending) {
        if (left >= 0) mm = mm - rho * (tl - th);
        if (right >= 0) mm = mm + rho * (th - tr);
        mu = mm;
      }
      cv = mm;
      if (left >= 0) cv = cv - rho * tl;
      if (right >= 0) cv = cv - rho * tr;
      x = th;
    }
    // -- chord Newton from the inverse at the previous own iterate (the chord steps' sigmoid by
    // inv1pexp_fast unless PersistArgs::dbg & 32: GADMM_NEWTON_FASTSIGM=0)
    const int kk_tl = it - a.start_iter;
    long long* tls = (a.timeline && kk_tl < 64) ? a.timeline + ((long)li * 128 + 64 + kk_tl) * 8 : nullptr;
    if (tls && lane == 0) tls[0] = (long long)__builtin_amdgcn_s_memrealtime();
    if (pend >= 0 && it - pend_it >= RLAG) {  // adopt the background refresh
      if (!wait_ready(pend)) { abort = 1; break; }
      cur = pend;
      pend = -1;
      cur_fresh = false;
    }
    if (!wait_ready(cur)) { abort = 1; break; }
    if (tls && lane == 0) tls[1] = (long long)__builtin_amdgcn_s_memrealtime();
    const double* hq = lds + L.buf(cur);
    double nd_prev = 0.0;
    used = 0;
    bool urgent = false;
    bool fresh = cur_fresh;  // the inverse in use was built at this solve's start point
    cur_fresh = false;
    for (int k = 0; k < NMAX; ++k) {
      const double z = quad_gemv<QT>(Xq, x, st);                     // margins
      const double ps = ini ? (fast_sig ? inv1pexp_fast(yv * z) : 1.0 / (1.0 + exp(yv * z))) : 0.0;  // sigma(-y z)
      const double gx = quad_gemv_lds<QT>(XTl, ini ? yv * ps : 0.0, st);  // (X^T (y . sigma))_j
      const double gr = inj ? -gx + shift * x + cv : 0.0;
      const double dx = quad_gemv_lds<QT>(hq, gr, st);
      const double dxl = inj ? dx : 0.0;
      x = inj ? x - dxl : 0.0;
      const double mdx = wave_max_abs(dxl), mx = wave_max_abs(x);
      used = k + 1;
      if (mdx < NTOL * fmax(1.0, mx)) break;
      if (k + 1 == NMAX) ++nfail;  // the step cap ends this solve unconverged
      if (chord <= 0.0 || (!fresh && k > 0 && mdx > chord * nd_prev)) {
        // contraction too slow: an inverse at the current x, from the crew (idle in this phase)
        const double z2 = quad_gemv<QT>(Xq, x, st);
        const double p2 = ini ? 1.0 / (1.0 + exp(yv * z2)) : 0.5;
        lds[L.wq + lane] = ini ? p2 * (1.0 - p2) : 0.0;
        if (pend >= 0) {  // the crew first finishes the background refresh (adopted: it is newer)
          if (!wait_ready(pend)) { abort = 1; break; }
          cur = pend;
          pend = -1;
        }
        cur = ++next_id;
        nc.src = -1;  // exact: Gauss-Jordan at the current x
        post(cur);
        urgent = true;
        if (!wait_ready(cur)) { abort = 1; break; }
        hq = lds + L.buf(cur);
        fresh = true;
        nd_prev = 0.0;
        continue;
      }
      fresh = false;
      nd_prev = mdx;
    }
    if (abort) break;
    if (tls && lane == 0) {
      tls[2] = (long long)__builtin_amdgcn_s_memrealtime();
      tls[3] = used;
      tls[4] = next_id;
    }
    // -- publish theta^it: own table + the remote neighbours' tables (first: the neighbours wait)
    const unsigned tag = make_tag(a.epoch, it);
    if (inj) {
      store_granule<SYS>(rth, (w * d + lane) * 16, tag, x);
      if (p0) store_granule<SYS>(rp0, (w * d + lane) * 16, tag, x);
      if (p1) store_granule<SYS>(rp1, (w * d + lane) * 16, tag, x);
    }
    if (!head) {  // tails: both neighbours are this iteration's heads -> dual update now
      double rp = 0.0;
      if (inj) {
        double mm = mu;
        if (left >= 0) mm = mm - rho * (tl - x);
        if (right >= 0) mm = mm + rho * (x - tr);
        mu = mm;
        if (left >= 0) rp = fma(tl - x, tl - x, rp);
        if (right >= 0) rp = fma(x - tr, x - tr, rp);
      }
      if (a.rres) {
        const double rs = wave_sum_f64(rp);
        if (lane == 0 && it - 1 < a.max_iter) a.rres[(long)(it - 1) * n + w] = rs;
      }
    } else {
      pending = 1;
    }
    th = x;
    // -- f_n(theta^it) -> monitor; the same margins give the crew its next refresh point (this worker's
    // new iterate), built while the other group solves
    const double z = quad_gemv<QT>(Xq, x, st);
    const double pz = ini ? 1.0 / (1.0 + exp(yv * z)) : 0.5;
    const double part = wave_sum_f64(ini ? softplus(-yv * z) : 0.0);
    const double xx = wave_sum_f64(inj ? x * x : 0.0);
    if (lane == 0) store_granule<SYS>(rob, ((it % a.ring) * n + w) * 16, tag, lam * 0.5 * xx + part);
    // background refresh at the new iterate only when this solve says the inverse is ageing (more
    // than bg_steps chord steps, or an urgent refresh): the crew then works while the other group
    // solves, and otherwise stays idle -- a busy crew shares this CU's SIMDs and LDS with the solver
    if ((used > bg_steps || urgent) && pend < 0) {  // the crew is idle (no refresh outstanding)
      lds[L.wq + lane] = ini ? pz * (1.0 - pz) : 0.0;
      pend = ++next_id;
      pend_it = it;
      nc.src = ns_bg ? cur : -1;  // background: one Newton-Schulz step from the inverse in use
      post(pend);
    }
  }
  lds_store_rel(&nc.quit, 1);  // crew: quit (after its current refresh, if any)
  if (inj) {
    a.theta[(long)w * d + lane] = th;
    a.mu[(long)li * d + lane] = mu;
  }
  if (lane == 0) {
    if (g.inner_iters) g.inner_iters[li] = used;
    if (nfail) atomicAdd(&a.ctl->inner_fail, nfail);  // read by the host after the launch
    if (abort) {
      a.ctl->done = 4;
    } else if (bid == 0 && stop_code) {
      a.ctl->done = stop_code;
      a.ctl->conv_iter = stop_iter;
      a.ctl->iter = it;
      a.ctl->pending = 1;
      a.ctl->monitored = stop_iter;
    }
  }
}

// ==================================================================================================
// GADMM_NEWTON_REC (default): the chord steps as a FOUR-wave pipeline. One chord step
//     z = X x,  s = y sigma(-y z),  dx = P (shift x + cv - X^T s),  x' = x - dx
// is three dependent GEMVs on one wave above (two of them from LDS: ~1.6 us per step,
// profiles/r03_newton). With the step's matrices formed once per inverse P (by the crew, MFMA):
//     B = P X^T (d x m),  XP = X P (m x d),  XB = X B (m x m),
// and y_k = shift x_k + cv, the step splits into
//     dx_k = P y_k - B s_k,   x_{k+1} = x_k - dx_k,   z_{k+1} = X x_{k+1} = z_k - XP y_k + XB s_k,
// so four waves, one register matrix each, run one GEMV per step in a pipeline:
//     S (margins, XB):  s_k = y sigma(-y z_k) -> ring; z_{k+1} = (z_k - w_k) + XB s_k
//     H (B):            b_k = B s_k -> ring
//     T (iterate, P):   dx_k = v_k - b_k; x_{k+1}; y_{k+1} -> ring; the stop and chord rules; then
//                       v_{k+1} = P y_{k+1} while H waits for s_{k+1}
//     W (XP):           w_k = XP y_k
// A step's dependent chain holds S's sigmoid and one GEMV; the loop s_k -> b_k -> y_{k+1} -> w_{k+1}
// -> s_{k+2} spans two steps (profiles/r05_l: ~0.76 us per step against 1.65 us on one wave). Every segment (a local solve, or its continuation after an urgent refresh) restarts
// the margins from the exact z_0 = X x_0 (wave W, X in LDS), which also gives the objective f_n and
// the refresh weights. The crew (4 waves) builds P exactly as the one-wave kernel's crew (Hessian,
// Gauss-Jordan or one Newton-Schulz step) plus the three products, into a per-worker global image
// (LogiArgs::scratch, refresh r in slot r % 3) that the pipeline waves load into VGPRs off the critical
// path (the next phase's inverse is known at the end of a phase). Which inverse each step uses is
// fixed by the iterates alone (deterministic); only the margins differ from the one-wave kernel in
// rounding (host emulation, tools/newton_recursion_emul.py: 424 iterations, theta within 1e-15).
namespace {

constexpr int RT = 512;           // 8 waves: S, T, H, W (SIMDs 0-3) + the crew (waves 4-7)
constexpr int RR = 4;             // ring slots (a producer runs at most two steps ahead)
constexpr int RSLOTS = 3;         // refresh images per worker
constexpr int RIMG = 4 * QB;      // one image: P | B | XP | XB, quad-LDS layout each
constexpr int REC_RLAG = 3;       // default refresh lag (iterations) and background-refresh step threshold: the
constexpr int REC_BG = 4;         // best of lag x threshold sweeps (profiles/r05_l: r5ls4 5.48-5.49 ms at 3 / 4, 5.56 at 3 / 3)

struct RLds {  // doubles
  int xt, xq, hs, hp, wq, slab, stage, sring, yring, vring, wring, z0v, xfin, total;
  __host__ __device__ RLds() {
    xt = 0;                    // [64][HS] X^T row-major, zero padded (crew operands: plain addressing)
    xq = xt + 64 * HS;         // X, quad-LDS layout (W's exact margins)
    hs = xq + QB;              // [64][HS] Hessian, then Newton-Schulz T, then B row-major (crew)
    hp = hs + 64 * HS;         // [64][HS] the new P row-major (crew)
    wq = hp + 64 * HS;         // [64] refresh weights
    slab = wq + 64;            // [2][4][64] Gauss-Jordan slabs
    stage = slab + 512;        // W's quad GEMV staging
    sring = stage + QSTAGE;    // [RR][4 QX] s_k (quad_gemv broadcast layout)
    yring = sring + RR * 4 * QX;  // [RR][4 QX] y_k
    vring = yring + RR * 4 * QX;  // [RR][64] b_k
    wring = vring + RR * 64;      // [RR][64] w_k
    z0v = wring + RR * 64;        // [64] exact margins of the next segment's start
    xfin = z0v + 64;              // [64] a segment's final iterate
    total = xfin + 64;
  }
};

enum { PC_Z0, PC_S, PC_Y, PC_V, PC_W, PC_END, PC_QUIT, PC_EKIND, PC_EREQ, PC_ESRC, PC_ENEXT,
       PC_EIT, PC_WDONE, PC_N };

// Ordering of the refresh images, which never leave the CU (the crew stores them, waves of the same
// workgroup load them): the crew waits for its stores (vmcnt 0) before `ready` is posted, and the
// loads bypass L1 (load_img: sc0), so no agent-scope fence (an L2 write-back / invalidate of the whole
// XCD, measured: refresh 15 -> 27 us) is needed.
__device__ __forceinline__ void wg_release() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
}
__device__ __forceinline__ void wg_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); }

// wave max of |v| by DPP row rotations (within 16 lanes) and two permlane swaps (across rows): a few
// dozen cycles instead of six ds_bpermute round trips (wave_max_abs)
template <int CTL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)u, CTL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), CTL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_max_abs_dpp(double v) {
  v = fabs(v);
  v = fmax(v, dpp_f64<0x128>(v));  // row_ror:8
  v = fmax(v, dpp_f64<0x124>(v));  // row_ror:4
  v = fmax(v, dpp_f64<0x122>(v));  // row_ror:2
  v = fmax(v, dpp_f64<0x121>(v));  // row_ror:1
  double a = v, b = v;
  swap16_f64(a, b);
  v = fmax(a, b);
  a = v;
  b = v;
  swap32_f64(a, b);
  return fmax(a, b);
}

// A pipeline hand-off post without the release fence: a wave's LDS operations are performed in order,
// so a flag written after the ring data cannot become visible before it (the fence's s_waitcnt only
// held the flag back by one LDS round trip). The compiler barrier keeps the data stores first.
// GADMM_NEWTON_POSTFENCE=1 (PersistArgs::dbg bit 17) restores the fenced post (A/B).
__device__ __forceinline__ void lds_post(int* p, int v, bool fenced) {
  if (fenced || !GADMM_LDS_IN_ORDER) {  // fence-free only where in-order LDS is documented
    lds_store_rel(p, v);
    return;
  }
  asm volatile("" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// C (64 x 64 tile column cw) = A B over k < 4 QT (operands zero beyond d / m): acc[R][reg] =
// C[16R + k4 + 4 reg][16 cw + c16]. The k loop is unrolled (a fixed 13 steps), so the operand LDS
// reads of later steps are issued ahead of the MFMAs.
template <class FA, class FB>
__device__ __forceinline__ void crew_mm(f64x4 (&acc)[4], int cw, FA fa, FB fb) {
  const int lane = threadIdx.x & 63, k4 = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int R = 0; R < 4; ++R) acc[R] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k0 = 0; k0 < 4 * QT; k0 += 4) {
    const int kk = k0 + k4;
    const double bv = fb(kk, 16 * cw + c16);
#pragma unroll
    for (int R = 0; R < 4; ++R) acc[R] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa(16 * R + c16, kk), bv, acc[R], 0, 0, 0);
  }
}

// quad_gemv's register matrix from a quad-LDS-layout image in global memory (one 16-B load per pair,
// sc0: past L1, which may still hold the slot's previous image)
__device__ __forceinline__ void load_img(double (&M)[4][QT], const double* img) {
  const int lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(img);
#pragma unroll
  for (int t = 0; t < QT; t += 2)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const u32x4 g = __builtin_amdgcn_raw_buffer_load_b128(rs, (((t >> 1) * 4 + r) * 128 + 2 * lane) * 8, 0, 1);
      M[r][t] = __longlong_as_double((long long)(((unsigned long long)g.y << 32) | g.x));
      if (t + 1 < QT) M[r][t + 1] = __longlong_as_double((long long)(((unsigned long long)g.w << 32) | g.z));
    }
}

// crew_sync with a deadline (the pipeline kernel ends even if a crew wave is gone)
__device__ __forceinline__ void crew_sync_dl(int* cnt, int& gen, unsigned long long dl) {
  gen += CREW;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  for (int spin = 0; __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < gen; ++spin) {
    __builtin_amdgcn_s_sleep(1);
    if ((spin & 255) == 255 && __builtin_amdgcn_s_memrealtime() > dl) break;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Coalesced write of a quad-LDS-layout image from a row-major LDS matrix M ([64][HS], element (row, col);
// trans: element (col, row)) by the crew's 256 threads: one 16-byte store per (t, t + 1) pair
__device__ __forceinline__ void crew_copy_out(double* img, const double* M, bool trans) {
  for (int e2 = (int)threadIdx.x - 256; 2 * e2 < QB; e2 += 256) {
    const int e = 2 * e2;  // elements e (t even) and e + 1 (t odd) of one lane's pair
    const int blk = e >> 7, within = e & 127;
    const int r = blk & 3, th = blk >> 2, lq = within >> 1;
    const int row = (lq & 15) + 16 * r, c0 = (lq >> 4) + 8 * th, c1 = c0 + 4;
    const double v0 = trans ? M[c0 * HS + row] : M[row * HS + c0];
    const double v1 = trans ? M[c1 * HS + row] : M[row * HS + c1];
    *reinterpret_cast<double2*>(img + e) = double2{v0, v1};
  }
}

// One refresh for the pipeline: P (Gauss-Jordan, or one Newton-Schulz step from the image `src`), then
// B = P X^T, XP = B^T (= X P: P symmetric) and XB = X B, all into the global image `out`.
__device__ __attribute__((noinline)) void crew_refresh_rec(double* lds, const RLds& L, int m, int d, double shift, int cw, int* cnt, int& gen,
                                 double* out, long long* tl, const double* src,
                                 unsigned long long dl) {
  const int lane = threadIdx.x & 63, k4 = lane >> 4, c16 = lane & 15, cc = 16 * cw + c16;
  const double* XT = lds + L.xt;  // X[i][j] = XT[j * HS + i] (zero for j >= d or i >= m)
  double* Hs = lds + L.hs;
  double* Hp = lds + L.hp;
  const double* wq = lds + L.wq;
  f64x4 acc[4];
  // Hessian tiles: H = X^T diag(w) X + shift I (identity padding)
  crew_mm(acc, cw, [&](int row, int kk) { return wq[kk] * XT[row * HS + kk]; },
          [&](int kk, int col) { return XT[col * HS + kk]; });
#pragma unroll
  for (int R = 0; R < 4; ++R)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int row = 16 * R + k4 + 4 * reg;
      Hs[row * HS + cc] = (row < d && cc < d) ? acc[R][reg] + (row == cc ? shift : 0.0) : (row == cc ? 1.0 : 0.0);
    }
  if (src) {  // the image's P into Hp (row-major, zero padding) while the Hessian completes (sc0 loads)
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(src);
    for (int e2 = (int)threadIdx.x - 256; 2 * e2 < QB; e2 += 256) {
      const u32x4 gv = __builtin_amdgcn_raw_buffer_load_b128(rs, e2 * 16, 0, 1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = 2 * e2 + h;
        const int blk = e >> 7, within = e & 127;
        const int r = blk & 3, th = blk >> 2, lq = within >> 1, t = 2 * th + (within & 1);
        Hp[((lq & 15) + 16 * r) * HS + (lq >> 4) + 4 * t] =
            __longlong_as_double((long long)(((unsigned long long)(h ? gv.w : gv.y) << 32) | (h ? gv.z : gv.x)));
      }
    }
    for (int e = (int)threadIdx.x - 256; e < 64 * 8; e += 256) Hp[(e >> 3) * HS + QCOLS + (e & 7)] = 0.0;
  }
  crew_sync_dl(cnt, gen, dl);
  if (tl && cw == 0 && lane == 0) tl[1] = (long long)__builtin_amdgcn_s_memrealtime();
  if (src) {
    // T = H X0 -> Hs;  U = X0 T;  X1 = 2 X0 - U -> Hp
    crew_mm(acc, cw, [&](int row, int kk) { return Hs[row * HS + kk]; }, [&](int kk, int col) { return Hp[kk * HS + col]; });
    crew_sync_dl(cnt, gen, dl);
#pragma unroll
    for (int R = 0; R < 4; ++R)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) Hs[(16 * R + k4 + 4 * reg) * HS + cc] = acc[R][reg];
    crew_sync_dl(cnt, gen, dl);
    crew_mm(acc, cw, [&](int row, int kk) { return Hp[row * HS + kk]; }, [&](int kk, int col) { return Hs[kk * HS + col]; });
    crew_sync_dl(cnt, gen, dl);  // every wave is done reading X0
#pragma unroll
    for (int R = 0; R < 4; ++R)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int row = 16 * R + k4 + 4 * reg;
        Hp[row * HS + cc] = (row < d && cc < d) ? 2.0 * Hp[row * HS + cc] - acc[R][reg] : 0.0;
      }
  } else {
    // in-place block Gauss-Jordan (the one-wave kernel's crew_refresh, same arithmetic)
    const int i = lane;
    double h[NCW];
#pragma unroll
    for (int c = 0; c < NCW; ++c) h[c] = Hs[i * HS + cw + CREW * c];
    const int nb = (d + 3) >> 2;
    double* slabs = lds + L.slab;
    for (int bb = 0; bb < nb; ++bb) {
      const int p = 4 * bb;
      double* slab = slabs + (bb & 1) * 256;
      {
        double hv = 0.0;
#pragma unroll
        for (int c = 0; c < NCW; ++c) hv = (c == bb) ? h[c] : hv;
        slab[cw * 64 + i] = hv;
      }
      crew_sync_dl(cnt, gen, dl);
      double P[4][4], Rr[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        Rr[q] = slab[q * 64 + i];
#pragma unroll
        for (int r = 0; r < 4; ++r) P[q][r] = slab[q * 64 + p + r];
      }
      const bool pivrow = (i >> 2) == bb;
      if (pivrow) {
#pragma unroll
        for (int q = 0; q < 4; ++q) Rr[q] = (q == (i & 3)) ? 1.0 : 0.0;
      }
      const double a00 = P[0][0], a01 = P[1][0], a11 = P[1][1];
      const double ia = rcp_nr(fma(a00, a11, -a01 * a01));
      const double A00 = a11 * ia, A01 = -a01 * ia, A11 = a00 * ia;
      const double b00 = P[2][0], b01 = P[3][0], b10 = P[2][1], b11 = P[3][1];
      const double w00 = fma(A00, b00, A01 * b10), w01 = fma(A00, b01, A01 * b11);
      const double w10 = fma(A01, b00, A11 * b10), w11 = fma(A01, b01, A11 * b11);
      const double s00 = P[2][2] - fma(b00, w00, b10 * w10);
      const double s01 = P[3][2] - fma(b00, w01, b10 * w11);
      const double s11 = P[3][3] - fma(b01, w01, b11 * w11);
      const double is = rcp_nr(fma(s00, s11, -s01 * s01));
      const double y0 = fma(A00, Rr[0], A01 * Rr[1]), y1 = fma(A01, Rr[0], A11 * Rr[1]);
      const double z2 = Rr[2] - fma(b00, y0, b10 * y1), z3 = Rr[3] - fma(b01, y0, b11 * y1);
      const double l2 = fma(s11, z2, -s01 * z3) * is, l3 = fma(s00, z3, -s01 * z2) * is;
      const double l0 = y0 - fma(w00, l2, w01 * l3), l1 = y1 - fma(w10, l2, w11 * l3);
      const double lw = cw == 0 ? l0 : (cw == 1 ? l1 : (cw == 2 ? l2 : l3));
#pragma unroll
      for (int c = 0; c < NCW; ++c) {
        const int j = cw + CREW * c;
        const double tq = fma(l0, slab[j], fma(l1, slab[64 + j], fma(l2, slab[128 + j], l3 * slab[192 + j])));
        const bool inK = c == bb;
        const double sg = j < p ? -1.0 : 1.0;
        double v;
        if (inK) v = pivrow ? lw : -lw;
        else v = pivrow ? sg * tq : fma(-sg, tq, h[c]);
        h[c] = v;
      }
    }
#pragma unroll
    for (int c = 0; c < NCW; ++c) {
      const int col = cw + CREW * c;
      Hp[i * HS + col] = (i < d && col < d) ? h[c] : 0.0;
    }
  }
  crew_sync_dl(cnt, gen, dl);
  if (tl && cw == 0 && lane == 0) tl[2] = (long long)__builtin_amdgcn_s_memrealtime();
  crew_copy_out(out, Hp, false);  // image 0: P
  // B = P X^T (rows: features, cols: samples) -> Hs row-major -> image 1, its transpose XP -> image 2
  crew_mm(acc, cw, [&](int row, int kk) { return Hp[row * HS + kk]; },
          [&](int kk, int col) { return XT[kk * HS + col]; });
#pragma unroll
  for (int R = 0; R < 4; ++R)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int row = 16 * R + k4 + 4 * reg;
      Hs[row * HS + cc] = (row < d && cc < m) ? acc[R][reg] : 0.0;
    }
  crew_sync_dl(cnt, gen, dl);  // B complete in Hs; every read of P in Hp done
  crew_copy_out(out + QB, Hs, false);
  crew_copy_out(out + 2 * QB, Hs, true);
  // XB = X B (m x m) -> image 3
  crew_mm(acc, cw, [&](int row, int kk) { return XT[kk * HS + row]; },
          [&](int kk, int col) { return Hs[kk * HS + col]; });
#pragma unroll
  for (int R = 0; R < 4; ++R)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int row = 16 * R + k4 + 4 * reg;
      Hp[row * HS + cc] = (row < m && cc < m) ? acc[R][reg] : 0.0;
    }
  crew_sync_dl(cnt, gen, dl);
  crew_copy_out(out + 3 * QB, Hp, false);
  wg_release();  // the image's global stores complete before `ready` is posted
  crew_sync_dl(cnt, gen, dl);
}

}  // namespace

template <bool SYS>
__global__ void __launch_bounds__(RT) chain_persistent_newton_rec_kernel(PersistArgs a, LogiArgs g) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ NCtl nc;
  __shared__ int pc[PC_N];
  const int d = a.d, n = a.n, m = g.m;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t rth = rsrc_of(a.thg);
  const __amdgpu_buffer_rsrc_t rob = rsrc_of(a.objg);
  const unsigned long long deadline = now_ticks() + (unsigned long long)a.timeout_ticks;
  // XCD packing (PersistArgs::xcd, one GPU): the launch has 8x the blocks and only every 8th works, so
  // all of them share one XCD's L2; with the placement verified, theta / objective granules are plain
  // write-back stores that stay in that L2 (a neighbour's poll is an L2 hit, not a fabric round trip)
  __shared__ int xcd_lds;
  const bool packed = !SYS && a.xcd > 0;
  if (packed && (blockIdx.x & 7u)) return;
  const int bid = packed ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
  bool local = false;
  if (!SYS && a.xcd > 1) local = xcd_verdict(a.xchk, bid, a.n_local + (a.has_monitor ? 1 : 0), deadline, &xcd_lds, (unsigned)a.xtag);
  if (!SYS && bid == 0 && threadIdx.x == 0) a.ctl->placed = a.xcd > 0 ? (local ? 2 : 1) : 0;
  const RLds L;

  if (a.has_monitor && bid == a.n_local) {  // the monitor: the one-wave kernel's
    if (wid != 0) return;
    double* vals = lds;
    for (int it = a.start_iter;; ++it) {
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
      }
      if (__shfl((int)code, 0, 64)) return;
    }
  }
  if (bid >= a.n_local) return;

  const PhaseSlot sl = a.slots[bid];
  const int li = sl.li, w = sl.gid, left = sl.left, right = sl.right;
  const bool head = (a.pos[bid] % 2) == 0;
  const double rho = a.rho, lam = g.lam, chord = g.step;
  const double shift = lam + rho * (double)((left >= 0 ? 1 : 0) + (right >= 0 ? 1 : 0));
  const double* Xg = g.X + (long)li * m * d;
  double* const img0 = g.scratch + (long)li * RSLOTS * RIMG;
  // per-step stamps of the first 24 segments (timeline_iters >= 512, tools/newton_rec_steps.py): row
  // 128 + 16 (sg - 1) + k; cols 0 S posted s_k, 1 T posted y_{k+1}, 2 H posted b_k, 3 W posted w_k,
  // 4 S got w_k, 5 T got b_k
  long long* const stp = (a.timeline && a.timeline_iters >= 512) ? a.timeline + ((long)li * a.timeline_iters + 128) * 8
                                                                 : nullptr;
#define REC_STAMP(col, sg_, k_)                                                                      \
  do {                                                                                             \
    if (stp && (threadIdx.x & 63) == 0 && (sg_) >= 1 && (sg_) <= 24 && (k_) < 16)                   \
      stp[((long)((sg_) - 1) * 16 + (k_)) * 8 + (col)] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
  const bool inj = lane < d, ini = lane < m;
  // set-up: X^T (row-major) and X (quad-LDS layout) into LDS, protocol words, the exact margins and refresh
  // weights at the start point theta^{start - 1}; the crew builds refresh 0 (Gauss-Jordan) from there
  for (int e = threadIdx.x; e < QB; e += RT) {
    const int blk = e >> 7, within = e & 127;
    const int r = blk & 3, th = blk >> 2, lq = within >> 1, t = 2 * th + (within & 1);
    const int row = (lq & 15) + 16 * r, col = (lq >> 4) + 4 * t;
    lds[L.xq + e] = (row < m && col < d && t < QT) ? Xg[(long)row * d + col] : 0.0;  // (sample, feature)
  }
  for (int e = threadIdx.x; e < 64 * 64; e += RT) {  // X^T row-major (feature j, sample i)
    const int j = e >> 6, i = e & 63;
    lds[L.xt + j * HS + i] = (j < d && i < m) ? Xg[(long)i * d + j] : 0.0;
  }
  if (threadIdx.x == 0) {
    nc.req = 0;
    nc.ready = -1;
    nc.cnt = 0;
    nc.src = -1;
    nc.shift = shift;
    nc.quit = 0;
  }
  if (threadIdx.x < PC_N) pc[threadIdx.x] = threadIdx.x == PC_Z0 ? 1 : 0;
  if (threadIdx.x < 64) {
    const int i = threadIdx.x;
    double z = 0.0, wi = 0.0;
    if (i < m) {
      for (int j = 0; j < d; ++j) z = fma(Xg[(long)i * d + j], a.theta[(long)w * d + j], z);
      const double pz = 1.0 / (1.0 + exp(g.Y[(long)li * m + i] * z));
      wi = pz * (1.0 - pz);
    }
    lds[L.wq + i] = wi;
    lds[L.z0v + i] = i < m ? z : 0.0;
  }
  lds_barrier();  // the only workgroup-wide barrier

  const double yv = ini ? g.Y[(long)li * m + lane] : 0.0;
  const bool post_fence = (a.dbg & (1 << 17)) != 0;
  auto ready_or_quit = [&](int r) -> bool {  // the crew finished refresh r (false: quit / deadline)
    for (int spin = 0;; ++spin) {
      if (lds_load_acq(&nc.ready) >= r) {
        wg_acquire();
        return true;
      }
      if (lds_load_acq(&pc[PC_QUIT])) return false;
      if ((spin & 63) == 63 && now_ticks() > deadline) return false;
      __builtin_amdgcn_s_sleep(1);
    }
  };
  // a pipeline wave's wait for pc[flag] >= want; 1: there, 0: segment sg ended, -1: quit / deadline
  // Issue priorities: a pipeline wave computes at 2 and spins at 0, the crew runs at 1, so a spinning
  // wave never takes a SIMD's issue slot from the crew wave it shares the SIMD with, nor the crew one
  // from a pipeline wave that has work.
  auto wait_step = [&](int flag, int want, int sg) -> int {
    if (lds_load_acq(&pc[flag]) >= want) return 1;
    __builtin_amdgcn_s_setprio(0);
    int res = 0;
    for (int spin = 0;; ++spin) {
      if (lds_load_acq(&pc[flag]) >= want) { res = 1; break; }
      if (lds_load_acq(&pc[PC_END]) >= sg) break;
      if ((spin & 63) == 63) {
        if (lds_load_acq(&pc[PC_QUIT]) || now_ticks() > deadline) { res = -1; break; }
      }
      if (spin >= 256) __builtin_amdgcn_s_sleep(1);  // a long wait (the idle phase): poll gently
    }
    __builtin_amdgcn_s_setprio(2);
    return res;
  };

  if (wid >= 4) {
    // ---------------------------------------------------------------- crew (waves 4-7)
    const int cw = wid - 4;
    int gen = 0, done_req = -1;
    __builtin_amdgcn_s_setprio(1);
    for (;;) {
      int r;  // quit before req (see the one-wave kernel's crew): W's last request precedes T's quit
      for (int spin = 0;; ++spin) {
        const int q = lds_load_acq(&nc.quit);
        r = lds_load_acq(&nc.req);
        if (r != done_req) break;
        if (q) return;
        if ((spin & 63) == 63 && now_ticks() > deadline + 100000000ull) return;
        __builtin_amdgcn_s_sleep(1);
      }
      long long* tl = (a.timeline && r < 64) ? a.timeline + ((long)li * a.timeline_iters + r) * 8 : nullptr;
      if (tl && cw == 0 && lane == 0) tl[0] = (long long)__builtin_amdgcn_s_memrealtime();
      const int srcr = nc.src;
      crew_refresh_rec(lds, L, m, d, nc.shift, cw, &nc.cnt, gen, img0 + (long)(r % RSLOTS) * RIMG, tl,
                       srcr >= 0 ? img0 + (long)(srcr % RSLOTS) * RIMG : nullptr, deadline + 50000000ull);
      if (tl && cw == 0 && lane == 0) tl[3] = (long long)__builtin_amdgcn_s_memrealtime();
      if (cw == 0 && lane == 0) lds_store_rel(&nc.ready, r);
      done_req = r;
    }
  }

  double* const sring = lds + L.sring;
  double* const yring = lds + L.yring;
  double* const vring = lds + L.vring;
  double* const wring = lds + L.wring;
  // This wave's register matrix (S: XB, T: P, H: B, W: XP), loaded at ONE place per loop (a conditional
  // reload of a loop-carried register array made the compiler keep two copies and spill): refresh 0
  // before the first segment, then at the end of every segment the matrix of the next one (pc[PC_ENEXT],
  // the phase's idle time except after an urgent refresh).
  double Mq[4][QT];
  const int part = wid == 0 ? 3 : wid == 1 ? 0 : wid == 2 ? 1 : 2;
  const double* const mimg = img0 + (long)part * QB;
  if (wid != 1) {
    // ------------------------------------------------ S (wave 0), H (wave 2), W (wave 3)
    const bool fast_sig = (a.dbg & 32) == 0;
    double* st = lds + L.stage;
    __builtin_amdgcn_s_setprio(2);
    if (!ready_or_quit(0)) return;
    load_img(Mq, mimg);
    // No wait for the segment's start: s_0 = y sigma(-y z_0) and b_0 = B s_0 depend only on the start
    // point (this worker's own iterate, exact margins from W) and the inverse announced at the previous
    // segment's end, so S and H form them during the idle phase; W waits for y_0 (the neighbours' theta).
    for (int sg = 1;; ++sg) {
      const int base = sg * 1024;
      if (wid == 0) {  // S: the margins
        for (int spin = 0;; ++spin) {
          if (lds_load_acq(&pc[PC_Z0]) >= sg) break;
          if ((spin & 63) == 63 && (lds_load_acq(&pc[PC_QUIT]) || now_ticks() > deadline)) return;
        }
        double z = lds[L.z0v + lane];
        for (int k = 0;; ++k) {
          const double sv = ini ? (fast_sig ? yv * inv1pexp_fast(yv * z) : yv / (1.0 + exp(yv * z))) : 0.0;
          double* slot = sring + (k % RR) * 4 * QX;
          slot[(lane & 3) * QX + (lane >> 2)] = sv;
          lds_post(&pc[PC_S], base + k + 1, post_fence);
          REC_STAMP(0, sg, k);
          const double u = quad_gemv_staged<QT>(Mq, slot);  // (XB s_k)_i
          const int got = wait_step(PC_W, base + k + 1, sg);
          if (got < 0) return;
          if (got == 0) break;
          REC_STAMP(4, sg, k);
          z = ini ? (z - wring[(k % RR) * 64 + lane]) + u : 0.0;
        }
      } else {  // H (wave 2): b_k = B s_k;  W: w_k = XP y_k
        const int flag = wid == 2 ? PC_V : PC_W;
        double* ring = wid == 2 ? vring : wring;
        const int src_flag = wid == 2 ? PC_S : PC_Y;
        double* const src_ring = wid == 2 ? sring : yring;
        for (int k = 0;; ++k) {
          const int got = wait_step(src_flag, base + k + 1, sg);
          if (got < 0) return;
          if (got == 0) break;
          const double v = quad_gemv_staged<QT>(Mq, src_ring + (k % RR) * 4 * QX);
          ring[(k % RR) * 64 + lane] = v;
          lds_post(&pc[flag], base + k + 1, post_fence);
          REC_STAMP(wid, sg, k);
        }
        if (wid == 3) {  // W: the segment's end -- exact margins at its final iterate
          for (int spin = 0;; ++spin) {
            if (lds_load_acq(&pc[PC_END]) >= sg) break;
            if ((spin & 63) == 63 && (lds_load_acq(&pc[PC_QUIT]) || now_ticks() > deadline)) return;
          }
          const double x = lds[L.xfin + lane];
          const double z = quad_gemv_lds<QT>(lds + L.xq, x, st);
          lds[L.z0v + lane] = ini ? z : 0.0;
          lds_store_rel(&pc[PC_Z0], sg + 1);
          const int kind = pc[PC_EKIND], req = pc[PC_EREQ], src = pc[PC_ESRC], it = pc[PC_EIT];
          if (kind == 1) {  // a local solve ended: f_n(theta^it) -> monitor
            const double partv = wave_sum_f64(ini ? softplus(-yv * z) : 0.0);
            const double xx = wave_sum_f64(inj ? x * x : 0.0);
            if (lane == 0)
              put_granule<SYS>(local, rob, ((it % a.ring) * n + w) * 16, make_tag(a.epoch, it), lam * 0.5 * xx + partv);
          }
          if (req >= 0) {  // a refresh at this iterate (the crew is idle: see the iterate wave)
            const double pz = ini ? 1.0 / (1.0 + exp(yv * z)) : 0.5;
            lds[L.wq + lane] = ini ? pz * (1.0 - pz) : 0.0;
            nc.src = src;
            lds_store_rel(&nc.req, req);
          }
          lds_store_rel(&pc[PC_WDONE], sg);  // T's quit waits for this (no request after the quit)
        }
      }
      if (wid != 3) {  // S / H: the segment is over once T posted its end
        for (int spin = 0;; ++spin) {
          if (lds_load_acq(&pc[PC_END]) >= sg) break;
          if ((spin & 63) == 63 && (lds_load_acq(&pc[PC_QUIT]) || now_ticks() > deadline)) return;
        }
      }
      const int nx = pc[PC_ENEXT];  // the next segment's matrix, loaded while idle
      if (!ready_or_quit(nx)) return;
      load_img(Mq, mimg + (long)(nx % RSLOTS) * RIMG);
    }
  }

  // ------------------------------------------------------------------ T (wave 1): iterate + protocol
  u32x4* const p0 = a.push ? a.push[2 * bid] : nullptr;
  u32x4* const p1 = a.push ? a.push[2 * bid + 1] : nullptr;
  const __amdgpu_buffer_rsrc_t rp0 = rsrc_of(p0 ? (const void*)p0 : (const void*)a.thg);
  const __amdgpu_buffer_rsrc_t rp1 = rsrc_of(p1 ? (const void*)p1 : (const void*)a.thg);
  double th = inj ? a.theta[(long)w * d + lane] : 0.0;
  double mu = inj ? a.mu[(long)li * d + lane] : 0.0;
  double tl = (inj && left >= 0) ? a.theta[(long)left * d + lane] : 0.0;
  double tr = (inj && right >= 0) ? a.theta[(long)right * d + lane] : 0.0;
  int pending = a.pending_in;
  int stop_code = 0, stop_iter = 0, abort = 0, used = 0, nfail = 0;
  // a background refresh requested at iteration i is adopted at i + RLAG; one is requested when a solve
  // took more than bg_steps chord steps (PersistArgs::dbg bits 8-11 / 12-15 override: GADMM_NEWTON_RLAG,
  // GADMM_NEWTON_BG)
  const int RLAG = ((a.dbg >> 8) & 15) ? ((a.dbg >> 8) & 15) : REC_RLAG;
  int cur = 0, pend = -1, pend_it = 0, next_id = 0, sg = 0;
  bool cur_fresh = true;
  const int bg_steps = ((a.dbg >> 12) & 15) ? ((a.dbg >> 12) & 15)
                                            : (g.max_inner >= 1 && g.max_inner < NMAX) ? g.max_inner : REC_BG;
  const bool ns_bg = g.inner_tol >= 0.0;
  const bool urgent_ns = ns_bg && (a.dbg & (1 << 16));  // GADMM_NEWTON_URGENT_NS=1
  auto wait_ready = [&](int r) -> bool {
    for (int spin = 0;; ++spin) {
      if (lds_load_acq(&nc.ready) >= r) {
        wg_acquire();
        return true;
      }
      if ((spin & 63) == 63 && now_ticks() > deadline) return false;
      __builtin_amdgcn_s_sleep(1);
    }
  };
  if (!wait_ready(0)) abort = 1;
  load_img(Mq, mimg);
  __builtin_amdgcn_s_setprio(2);

  int it = a.start_iter;
  for (; !abort; ++it) {
    if (it > a.max_iter + a.lag) break;
    const bool check = it - a.start_iter >= a.lag;
    const int jdec = it - a.lag;
    const bool need_nb = head ? it > a.start_iter : true;
    const int jnb = head ? it - 1 : it;
    const unsigned tnb = make_tag(a.epoch, jnb), tj = make_tag(a.epoch, jdec);
    const int ra = need_nb ? left : -1, rb = need_nb ? right : -1;
    bool decided = !check;
    unsigned long long dv = 0;
    int outcome = 0;
    const int kk_tl = it - a.start_iter;
    long long* tls = (a.timeline && kk_tl < 64) ? a.timeline + ((long)li * a.timeline_iters + 64 + kk_tl) * 8 : nullptr;
    long long t_nb = 0, t_dec = 0;  // (instrumented runs) when the neighbours' theta / the decision arrived
    for (int spin = 0;; ++spin) {
      bool nb = true;
      if (inj) {
        if (ra >= 0) nb &= load_granule<SYS>(rth, (ra * d + lane) * 16, tnb, &tl);
        if (rb >= 0) nb &= load_granule<SYS>(rth, (rb * d + lane) * 16, tnb, &tr);
      }
      if (!decided) {
        dv = __shfl(load_dec<SYS>(&a.decg[jdec % a.ring]), 0, 64);
        decided = (unsigned)(dv >> 32) == tj;
      }
      if (tls) {
        const long long now = (long long)__builtin_amdgcn_s_memrealtime();
        if (!t_nb && __all(nb)) t_nb = now;
        if (!t_dec && decided) t_dec = now;
      }
      if (decided && (unsigned)(dv & 0xffffffffu) != 0u) { outcome = 2; break; }
      if (decided && __all(nb)) { outcome = 1; break; }
      if ((spin & 7) == 7 && now_ticks() > deadline) { outcome = 3; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (outcome != 1) {
      if (outcome == 2) {
        stop_code = (int)(unsigned)(dv & 0xffffffffu);
        stop_iter = jdec;
      } else {
        abort = 1;
      }
      break;
    }
    double cv = 0.0, x = 0.0;
    if (inj) {
      double mm = mu;
      if (head && pending) {
        if (left >= 0) mm = mm - rho * (tl - th);
        if (right >= 0) mm = mm + rho * (th - tr);
        mu = mm;
      }
      cv = mm;
      if (left >= 0) cv = cv - rho * tl;
      if (right >= 0) cv = cv - rho * tr;
      x = th;
    }
    if (tls && lane == 0) {
      tls[0] = (long long)__builtin_amdgcn_s_memrealtime();
      tls[6] = t_nb;
      tls[7] = t_dec;
    }
    if (pend >= 0 && it - pend_it >= RLAG) {  // adopt the background refresh (preloaded by S, H, W)
      cur = pend;
      pend = -1;
      cur_fresh = false;
    }
    double nd_prev = 0.0;
    used = 0;
    bool urgent = false, fresh = cur_fresh;
    cur_fresh = false;
    int ks = 0;  // chord steps of this local solve (all segments)
    for (;;) {   // segments: the solve, and its continuation after each urgent refresh (Mq: refresh cur)
      if (tls && lane == 0 && ks == 0) tls[1] = (long long)__builtin_amdgcn_s_memrealtime();
      ++sg;
      const int base = sg * 1024;
      yring[(lane & 3) * QX + (lane >> 2)] = inj ? fma(shift, x, cv) : 0.0;  // y_0 (slot 0)
      lds_post(&pc[PC_Y], base + 1, post_fence);
      double v = quad_gemv_staged<QT>(Mq, yring);  // v_0 = P y_0 (T's register matrix: P)
      int reason = 0;  // 1: the solve ends, 2: urgent refresh
      for (int k = 0;; ++k) {
        const int want = base + k + 1;
        bool got = lds_load_acq(&pc[PC_V]) >= want;  // b_k = B s_k from H
        if (!got) {
          __builtin_amdgcn_s_setprio(0);
          for (int spin = 0;; ++spin) {
            if (lds_load_acq(&pc[PC_V]) >= want) { got = true; break; }
            if ((spin & 63) == 63 && now_ticks() > deadline) break;
          }
          __builtin_amdgcn_s_setprio(2);
        }
        if (!got) { abort = 1; break; }
        REC_STAMP(5, sg, k);
        const double dxl = inj ? v - vring[(k % RR) * 64 + lane] : 0.0;  // dx_k = P y_k - B s_k
        x = inj ? x - dxl : 0.0;
        double* const ynext = yring + ((k + 1) % RR) * 4 * QX;
        ynext[(lane & 3) * QX + (lane >> 2)] = inj ? fma(shift, x, cv) : 0.0;
        lds_post(&pc[PC_Y], want + 1, post_fence);
        REC_STAMP(1, sg, k);
        const double mdx = wave_max_abs_dpp(dxl), mx = wave_max_abs_dpp(x);
        used = ++ks;
        if (mdx < NTOL * fmax(1.0, mx) || ks >= NMAX) {
          if (!(mdx < NTOL * fmax(1.0, mx))) ++nfail;  // the step cap ends this solve unconverged
          reason = 1;
          break;
        }
        if (chord <= 0.0 || (!fresh && ks > 1 && mdx > chord * nd_prev)) { reason = 2; break; }
        fresh = false;
        nd_prev = mdx;
        v = quad_gemv_staged<QT>(Mq, ynext);  // v_{k+1} = P y_{k+1}, while H waits for s_{k+1}
      }
      if (abort) break;
      lds[L.xfin + lane] = x;
      if (reason == 2) {
        // contraction too slow: an exact inverse at the current x (W posts the request once it has the
        // weights there); the crew first finishes a background refresh in progress
        if (pend >= 0) {
          if (!wait_ready(pend)) { abort = 1; break; }
          pend = -1;
        }
        const int src_u = urgent_ns ? cur : -1;  // one Newton-Schulz step from the inverse in use, or exact
        cur = ++next_id;
        pc[PC_EKIND] = 0;
        pc[PC_EREQ] = cur;
        pc[PC_ESRC] = src_u;
        pc[PC_ENEXT] = cur;
        pc[PC_EIT] = it;
        lds_store_rel(&pc[PC_END], sg);
        urgent = true;
        fresh = true;
        nd_prev = 0.0;
        if (!wait_ready(cur)) { abort = 1; break; }
        load_img(Mq, mimg + (long)(cur % RSLOTS) * RIMG);
        continue;
      }
      break;
    }
    if (abort) break;
    if (tls && lane == 0) {
      tls[2] = (long long)__builtin_amdgcn_s_memrealtime();
      tls[3] = used;
      tls[4] = next_id;
    }
    // publish theta^it first (the neighbours wait for it)
    const unsigned tag = make_tag(a.epoch, it);
    if (inj) {
      put_granule<SYS>(local, rth, (w * d + lane) * 16, tag, x);
      if (p0) store_granule<SYS>(rp0, (w * d + lane) * 16, tag, x);
      if (p1) store_granule<SYS>(rp1, (w * d + lane) * 16, tag, x);
    }
    // end of the solve: W takes f_n, the exact margins and (maybe) a background refresh request from here
    int req = -1, src = -1;
    if ((used > bg_steps || urgent) && pend < 0) {
      pend = req = ++next_id;
      pend_it = it;
      src = ns_bg ? cur : -1;
    }
    const int nx = (pend >= 0 && it + 1 - pend_it >= RLAG) ? pend : cur;  // the next phase's inverse
    pc[PC_EKIND] = 1;
    pc[PC_EREQ] = req;
    pc[PC_ESRC] = src;
    pc[PC_ENEXT] = nx;
    pc[PC_EIT] = it;
    lds_store_rel(&pc[PC_END], sg);
    if (!head) {
      double rp = 0.0;
      if (inj) {
        double mm = mu;
        if (left >= 0) mm = mm - rho * (tl - x);
        if (right >= 0) mm = mm + rho * (x - tr);
        mu = mm;
        if (left >= 0) rp = fma(tl - x, tl - x, rp);
        if (right >= 0) rp = fma(x - tr, x - tr, rp);
      }
      if (a.rres) {
        const double rs = wave_sum_f64(rp);
        if (lane == 0 && it - 1 < a.max_iter) a.rres[(long)(it - 1) * n + w] = rs;
      }
    } else {
      pending = 1;
    }
    th = x;
    if (!wait_ready(nx)) { abort = 1; break; }
    load_img(Mq, mimg + (long)(nx % RSLOTS) * RIMG);
    if (tls && lane == 0) tls[5] = (long long)__builtin_amdgcn_s_memrealtime();  // next inverse in VGPRs
  }
  if (!abort) {  // W's end-of-segment work (and its refresh request, if any) precedes the quit
    for (int spin = 0;; ++spin) {
      if (lds_load_acq(&pc[PC_WDONE]) >= sg) break;
      if ((spin & 63) == 63 && now_ticks() > deadline) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  lds_store_rel(&pc[PC_QUIT], 1);  // S, H, W leave
  lds_store_rel(&nc.quit, 1);      // the crew leaves after serving every request
  if (inj) {
    a.theta[(long)w * d + lane] = th;
    a.mu[(long)li * d + lane] = mu;
  }
  if (lane == 0) {
    if (g.inner_iters) g.inner_iters[li] = used;
    if (nfail) atomicAdd(&a.ctl->inner_fail, nfail);  // read by the host after the launch
    if (abort) {
      a.ctl->done = 4;
    } else if (bid == 0 && stop_code) {
      a.ctl->done = stop_code;
      a.ctl->conv_iter = stop_iter;
      a.ctl->iter = it;
      a.ctl->pending = 1;
      a.ctl->monitored = stop_iter;
    }
  }
}

extern "C" long gadmm_resident_capacity(const void* fn, int threads, size_t shm);
extern "C" int gadmm_xcd_mode(const PersistArgs* a, int blocks, long cap_total);  // chain_persistent.hip
extern "C" unsigned gadmm_next_xtag();  // chain_persistent.hip

// The pipeline kernel is the default; GADMM_NEWTON_REC=0 selects the one-wave solver kernel.
static bool newton_rec(const LogiArgs& g) {
  const char* e = getenv("GADMM_NEWTON_REC");
  return g.scratch != nullptr && !(e && e[0] == '0');
}

static const void* newton_variant(const PersistArgs& a, const LogiArgs& g) {
  if (a.d > 4 * QT || g.m > 4 * QT || a.d < 1 || g.m < 1 || a.n_epochs > 0) return nullptr;
  if (newton_rec(g))
    return a.sys_scope ? (const void*)chain_persistent_newton_rec_kernel<true>
                       : (const void*)chain_persistent_newton_rec_kernel<false>;
  return a.sys_scope ? (const void*)chain_persistent_newton_kernel<true>
                     : (const void*)chain_persistent_newton_kernel<false>;
}

static int newton_threads(const LogiArgs& g) { return newton_rec(g) ? RT : NT; }

static size_t newton_shm(const PersistArgs& a, const LogiArgs& g) {
  size_t b = newton_rec(g) ? (size_t)RLds().total * 8 : (size_t)NLds(g.m, a.d).total * 8;
  if (b < (size_t)a.n * 8) b = (size_t)a.n * 8;  // the monitor stages one double per worker
  return b;
}

extern "C" {

long gadmm_chain_persistent_newton_capacity(const PersistArgs* args, const LogiArgs* g) {
  const void* fn = newton_variant(*args, *g);
  return fn ? gadmm_resident_capacity(fn, newton_threads(*g), newton_shm(*args, *g)) : 0;
}

int gadmm_chain_persistent_newton_launch(const PersistArgs* args, const LogiArgs* gargs, hipStream_t st) {
  const PersistArgs& a = *args;
  const LogiArgs& g = *gargs;
  const void* fn = newton_variant(a, g);
  if (!fn || !g.X || !g.Y || a.ring <= a.lag + 1 || a.start_iter + a.max_iter + a.lag >= (1 << 20) ||
      (a.has_monitor && !a.dec_push)) {
    gadmm_set_error("persistent Newton kernel: unsupported configuration (d=%d m=%d)", a.d, g.m);
    return -1;
  }
  const size_t shm = newton_shm(a, g);
  if (shm > 160 * 1024) {
    gadmm_set_error("persistent Newton kernel: %zu B of LDS", shm);
    return -1;
  }
  const int blocks = a.n_local + (a.has_monitor ? 1 : 0);
  const int nt = newton_threads(g);
  const long cap = gadmm_resident_capacity(fn, nt, shm);
  if (blocks > cap) {
    gadmm_set_error("persistent Newton kernel: %d workgroups but only %ld can be resident", blocks, cap);
    return -2;
  }
  if (shm > 65536) GADMM_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  PersistArgs ka = a;
  ka.xcd = newton_rec(g) ? gadmm_xcd_mode(&a, blocks, cap) : 0;  // the pipeline kernel packs onto one XCD
  ka.xtag = (int)gadmm_next_xtag();  // fresh placement-check tag: no memset of xchk
  const char* fs = getenv("GADMM_NEWTON_FASTSIGM");
  if (fs && fs[0] == '0') ka.dbg |= 32;
  const char* rl = getenv("GADMM_NEWTON_RLAG");
  if (rl && atoi(rl) > 0) ka.dbg |= (atoi(rl) & 15) << 8;
  const char* bg = getenv("GADMM_NEWTON_BG");
  if (bg && atoi(bg) > 0) ka.dbg |= (atoi(bg) & 15) << 12;
  const char* pf = getenv("GADMM_NEWTON_POSTFENCE");
  if (pf && pf[0] == '1') ka.dbg |= 1 << 17;
  const char* un = getenv("GADMM_NEWTON_URGENT_NS");
  if (un && un[0] == '1') ka.dbg |= 1 << 16;
  void* kargs[] = {&ka, const_cast<LogiArgs*>(&g)};
  GADMM_CHECK(hipLaunchKernel(fn, dim3(ka.xcd > 0 ? 8 * blocks : blocks), dim3(nt), kargs, shm, st));
  GADMM_CHECK(hipGetLastError());
  return 0;
}

// doubles of LogiArgs::scratch per local worker for the pipeline kernel
long gadmm_newton_rec_scratch_doubles(void) { return (long)RSLOTS * RIMG; }

}  // extern "C"
