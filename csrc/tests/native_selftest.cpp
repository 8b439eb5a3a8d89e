// Native self-test of libgadmm_native's C API, without Python: the kernels and the C++ runtime
// against a plain host (double) reference of the same algorithms. Built twice by
// tools/build_selftest.py: plain, and with host AddressSanitizer + UndefinedBehaviorSanitizer
// (-Xarch_host -fsanitize=...; device code is never instrumented - GPU ASan is not available).
//
//   native_selftest --host-only   ABI, planning and argument-validation paths (no GPU needed)
//   native_selftest               + Gram, inverses, multi-kernel engine (hipGraph), per-worker and
//                                 temporally blocked persistent kernels, first-order engine (GPU)
//
// This is the "race detection / sanitizers" subsystem of SURVEY.md §5 for the native layer: the
// hand-off protocols are exercised end to end under the sanitizers, and every engine's iterates are
// checked against an independent host implementation (a stale neighbour read changes the iterates).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gadmm_chain.h"
#include "gadmm_fo.h"
#include "gadmm_star.h"

extern "C" {
const char* gadmm_last_error();
int gadmm_native_version();
int gadmm_abi_layout(long long* out, int n);
int gadmm_fo_abi_layout(long long* out, int n);
int gadmm_gram_f64(const double* X, const double* Y, int N, int m, int d, int ksplit, double* A, double* B,
                   double* YY, double* slab, hipStream_t st);
int gadmm_spd_inverse_small_f64(const double* A, const double* shift, int N, int d, int nvar, double* out,
                                int* status, hipStream_t st);
void* gadmm_chain_engine_create(const EngineDesc* desc);
void gadmm_chain_engine_destroy(void* h);
int gadmm_chain_engine_set_plan(void* h, int nh, const PhaseSlot* head, int nt, const PhaseSlot* tail, int nxh,
                                const XchgOp* xh, int nxt, const XchgOp* xt);
int gadmm_chain_engine_reset(void* h, int start_iter, int pending);
int gadmm_chain_engine_run(void* h, int block, int stop_iter, int use_graph, RunStats* out);
int gadmm_chain_persistent_launch(const PersistArgs* a, hipStream_t st);
int gadmm_chain_blocked_plan(int n, int d, int want_k, int* k_out, int* len_out);
long gadmm_chain_blocked_tab_granules(int n, int d, int ring);
int gadmm_chain_blocked_launch(const PersistArgs* a, hipStream_t st);
int gadmm_fo_launch(const FoArgs* a, void* stream);
long gadmm_fo_tab_granules(int n, int d, int slots);
long gadmm_spd_inverse_blocked_workspace(int d, int nb);
int gadmm_spd_inverse_blocked_f64(const double* A, const double* shift_host, int N, int d, int nvar, double* out,
                                  double* ws, int* status, int nb, hipStream_t st);
int gadmm_star_launch(const StarArgs* a, hipStream_t st);
int gadmm_star_abi_layout(long long* out, int n);
}

namespace {

int failures = 0;
#define EXPECT(cond, ...)                           \
  do {                                              \
    if (!(cond)) {                                  \
      ++failures;                                   \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);            \
      std::fprintf(stderr, "\n");                   \
    }                                               \
  } while (0)
#define HIPOK(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(2);                                                                      \
    }                                                                                    \
  } while (0)

// ------------------------------------------------------------------ host reference (double)
struct Problem {
  int N, m, d;
  std::vector<double> X, Y, A, b, yy;
};

double lcg_normal(unsigned long long& s) {  // Box-Muller on a 64-bit LCG
  auto u = [&]() {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return ((s >> 11) + 0.5) / 9007199254740992.0;
  };
  const double u1 = u(), u2 = u();
  return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
}

Problem make_problem(int N, int m, int d) {
  Problem p{N, m, d};
  unsigned long long s = 12345;
  p.X.resize((size_t)N * m * d);
  p.Y.resize((size_t)N * m);
  std::vector<double> ts(d);
  for (auto& t : ts) t = lcg_normal(s);
  for (int n = 0; n < N; ++n)
    for (int i = 0; i < m; ++i) {
      double acc = 0.0;
      for (int j = 0; j < d; ++j) {
        const double v = lcg_normal(s);
        p.X[((size_t)n * m + i) * d + j] = v;
        acc += v * ts[j];
      }
      p.Y[(size_t)n * m + i] = acc + 0.3 * lcg_normal(s);
    }
  p.A.assign((size_t)N * d * d, 0.0);
  p.b.assign((size_t)N * d, 0.0);
  p.yy.assign(N, 0.0);
  for (int n = 0; n < N; ++n)
    for (int i = 0; i < m; ++i) {
      const double* x = &p.X[((size_t)n * m + i) * d];
      const double y = p.Y[(size_t)n * m + i];
      for (int j = 0; j < d; ++j) {
        for (int k = 0; k < d; ++k) p.A[((size_t)n * d + j) * d + k] += x[j] * x[k];
        p.b[(size_t)n * d + j] += x[j] * y;
      }
      p.yy[n] += y * y;
    }
  return p;
}

// Solve (M) x = r for SPD M (d x d) by Cholesky.
void chol_solve(std::vector<double> M, const double* r, double* x, int d) {
  for (int j = 0; j < d; ++j) {
    double s = M[j * d + j];
    for (int k = 0; k < j; ++k) s -= M[j * d + k] * M[j * d + k];
    M[j * d + j] = std::sqrt(s);
    for (int i = j + 1; i < d; ++i) {
      double t = M[i * d + j];
      for (int k = 0; k < j; ++k) t -= M[i * d + k] * M[j * d + k];
      M[i * d + j] = t / M[j * d + j];
    }
  }
  std::vector<double> z(d);
  for (int i = 0; i < d; ++i) {
    double t = r[i];
    for (int k = 0; k < i; ++k) t -= M[i * d + k] * z[k];
    z[i] = t / M[i * d + i];
  }
  for (int i = d - 1; i >= 0; --i) {
    double t = z[i];
    for (int k = i + 1; k < d; ++k) t -= M[k * d + i] * x[k];
    x[i] = t / M[i * d + i];
  }
}

double objective(const Problem& p, const std::vector<double>& th) {
  double f = 0.0;
  const int d = p.d;
  for (int n = 0; n < p.N; ++n) {
    const double* A = &p.A[(size_t)n * d * d];
    const double* t = &th[(size_t)n * d];
    for (int i = 0; i < d; ++i) {
      double q = 0.0;
      for (int j = 0; j < d; ++j) q += A[i * d + j] * t[j];
      f += 0.5 * q * t[i] - p.b[(size_t)n * d + i] * t[i];
    }
    f += 0.5 * p.yy[n];
  }
  return f;
}

double optimum(const Problem& p) {
  const int d = p.d;
  std::vector<double> As(d * d, 0.0), bs(d, 0.0), x(d);
  double yy = 0.0;
  for (int n = 0; n < p.N; ++n) {
    for (int e = 0; e < d * d; ++e) As[e] += p.A[(size_t)n * d * d + e];
    for (int i = 0; i < d; ++i) bs[i] += p.b[(size_t)n * d + i];
    yy += p.yy[n];
  }
  chol_solve(As, bs.data(), x.data(), d);
  double f = 0.5 * yy;
  for (int i = 0; i < d; ++i) {
    double q = 0.0;
    for (int j = 0; j < d; ++j) q += As[i * d + j] * x[j];
    f += 0.5 * q * x[i] - bs[i] * x[i];
  }
  return f;
}

// Star ADMM (standared_ADMM.m): hub = worker N - 1; returns iterations to |obj - obj0| < tol.
int host_star(const Problem& p, double rho, double obj0, double tol, int max_iter) {
  const int N = p.N, d = p.d, hub = N - 1;
  std::vector<double> th((size_t)N * d, 0.0), lam((size_t)N * d, 0.0), thh(d, 0.0), r(d);
  for (int it = 1; it <= max_iter; ++it) {
    for (int n = 0; n < hub; ++n) {
      std::vector<double> M(p.A.begin() + (size_t)n * d * d, p.A.begin() + (size_t)(n + 1) * d * d);
      for (int i = 0; i < d; ++i) M[i * d + i] += rho;
      for (int i = 0; i < d; ++i) r[i] = p.b[(size_t)n * d + i] - lam[(size_t)n * d + i] + rho * thh[i];
      chol_solve(M, r.data(), &th[(size_t)n * d], d);
    }
    std::vector<double> M(p.A.begin() + (size_t)hub * d * d, p.A.end());
    for (int i = 0; i < d; ++i) M[i * d + i] += (N - 1) * rho;
    for (int i = 0; i < d; ++i) {
      double c1 = 0.0, s1 = 0.0;
      for (int n = 0; n < hub; ++n) {
        c1 += lam[(size_t)n * d + i];
        s1 += th[(size_t)n * d + i];
      }
      r[i] = p.b[(size_t)hub * d + i] + c1 + rho * s1;
    }
    chol_solve(M, r.data(), &th[(size_t)hub * d], d);
    for (int i = 0; i < d; ++i) thh[i] = th[(size_t)hub * d + i];
    for (int n = 0; n < hub; ++n)
      for (int i = 0; i < d; ++i) lam[(size_t)n * d + i] += rho * (th[(size_t)n * d + i] - thh[i]);
    if (std::fabs(objective(p, th) - obj0) < tol) return it;
  }
  return -1;
}

// GADMM on the identity chain, per-worker duals (dynamic_group_ADMM_closedForm.m form).
int host_gadmm(const Problem& p, double rho, double obj0, double tol, int max_iter, std::vector<double>& th) {
  const int N = p.N, d = p.d;
  th.assign((size_t)N * d, 0.0);
  std::vector<double> mu((size_t)N * d, 0.0), r(d);
  auto solve = [&](int n) {
    const bool l = n > 0, rr = n < N - 1;
    const int deg = (int)l + (int)rr;
    std::vector<double> M(p.A.begin() + (size_t)n * d * d, p.A.begin() + (size_t)(n + 1) * d * d);
    for (int i = 0; i < d; ++i) M[i * d + i] += deg * rho;
    for (int i = 0; i < d; ++i) {
      double v = p.b[(size_t)n * d + i] - mu[(size_t)n * d + i];
      if (l) v += rho * th[(size_t)(n - 1) * d + i];
      if (rr) v += rho * th[(size_t)(n + 1) * d + i];
      r[i] = v;
    }
    chol_solve(M, r.data(), &th[(size_t)n * d], d);
  };
  for (int it = 1; it <= max_iter; ++it) {
    for (int n = 0; n < N; n += 2) solve(n);
    for (int n = 1; n < N; n += 2) solve(n);
    for (int n = 0; n < N; ++n)
      for (int i = 0; i < d; ++i) {
        double m = mu[(size_t)n * d + i];
        const double t = th[(size_t)n * d + i];
        if (n > 0) m -= rho * (th[(size_t)(n - 1) * d + i] - t);
        if (n < N - 1) m += rho * (t - th[(size_t)(n + 1) * d + i]);
        mu[(size_t)n * d + i] = m;
      }
    if (std::fabs(objective(p, th) - obj0) < tol) return it;
  }
  return -1;
}

double max_rel(const std::vector<double>& a, const std::vector<double>& b) {
  double num = 0.0, den = 1e-300;
  for (size_t i = 0; i < a.size(); ++i) {
    num = std::fmax(num, std::fabs(a[i] - b[i]));
    den = std::fmax(den, std::fabs(b[i]));
  }
  return num / den;
}

template <typename T>
T* dalloc(size_t n) {
  T* p = nullptr;
  HIPOK(hipMalloc((void**)&p, n * sizeof(T) + 16));
  HIPOK(hipMemset(p, 0, n * sizeof(T) + 16));
  return p;
}
template <typename T>
std::vector<T> fetch(const T* d, size_t n) {
  std::vector<T> h(n);
  HIPOK(hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost));
  return h;
}

// ------------------------------------------------------------------ host-only checks
void host_only_checks() {
  EXPECT(gadmm_native_version() >= 1, "native version");
  long long buf[32];
  EXPECT(gadmm_abi_layout(buf, 32) >= 10 && buf[3] == (long long)sizeof(PhaseArgs), "abi layout");
  EXPECT(gadmm_fo_abi_layout(buf, 32) >= 6 && buf[1] == (long long)sizeof(FoArgs), "fo abi layout");
  int k = 0, len = 0;
  const int W = gadmm_chain_blocked_plan(24, 50, 0, &k, &len);
  // k = 2; the owned length is the shortest (1..4) whose launch fits one XCD (device-dependent)
  EXPECT(k == 2 && len >= 1 && len <= 4 && W == (24 + len - 1) / len, "blocked plan 24x50 -> W=%d k=%d len=%d", W,
         k, len);
  EXPECT(gadmm_chain_blocked_plan(24, 100, 0, &k, &len) == 0, "blocked plan rejects d > 52");
  // argument validation returns before touching the device
  EXPECT(gadmm_spd_inverse_small_f64(nullptr, nullptr, 4, 200, 1, nullptr, nullptr, nullptr) != 0 &&
             std::strlen(gadmm_last_error()) > 0,
         "spd_inverse rejects d > 128");
  FoArgs fa;
  std::memset(&fa, 0, sizeof(fa));
  fa.d = 500;
  fa.n = 4;
  fa.ring = 64;
  EXPECT(gadmm_fo_launch(&fa, nullptr) == -2, "fo_launch rejects d > 128");
  PersistArgs pa;
  std::memset(&pa, 0, sizeof(pa));
  pa.d = 50;
  EXPECT(gadmm_chain_blocked_launch(&pa, nullptr) != 0, "blocked launch rejects an empty plan");
  EXPECT(gadmm_star_abi_layout(buf, 32) >= 2 && buf[0] == (long long)sizeof(StarArgs), "star abi layout");
  StarArgs sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.d = 50;
  sa.n = 1;
  EXPECT(gadmm_star_launch(&sa, nullptr) == -1, "star launch rejects n < 2");
  EXPECT(gadmm_spd_inverse_blocked_f64(nullptr, nullptr, 1, 300, 1, nullptr, nullptr, nullptr, 100, nullptr) == -1,
         "blocked inverse rejects nb = 100");
  EXPECT(gadmm_spd_inverse_blocked_workspace(300, 128) > gadmm_spd_inverse_blocked_workspace(300, 64),
         "blocked inverse workspace grows with the block");
}

// ------------------------------------------------------------------ GPU checks
void gpu_checks() {
  const int N = 8, m = 20, d = 12;
  const double rho = 4.0, tol = 1e-8;
  const int max_iter = 3000;
  Problem p = make_problem(N, m, d);
  const double obj0 = optimum(p);
  std::vector<double> th_ref;
  const int it_ref = host_gadmm(p, rho, obj0, tol, max_iter, th_ref);
  EXPECT(it_ref > 0, "host GADMM did not converge");
  std::printf("host reference: %d iterations to %.0e, obj0 = %.12f\n", it_ref, tol, obj0);

  hipStream_t st;
  HIPOK(hipStreamCreate(&st));
  double* X = dalloc<double>(p.X.size());
  double* Y = dalloc<double>(p.Y.size());
  HIPOK(hipMemcpy(X, p.X.data(), p.X.size() * 8, hipMemcpyHostToDevice));
  HIPOK(hipMemcpy(Y, p.Y.data(), p.Y.size() * 8, hipMemcpyHostToDevice));
  double* A = dalloc<double>((size_t)N * d * d);
  double* b = dalloc<double>((size_t)N * d);
  double* yy = dalloc<double>(N);
  EXPECT(gadmm_gram_f64(X, Y, N, m, d, 1, A, b, yy, nullptr, st) == 0, "gram: %s", gadmm_last_error());
  HIPOK(hipStreamSynchronize(st));
  EXPECT(max_rel(fetch(A, p.A.size()), p.A) < 1e-13, "gram A");
  EXPECT(max_rel(fetch(b, p.b.size()), p.b) < 1e-13, "gram b");
  EXPECT(max_rel(fetch(yy, p.yy.size()), p.yy) < 1e-13, "gram yy");

  std::vector<double> shifts(2 * N);
  for (int n = 0; n < N; ++n) {
    shifts[2 * n] = rho;
    shifts[2 * n + 1] = 2 * rho;
  }
  double* sh = dalloc<double>(shifts.size());
  HIPOK(hipMemcpy(sh, shifts.data(), shifts.size() * 8, hipMemcpyHostToDevice));
  double* Minv = dalloc<double>((size_t)N * 2 * d * d);
  int* status = dalloc<int>(1);
  EXPECT(gadmm_spd_inverse_small_f64(A, sh, N, d, 2, Minv, status, st) == 0, "inverse");
  HIPOK(hipStreamSynchronize(st));
  EXPECT(fetch(status, 1)[0] == 0, "inverse status");

  // chain slots, identity path
  std::vector<PhaseSlot> heads, tails, all(N);
  for (int n = 0; n < N; ++n) {
    PhaseSlot s{n, n, n > 0 ? n - 1 : -1, n < N - 1 ? n + 1 : -1};
    all[n] = s;
    (n % 2 == 0 ? heads : tails).push_back(s);
  }
  double* theta = dalloc<double>((size_t)N * d);
  double* mu = dalloc<double>((size_t)N * d);
  double* trace = dalloc<double>(max_iter);
  ChainCtl* ctl = dalloc<ChainCtl>(1);

  // ---- multi-kernel engine (graph-replayed phases)
  {
    const int block = 16;
    double* objw = dalloc<double>(N);
    double* part = dalloc<double>(block);
    double* reduced = dalloc<double>(block);
    int* inner = dalloc<int>(N);
    PhaseSlot* dslots = dalloc<PhaseSlot>(2 * N);
    EngineDesc desc;
    std::memset(&desc, 0, sizeof(desc));
    PhaseArgs& a = desc.base;
    a.d = d;
    a.n_local = N;
    a.nvar = 2;
    a.deg_to_var[0] = 0;
    a.deg_to_var[1] = 0;
    a.deg_to_var[2] = 1;
    a.model = 0;
    a.Minv = Minv;
    a.A = A;
    a.b = b;
    a.yy = yy;
    a.mu = mu;
    a.theta = theta;
    a.rho = rho;
    a.objw = objw;
    a.ctl = ctl;
    a.trace = trace;
    a.part = part;
    a.ring = block;
    a.max_iter = max_iter;
    a.obj0 = obj0;
    a.tol = tol;
    a.m = m;
    a.inner_iters = inner;
    a.n_total = N;
    desc.d_slots = dslots;
    desc.reduced = reduced;
    desc.stream = st;
    desc.nranks = 1;
    void* h = gadmm_chain_engine_create(&desc);
    EXPECT(h != nullptr, "engine create");
    EXPECT(gadmm_chain_engine_set_plan(h, (int)heads.size(), heads.data(), (int)tails.size(), tails.data(), 0,
                                       nullptr, 0, nullptr) == 0,
           "set_plan: %s", gadmm_last_error());
    EXPECT(gadmm_chain_engine_reset(h, 1, 0) == 0, "reset");
    RunStats rs;
    std::memset(&rs, 0, sizeof(rs));
    EXPECT(gadmm_chain_engine_run(h, block, 0, 1, &rs) == 0, "run: %s", gadmm_last_error());
    EXPECT(rs.done == 1 && std::abs(rs.iters - it_ref) <= 1, "graph engine: done=%d iters=%d (host %d)", rs.done,
           rs.iters, it_ref);
    std::printf("graph engine: %d iterations, %d replays\n", rs.iters, rs.replays);
    gadmm_chain_engine_destroy(h);
    for (void* q : {(void*)objw, (void*)part, (void*)reduced, (void*)inner, (void*)dslots}) HIPOK(hipFree(q));
  }

  // ---- persistent kernels: per-worker and temporally blocked
  auto run_persistent = [&](bool blocked, unsigned epoch) {
    HIPOK(hipMemset(theta, 0, (size_t)N * d * 8));
    HIPOK(hipMemset(mu, 0, (size_t)N * d * 8));
    HIPOK(hipMemset(ctl, 0, sizeof(ChainCtl)));
    const int lag = blocked ? 8 : 4, ring = lag + 4;
    PhaseSlot* dslots = dalloc<PhaseSlot>(N);
    int* dpos = dalloc<int>(N);
    std::vector<int> pos(N);
    for (int n = 0; n < N; ++n) pos[n] = n;
    HIPOK(hipMemcpy(dslots, all.data(), N * sizeof(PhaseSlot), hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(dpos, pos.data(), N * sizeof(int), hipMemcpyHostToDevice));
    u32x4* thg = dalloc<u32x4>((size_t)N * d);
    u32x4* objg = dalloc<u32x4>((size_t)ring * N);
    unsigned long long* decg = dalloc<unsigned long long>(ring);
    unsigned long long** decp = dalloc<unsigned long long*>(1);
    HIPOK(hipMemcpy(decp, &decg, sizeof(void*), hipMemcpyHostToDevice));
    PersistArgs pa;
    std::memset(&pa, 0, sizeof(pa));
    pa.d = d;
    pa.n = N;
    pa.n_local = N;
    pa.start_iter = 1;
    pa.max_iter = max_iter;
    pa.lag = lag;
    pa.ring = ring;
    pa.nvar = 2;
    pa.obj_mode = 0;
    pa.deg_to_var[0] = 0;
    pa.deg_to_var[1] = 0;
    pa.deg_to_var[2] = 1;
    pa.has_monitor = 1;
    pa.nranks = 1;
    pa.epoch = epoch;
    pa.rho = rho;
    pa.obj0 = obj0;
    pa.tol = tol;
    pa.timeout_ticks = 20LL * 100000000LL;
    pa.slots = dslots;
    pa.pos = dpos;
    pa.Minv = Minv;
    pa.A = A;
    pa.b = b;
    pa.yy = yy;
    pa.theta = theta;
    pa.mu = mu;
    pa.thg = thg;
    pa.objg = objg;
    pa.decg = decg;
    pa.dec_push = decp;
    pa.trace = trace;
    pa.ctl = ctl;
    u32x4* tab = nullptr;
    int rc;
    if (blocked) {
      int k = 0, len = 0;
      EXPECT(gadmm_chain_blocked_plan(N, d, 0, &k, &len) > 0, "blocked plan");
      pa.blk_k = k;
      pa.blk_len = len;
      tab = dalloc<u32x4>(gadmm_chain_blocked_tab_granules(N, d, ring));
      pa.blk_tab = tab;
      rc = gadmm_chain_blocked_launch(&pa, st);
    } else {
      rc = gadmm_chain_persistent_launch(&pa, st);
    }
    EXPECT(rc == 0, "persistent launch: %s", gadmm_last_error());
    HIPOK(hipStreamSynchronize(st));
    const ChainCtl c = fetch(ctl, 1)[0];
    EXPECT(c.done == 1 && std::abs(c.conv_iter - it_ref) <= 1,
           "%s persistent: done=%d iters=%d (host %d) ctl={iter %d pending %d ticket %u monitored %d} last error '%s'",
           blocked ? "blocked" : "per-worker", c.done, c.conv_iter, it_ref, c.iter, c.pending, c.ticket, c.monitored,
           hipGetErrorString(hipGetLastError()));
    std::printf("%s persistent kernel: %d iterations\n", blocked ? "blocked" : "per-worker", c.conv_iter);
    for (void* q : {(void*)dslots, (void*)dpos, (void*)thg, (void*)objg, (void*)decg, (void*)decp}) HIPOK(hipFree(q));
    if (tab) HIPOK(hipFree(tab));
  };
  run_persistent(false, 1);
  run_persistent(true, 2);
  run_persistent(false, 3);

  // ---- first-order engine: faithful GD (ones at iteration 1) vs host GD, objective traces
  {
    const int iters = 300;
    double lmax = 0.0;  // power iteration on sum A_n
    {
      std::vector<double> As(d * d, 0.0), v(d, 1.0), w(d);
      for (int n = 0; n < N; ++n)
        for (int e = 0; e < d * d; ++e) As[e] += p.A[(size_t)n * d * d + e];
      for (int r = 0; r < 500; ++r) {
        double nrm = 0.0;
        for (int i = 0; i < d; ++i) {
          w[i] = 0.0;
          for (int j = 0; j < d; ++j) w[i] += As[i * d + j] * v[j];
          nrm += w[i] * w[i];
        }
        nrm = std::sqrt(nrm);
        lmax = nrm;
        for (int i = 0; i < d; ++i) v[i] = w[i] / nrm;
      }
    }
    const double step = 1.0 / lmax;
    std::vector<double> th(d, 0.0), obj_ref(iters);
    for (int it = 1; it <= iters; ++it) {
      std::vector<double> rep((size_t)N * d);
      for (int n = 0; n < N; ++n)
        for (int i = 0; i < d; ++i) rep[(size_t)n * d + i] = th[i];
      obj_ref[it - 1] = objective(p, rep);
      std::vector<double> g(d, 0.0);
      if (it == 1) {
        for (auto& x : g) x = 1.0;
      } else {
        for (int n = 0; n < N; ++n)
          for (int i = 0; i < d; ++i) {
            double q = 0.0;
            for (int j = 0; j < d; ++j) q += p.A[((size_t)n * d + i) * d + j] * th[j];
            g[i] += q - p.b[(size_t)n * d + i];
          }
      }
      for (int i = 0; i < d; ++i) th[i] -= step * g[i];
    }
    FoArgs fa;
    std::memset(&fa, 0, sizeof(fa));
    fa.alg = FO_GD;
    fa.model = FO_LINEAR;
    fa.n = N;
    fa.d = d;
    fa.m = m;
    fa.max_iter = iters;
    fa.faithful = 1;
    fa.ring = 64;
    fa.epoch = 1;
    fa.step = step;
    fa.obj0 = obj0;
    fa.tol = -1.0;
    fa.timeout_ticks = 20LL * 100000000LL;
    fa.A = A;
    fa.b = b;
    fa.yy = yy;
    fa.slots = 2;  // one GPU: every worker's row per iteration, lock-step readers
    fa.nranks = 1;
    fa.n_local = N;
    fa.has_monitor = 1;
    u32x4* tab = dalloc<u32x4>((size_t)gadmm_fo_tab_granules(N, d, fa.slots));
    u32x4* part = dalloc<u32x4>((size_t)64 * N * 2);
    double* ot = dalloc<double>(iters);
    double* ct = dalloc<double>(iters);
    long long* tt = dalloc<long long>(iters);
    double* tho = dalloc<double>((size_t)N * d);
    FoCtl* fc = dalloc<FoCtl>(1);
    fa.tab = tab;
    fa.part = part;
    fa.obj_trace = ot;
    fa.cnt_trace = ct;
    fa.time_trace = tt;
    fa.theta_out = tho;
    fa.ctl = fc;
    fa.wmon = &fc->monitored;  // one GPU: the run-wide words are the control block's
    fa.wstop = &fc->stop_iter;
    EXPECT(gadmm_fo_launch(&fa, st) == 0, "fo launch");
    HIPOK(hipStreamSynchronize(st));
    const FoCtl c = fetch(fc, 1)[0];
    EXPECT(c.status == 2 && c.iters == iters, "fo status=%d iters=%d", c.status, c.iters);
    EXPECT(max_rel(fetch(ot, iters), obj_ref) < 1e-11, "fo GD objective trace vs host: %.3e",
           max_rel(fetch(ot, iters), obj_ref));
    std::printf("first-order GD: %d iterations, trace rel err %.2e\n", c.iters, max_rel(fetch(ot, iters), obj_ref));
    for (void* q : {(void*)tab, (void*)part, (void*)ot, (void*)ct, (void*)tt, (void*)tho, (void*)fc}) HIPOK(hipFree(q));
  }

  // ---- star ADMM kernel (one launch) vs the host star ADMM
  {
    const double srho = 1.0, stol = 1e-6;
    const int it_star = host_star(p, srho, obj0, stol, 20000);
    EXPECT(it_star > 0, "host star ADMM did not converge");
    std::vector<double> sshift(N);
    for (int n = 0; n < N; ++n) sshift[n] = n == N - 1 ? (N - 1) * srho : srho;
    double* ssh = dalloc<double>(N);
    HIPOK(hipMemcpy(ssh, sshift.data(), N * 8, hipMemcpyHostToDevice));
    double* SMinv = dalloc<double>((size_t)N * d * d);
    EXPECT(gadmm_spd_inverse_small_f64(A, ssh, N, d, 1, SMinv, status, st) == 0, "star inverses");
    const int lag = 4, ring = 8, smax = 20000;
    std::vector<int> gid(N);
    for (int n = 0; n < N; ++n) gid[n] = n;
    int* dgid = dalloc<int>(N);
    HIPOK(hipMemcpy(dgid, gid.data(), N * sizeof(int), hipMemcpyHostToDevice));
    double* sth = dalloc<double>((size_t)N * d);
    double* slam = dalloc<double>((size_t)N * d);
    double* slamh = dalloc<double>((size_t)N * d);
    double* strace = dalloc<double>(smax);
    u32x4* sthg = dalloc<u32x4>((size_t)N * d);
    u32x4* sobjg = dalloc<u32x4>((size_t)ring * N);
    unsigned long long* sdecg = dalloc<unsigned long long>(ring);
    unsigned long long** sdecp = dalloc<unsigned long long*>(1);
    u32x4** speer = dalloc<u32x4*>(1);
    HIPOK(hipMemcpy(sdecp, &sdecg, sizeof(void*), hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(speer, &sthg, sizeof(void*), hipMemcpyHostToDevice));
    ChainCtl* sctl = dalloc<ChainCtl>(1);
    StarArgs sa;
    std::memset(&sa, 0, sizeof(sa));
    sa.d = d;
    sa.n = N;
    sa.n_local = N;
    sa.max_iter = smax;
    sa.lag = lag;
    sa.ring = ring;
    sa.has_monitor = 1;
    sa.nranks = 1;
    sa.epoch = 1;
    sa.rho = srho;
    sa.obj0 = obj0;
    sa.tol = stol;
    sa.timeout_ticks = 20LL * 100000000LL;
    sa.gid = dgid;
    sa.Minv = SMinv;
    sa.A = A;
    sa.b = b;
    sa.yy = yy;
    sa.theta = sth;
    sa.lam = slam;
    sa.lam_hub = slamh;
    sa.thg = sthg;
    sa.peer_thg = speer;
    sa.objg = sobjg;
    sa.decg = sdecg;
    sa.dec_push = sdecp;
    sa.trace = strace;
    sa.ctl = sctl;
    EXPECT(gadmm_star_launch(&sa, st) == 0, "star launch: %s", gadmm_last_error());
    HIPOK(hipStreamSynchronize(st));
    const ChainCtl c = fetch(sctl, 1)[0];
    EXPECT(c.done == 1 && std::abs(c.conv_iter - it_star) <= 1, "star kernel: done=%d iters=%d (host %d)", c.done,
           c.conv_iter, it_star);
    std::printf("star kernel: %d iterations (host %d)\n", c.conv_iter, it_star);
    for (void* q : {(void*)ssh, (void*)SMinv, (void*)dgid, (void*)sth, (void*)slam, (void*)slamh, (void*)strace,
                    (void*)sthg, (void*)sobjg, (void*)sdecg, (void*)sdecp, (void*)speer, (void*)sctl})
      HIPOK(hipFree(q));
  }

  // ---- blocked large-d inverse (d = 200: a recursive 72-pivot last block) vs M Minv = I on the host
  {
    const int D = 200;
    std::vector<double> Mh((size_t)D * D);
    unsigned long long sd = 777;
    std::vector<double> G((size_t)2 * D * D);
    for (auto& v : G) v = lcg_normal(sd);
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) {
        double acc = 0.0;
        for (int k = 0; k < 2 * D; ++k) acc += G[(size_t)k * D + i] * G[(size_t)k * D + j];
        Mh[(size_t)i * D + j] = acc / (2 * D);
      }
    double* dA = dalloc<double>((size_t)D * D);
    double* dout = dalloc<double>((size_t)D * D);
    const long nws = gadmm_spd_inverse_blocked_workspace(D, 128);
    double* ws = dalloc<double>((size_t)nws);
    HIPOK(hipMemcpy(dA, Mh.data(), Mh.size() * 8, hipMemcpyHostToDevice));
    const double shift = 0.25;
    EXPECT(gadmm_spd_inverse_blocked_f64(dA, &shift, 1, D, 1, dout, ws, status, 128, st) == 0, "blocked inverse: %s",
           gadmm_last_error());
    HIPOK(hipStreamSynchronize(st));
    const std::vector<double> inv = fetch(dout, (size_t)D * D);
    double err = 0.0;
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) {
        double acc = 0.0;
        for (int k = 0; k < D; ++k) acc += (Mh[(size_t)i * D + k] + (i == k ? shift : 0.0)) * inv[(size_t)k * D + j];
        err = std::fmax(err, std::fabs(acc - (i == j ? 1.0 : 0.0)));
      }
    EXPECT(err < 1e-11 && fetch(status, 1)[0] == 0, "blocked inverse: max |M Minv - I| = %.3e", err);
    std::printf("blocked inverse d=%d: max |M Minv - I| = %.2e\n", D, err);
    for (void* q : {(void*)dA, (void*)dout, (void*)ws}) HIPOK(hipFree(q));
  }

  for (void* q : {(void*)X, (void*)Y, (void*)A, (void*)b, (void*)yy, (void*)sh, (void*)Minv, (void*)status,
                  (void*)theta, (void*)mu, (void*)trace, (void*)ctl})
    HIPOK(hipFree(q));
  HIPOK(hipStreamDestroy(st));
}

}  // namespace

int main(int argc, char** argv) {
  const bool host_only = argc > 1 && std::strcmp(argv[1], "--host-only") == 0;
  host_only_checks();
  if (!host_only) gpu_checks();
  if (failures) {
    std::fprintf(stderr, "native_selftest: %d failure(s)\n", failures);
    return 1;
  }
  std::printf("native_selftest: OK (%s)\n", host_only ? "host-only" : "host + GPU");
  return 0;
}
