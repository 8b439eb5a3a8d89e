// D-GADMM chain construction on the host, for a batch of epochs (K15: findPath.m:16-30 /
// findPath2.m:43-59 semantics). Python draws the node positions (the seeded numpy stream the
// reference-semantics schedule defines); this routine does the O(E N^2) part -- squared distances,
// the greedy nearest-unvisited chain from node 0 (lowest index wins ties, as numpy argmin), and the
// per-hop cost -- so pre-drawing ~300 epochs for a one-launch D-GADMM run costs tens of us instead
// of milliseconds of numpy dispatch. Bit-identical to PathSchedule.prefetch_arrays' numpy path: no
// FMA contraction, the same operation order ((dx*dx) + (dy*dy); ((d2*eta)*bw)*f for energies).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <limits>
#include <mutex>
#include <thread>
#include <vector>

#pragma clang fp contract(off)

namespace {

// Epochs [e0, e1) of the batch: one geometry + greedy chain each (independent of the others).
// Only the distances the greedy walk reads are formed: the row of the current node, restricted to
// the still-unvisited nodes kept compacted in `left` (N^2/2 pairs instead of N^2). Each pair is
// computed exactly as the full matrix would hold it, and candidates are scanned in ascending index
// order, so the chain and costs are unchanged.
void greedy_range(const double* uv, int e0, int e1, int n, double side, int energy, double eta, double bw, double f,
                  long long* paths, double* costs) {
  std::vector<double> x(n), y(n);
  std::vector<int> left(n);
  std::vector<double> v(n);
  const double inf = std::numeric_limits<double>::infinity();
  for (int e = e0; e < e1; ++e) {
    const double* g = uv + (size_t)e * n * 2;
    for (int i = 0; i < n; ++i) {
      x[i] = g[2 * i] * side;
      y[i] = g[2 * i + 1] * side;
    }
    long long* p = paths + (size_t)e * n;
    int nleft = 0;
    for (int j = 1; j < n; ++j) left[nleft++] = j;  // ascending: lowest index wins ties
    int cur = 0;
    p[0] = 0;
    for (int k = 1; k < n; ++k) {
      // distances first (independent, vectorisable), then the minimum (exact in any order), then the
      // first candidate holding it: the same choice as a sequential strict-< scan
      const double xc = x[cur], yc = y[cur];
      double bv = inf;
      for (int q = 0; q < nleft; ++q) {
        const int j = left[q];
        const double dx = xc - x[j], dy = yc - y[j];
        const double a = dx * dx, b = dy * dy;
        v[q] = a + b;
      }
      double m4[4] = {inf, inf, inf, inf};  // four independent running minima (short dependent chain)
      int q = 0;
      for (; q + 4 <= nleft; q += 4)
        for (int u = 0; u < 4; ++u) m4[u] = v[q + u] < m4[u] ? v[q + u] : m4[u];
      for (; q < nleft; ++q) m4[0] = v[q] < m4[0] ? v[q] : m4[0];
      for (int u = 0; u < 4; ++u) bv = m4[u] < bv ? m4[u] : bv;
      int bi = 0;
      if (bv < inf)
        while (v[bi] != bv) ++bi;
      // every candidate at +inf / NaN: numpy argmin takes the first unvisited (bi = 0 above)
      const int best = left[bi];
      double c = v[bi];
      for (int q = bi + 1; q < nleft; ++q) left[q - 1] = left[q];  // keep ascending order
      --nleft;
      p[k] = best;
      if (energy) {
        c = c * eta;
        c = c * bw;
        c = c * f;
      }
      costs[(size_t)e * (n - 1) + (k - 1)] = c;
      cur = best;
    }
  }
}

}  // namespace

// The epochs are independent: large batches are split over up to 8 host threads.
extern "C" int gadmm_greedy_chains(const double* uv, int E, int n, double side, int energy, double eta, double bw,
                                   double f, long long* paths, double* costs) {
  if (E < 0 || n < 1 || !uv || !paths || (n > 1 && !costs)) return -1;
  const long work = (long)E * n * n;
  int nt = 1;
  if (work > 400000) {  // below this one core beats spawning threads (~300 epochs x 24 nodes: ~40 us)
    const unsigned hw = std::thread::hardware_concurrency();
    nt = (int)std::min<long>(std::min<unsigned>(hw ? hw : 1, 8u), std::max<long>(1, work / 40000));
  }
  static const int env_nt = getenv("GADMM_CHAIN_THREADS") ? atoi(getenv("GADMM_CHAIN_THREADS")) : 0;  // A/B
  if (env_nt >= 1) nt = std::min(env_nt, 8);
  if (nt > E) nt = E;
  if (nt <= 1) {
    greedy_range(uv, 0, E, n, side, energy, eta, bw, f, paths, costs);
    return 0;
  }
  std::vector<std::thread> pool;
  pool.reserve(nt - 1);
  const int per = (E + nt - 1) / nt;
  for (int t = 1; t < nt; ++t) {
    const int e0 = t * per, e1 = std::min(E, e0 + per);
    if (e0 < e1) pool.emplace_back(greedy_range, uv, e0, e1, n, side, energy, eta, bw, f, paths, costs);
  }
  greedy_range(uv, 0, std::min(E, per), n, side, energy, eta, bw, f, paths, costs);
  for (auto& th : pool) th.join();
  return 0;
}

// The blocked kernel's D-GADMM tables (one GPU, every worker local: li == worker id) from the chains
// P [E][n]: per (epoch, chain POSITION) the slot (li, gid, left, right); per (epoch, worker) its
// position; and per (epoch, position) the flush pair (PersistArgs::ep_flush): the old-chain
// neighbours of the worker placed there if it was a head of the previous epoch's chain, else -1.
// The numpy equivalent (chain_engine.py: epoch_flush_table) cost ~0.1-0.2 ms per solve.
// Every row of P must be a permutation of 0..n-1 (-2 otherwise: a duplicate would leave a stale
// position of the previous epoch in pos / the flush pairs).
extern "C" int gadmm_epoch_tables_blocked(const long long* P, int E, int n, int* slots, int* pos, int* flush) {
  if (E < 0 || n < 1 || !P || (E > 0 && (!slots || !pos || !flush))) return -1;
  std::vector<int> pos_prev(n), pos_cur(n), seen(n, -1);
  for (int e = 0; e < E; ++e) {
    const long long* pe = P + (size_t)e * n;
    for (int p = 0; p < n; ++p) {
      const long long w = pe[p];
      if (w < 0 || w >= n || seen[w] == e) return -2;
      seen[w] = e;
      pos_cur[w] = p;
    }
    for (int p = 0; p < n; ++p) {
      int* s = slots + ((size_t)e * n + p) * 4;
      s[0] = (int)pe[p];
      s[1] = (int)pe[p];
      s[2] = p > 0 ? (int)pe[p - 1] : -1;
      s[3] = p + 1 < n ? (int)pe[p + 1] : -1;
      int* f = flush + ((size_t)e * n + p) * 2;
      f[0] = f[1] = -1;
      if (e > 0) {
        const long long* pp = P + (size_t)(e - 1) * n;
        const int po = pos_prev[pe[p]];
        if (po % 2 == 0) {
          f[0] = po > 0 ? (int)pp[po - 1] : -1;
          f[1] = po + 1 < n ? (int)pp[po + 1] : -1;
        }
      }
    }
    for (int w = 0; w < n; ++w) pos[(size_t)e * n + w] = pos_cur[w];
    pos_prev.swap(pos_cur);
  }
  return 0;
}

// Per-epoch device tables of the one-launch D-GADMM kernel (chain_persistent.hip, dynamic mode),
// from the chains P [E][n] (position -> worker): for each local worker li (global id loc[li]) its
// slot (li, gid, left, right) and chain position in every epoch. Replaces ~0.5 ms of numpy per
// solve (argsort + fancy indexing over ~300 epochs) on the host path of every D-GADMM solve.
// Rows of P must be permutations (-2 otherwise).
extern "C" int gadmm_epoch_tables(const long long* P, int E, int n, const long long* loc, int nloc, int* slots,
                                  int* pos) {
  if (E < 0 || n < 1 || nloc < 0 || !P || (nloc > 0 && (!loc || !slots || !pos))) return -1;
  std::vector<int> pos_of(n), seen(n, -1);
  for (int e = 0; e < E; ++e) {
    const long long* pe = P + (size_t)e * n;
    for (int p = 0; p < n; ++p) {
      const long long w = pe[p];
      if (w < 0 || w >= n || seen[w] == e) return -2;
      seen[w] = e;
      pos_of[w] = p;
    }
    for (int li = 0; li < nloc; ++li) {
      const long long w = loc[li];
      if (w < 0 || w >= n) return -3;
      const int k = pos_of[w];
      int* s = slots + ((size_t)e * nloc + li) * 4;
      s[0] = li;
      s[1] = (int)w;
      s[2] = k > 0 ? (int)pe[k - 1] : -1;
      s[3] = k + 1 < n ? (int)pe[k + 1] : -1;
      pos[(size_t)e * nloc + li] = k;
    }
  }
  return 0;
}

// numpy's PCG64 (XSL-RR output of a 128-bit LCG; Generator.random() = (next64 >> 11) * 2^-53), so the
// node geometries of a seeded D-GADMM schedule can be drawn here, bit for bit, from a state the caller
// hands over (the numpy Generator is then advanced by the same count, or not materialised at all).
namespace {
typedef unsigned __int128 u128;
constexpr u128 PCG_MULT = ((u128)0x2360ED051FC65DA4ULL << 64) | (u128)0x4385DF649FCCF645ULL;

inline u128 pcg_advance(u128 state, u128 inc, unsigned long long delta) {
  u128 acc_mult = 1, acc_plus = 0, cur_mult = PCG_MULT, cur_plus = inc;
  while (delta > 0) {
    if (delta & 1) {
      acc_mult *= cur_mult;
      acc_plus = acc_plus * cur_mult + cur_plus;
    }
    cur_plus = (cur_mult + 1) * cur_plus;
    cur_mult *= cur_mult;
    delta >>= 1;
  }
  return acc_mult * state + acc_plus;
}

inline void pcg_uniform(u128& state, u128 inc, long count, double* out) {
  for (long i = 0; i < count; ++i) {
    state = state * PCG_MULT + inc;
    const unsigned long long x = (unsigned long long)(state >> 64) ^ (unsigned long long)state;
    const unsigned rot = (unsigned)(state >> 122);
    const unsigned long long r = (x >> rot) | (x << ((64 - rot) & 63));
    out[i] = (double)(r >> 11) * (1.0 / 9007199254740992.0);
  }
}
}  // namespace

// `count` doubles of numpy's PCG64 Generator.random() from the state (s_hi:s_lo, increment i_hi:i_lo)
// advanced by `ahead` outputs first.
extern "C" int gadmm_pcg64_uniform(unsigned long long s_hi, unsigned long long s_lo, unsigned long long i_hi,
                                   unsigned long long i_lo, unsigned long long ahead, long count, double* out) {
  if (count < 0 || (count > 0 && !out)) return -1;
  const u128 inc = ((u128)i_hi << 64) | i_lo;
  u128 st = pcg_advance(((u128)s_hi << 64) | s_lo, inc, ahead);
  pcg_uniform(st, inc, count, out);
  return 0;
}

// Asynchronous greedy chains: one process-wide host worker thread runs gadmm_greedy_chains on a batch
// while the caller keeps going (a D-GADMM solve draws its first launch's chains at the top of the
// solve and joins them just before it builds the epoch tables: the greedy walks overlap the engine
// refresh / reset / schedule set-up on the Python side instead of preceding the launch). One job at a
// time: a submit while a job is pending first waits for it, and a submit from another thread waits until
// the owning thread's gadmm_greedy_chains_wait. The caller keeps uv / paths / costs alive until
// gadmm_greedy_chains_wait returns.
// Hand-offs are lock-free spins on an atomic state (a futex wake and a condition-variable round trip
// cost tens of us on the sandboxed hosts measured, more than the walks themselves); the worker spins
// for at most SPIN_NS after a job and then sleeps on the condition variable until the next submit.
namespace {
struct GreedyJob {
  double* uv = nullptr;  // drawn first by the worker when rng is set
  int E = 0, n = 0, energy = 0, rng = 0;
  unsigned long long s_hi = 0, s_lo = 0, i_hi = 0, i_lo = 0, ahead = 0;
  double side = 0, eta = 0, bw = 0, f = 0;
  long long* paths = nullptr;
  double* costs = nullptr;
  int rc = 0;
};
enum { G_IDLE = 0, G_PENDING = 1, G_RUNNING = 2 };
constexpr long long SPIN_NS = 3000000;  // 3 ms: covers back-to-back solves, then the worker sleeps

// Heap-allocated and never destroyed: a static condition variable would be destroyed at process exit
// while the detached worker still waits on it (glibc's pthread_cond_destroy then blocks the exit).
struct GreedyPool {
  std::mutex mu;
  std::condition_variable cv;
  GreedyJob job;
  std::atomic<int> state{G_IDLE};
  std::atomic<bool> sleeping{false};
  std::once_flag started;
  // One caller thread at a time owns the worker from its submit until its wait: a second thread's
  // submit blocks until the owner has joined (it could otherwise overwrite the pending job, and the
  // owner would read the other caller's paths / return code). Re-submitting by the owner is allowed.
  std::atomic<bool> claimed{false};
  std::atomic<std::thread::id> owner{};
};
GreedyPool& pool() {
  static GreedyPool* p = new GreedyPool();
  return *p;
}

inline void cpu_relax() { __builtin_ia32_pause(); }

void greedy_worker() {
  GreedyPool& P = pool();
  for (;;) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned k = 1; P.state.load(std::memory_order_acquire) != G_PENDING; ++k) {
      cpu_relax();
      if ((k & 1023) == 0 && std::chrono::duration_cast<std::chrono::nanoseconds>(
                                 std::chrono::steady_clock::now() - t0).count() > SPIN_NS) {
        std::unique_lock<std::mutex> lk(P.mu);
        P.sleeping.store(true);  // seq_cst: ordered against the submitter's state store / sleeping load
        P.cv.wait(lk, [&] { return P.state.load() == G_PENDING; });
        P.sleeping.store(false);
        break;
      }
    }
    P.state.store(G_RUNNING, std::memory_order_relaxed);
    const GreedyJob& j = P.job;
    int rc = 0;
    if (j.rng) rc = gadmm_pcg64_uniform(j.s_hi, j.s_lo, j.i_hi, j.i_lo, j.ahead, (long)j.E * j.n * 2, j.uv);
    if (rc == 0) rc = gadmm_greedy_chains(j.uv, j.E, j.n, j.side, j.energy, j.eta, j.bw, j.f, j.paths, j.costs);
    P.job.rc = rc;
    P.state.store(G_IDLE, std::memory_order_release);
  }
}

void wait_idle(GreedyPool& P) {
  while (P.state.load(std::memory_order_acquire) != G_IDLE) cpu_relax();
}
}  // namespace

namespace {
int submit(const GreedyJob& nj) {
  GreedyPool& P = pool();
  std::call_once(P.started, [] { std::thread(greedy_worker).detach(); });  // lives for the process
  const std::thread::id me = std::this_thread::get_id();
  if (!(P.claimed.load(std::memory_order_acquire) && P.owner.load() == me)) {
    while (P.claimed.exchange(true, std::memory_order_acquire)) std::this_thread::yield();
    P.owner.store(me);
  }
  wait_idle(P);
  P.job = nj;
  P.state.store(G_PENDING);  // seq_cst (see the worker's sleeping store)
  if (P.sleeping.load()) {
    std::lock_guard<std::mutex> lk(P.mu);
    P.cv.notify_one();
  }
  return 0;
}
}  // namespace

extern "C" int gadmm_greedy_chains_async(const double* uv, int E, int n, double side, int energy, double eta,
                                         double bw, double f, long long* paths, double* costs) {
  if (E < 0 || n < 1 || !uv || !paths || (n > 1 && !costs)) return -1;
  GreedyJob j;
  j.uv = const_cast<double*>(uv);
  j.E = E;
  j.n = n;
  j.side = side;
  j.energy = energy;
  j.eta = eta;
  j.bw = bw;
  j.f = f;
  j.paths = paths;
  j.costs = costs;
  return submit(j);
}

// The same, with the node geometries drawn by the worker too: uv (E x n x 2, written) from numpy's PCG64
// state (s_hi:s_lo, inc i_hi:i_lo) advanced by `ahead` outputs -- exactly Generator.random((E, n, 2)).
extern "C" int gadmm_draw_chains_async(unsigned long long s_hi, unsigned long long s_lo, unsigned long long i_hi,
                                       unsigned long long i_lo, unsigned long long ahead, double* uv, int E, int n,
                                       double side, int energy, double eta, double bw, double f, long long* paths,
                                       double* costs) {
  if (E < 0 || n < 1 || !uv || !paths || (n > 1 && !costs)) return -1;
  GreedyJob j;
  j.uv = uv;
  j.E = E;
  j.n = n;
  j.side = side;
  j.energy = energy;
  j.eta = eta;
  j.bw = bw;
  j.f = f;
  j.paths = paths;
  j.costs = costs;
  j.rng = 1;
  j.s_hi = s_hi;
  j.s_lo = s_lo;
  j.i_hi = i_hi;
  j.i_lo = i_lo;
  j.ahead = ahead;
  return submit(j);
}

// Waits for the job of the last gadmm_greedy_chains_async; its return code (0 when none is pending).
extern "C" int gadmm_greedy_chains_wait() {
  GreedyPool& P = pool();
  wait_idle(P);
  const int rc = P.job.rc;
  if (P.claimed.load(std::memory_order_acquire) && P.owner.load() == std::this_thread::get_id()) {
    P.owner.store(std::thread::id());
    P.claimed.store(false, std::memory_order_release);  // the next caller's submit may take the worker
  }
  return rc;
}
