// D-GADMM chain construction on the host, for a batch of epochs (K15: findPath.m:16-30 /
// findPath2.m:43-59 semantics). Python draws the node positions (the seeded numpy stream the
// reference-semantics schedule defines); this routine does the O(E N^2) part -- squared distances,
// the greedy nearest-unvisited chain from node 0 (lowest index wins ties, as numpy argmin), and the
// per-hop cost -- so pre-drawing ~300 epochs for a one-launch D-GADMM run costs tens of us instead
// of milliseconds of numpy dispatch. Bit-identical to PathSchedule.prefetch_arrays' numpy path: no
// FMA contraction, the same operation order ((dx*dx) + (dy*dy); ((d2*eta)*bw)*f for energies).
#include <algorithm>
#include <cstdlib>
#include <limits>
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
