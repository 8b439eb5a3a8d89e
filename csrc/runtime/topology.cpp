// D-GADMM chain construction on the host, for a batch of epochs (K15: findPath.m:16-30 /
// findPath2.m:43-59 semantics). Python draws the node positions (the seeded numpy stream the
// reference-semantics schedule defines); this routine does the O(E N^2) part -- squared distances,
// the greedy nearest-unvisited chain from node 0 (lowest index wins ties, as numpy argmin), and the
// per-hop cost -- so pre-drawing ~300 epochs for a one-launch D-GADMM run costs tens of us instead
// of milliseconds of numpy dispatch. Bit-identical to PathSchedule.prefetch_arrays' numpy path: no
// FMA contraction, the same operation order ((dx*dx) + (dy*dy); ((d2*eta)*bw)*f for energies).
#include <algorithm>
#include <limits>
#include <thread>
#include <vector>

#pragma clang fp contract(off)

namespace {

// Epochs [e0, e1) of the batch: one geometry + greedy chain each (independent of the others).
void greedy_range(const double* uv, int e0, int e1, int n, double side, int energy, double eta, double bw, double f,
                  long long* paths, double* costs) {
  std::vector<double> x(n), y(n), d2((size_t)n * n);
  std::vector<char> visited(n);
  const double inf = std::numeric_limits<double>::infinity();
  for (int e = e0; e < e1; ++e) {
    const double* g = uv + (size_t)e * n * 2;
    for (int i = 0; i < n; ++i) {
      x[i] = g[2 * i] * side;
      y[i] = g[2 * i + 1] * side;
    }
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        const double dx = x[i] - x[j], dy = y[i] - y[j];
        const double a = dx * dx, b = dy * dy;
        d2[(size_t)i * n + j] = i == j ? 0.0 : a + b;
      }
    long long* p = paths + (size_t)e * n;
    std::fill(visited.begin(), visited.end(), 0);
    int cur = 0;
    p[0] = 0;
    visited[0] = 1;
    for (int k = 1; k < n; ++k) {
      int best = -1;
      double bv = inf;
      const double* row = d2.data() + (size_t)cur * n;
      for (int j = 0; j < n; ++j)
        if (!visited[j] && row[j] < bv) {
          bv = row[j];
          best = j;
        }
      if (best < 0)  // every candidate at +inf / NaN: numpy argmin takes the first unvisited
        for (int j = 0; j < n && best < 0; ++j)
          if (!visited[j]) best = j;
      p[k] = best;
      visited[best] = 1;
      double c = d2[(size_t)cur * n + best];
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

// The epochs are independent: large batches are split over up to 8 host threads (the ~300-epoch
// batch of a one-launch D-GADMM solve took ~0.5-1 ms on one core, a third of the solve).
extern "C" int gadmm_greedy_chains(const double* uv, int E, int n, double side, int energy, double eta, double bw,
                                   double f, long long* paths, double* costs) {
  if (E < 0 || n < 1 || !uv || !paths || (n > 1 && !costs)) return -1;
  const long work = (long)E * n * n;
  int nt = 1;
  if (work > 40000) {
    const unsigned hw = std::thread::hardware_concurrency();
    nt = (int)std::min<long>(std::min<unsigned>(hw ? hw : 1, 8u), std::max<long>(1, work / 40000));
    if (nt > E) nt = E;
  }
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

// Per-epoch device tables of the one-launch D-GADMM kernel (chain_persistent.hip, dynamic mode),
// from the chains P [E][n] (position -> worker): for each local worker li (global id loc[li]) its
// slot (li, gid, left, right) and chain position in every epoch. Replaces ~0.5 ms of numpy per
// solve (argsort + fancy indexing over ~300 epochs) on the host path of every D-GADMM solve.
extern "C" int gadmm_epoch_tables(const long long* P, int E, int n, const long long* loc, int nloc, int* slots,
                                  int* pos) {
  if (E < 0 || n < 1 || nloc < 0 || !P || (nloc > 0 && (!loc || !slots || !pos))) return -1;
  std::vector<int> pos_of(n);
  for (int e = 0; e < E; ++e) {
    const long long* pe = P + (size_t)e * n;
    for (int p = 0; p < n; ++p) {
      const long long w = pe[p];
      if (w < 0 || w >= n) return -2;
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
