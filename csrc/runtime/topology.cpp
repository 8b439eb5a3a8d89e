// D-GADMM chain construction on the host, for a batch of epochs (K15: findPath.m:16-30 /
// findPath2.m:43-59 semantics). Python draws the node positions (the seeded numpy stream the
// reference-semantics schedule defines); this routine does the O(E N^2) part -- squared distances,
// the greedy nearest-unvisited chain from node 0 (lowest index wins ties, as numpy argmin), and the
// per-hop cost -- so pre-drawing ~300 epochs for a one-launch D-GADMM run costs tens of us instead
// of milliseconds of numpy dispatch. Bit-identical to PathSchedule.prefetch_arrays' numpy path: no
// FMA contraction, the same operation order ((dx*dx) + (dy*dy); ((d2*eta)*bw)*f for energies).
#include <limits>
#include <vector>

#pragma clang fp contract(off)

extern "C" int gadmm_greedy_chains(const double* uv, int E, int n, double side, int energy, double eta, double bw,
                                   double f, long long* paths, double* costs) {
  if (E < 0 || n < 1 || !uv || !paths || (n > 1 && !costs)) return -1;
  std::vector<double> x(n), y(n), d2((size_t)n * n);
  std::vector<char> visited(n);
  const double inf = std::numeric_limits<double>::infinity();
  for (int e = 0; e < E; ++e) {
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
  return 0;
}
