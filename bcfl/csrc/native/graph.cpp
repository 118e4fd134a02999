// Host-side trust/network analytics (SURVEY.md §2.3 N1–N7), native C++.
//
// The reference computes these offline in notebooks with networkx / sklearn
// (All_graphs_IMDB_dataset.ipynb:168-180 PageRank, :300-314 DBSCAN, :362-366/:463-472 modified
// Z-score, :509/:544-650 greedy modularity) and hand-computes information-passing times in
// markdown (Medical_Transcriptions_All_graphs.ipynb:974-999). Here they are library functions
// that run inside the training loop (topology filter at start-up, update filter every round).
#include "graph.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>
#include <queue>
#include <stdexcept>

namespace bcfl {

// networkx 3.x pagerank (scipy variant): row-normalised weights, uniform personalisation,
// dangling mass redistributed uniformly, L1 convergence test err < N * tol.
PageRankResult pagerank(const std::vector<double>& W, int n, double alpha, double tol, int max_iter) {
  if ((int)W.size() != n * n) throw std::invalid_argument("pagerank: W must be n*n");
  std::vector<double> S(n, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) S[i] += W[i * n + j];
  std::vector<double> inv(n, 0.0);
  std::vector<int> dangling;
  for (int i = 0; i < n; ++i) {
    if (S[i] != 0.0) inv[i] = 1.0 / S[i];
    else dangling.push_back(i);
  }
  std::vector<double> x(n, 1.0 / n), xl(n), p(n, 1.0 / n);
  PageRankResult r;
  for (int it = 0; it < max_iter; ++it) {
    xl = x;
    double dsum = 0.0;
    for (int i : dangling) dsum += xl[i];
    for (int j = 0; j < n; ++j) {
      double acc = 0.0;
      for (int i = 0; i < n; ++i) {
        double q = W[i * n + j] * inv[i];
        if (q != 0.0) acc += xl[i] * q;
      }
      x[j] = alpha * (acc + dsum * p[j]) + (1.0 - alpha) * p[j];
    }
    double err = 0.0;
    for (int j = 0; j < n; ++j) err += std::fabs(x[j] - xl[j]);
    r.iterations = it + 1;
    if (err < n * tol) {
      r.ranks = x;
      r.converged = true;
      return r;
    }
  }
  r.ranks = x;
  r.converged = false;
  return r;
}

SigmaFlags sigma_flags(const std::vector<double>& v, double k, bool low_only) {
  SigmaFlags f;
  int n = (int)v.size();
  double mu = 0.0;
  for (double x : v) mu += x;
  mu /= std::max(n, 1);
  double var = 0.0;
  for (double x : v) var += (x - mu) * (x - mu);
  double sd = std::sqrt(var / std::max(n, 1));
  f.lo = mu - k * sd;
  f.hi = mu + k * sd;
  f.flags.assign(n, 0);
  for (int i = 0; i < n; ++i)
    f.flags[i] = (v[i] < f.lo) || (!low_only && v[i] > f.hi);
  return f;
}

static double median_of(std::vector<double> v) {
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  size_t n = v.size();
  return n % 2 ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2]);
}

std::vector<double> modified_z(const std::vector<double>& v) {
  double med = median_of(v);
  std::vector<double> dev(v.size());
  for (size_t i = 0; i < v.size(); ++i) dev[i] = std::fabs(v[i] - med);
  double mad = median_of(dev);
  std::vector<double> z(v.size());
  for (size_t i = 0; i < v.size(); ++i)
    z[i] = mad == 0.0 ? (v[i] == med ? 0.0 : std::copysign(std::numeric_limits<double>::infinity(), v[i] - med))
                      : 0.6745 * (v[i] - med) / mad;
  return z;
}

// sklearn DBSCAN semantics: neighbourhood = points within eps (inclusive, self included),
// core = |neighbourhood| >= min_samples, clusters grown from cores in index order.
std::vector<int> dbscan(const std::vector<double>& X, int n, int d, double eps, int min_samples) {
  std::vector<std::vector<int>> nb(n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int k = 0; k < d; ++k) {
        double t = X[i * d + k] - X[j * d + k];
        s += t * t;
      }
      if (std::sqrt(s) <= eps) nb[i].push_back(j);
    }
  std::vector<int> label(n, -1);
  std::vector<char> core(n, 0);
  for (int i = 0; i < n; ++i) core[i] = (int)nb[i].size() >= min_samples;
  int cid = 0;
  for (int i = 0; i < n; ++i) {
    if (!core[i] || label[i] != -1) continue;
    std::vector<int> stack{i};
    label[i] = cid;
    while (!stack.empty()) {
      int u = stack.back();
      stack.pop_back();
      if (!core[u]) continue;
      for (int v : nb[u])
        if (label[v] == -1) {
          label[v] = cid;
          if (core[v]) stack.push_back(v);
        }
    }
    ++cid;
  }
  return label;
}

std::vector<double> weighted_degree(const std::vector<double>& W, int n) {
  std::vector<double> deg(n, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) deg[i] += W[i * n + j];
  return deg;
}

std::vector<double> dijkstra(const std::vector<double>& L, int n, int src,
                             const std::vector<char>& active) {
  const double INF = std::numeric_limits<double>::infinity();
  std::vector<double> dist(n, INF);
  std::vector<char> done(n, 0);
  if (!active[src]) return dist;
  dist[src] = 0.0;
  using P = std::pair<double, int>;
  std::priority_queue<P, std::vector<P>, std::greater<P>> pq;
  pq.push({0.0, src});
  while (!pq.empty()) {
    auto [du, u] = pq.top();
    pq.pop();
    if (done[u]) continue;
    done[u] = 1;
    for (int v = 0; v < n; ++v) {
      if (!active[v] || v == u) continue;
      double w = L[u * n + v];
      if (!(w < INF) || w < 0) continue;
      if (du + w < dist[v]) {
        dist[v] = du + w;
        pq.push({dist[v], v});
      }
    }
  }
  return dist;
}

PassingTime info_passing_time(const std::vector<double>& L, int n, int src,
                              const std::vector<char>& active) {
  auto d = dijkstra(L, n, src, active);
  PassingTime t{0.0, 0.0, 0};
  for (int j = 0; j < n; ++j) {
    if (j == src || !active[j]) continue;
    if (!std::isfinite(d[j])) continue;
    t.sync += d[j];
    t.async_ = std::max(t.async_, d[j]);
    t.reached++;
  }
  return t;
}

BestSource best_source(const std::vector<double>& L, int n, const std::vector<char>& active,
                       double d_g) {
  BestSource b{-1, std::numeric_limits<double>::infinity()};
  for (int s = 0; s < n; ++s) {
    if (!active[s]) continue;
    auto t = info_passing_time(L, n, s, active);
    double obj = d_g + t.async_;
    if (obj < b.objective) { b.objective = obj; b.source = s; }
  }
  return b;
}

// Clauset–Newman–Moore greedy modularity agglomeration on a weighted undirected graph.
std::vector<int> greedy_modularity(const std::vector<double>& A, int n) {
  std::vector<int> comm(n);
  std::iota(comm.begin(), comm.end(), 0);
  double m2 = 0.0;
  for (double w : A) m2 += w;
  if (m2 <= 0.0) return comm;
  std::vector<double> k(n, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) k[i] += A[i * n + j];
  while (true) {
    int nc = *std::max_element(comm.begin(), comm.end()) + 1;
    std::vector<double> E(nc * nc, 0.0), a(nc, 0.0);
    for (int i = 0; i < n; ++i) {
      a[comm[i]] += k[i] / m2;
      for (int j = 0; j < n; ++j) E[comm[i] * nc + comm[j]] += A[i * n + j] / m2;
    }
    double best = 0.0;
    int bi = -1, bj = -1;
    for (int i = 0; i < nc; ++i)
      for (int j = i + 1; j < nc; ++j) {
        double dq = 2.0 * (E[i * nc + j] - a[i] * a[j]);
        if (dq > best + 1e-15) { best = dq; bi = i; bj = j; }
      }
    if (bi < 0) break;
    for (int& c : comm) {
      if (c == bj) c = bi;
      else if (c > bj) --c;
    }
  }
  return comm;
}

double modularity(const std::vector<double>& A, int n, const std::vector<int>& comm) {
  double m2 = 0.0;
  for (double w : A) m2 += w;
  if (m2 <= 0.0) return 0.0;
  std::vector<double> k(n, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) k[i] += A[i * n + j];
  double q = 0.0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j)
      if (comm[i] == comm[j]) q += A[i * n + j] - k[i] * k[j] / m2;
  return q / m2;
}

}  // namespace bcfl
