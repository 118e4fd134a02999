#pragma once
#include <vector>

namespace bcfl {

struct PageRankResult {
  std::vector<double> ranks;
  int iterations = 0;
  bool converged = false;
};
PageRankResult pagerank(const std::vector<double>& W, int n, double alpha = 0.85,
                        double tol = 1e-6, int max_iter = 100);

struct SigmaFlags {
  double lo, hi;
  std::vector<int> flags;
};
SigmaFlags sigma_flags(const std::vector<double>& v, double k, bool low_only);

std::vector<double> modified_z(const std::vector<double>& v);
std::vector<int> dbscan(const std::vector<double>& X, int n, int d, double eps, int min_samples);
std::vector<double> weighted_degree(const std::vector<double>& W, int n);
std::vector<double> dijkstra(const std::vector<double>& L, int n, int src,
                             const std::vector<char>& active);

struct PassingTime {
  double sync;    // sum over destinations (sequential sends)
  double async_;  // max over destinations (concurrent sends)
  int reached;
};
PassingTime info_passing_time(const std::vector<double>& L, int n, int src,
                              const std::vector<char>& active);

struct BestSource {
  int source;
  double objective;
};
BestSource best_source(const std::vector<double>& L, int n, const std::vector<char>& active,
                       double d_g);

std::vector<int> greedy_modularity(const std::vector<double>& A, int n);
double modularity(const std::vector<double>& A, int n, const std::vector<int>& comm);

}  // namespace bcfl
