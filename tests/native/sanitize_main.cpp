// Host-runtime self-test built with -fsanitize=address,undefined: exercises the
// SHA-256 / Merkle, hash-chain ledger and graph code paths the Python bindings use, so memory and
// UB errors in the native host components surface on the CPU (GPU sanitizers are unavailable).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "graph.h"
#include "ledger.h"
#include "sha256.h"

#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                     \
    }                                                               \
  } while (0)

int main() {
  // SHA-256 known answers (FIPS 180-2)
  CHECK(bcfl::sha256_hex("abc") ==
        "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad");
  CHECK(bcfl::sha256_hex("") ==
        "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855");
  std::string m(1000003, 'a');
  for (size_t i = 0; i < m.size(); ++i) m[i] = char('a' + (i * 7) % 26);
  auto one = bcfl::sha256(m.data(), m.size());
  bcfl::Sha256 h;  // streaming in odd chunks == one shot
  for (size_t i = 0; i < m.size(); i += 777) h.update(m.data() + i, std::min<size_t>(777, m.size() - i));
  CHECK(h.digest() == one);
  // Merkle: tail leaf shorter than leaf_bytes, odd leaf counts
  for (size_t n : {1u, 4095u, 4096u, 4097u, 3u * 4096u + 5u}) {
    auto r1 = bcfl::merkle_root(reinterpret_cast<const uint8_t*>(m.data()), n, 4096);
    auto r2 = bcfl::merkle_root(reinterpret_cast<const uint8_t*>(m.data()), n, 4096);
    CHECK(r1 == r2);
  }
  // ledger: append, verify, tamper detection
  bcfl::Ledger L("{\"genesis\":1}", 0.0);
  for (int r = 0; r < 50; ++r)
    for (int c = 0; c < 4; ++c) L.append(r, c, "update", bcfl::sha256_hex(std::to_string(r * 4 + c)), "accept", "{}", r + 0.001 * c);
  CHECK(L.size() == 201 && L.verify() == -1);
  L.mutable_at(77).verdict = "reject";
  CHECK(L.verify() == 77);
  // graph analytics on a random complete digraph
  const int n = 12;
  std::vector<double> W(n * n, 0.0), Lat(n * n, 0.0);
  unsigned s = 12345;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j)
      if (i != j) {
        s = s * 1103515245u + 12345u;
        const double bw = 50.0 + (s >> 16) % 450;
        W[i * n + j] = 1.0 / bw;
        Lat[i * n + j] = 0.4 / bw;
      }
  auto pr = bcfl::pagerank(W, n);
  double sum = 0;
  for (double x : pr.ranks) sum += x;
  CHECK(pr.converged && std::fabs(sum - 1.0) < 1e-9);
  auto sf = bcfl::sigma_flags(pr.ranks, 1.0, false);
  CHECK(sf.lo < sf.hi);
  auto z = bcfl::modified_z(bcfl::weighted_degree(W, n));
  CHECK((int)z.size() == n);
  std::vector<double> X(n);
  for (int i = 0; i < n; ++i) X[i] = i < 10 ? 1.0 + 0.01 * i : 50.0 + i;
  auto lab = bcfl::dbscan(X, n, 1, 0.5, 2);
  CHECK(lab[11] == -1 && lab[0] != -1);
  std::vector<char> act(n, 1);
  act[3] = 0;
  auto pt = bcfl::info_passing_time(Lat, n, 0, act);
  CHECK(pt.reached == n - 2 && pt.async_ <= pt.sync);
  auto bs = bcfl::best_source(Lat, n, act, 1.0);
  CHECK(bs.source >= 0 && bs.source != 3);
  auto comm = bcfl::greedy_modularity(W, n);
  CHECK((int)comm.size() == n);
  std::printf("native host sanitizer self-test OK\n");
  return 0;
}
