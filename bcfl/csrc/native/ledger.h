// Append-only hash-chained ledger of federated updates ("BC-FL").
//
// The reference only *names* a blockchain layer (chart titles and a hand sum at
// All_graphs_IMDB_dataset.ipynb:1048,1070-1071; Medical_Transcriptions_All_graphs.ipynb:1091-1098;
// no ledger, hashing or block code exists — SURVEY.md N8). This is a real one: every block
// commits to its predecessor's hash, the round, the client, the SHA-256 Merkle root of the
// client's flat update buffer (hashed on the GPU) and the anomaly verdict; verify() walks the
// chain and returns the first height whose hash or back-link does not match.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace bcfl {

struct Block {
  int64_t height = 0;
  std::string prev_hash;
  double ts = 0.0;
  int64_t round = -1;
  int64_t client = -1;
  std::string kind;
  std::string update_root;
  std::string verdict;
  std::string payload;
  std::string hash;
};

std::string block_preimage(const Block& b);
std::string block_hash(const Block& b);

class Ledger {
 public:
  Ledger(const std::string& genesis_payload, double ts);
  const Block& append(int64_t round, int64_t client, const std::string& kind,
                      const std::string& update_root, const std::string& verdict,
                      const std::string& payload, double ts);
  // -1 when the whole chain verifies, else the first failing height
  int64_t verify() const;
  const std::string& tip() const { return chain_.back().hash; }
  size_t size() const { return chain_.size(); }
  const Block& at(size_t i) const { return chain_.at(i); }
  Block& mutable_at(size_t i) { return chain_.at(i); }  // fault-injection tests only
  void push_raw(const Block& b) { chain_.push_back(b); }
  void clear() { chain_.clear(); }

 private:
  std::vector<Block> chain_;
};

}  // namespace bcfl
