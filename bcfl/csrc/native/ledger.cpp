#include "ledger.h"

#include <cstdio>

#include "sha256.h"

namespace bcfl {

std::string block_preimage(const Block& b) {
  char ts[64];
  std::snprintf(ts, sizeof(ts), "%.6f", b.ts);
  std::string s;
  s.reserve(256 + b.payload.size());
  s += std::to_string(b.height); s += '|';
  s += b.prev_hash; s += '|';
  s += ts; s += '|';
  s += std::to_string(b.round); s += '|';
  s += std::to_string(b.client); s += '|';
  s += b.kind; s += '|';
  s += b.update_root; s += '|';
  s += b.verdict; s += '|';
  s += b.payload;
  return s;
}

std::string block_hash(const Block& b) { return sha256_hex(block_preimage(b)); }

Ledger::Ledger(const std::string& genesis_payload, double ts) {
  Block g;
  g.height = 0;
  g.prev_hash = std::string(64, '0');
  g.ts = ts;
  g.kind = "genesis";
  g.payload = genesis_payload;
  g.hash = block_hash(g);
  chain_.push_back(g);
}

const Block& Ledger::append(int64_t round, int64_t client, const std::string& kind,
                            const std::string& update_root, const std::string& verdict,
                            const std::string& payload, double ts) {
  Block b;
  b.height = (int64_t)chain_.size();
  b.prev_hash = chain_.back().hash;
  b.ts = ts;
  b.round = round;
  b.client = client;
  b.kind = kind;
  b.update_root = update_root;
  b.verdict = verdict;
  b.payload = payload;
  b.hash = block_hash(b);
  chain_.push_back(b);
  return chain_.back();
}

int64_t Ledger::verify() const {
  for (size_t i = 0; i < chain_.size(); ++i) {
    const Block& b = chain_[i];
    if (b.height != (int64_t)i) return (int64_t)i;
    if (i == 0 ? b.prev_hash != std::string(64, '0') : b.prev_hash != chain_[i - 1].hash)
      return (int64_t)i;
    if (block_hash(b) != b.hash) return (int64_t)i;
  }
  return -1;
}

}  // namespace bcfl
