// SHA-256 (FIPS 180-4), host implementation used by the ledger and the Merkle verifier.
// The device-side leaf/inner hashing lives in csrc/kernels/sha256.hip; both must agree
// bit-for-bit (tests compare against Python's hashlib).
#pragma once
#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace bcfl {

class Sha256 {
 public:
  Sha256() { reset(); }
  void reset() {
    static const uint32_t iv[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    std::memcpy(h_, iv, sizeof(iv));
    len_ = 0;
    buf_len_ = 0;
  }
  void update(const void* data, size_t n);
  std::array<uint8_t, 32> digest();

 private:
  void block(const uint8_t* p);
  uint32_t h_[8];
  uint64_t len_;
  uint8_t buf_[64];
  size_t buf_len_;
};

std::array<uint8_t, 32> sha256(const void* data, size_t n);
std::string to_hex(const uint8_t* d, size_t n);
std::string sha256_hex(const std::string& s);

// RFC-6962-style Merkle tree: leaf = H(0x00 || leaf bytes), node = H(0x01 || L || R),
// an odd node at the end of a level is promoted unchanged.
std::array<uint8_t, 32> merkle_root(const uint8_t* data, size_t n, size_t leaf_bytes);
std::array<uint8_t, 32> merkle_from_leaves(const std::vector<std::array<uint8_t, 32>>& leaves);

}  // namespace bcfl
