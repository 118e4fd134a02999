#include "sha256.h"

namespace bcfl {
namespace {
constexpr uint32_t K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};
inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
}  // namespace

void Sha256::block(const uint8_t* p) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i)
    w[i] = (uint32_t(p[4 * i]) << 24) | (uint32_t(p[4 * i + 1]) << 16) |
           (uint32_t(p[4 * i + 2]) << 8) | uint32_t(p[4 * i + 3]);
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h_[0], b = h_[1], c = h_[2], d = h_[3], e = h_[4], f = h_[5], g = h_[6], h = h_[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + K[i] + w[i];
    uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h_[0] += a; h_[1] += b; h_[2] += c; h_[3] += d; h_[4] += e; h_[5] += f; h_[6] += g; h_[7] += h;
}

void Sha256::update(const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  len_ += n;
  if (buf_len_) {
    size_t take = std::min(n, 64 - buf_len_);
    std::memcpy(buf_ + buf_len_, p, take);
    buf_len_ += take; p += take; n -= take;
    if (buf_len_ == 64) { block(buf_); buf_len_ = 0; }
  }
  while (n >= 64) { block(p); p += 64; n -= 64; }
  if (n) { std::memcpy(buf_, p, n); buf_len_ = n; }
}

std::array<uint8_t, 32> Sha256::digest() {
  uint64_t bits = len_ * 8;
  uint8_t pad = 0x80;
  update(&pad, 1);
  uint8_t z = 0;
  while (buf_len_ != 56) update(&z, 1);
  uint8_t lb[8];
  for (int i = 0; i < 8; ++i) lb[i] = uint8_t(bits >> (56 - 8 * i));
  update(lb, 8);
  std::array<uint8_t, 32> out;
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = uint8_t(h_[i] >> 24); out[4 * i + 1] = uint8_t(h_[i] >> 16);
    out[4 * i + 2] = uint8_t(h_[i] >> 8); out[4 * i + 3] = uint8_t(h_[i]);
  }
  return out;
}

std::array<uint8_t, 32> sha256(const void* data, size_t n) {
  Sha256 s;
  s.update(data, n);
  return s.digest();
}

std::string to_hex(const uint8_t* d, size_t n) {
  static const char* hx = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) { s[2 * i] = hx[d[i] >> 4]; s[2 * i + 1] = hx[d[i] & 15]; }
  return s;
}

std::string sha256_hex(const std::string& s) {
  auto d = sha256(s.data(), s.size());
  return to_hex(d.data(), 32);
}

std::array<uint8_t, 32> merkle_from_leaves(const std::vector<std::array<uint8_t, 32>>& leaves) {
  if (leaves.empty()) return sha256(nullptr, 0);
  std::vector<std::array<uint8_t, 32>> lvl = leaves, nxt;
  while (lvl.size() > 1) {
    nxt.clear();
    for (size_t i = 0; i + 1 < lvl.size(); i += 2) {
      uint8_t buf[65];
      buf[0] = 0x01;
      std::memcpy(buf + 1, lvl[i].data(), 32);
      std::memcpy(buf + 33, lvl[i + 1].data(), 32);
      nxt.push_back(sha256(buf, 65));
    }
    if (lvl.size() % 2) nxt.push_back(lvl.back());
    lvl.swap(nxt);
  }
  return lvl[0];
}

std::array<uint8_t, 32> merkle_root(const uint8_t* data, size_t n, size_t leaf_bytes) {
  size_t nl = n ? (n + leaf_bytes - 1) / leaf_bytes : 1;
  std::vector<std::array<uint8_t, 32>> leaves(nl);
  for (size_t i = 0; i < nl; ++i) {
    Sha256 s;
    uint8_t z = 0x00;
    s.update(&z, 1);
    size_t lo = i * leaf_bytes, len = std::min(leaf_bytes, n - std::min(n, lo));
    if (len) s.update(data + lo, len);
    leaves[i] = s.digest();
  }
  return merkle_from_leaves(leaves);
}

}  // namespace bcfl
