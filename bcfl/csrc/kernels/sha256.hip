// GPU SHA-256 Merkle hashing of a flat parameter buffer (the ledger's update_root).
//
// SHA-256 of a 433 MB BERT-base update on one CPU core takes 0.2-0.4 s and
// would dominate a ms-scale round. Here every leaf (default 4 KiB) is hashed by one GPU thread —
// ~100k independent leaves keep all 256 CUs busy — and the tree levels are reduced on the device;
// only the 32-byte root crosses PCIe. Domain separation as RFC 6962: leaf = H(0x00 || bytes),
// node = H(0x01 || left || right), an odd node is promoted. Bit-identical to hashlib (tests).
#include "common.h"
#include "kernels.h"

namespace bcfl {
namespace {

__device__ __constant__ uint32_t K256[64] = {
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

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_rotateright32(x, n); }
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ void compress(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      const uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
    }
    const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = hh + S1 + ch + K256[i] + wi;
    const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

__device__ __forceinline__ void init_h(uint32_t h[8]) {
  h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
  h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
}

__device__ __forceinline__ void store_digest(uint8_t* out, const uint32_t h[8]) {
  uint4* o = reinterpret_cast<uint4*>(out);
  o[0] = make_uint4(bswap(h[0]), bswap(h[1]), bswap(h[2]), bswap(h[3]));
  o[1] = make_uint4(bswap(h[4]), bswap(h[5]), bswap(h[6]), bswap(h[7]));
}

// message = 0x00 || leaf (L bytes, L % 4 == 0). Word i < L/4 of the message is the 1-byte-shifted
// big-endian view of data words i-1, i; then 0x80 after the last byte, zeros, 64-bit bit length.
__global__ __launch_bounds__(256) void sha_leaf_kernel(const uint8_t* __restrict__ data,
                                                      int64_t nbytes, int64_t leaf,
                                                      uint8_t* __restrict__ out, int64_t nleaves) {
  const int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (id >= nleaves) return;
  const int64_t lo = id * leaf;
  const int64_t L = (lo + leaf <= nbytes) ? leaf : (nbytes - lo > 0 ? nbytes - lo : 0);
  const uint32_t* D = reinterpret_cast<const uint32_t*>(data + lo);
  const int64_t nw = L / 4;                      // data words
  const int64_t M = 1 + L;                       // message bytes
  const int64_t P = ((M + 9 + 63) / 64) * 64;    // padded bytes
  const int64_t nblk = P / 64;
  const uint64_t bits = (uint64_t)M * 8u;
  uint32_t h[8];
  init_h(h);
  uint32_t prev = 0;  // BE of previous data word (low byte carries into the next message word)
  for (int64_t blk = 0; blk < nblk; ++blk) {
    uint32_t w[16];
    const int64_t k0 = blk * 16;
    if (k0 + 16 <= nw) {  // fast path: whole block inside the data
      const uint4* D4 = reinterpret_cast<const uint4*>(D + k0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 v = D4[q];
        const uint32_t be[4] = {bswap(v.x), bswap(v.y), bswap(v.z), bswap(v.w)};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          w[q * 4 + t] = (prev << 24) | (be[t] >> 8);
          prev = be[t];
        }
      }
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int64_t k = k0 + t;
        uint32_t x;
        if (k < nw) {
          const uint32_t be = bswap(D[k]);
          x = (prev << 24) | (be >> 8);
          prev = be;
        } else if (k == nw) {
          x = (prev << 24) | 0x00800000u;
        } else if (k == P / 4 - 2) {
          x = (uint32_t)(bits >> 32);
        } else if (k == P / 4 - 1) {
          x = (uint32_t)bits;
        } else {
          x = 0u;
        }
        w[t] = x;
      }
    }
    compress(h, w);
  }
  store_digest(out + id * 32, h);
}

// node i = H(0x01 || in[2i] || in[2i+1]) ; odd tail promoted
__global__ __launch_bounds__(256) void sha_node_kernel(const uint8_t* __restrict__ in, int64_t n,
                                                      uint8_t* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t m = (n + 1) / 2;
  if (i >= m) return;
  if (2 * i + 1 >= n) {  // promote
    const uint4* s = reinterpret_cast<const uint4*>(in + 2 * i * 32);
    uint4* d = reinterpret_cast<uint4*>(out + i * 32);
    d[0] = s[0];
    d[1] = s[1];
    return;
  }
  const uint32_t* c = reinterpret_cast<const uint32_t*>(in + 2 * i * 32);  // 16 words L||R
  uint32_t be[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) be[t] = bswap(c[t]);
  uint32_t h[8];
  init_h(h);
  uint32_t w[16];
  uint32_t prev = 0x01u;  // prefix byte
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    w[t] = (prev << 24) | (be[t] >> 8);
    prev = be[t];
  }
  compress(h, w);
  // second block: last byte of R, 0x80, zeros, length = 65 * 8 = 520 bits
#pragma unroll
  for (int t = 0; t < 16; ++t) w[t] = 0u;
  w[0] = (prev << 24) | 0x00800000u;
  w[15] = 520u;
  compress(h, w);
  store_digest(out + i * 32, h);
}

}  // namespace

int launch_sha256_leaves(const uint8_t* data, int64_t nbytes, int64_t leaf_bytes, uint8_t* out,
                         int64_t nleaves, hipStream_t s) {
  if (leaf_bytes % 64 || nbytes % 4 || ((uintptr_t)data & 15)) return -2;
  hipLaunchKernelGGL(sha_leaf_kernel, dim3((unsigned)((nleaves + 255) / 256)), dim3(256), 0, s,
                     data, nbytes, leaf_bytes, out, nleaves);
  return 0;
}

int launch_sha256_merkle(uint8_t* level, uint8_t* scratch, int64_t n, uint8_t* root, hipStream_t s) {
  uint8_t* a = level;
  uint8_t* b = scratch;
  while (n > 1) {
    const int64_t m = (n + 1) / 2;
    hipLaunchKernelGGL(sha_node_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, a, n, b);
    uint8_t* t = a; a = b; b = t;
    n = m;
  }
  return hipMemcpyAsync(root, a, 32, hipMemcpyDeviceToDevice, s) == hipSuccess ? 0 : -3;
}

}  // namespace bcfl
