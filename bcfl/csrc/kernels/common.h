// Shared device helpers for bcfl's gfx950 (CDNA4) kernels.
//   * 64-lane wave reductions (wave64 — never warp-32 idioms)
//   * bf16 <-> f32 bit conversions and 8/16-byte vector types
//   * the counter-based dropout hash, bit-identical to bcfl/ops/rng.py
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bcfl {

constexpr int WAVE = 64;

typedef uint16_t bf16_t;  // raw bf16 bits
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;   // MFMA A/B fragment (4 VGPRs)
typedef __attribute__((ext_vector_type(16))) float f32x16_t;   // 32x32 MFMA accumulator
typedef __attribute__((ext_vector_type(4))) float f32x4_t;     // 16x16 MFMA accumulator
typedef __attribute__((ext_vector_type(2))) float f32x2_t;     // packed-fp32 VALU pair
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2_t;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

// round-to-nearest-even f32 -> bf16: gfx950 has v_cvt_pk_bf16_f32 (RNE, NaN quieted), one
// instruction per pair instead of the ~7-op integer rounding sequence.
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}

__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  bf16x2_t v;
  v[0] = (__bf16)a;
  v[1] = (__bf16)b;
  return __builtin_bit_cast(uint32_t, v);
}

// generic element load/store for float / bf16 buffers
template <typename T> __device__ __forceinline__ float ld(const T* p, size_t i);
template <> __device__ __forceinline__ float ld<float>(const float* p, size_t i) { return p[i]; }
template <> __device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, size_t i) { return bf2f(p[i]); }
template <typename T> __device__ __forceinline__ void st(T* p, size_t i, float v);
template <> __device__ __forceinline__ void st<float>(float* p, size_t i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void st<bf16_t>(bf16_t* p, size_t i, float v) { p[i] = f2bf(v); }

// 4-wide vector load/store (8 B for bf16, 16 B for f32)
template <typename T> struct Vec4;
template <> struct Vec4<float> {
  __device__ __forceinline__ static void load(const float* p, float v[4]) {
    float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  }
  __device__ __forceinline__ static void store(float* p, const float v[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct Vec4<bf16_t> {
  __device__ __forceinline__ static void load(const bf16_t* p, float v[4]) {
    uint2 x = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(x.x << 16); v[1] = __uint_as_float(x.x & 0xffff0000u);
    v[2] = __uint_as_float(x.y << 16); v[3] = __uint_as_float(x.y & 0xffff0000u);
  }
  __device__ __forceinline__ static void store(bf16_t* p, const float v[4]) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
  }
};

// 8-wide vector load/store (16 B for bf16 — the 1 KiB-per-wave-instruction sweet spot)
template <typename T> struct Vec8;
template <> struct Vec8<float> {
  __device__ __forceinline__ static void load(const float* p, float v[8]) {
    Vec4<float>::load(p, v);
    Vec4<float>::load(p + 4, v + 4);
  }
  __device__ __forceinline__ static void store(float* p, const float v[8]) {
    Vec4<float>::store(p, v);
    Vec4<float>::store(p + 4, v + 4);
  }
};
template <> struct Vec8<bf16_t> {
  __device__ __forceinline__ static void load(const bf16_t* p, float v[8]) {
    uint4 x = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void store(bf16_t* p, const float v[8]) {
    *reinterpret_cast<uint4*>(p) = make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]),
                                              pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
  }
};

// sum over the 32 lanes of a half-wave (lanes l and l^k for k < 32 share a half)
__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- dropout hash (bcfl/ops/rng.py::hash32) --------------------------------------------------
__device__ __forceinline__ uint32_t hash32(uint32_t x, uint32_t ka, uint32_t kb) {
  x ^= ka;
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= kb;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// keep bit for element index e (uint32 wrap), 8-bit threshold p8
__device__ __forceinline__ bool keep_elem(uint32_t e, uint32_t p8, uint32_t ka, uint32_t kb) {
  uint32_t h = hash32(e >> 2, ka, kb);
  return ((h >> ((e & 3u) * 8u)) & 0xffu) >= p8;
}
__device__ __forceinline__ float keep_scale(uint32_t p8) { return 256.0f / (256.0f - (float)p8); }

}  // namespace bcfl
