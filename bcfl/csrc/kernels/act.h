// Activation functions and their derivatives, shared by the bias+activation kernels
// (elementwise.hip) and the fused GEMM epilogues (linear.hip). Ids match bcfl/ops/functional.py
// _ACT_ID: HF BERT "gelu" (erf), ALBERT "gelu_new" (tanh approximation), ReLU, tanh, SiLU.
#pragma once
#include "common.h"

namespace bcfl {
namespace {

enum Act { ACT_GELU = 0, ACT_GELU_TANH = 1, ACT_RELU = 2, ACT_TANH = 3, ACT_SILU = 4 };

// erf(x) by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16 output rounding):
// one v_rcp, one v_exp and 5 FMAs, no branches. The libm erff is a piecewise polynomial whose
// divergent branches both run in a wave; in the fused GEMM epilogues (64 outputs per lane) that
// VALU work is not hidden behind MFMA (the GELU variants ran ~30 % below the plain GEMMs,
// profiles/linear_gemm_vs_hipblaslt.md). Returns erf(z) and e = exp(-z^2) (GELU' reuses it:
// exp(-x^2 / 2) with z = x / sqrt(2)).
__device__ __forceinline__ float fast_erf(float z, float& e) {
  const float a = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  e = __builtin_amdgcn_exp2f(-1.4426950408889634f * a * a);
  return copysignf(fmaf(-p, e, 1.f), z);
}

// tanh(u) = 1 - 2 / (1 + exp(2u)): one exp2 + one reciprocal (saturates cleanly at +-1)
__device__ __forceinline__ float fast_tanh(float u) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(2.8853900817779268f * u));
}

__device__ __forceinline__ float gelu_f(float x) {
  float e;
  return 0.5f * x * (1.f + fast_erf(x * 0.70710678118654752f, e));
}

__device__ __forceinline__ float gelu_d(float x) {
  float e;
  const float r = fast_erf(x * 0.70710678118654752f, e);
  return fmaf(x * 0.3989422804014327f, e, 0.5f * (1.f + r));
}

__device__ __forceinline__ float gelu_tanh_f(float x) {
  const float u = 0.7978845608028654f * fmaf(0.044715f * x, x * x, x);
  return 0.5f * x * (1.f + fast_tanh(u));
}

__device__ __forceinline__ float gelu_tanh_d(float x) {
  const float k = 0.7978845608028654f;
  const float u = k * fmaf(0.044715f * x, x * x, x);
  const float t = fast_tanh(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * x * x);
}

__device__ __forceinline__ float act_f(float x, int act) {
  switch (act) {
    case ACT_GELU: return gelu_f(x);
    case ACT_GELU_TANH: return gelu_tanh_f(x);
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_TANH: return fast_tanh(x);
    default: return x / (1.f + __expf(-x));
  }
}

__device__ __forceinline__ float act_d(float x, int act) {
  switch (act) {
    case ACT_GELU: return gelu_d(x);
    case ACT_GELU_TANH: return gelu_tanh_d(x);
    case ACT_RELU: return x > 0.f ? 1.f : 0.f;
    case ACT_TANH: { const float t = fast_tanh(x); return 1.f - t * t; }
    default: { const float sg = 1.f / (1.f + __expf(-x)); return sg * (1.f + x * (1.f - sg)); }
  }
}

// compile-time activation (GEMM epilogues: no switch, no call, fully inlined)
template <int ACT>
__device__ __forceinline__ float act_ft(float x) {
  if constexpr (ACT == ACT_GELU) {
    return gelu_f(x);
  } else if constexpr (ACT == ACT_GELU_TANH) {
    return gelu_tanh_f(x);
  } else {
    return x > 0.f ? x : 0.f;
  }
}

template <int ACT>
__device__ __forceinline__ float act_dt(float x) {
  if constexpr (ACT == ACT_GELU) {
    return gelu_d(x);
  } else if constexpr (ACT == ACT_GELU_TANH) {
    return gelu_tanh_d(x);
  } else {
    return x > 0.f ? 1.f : 0.f;
  }
}

}  // namespace
}  // namespace bcfl
