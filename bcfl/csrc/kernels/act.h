// Activation functions and their derivatives, shared by the bias+activation kernels
// (elementwise.hip) and the fused GEMM epilogues (linear.hip). Ids match bcfl/ops/functional.py
// _ACT_ID: HF BERT "gelu" (erf), ALBERT "gelu_new" (tanh approximation), ReLU, tanh, SiLU.
#pragma once
#include "common.h"

namespace bcfl {
namespace {

enum Act { ACT_GELU = 0, ACT_GELU_TANH = 1, ACT_RELU = 2, ACT_TANH = 3, ACT_SILU = 4 };

__device__ __forceinline__ float act_f(float x, int act) {
  switch (act) {
    case ACT_GELU: return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
    case ACT_GELU_TANH: {
      const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
      return 0.5f * x * (1.f + tanhf(u));
    }
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_TANH: return tanhf(x);
    default: return x / (1.f + __expf(-x));
  }
}

__device__ __forceinline__ float act_d(float x, int act) {
  switch (act) {
    case ACT_GELU:
      return 0.5f * (1.f + erff(x * 0.70710678118654752f)) +
             x * 0.3989422804014327f * __expf(-0.5f * x * x);
    case ACT_GELU_TANH: {
      const float k = 0.7978845608028654f;
      const float u = k * (x + 0.044715f * x * x * x);
      const float t = tanhf(u);
      return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * x * x);
    }
    case ACT_RELU: return x > 0.f ? 1.f : 0.f;
    case ACT_TANH: { const float t = tanhf(x); return 1.f - t * t; }
    default: { const float sg = 1.f / (1.f + __expf(-x)); return sg * (1.f + x * (1.f - sg)); }
  }
}

// compile-time activation (GEMM epilogues: no switch, no call, fully inlined)
template <int ACT>
__device__ __forceinline__ float act_ft(float x) {
  if constexpr (ACT == ACT_GELU) {
    return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
  } else if constexpr (ACT == ACT_GELU_TANH) {
    const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
    return 0.5f * x * (1.f + tanhf(u));
  } else {
    return x > 0.f ? x : 0.f;
  }
}

template <int ACT>
__device__ __forceinline__ float act_dt(float x) {
  if constexpr (ACT == ACT_GELU) {
    return 0.5f * (1.f + erff(x * 0.70710678118654752f)) +
           x * 0.3989422804014327f * __expf(-0.5f * x * x);
  } else if constexpr (ACT == ACT_GELU_TANH) {
    const float k = 0.7978845608028654f;
    const float u = k * (x + 0.044715f * x * x * x);
    const float t = tanhf(u);
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * x * x);
  } else {
    return x > 0.f ? 1.f : 0.f;
  }
}

}  // namespace
}  // namespace bcfl
