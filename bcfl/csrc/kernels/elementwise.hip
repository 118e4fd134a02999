// Memory-bound fused kernels (SURVEY.md §2.6 K6, K10, K11 + Llama SwiGLU/RoPE).
//
//   bias_act_fwd/bwd   GEMM epilogue: bias + GELU(erf) / gelu_new(tanh) / ReLU / tanh / SiLU, and
//                      its backward with the bias-gradient column sum fused in (K6)
//   swiglu_fwd/bwd     silu(gate) * up on the fused [T, 2I] gate|up projection
//   rope               rotate the q|k column blocks of a packed qkv projection (HF rotate_half)
//   adamw              ONE launch over the whole flat parameter buffer (K10), HF or torch semantics
//   mix / axpby / delta_encode / cast_copy   FedAvg scale-accumulate + gossip mixing (K11) and the
//                      error-feedback bf16 delta codec of the P2P wire
//   block_sketch       signed block sketch of a flat update for the anomaly filter
//
// All kernels use 4-wide vector accesses (8 B bf16 / 16 B fp32 per lane) and grid-stride loops
// sized to the CU count (Guideline 11: ≤ 8 blocks per CU resident, rest grid-strided).
#include "act.h"
#include "common.h"
#include "kernels.h"

namespace bcfl {
namespace {

constexpr int EW_THREADS = 256;

inline int ew_grid(int64_t nvec) {
  int64_t g = (nvec + EW_THREADS - 1) / EW_THREADS;
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

// 2-D launch for row-structured elementwise kernels: grid.x covers the columns in 8-element
// chunks (one 16-byte access per lane), grid.y strides over rows — no per-element 64-bit
// division (which the compiler would expand into a software divide).
constexpr int COLS_PER_BLOCK = EW_THREADS * 8;

template <typename T>
__global__ __launch_bounds__(EW_THREADS) void bias_act_fwd_kernel(const T* __restrict__ y,
                                                                  const T* __restrict__ bias,
                                                                  T* __restrict__ out,
                                                                  int64_t rows, int N, int act) {
  const int col = (blockIdx.x * EW_THREADS + threadIdx.x) * 8;
  if (col >= N) return;
  float b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (bias) Vec8<T>::load(bias + col, b);
  for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
    const int64_t e = r * N + col;
    float v[8];
    Vec8<T>::load(y + e, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = act_f(v[k] + b[k], act);
    Vec8<T>::store(out + e, v);
  }
}

// grid (ceil(N / 2048), nblk_rows); partial[blockIdx.y][N]
template <typename T>
__global__ __launch_bounds__(EW_THREADS) void bias_act_bwd_kernel(
    const T* __restrict__ dout, const T* __restrict__ y, const T* __restrict__ bias,
    T* __restrict__ dy, float* __restrict__ partial, int64_t rows, int N, int act) {
  const int col = (blockIdx.x * EW_THREADS + threadIdx.x) * 8;
  if (col >= N) return;
  float b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (bias) Vec8<T>::load(bias + col, b);
  for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
    const int64_t e = r * N + col;
    float d[8], v[8], o[8];
    Vec8<T>::load(dout + e, d);
    Vec8<T>::load(y + e, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o[k] = d[k] * act_d(v[k] + b[k], act);
      acc[k] += o[k];
    }
    Vec8<T>::store(dy + e, o);
  }
  if (partial) Vec8<float>::store(partial + (size_t)blockIdx.y * N + col, acc);
}

template <typename T>
__global__ __launch_bounds__(EW_THREADS) void swiglu_fwd_kernel(const T* __restrict__ gu,
                                                                T* __restrict__ out, int64_t rows,
                                                                int I) {
  const int c = (blockIdx.x * EW_THREADS + threadIdx.x) * 8;
  if (c >= I) return;
  for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
    float g[8], u[8], o[8];
    Vec8<T>::load(gu + r * 2 * I + c, g);
    Vec8<T>::load(gu + r * 2 * I + I + c, u);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = g[k] / (1.f + __expf(-g[k])) * u[k];
    Vec8<T>::store(out + r * I + c, o);
  }
}

template <typename T>
__global__ __launch_bounds__(EW_THREADS) void swiglu_bwd_kernel(const T* __restrict__ dout,
                                                                const T* __restrict__ gu,
                                                                T* __restrict__ dgu, int64_t rows,
                                                                int I) {
  const int c = (blockIdx.x * EW_THREADS + threadIdx.x) * 8;
  if (c >= I) return;
  for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
    float d[8], g[8], u[8], dg[8], du[8];
    Vec8<T>::load(dout + r * I + c, d);
    Vec8<T>::load(gu + r * 2 * I + c, g);
    Vec8<T>::load(gu + r * 2 * I + I + c, u);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float sg = 1.f / (1.f + __expf(-g[k]));
      const float sl = g[k] * sg;
      du[k] = d[k] * sl;
      dg[k] = d[k] * u[k] * sg * (1.f + g[k] * (1.f - sg));
    }
    Vec8<T>::store(dgu + r * 2 * I + c, dg);
    Vec8<T>::store(dgu + r * 2 * I + I + c, du);
  }
}

// one thread per (row, rotated pair) or per copied element pair
template <typename T>
__global__ __launch_bounds__(EW_THREADS) void rope_kernel(const T* __restrict__ x, T* __restrict__ out,
                                                         const int* __restrict__ pos,
                                                         const float* __restrict__ cosb,
                                                         const float* __restrict__ sinb,
                                                         int64_t rows, int stride, int nrot, int d,
                                                         int inverse) {
  const int half = d / 2;
  const int per_row = stride / 2;  // work items per row
  const int64_t total = rows * per_row;
  for (int64_t i = blockIdx.x * (int64_t)EW_THREADS + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * EW_THREADS) {
    const int64_t r = i / per_row;
    const int w = (int)(i % per_row);
    const int64_t rb = r * stride;
    const int rot_items = nrot * half;
    if (w < rot_items) {
      const int h = w / half, j = w % half;
      const int p = pos[r];
      const float c = cosb[(int64_t)p * half + j];
      const float s = inverse ? -sinb[(int64_t)p * half + j] : sinb[(int64_t)p * half + j];
      const int64_t a = rb + (int64_t)h * d + j;
      const float x1 = ld<T>(x, a), x2 = ld<T>(x, a + half);
      st<T>(out, a, x1 * c - x2 * s);
      st<T>(out, a + half, x2 * c + x1 * s);
    } else {
      const int64_t a = rb + (int64_t)nrot * d + 2 * (w - rot_items);
      st<T>(out, a, ld<T>(x, a));
      st<T>(out, a + 1, ld<T>(x, a + 1));
    }
  }
}

// bf16, 16-byte vectors: one thread rotates 8 consecutive pairs (x[j], x[j + d/2]) of one head
// (cos / sin as two float4 loads each from the table row of the token's position) or copies 8
// elements of the non-rotated tail (v); ~5x less time than the element-pair kernel at the
// Llama-3-8B qkv shape ([8k, 6144], profiles/config5_kernel_stats_r4.md: 163 us per call)
__global__ __launch_bounds__(EW_THREADS) void rope_vec_kernel(const bf16_t* __restrict__ x,
                                                             bf16_t* __restrict__ out,
                                                             const int* __restrict__ pos,
                                                             const float* __restrict__ cosb,
                                                             const float* __restrict__ sinb,
                                                             int64_t rows, int stride, int nrot,
                                                             int d, int inverse) {
  const int half = d / 2, hv = half / 8;
  const int rot_v = nrot * hv, cp_v = (stride - nrot * d) / 8;
  const int per_row = rot_v + cp_v;
  const int64_t total = rows * per_row;
  for (int64_t i = blockIdx.x * (int64_t)EW_THREADS + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * EW_THREADS) {
    const int64_t r = i / per_row;
    const int w = (int)(i - r * per_row);
    const int64_t rb = r * stride;
    if (w < rot_v) {
      const int h = w / hv, j0 = (w - h * hv) * 8;
      const int64_t t = (int64_t)pos[r] * half + j0;
      float c[8], sn[8], x1[8], x2[8], y1[8], y2[8];
      Vec8<float>::load(cosb + t, c);
      Vec8<float>::load(sinb + t, sn);
      const int64_t a = rb + (int64_t)h * d + j0;
      Vec8<bf16_t>::load(x + a, x1);
      Vec8<bf16_t>::load(x + a + half, x2);
      const float sg = inverse ? -1.f : 1.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float se = sg * sn[e];
        y1[e] = x1[e] * c[e] - x2[e] * se;
        y2[e] = x2[e] * c[e] + x1[e] * se;
      }
      Vec8<bf16_t>::store(out + a, y1);
      Vec8<bf16_t>::store(out + a + half, y2);
    } else {
      const int64_t a = rb + (int64_t)nrot * d + 8 * (w - rot_v);
      *reinterpret_cast<uint4*>(out + a) = *reinterpret_cast<const uint4*>(x + a);
    }
  }
}

template <typename TD, typename TS>
__global__ __launch_bounds__(EW_THREADS) void cast_kernel(TD* __restrict__ dst,
                                                         const TS* __restrict__ src, int64_t n) {
  const int64_t nvec = n / 4;
  for (int64_t i = blockIdx.x * (int64_t)EW_THREADS + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * EW_THREADS) {
    float v[4];
    Vec4<TS>::load(src + i * 4, v);
    Vec4<TD>::store(dst + i * 4, v);
  }
  for (int64_t i = nvec * 4 + blockIdx.x * (int64_t)EW_THREADS + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * EW_THREADS)
    st<TD>(dst, i, ld<TS>(src, i));
}

template <typename TX>
__global__ __launch_bounds__(EW_THREADS) void axpby_kernel(float* __restrict__ y, const TX* x,
                                                          float a, float b, int64_t n) {
  const int64_t nvec = n / 4;
  for (int64_t i = blockIdx.x * (int64_t)EW_THREADS + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * EW_THREADS) {
    float yv[4], xv[4];
    Vec4<float>::load(y + i * 4, yv);
    if (a != 0.f) Vec4<TX>::load(x + i * 4, xv);
#pragma unroll
    for (int k = 0; k < 4; ++k) yv[k] = (a != 0.f ? a * xv[k] : 0.f) + b * yv[k];
    Vec4<float>::store(y + i * 4, yv);
  }
  for (int64_t i = nvec * 4 + blockIdx.x * (int64_t)EW_THREADS + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * EW_THREADS)
    y[i] = (a != 0.f ? a * ld<TX>(x, i) : 0.f) + b * y[i];
}

constexpr int MAX_NBRS = 16;
struct MixArgs {
  const void* p[MAX_NBRS];
  int dt[MAX_NBRS];
  float w[MAX_NBRS];
};

__global__ __launch_bounds__(EW_THREADS) void mix_kernel(float* __restrict__ master, MixArgs args,
                                                        int nn, float self_w,
                                                        bf16_t* __restrict__ pout_bf,
                                                        float* __restrict__ pout_f, int64_t n) {
  const int64_t nvec = n / 4;  // n is a multiple of 64 (flat buffers are padded)
  for (int64_t i = blockIdx.x * (int64_t)EW_THREADS + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * EW_THREADS) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (self_w != 0.f) {  // self_w = 0: master is overwritten, never read (formed sums, d_c)
      Vec4<float>::load(master + i * 4, acc);
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] *= self_w;
    }
    for (int j = 0; j < nn; ++j) {
      float v[4];
      if (args.dt[j] == DT_BF16) Vec4<bf16_t>::load((const bf16_t*)args.p[j] + i * 4, v);
      else Vec4<float>::load((const float*)args.p[j] + i * 4, v);
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += args.w[j] * v[k];
    }
    Vec4<float>::store(master + i * 4, acc);
    if (pout_bf) Vec4<bf16_t>::store(pout_bf + i * 4, acc);
    if (pout_f) Vec4<float>::store(pout_f + i * 4, acc);
  }
}

// Round end of one client under round-complete delta gossip (bcfl/parallel/gossip.py publish),
// one pass instead of five (u, S, the two wire casts, the own-progress retraction) plus the
// client's new SCAFFOLD control variate (fl/drift.py after_train, deferred to here):
//   u = y - x;  S += u;  wire[:n] = S;  [c = (x - y) / L - s d;  cv = c;  wire[n:] = c]
//   y <- x;  param <- x            (the client's own progress waits for its round to complete:
//                                   the model IS its round-start record again, bit for bit)
// Every term is rounded as the separate kernels rounded it (axpby / mix order of operations).
template <typename TW>
__global__ __launch_bounds__(EW_THREADS) void delta_round_end_kernel(
    float* __restrict__ y, const float* __restrict__ x, float* __restrict__ cum,
    const float* __restrict__ d, float* __restrict__ cv, TW* __restrict__ wire_m,
    TW* __restrict__ wire_a, bf16_t* __restrict__ pout_bf, float* __restrict__ pout_f,
    float inv_l, float s, int64_t n) {
  const int64_t nvec = n / 4;  // n is a multiple of 64 (flat buffers are padded)
  for (int64_t i = blockIdx.x * (int64_t)EW_THREADS + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * EW_THREADS) {
    float yv[4], xv[4], sv[4], dv[4] = {0.f, 0.f, 0.f, 0.f}, u[4], c[4];
    Vec4<float>::load(y + i * 4, yv);
    Vec4<float>::load(x + i * 4, xv);
    Vec4<float>::load(cum + i * 4, sv);
    if (d) Vec4<float>::load(d + i * 4, dv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      u[k] = yv[k] - xv[k];
      sv[k] = u[k] + sv[k];
      c[k] = inv_l * xv[k];
      c[k] = c[k] + (-inv_l) * yv[k];
      if (d) c[k] = (-s) * dv[k] + c[k];
    }
    Vec4<float>::store(cum + i * 4, sv);
    Vec4<TW>::store(wire_m + i * 4, sv);
    if (cv) {
      Vec4<float>::store(cv + i * 4, c);
      Vec4<TW>::store(wire_a + i * 4, c);
    }
    Vec4<float>::store(y + i * 4, xv);
    if (pout_bf) Vec4<bf16_t>::store(pout_bf + i * 4, xv);
    if (pout_f) Vec4<float>::store(pout_f + i * 4, xv);
  }
}

template <typename TO>
__global__ __launch_bounds__(EW_THREADS) void delta_encode_kernel(const float* __restrict__ x,
                                                                 float* __restrict__ ref,
                                                                 TO* __restrict__ out, int64_t n) {
  const int64_t nvec = n / 4;
  for (int64_t i = blockIdx.x * (int64_t)EW_THREADS + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * EW_THREADS) {
    float xv[4], rv[4], q[4];
    Vec4<float>::load(x + i * 4, xv);
    Vec4<float>::load(ref + i * 4, rv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d = xv[k] - rv[k];
      q[k] = sizeof(TO) == 2 ? bf2f(f2bf(d)) : d;
      rv[k] += q[k];
    }
    Vec4<TO>::store(out + i * 4, q);
    Vec4<float>::store(ref + i * 4, rv);
  }
}

template <typename TG>
__global__ __launch_bounds__(EW_THREADS) void adamw_kernel(
    float* __restrict__ master, const TG* __restrict__ grad, float* __restrict__ m,
    float* __restrict__ v, bf16_t* __restrict__ pout_bf, float* __restrict__ pout_f, float b1,
    float b2, float eps, float step_size, float decay_mul, float denom_scale, int hf_mode,
    float grad_scale, int64_t n) {
  const int64_t nvec = n / 4;
  for (int64_t i = blockIdx.x * (int64_t)EW_THREADS + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * EW_THREADS) {
    float p[4], g[4], mm[4], vv[4];
    Vec4<float>::load(master + i * 4, p);
    Vec4<TG>::load(grad + i * 4, g);
    Vec4<float>::load(m + i * 4, mm);
    Vec4<float>::load(v + i * 4, vv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = g[k] * grad_scale;
      mm[k] = b1 * mm[k] + (1.f - b1) * gk;
      vv[k] = b2 * vv[k] + (1.f - b2) * gk * gk;
      if (hf_mode) {
        p[k] -= step_size * mm[k] / (sqrtf(vv[k]) + eps);
        p[k] *= decay_mul;
      } else {
        p[k] *= decay_mul;
        p[k] -= step_size * mm[k] / (sqrtf(vv[k]) * denom_scale + eps);
      }
    }
    Vec4<float>::store(master + i * 4, p);
    Vec4<float>::store(m + i * 4, mm);
    Vec4<float>::store(v + i * 4, vv);
    if (pout_bf) Vec4<bf16_t>::store(pout_bf + i * 4, p);
    if (pout_f) Vec4<float>::store(pout_f + i * 4, p);
  }
}

// Multi-tensor AdamW: gradients are separate tensors (as autograd produced them); master / m / v /
// param are flat. The launch covers up to MT_MAX tensors concatenated (each padded to a multiple
// of 4 elements); block b owns a fixed range of that concatenation and walks the tensor table.
constexpr int MT_MAX = 40;
struct MTArgs {
  const void* g[MT_MAX];
  const void* g2[MT_MAX];  // optional second gradient of the same tensor (micro-batch replica), summed
  int64_t off[MT_MAX];
  int64_t numel[MT_MAX];
  int64_t start[MT_MAX + 1];
  int aligned[MT_MAX];
  int n;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& mm, float& vv, float b1,
                                          float b2, float eps, float step_size, float decay_mul,
                                          float denom_scale, int hf) {
  mm = b1 * mm + (1.f - b1) * g;
  vv = b2 * vv + (1.f - b2) * g * g;
  if (hf) {
    p -= step_size * mm / (sqrtf(vv) + eps);
    p *= decay_mul;
  } else {
    p *= decay_mul;
    p -= step_size * mm / (sqrtf(vv) * denom_scale + eps);
  }
}

template <typename TG>
__global__ __launch_bounds__(EW_THREADS) void adamw_mt_kernel(
    float* __restrict__ master, float* __restrict__ m, float* __restrict__ v,
    bf16_t* __restrict__ pout_bf, float* __restrict__ pout_f, MTArgs a, int64_t chunk, float b1,
    float b2, float eps, float step_size, float decay_mul, float denom_scale, int hf,
    float grad_scale, const float* __restrict__ corr, float corr_lr,
    const float* __restrict__ gscale) {
  // corr (optional): drift-correction direction in update space (SCAFFOLD-style control variate
  // difference c - c_i, bcfl/fl/drift.py); the step becomes p -= lr * (adam_update + corr)
  // gscale (optional, device): global-norm clip coefficient from clip_coef_kernel, multiplied
  // into grad_scale (no host round trip between the norm and the step)
  if (gscale) grad_scale *= gscale[0];
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  int64_t hi = lo + chunk;
  if (hi > a.start[a.n]) hi = a.start[a.n];
  int t = 0;
  while (t + 1 < a.n && a.start[t + 1] <= lo) ++t;
  for (int64_t e = lo + threadIdx.x * 4; e < hi; e += EW_THREADS * 4) {
    while (e >= a.start[t + 1]) ++t;
    const int64_t loc = e - a.start[t];
    const int64_t n = a.numel[t];
    if (loc >= n) continue;
    const TG* g = reinterpret_cast<const TG*>(a.g[t]) + loc;
    const int64_t f = a.off[t] + loc;
    if (loc + 4 <= n && a.aligned[t]) {
      float p[4], gv[4], mm[4], vv[4];
      Vec4<float>::load(master + f, p);
      Vec4<TG>::load(g, gv);
      if (a.g2[t]) {
        float gw[4];
        Vec4<TG>::load(reinterpret_cast<const TG*>(a.g2[t]) + loc, gw);
#pragma unroll
        for (int k = 0; k < 4; ++k) gv[k] += gw[k];
      }
      Vec4<float>::load(m + f, mm);
      Vec4<float>::load(v + f, vv);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        adam_elem(p[k], gv[k] * grad_scale, mm[k], vv[k], b1, b2, eps, step_size, decay_mul,
                  denom_scale, hf);
      if (corr) {
        float cv[4];
        Vec4<float>::load(corr + f, cv);
#pragma unroll
        for (int k = 0; k < 4; ++k) p[k] -= corr_lr * cv[k];
      }
      Vec4<float>::store(master + f, p);
      Vec4<float>::store(m + f, mm);
      Vec4<float>::store(v + f, vv);
      if (pout_bf) Vec4<bf16_t>::store(pout_bf + f, p);
      if (pout_f) Vec4<float>::store(pout_f + f, p);
    } else {
      for (int k = 0; k < 4 && loc + k < n; ++k) {
        float p = master[f + k], mm = m[f + k], vv = v[f + k];
        float gk = ld<TG>(g, k);
        if (a.g2[t]) gk += ld<TG>(reinterpret_cast<const TG*>(a.g2[t]) + loc, k);
        adam_elem(p, gk * grad_scale, mm, vv, b1, b2, eps, step_size, decay_mul, denom_scale, hf);
        if (corr) p -= corr_lr * corr[f + k];
        master[f + k] = p;
        m[f + k] = mm;
        v[f + k] = vv;
        if (pout_bf) pout_bf[f + k] = f2bf(p);
        if (pout_f) pout_f[f + k] = p;
      }
    }
  }
}

// Global gradient norm for clipping: per-block partial sums of squares over the same
// multi-tensor table as adamw_mt_kernel (g + g2 when a micro-batch replica is attached), then ONE
// block reduces the partials in a fixed order (deterministic) into [coef, norm] with
// coef = min(1, max_norm / (norm + 1e-6)) — torch.nn.utils.clip_grad_norm_ semantics.
template <typename TG>
__global__ __launch_bounds__(EW_THREADS) void sumsq_mt_kernel(MTArgs a, int64_t chunk,
                                                               float* __restrict__ partial) {
  __shared__ float red[EW_THREADS / WAVE];
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  int64_t hi = lo + chunk;
  if (hi > a.start[a.n]) hi = a.start[a.n];
  int t = 0;
  while (t + 1 < a.n && a.start[t + 1] <= lo) ++t;
  float acc = 0.f;
  for (int64_t e = lo + threadIdx.x * 4; e < hi; e += EW_THREADS * 4) {
    while (e >= a.start[t + 1]) ++t;
    const int64_t loc = e - a.start[t];
    const int64_t n = a.numel[t];
    if (loc >= n) continue;
    const TG* g = reinterpret_cast<const TG*>(a.g[t]) + loc;
    if (loc + 4 <= n && a.aligned[t]) {
      float gv[4];
      Vec4<TG>::load(g, gv);
      if (a.g2[t]) {
        float gw[4];
        Vec4<TG>::load(reinterpret_cast<const TG*>(a.g2[t]) + loc, gw);
#pragma unroll
        for (int k = 0; k < 4; ++k) gv[k] += gw[k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) acc += gv[k] * gv[k];
    } else {
      for (int k = 0; k < 4 && loc + k < n; ++k) {
        float gk = ld<TG>(g, k);
        if (a.g2[t]) gk += ld<TG>(reinterpret_cast<const TG*>(a.g2[t]) + loc, k);
        acc += gk * gk;
      }
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = 0.f;
    for (int w = 0; w < EW_THREADS / WAVE; ++w) b += red[w];
    partial[blockIdx.x] = b;
  }
}

__global__ __launch_bounds__(EW_THREADS) void clip_coef_kernel(const float* __restrict__ partial,
                                                                int n, float max_norm,
                                                                float* __restrict__ out) {
  __shared__ float red[EW_THREADS / WAVE];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += EW_THREADS) acc += partial[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < EW_THREADS / WAVE; ++w) s += red[w];
    const float norm = sqrtf(s);
    const float c = max_norm / (norm + 1e-6f);
    out[0] = c < 1.f ? c : 1.f;
    out[1] = norm;
  }
}

template <typename TX>
__global__ __launch_bounds__(EW_THREADS) void block_sketch_kernel(const TX* __restrict__ x,
                                                                 int64_t n, int64_t blk,
                                                                 uint32_t ka, uint32_t kb,
                                                                 float* __restrict__ out) {
  __shared__ float red[EW_THREADS / WAVE];
  const int64_t lo = (int64_t)blockIdx.x * blk;
  const int64_t hi = lo + blk < n ? lo + blk : n;
  float a = 0.f;
  for (int64_t i = lo + threadIdx.x; i < hi; i += EW_THREADS) {
    const uint32_t h = hash32((uint32_t)i, ka, kb);
    const float s = (h & 1u) ? 1.f : -1.f;
    a += s * ld<TX>(x, i);
  }
  a = wave_sum(a);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < EW_THREADS / WAVE; ++w) t += red[w];
    out[blockIdx.x] = t;
  }
}

// update statistics of the anomaly filter, measured by the RECEIVER on what it is about to apply:
// the signed block sketch of d = a - b (a = a source's newest cumulative update, b = the one
// already applied) in out[0, dim) and the per-block sum of d^2 in out[dim, 2 dim) — one read of
// each operand, no materialised difference
template <typename T>
__global__ __launch_bounds__(EW_THREADS) void update_stats_kernel(const T* __restrict__ a,
                                                                  const T* __restrict__ b,
                                                                  int64_t n, int64_t blk,
                                                                  uint32_t ka, uint32_t kb,
                                                                  float* __restrict__ out) {
  __shared__ float red[2][EW_THREADS / WAVE];
  const int64_t lo = (int64_t)blockIdx.x * blk;
  const int64_t hi = lo + blk < n ? lo + blk : n;
  float sk = 0.f, sq = 0.f;
  for (int64_t i = lo + threadIdx.x; i < hi; i += EW_THREADS) {
    const float d = ld<T>(a, i) - ld<T>(b, i);
    const uint32_t h = hash32((uint32_t)i, ka, kb);
    sk += (h & 1u) ? d : -d;
    sq += d * d;
  }
  sk = wave_sum(sk);
  sq = wave_sum(sq);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = sk;
    red[1][threadIdx.x >> 6] = sq;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f, q = 0.f;
    for (int w = 0; w < EW_THREADS / WAVE; ++w) {
      t += red[0][w];
      q += red[1][w];
    }
    out[blockIdx.x] = t;
    out[gridDim.x + blockIdx.x] = q;
  }
}

// dropout multiplier m[i] = keep(i) / (1 - p) or 0 (bcfl/ops/rng.py element layout): the pooled
// [B, H] head dropout applies it with one multiply forward and one backward
template <typename T>
__global__ __launch_bounds__(EW_THREADS) void drop_mask_kernel(T* __restrict__ m, int64_t n,
                                                               uint32_t p8, uint32_t ka,
                                                               uint32_t kb, float scale) {
  for (int64_t i4 = blockIdx.x * (int64_t)EW_THREADS + threadIdx.x; i4 * 4 < n;
       i4 += (int64_t)gridDim.x * EW_THREADS) {
    const uint32_t h = hash32((uint32_t)i4, ka, kb);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t i = i4 * 4 + e;
      if (i < n) m[i] = (T)(((h >> (8 * e)) & 0xffu) >= p8 ? scale : 0.f);
    }
  }
}

}  // namespace

int launch_drop_mask(void* m, int dt, int64_t n, uint32_t p8, uint32_t ka, uint32_t kb,
                     hipStream_t s) {
  if (n <= 0) return 0;
  const float scale = 256.0f / (256.0f - (float)p8);  // host copy of keep_scale()
  if (dt == DT_BF16)
    hipLaunchKernelGGL(drop_mask_kernel<__bf16>, dim3(ew_grid((n + 3) / 4)), dim3(EW_THREADS), 0, s,
                       (__bf16*)m, n, p8, ka, kb, scale);
  else
    hipLaunchKernelGGL(drop_mask_kernel<float>, dim3(ew_grid((n + 3) / 4)), dim3(EW_THREADS), 0, s,
                       (float*)m, n, p8, ka, kb, scale);
  return 0;
}

int launch_bias_act_fwd(const void* y, const void* bias, void* out, int64_t rows, int N, int act,
                        int dt, hipStream_t s) {
  if (N % 8) return -2;
  dim3 grid((N + COLS_PER_BLOCK - 1) / COLS_PER_BLOCK, (unsigned)(rows < 8192 ? rows : 8192));
  if (rows == 0) return 0;
  if (dt == DT_BF16)
    hipLaunchKernelGGL(bias_act_fwd_kernel<bf16_t>, grid, dim3(EW_THREADS), 0, s,
                       (const bf16_t*)y, (const bf16_t*)bias, (bf16_t*)out, rows, N, act);
  else
    hipLaunchKernelGGL(bias_act_fwd_kernel<float>, grid, dim3(EW_THREADS), 0, s,
                       (const float*)y, (const float*)bias, (float*)out, rows, N, act);
  return 0;
}

int launch_bias_act_bwd(const void* dout, const void* y, const void* bias, void* dy,
                        float* partial, int nblk_rows, int64_t rows, int N, int act, int dt,
                        hipStream_t s) {
  if (N % 8) return -2;
  dim3 grid((N + COLS_PER_BLOCK - 1) / COLS_PER_BLOCK, nblk_rows);
  if (dt == DT_BF16)
    hipLaunchKernelGGL(bias_act_bwd_kernel<bf16_t>, grid, dim3(EW_THREADS), 0, s,
                       (const bf16_t*)dout, (const bf16_t*)y, (const bf16_t*)bias, (bf16_t*)dy,
                       partial, rows, N, act);
  else
    hipLaunchKernelGGL(bias_act_bwd_kernel<float>, grid, dim3(EW_THREADS), 0, s,
                       (const float*)dout, (const float*)y, (const float*)bias, (float*)dy,
                       partial, rows, N, act);
  return 0;
}

int launch_swiglu_fwd(const void* gu, void* out, int64_t rows, int I, int dt, hipStream_t s) {
  if (I % 8) return -2;
  if (rows == 0) return 0;
  dim3 grid((I + COLS_PER_BLOCK - 1) / COLS_PER_BLOCK, (unsigned)(rows < 8192 ? rows : 8192));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(swiglu_fwd_kernel<bf16_t>, grid, dim3(EW_THREADS), 0, s,
                       (const bf16_t*)gu, (bf16_t*)out, rows, I);
  else
    hipLaunchKernelGGL(swiglu_fwd_kernel<float>, grid, dim3(EW_THREADS), 0, s,
                       (const float*)gu, (float*)out, rows, I);
  return 0;
}

int launch_swiglu_bwd(const void* dout, const void* gu, void* dgu, int64_t rows, int I, int dt,
                      hipStream_t s) {
  if (I % 8) return -2;
  if (rows == 0) return 0;
  dim3 grid((I + COLS_PER_BLOCK - 1) / COLS_PER_BLOCK, (unsigned)(rows < 8192 ? rows : 8192));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(swiglu_bwd_kernel<bf16_t>, grid, dim3(EW_THREADS), 0, s,
                       (const bf16_t*)dout, (const bf16_t*)gu, (bf16_t*)dgu, rows, I);
  else
    hipLaunchKernelGGL(swiglu_bwd_kernel<float>, grid, dim3(EW_THREADS), 0, s,
                       (const float*)dout, (const float*)gu, (float*)dgu, rows, I);
  return 0;
}

int launch_rope(const void* x, void* out, const int* pos, const float* cos, const float* sin,
                int64_t rows, int row_stride, int nrot, int d, int inverse, int dt, hipStream_t s) {
  if (row_stride % 2 || d % 2 || nrot * d > row_stride) return -2;
  const int64_t total = rows * (row_stride / 2);
  const bool aligned = ((uintptr_t)x % 16 == 0) && ((uintptr_t)out % 16 == 0) &&
                       ((uintptr_t)cos % 16 == 0) && ((uintptr_t)sin % 16 == 0);
  if (dt == DT_BF16 && d % 16 == 0 && row_stride % 8 == 0 && aligned) {
    const int64_t tv = rows * (nrot * (d / 16) + (row_stride - nrot * d) / 8);
    hipLaunchKernelGGL(rope_vec_kernel, dim3(ew_grid(tv)), dim3(EW_THREADS), 0, s,
                       (const bf16_t*)x, (bf16_t*)out, pos, cos, sin, rows, row_stride, nrot, d,
                       inverse);
    return 0;
  }
  if (dt == DT_BF16)
    hipLaunchKernelGGL(rope_kernel<bf16_t>, dim3(ew_grid(total)), dim3(EW_THREADS), 0, s,
                       (const bf16_t*)x, (bf16_t*)out, pos, cos, sin, rows, row_stride, nrot, d, inverse);
  else
    hipLaunchKernelGGL(rope_kernel<float>, dim3(ew_grid(total)), dim3(EW_THREADS), 0, s,
                       (const float*)x, (float*)out, pos, cos, sin, rows, row_stride, nrot, d, inverse);
  return 0;
}

int launch_cast_copy(void* dst, int dst_dt, const void* src, int src_dt, int64_t n, hipStream_t s) {
  const int g = ew_grid(n / 4 + 1);
  if (dst_dt == DT_BF16 && src_dt == DT_F32)
    hipLaunchKernelGGL((cast_kernel<bf16_t, float>), dim3(g), dim3(EW_THREADS), 0, s, (bf16_t*)dst, (const float*)src, n);
  else if (dst_dt == DT_F32 && src_dt == DT_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16_t>), dim3(g), dim3(EW_THREADS), 0, s, (float*)dst, (const bf16_t*)src, n);
  else if (dst_dt == DT_F32 && src_dt == DT_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), dim3(g), dim3(EW_THREADS), 0, s, (float*)dst, (const float*)src, n);
  else
    hipLaunchKernelGGL((cast_kernel<bf16_t, bf16_t>), dim3(g), dim3(EW_THREADS), 0, s, (bf16_t*)dst, (const bf16_t*)src, n);
  return 0;
}

int launch_axpby(float* y, const void* x, int x_dt, float a, float b, int64_t n, hipStream_t s) {
  const int g = ew_grid(n / 4 + 1);
  if (x_dt == DT_BF16)
    hipLaunchKernelGGL(axpby_kernel<bf16_t>, dim3(g), dim3(EW_THREADS), 0, s, y, (const bf16_t*)x, a, b, n);
  else
    hipLaunchKernelGGL(axpby_kernel<float>, dim3(g), dim3(EW_THREADS), 0, s, y, (const float*)x, a, b, n);
  return 0;
}

int launch_mix(float* master, const void* const* nbrs, const int* nbr_dt, const float* w, int nn,
               float self_w, void* param_out, int param_dt, int64_t n, hipStream_t s) {
  if (n % 4) return -2;
  if (nn > MAX_NBRS) {  // fold in chunks of MAX_NBRS
    int r = launch_mix(master, nbrs, nbr_dt, w, MAX_NBRS, self_w, nullptr, param_dt, n, s);
    if (r) return r;
    return launch_mix(master, nbrs + MAX_NBRS, nbr_dt + MAX_NBRS, w + MAX_NBRS, nn - MAX_NBRS,
                      1.f, param_out, param_dt, n, s);
  }
  MixArgs a;
  for (int j = 0; j < nn; ++j) { a.p[j] = nbrs[j]; a.dt[j] = nbr_dt[j]; a.w[j] = w[j]; }
  hipLaunchKernelGGL(mix_kernel, dim3(ew_grid(n / 4)), dim3(EW_THREADS), 0, s, master, a, nn,
                     self_w, param_dt == DT_BF16 ? (bf16_t*)param_out : nullptr,
                     param_dt == DT_F32 ? (float*)param_out : nullptr, n);
  return 0;
}

int launch_delta_round_end(float* y, const float* x, float* cum, const float* d, float* cv,
                           void* wire, int wire_dt, void* param_out, int param_dt, float inv_l,
                           float scale, int64_t n, hipStream_t s) {
  if (n % 4) return -2;
  bf16_t* pb = param_dt == DT_BF16 ? (bf16_t*)param_out : nullptr;
  float* pf = param_dt == DT_F32 ? (float*)param_out : nullptr;
  if (wire_dt == DT_BF16)
    hipLaunchKernelGGL(delta_round_end_kernel<bf16_t>, dim3(ew_grid(n / 4)), dim3(EW_THREADS), 0, s,
                       y, x, cum, d, cv, (bf16_t*)wire, cv ? (bf16_t*)wire + n : nullptr, pb, pf,
                       inv_l, scale, n);
  else if (wire_dt == DT_F32)
    hipLaunchKernelGGL(delta_round_end_kernel<float>, dim3(ew_grid(n / 4)), dim3(EW_THREADS), 0, s,
                       y, x, cum, d, cv, (float*)wire, cv ? (float*)wire + n : nullptr, pb, pf,
                       inv_l, scale, n);
  else
    return -3;
  return 0;
}

int launch_delta_encode(const float* x, float* ref, void* out, int out_dt, int64_t n, hipStream_t s) {
  if (n % 4) return -2;
  if (out_dt == DT_BF16)
    hipLaunchKernelGGL(delta_encode_kernel<bf16_t>, dim3(ew_grid(n / 4)), dim3(EW_THREADS), 0, s, x, ref, (bf16_t*)out, n);
  else
    hipLaunchKernelGGL(delta_encode_kernel<float>, dim3(ew_grid(n / 4)), dim3(EW_THREADS), 0, s, x, ref, (float*)out, n);
  return 0;
}

int launch_adamw(float* master, const void* grad, int grad_dt, float* m, float* v,
                 void* param_out, int param_dt, float lr, float b1, float b2, float eps, float wd,
                 int step, int mode, float grad_scale, int64_t n, hipStream_t s) {
  if (n % 4) return -2;
  const double bc1 = 1.0 - __builtin_pow((double)b1, step);
  const double bc2 = 1.0 - __builtin_pow((double)b2, step);
  float step_size, decay_mul, denom_scale = 1.f;
  const int hf = mode == 0;
  if (hf) {
    step_size = (float)(lr * __builtin_sqrt(bc2) / bc1);
    decay_mul = 1.f - lr * wd;
  } else {
    step_size = (float)(lr / bc1);
    decay_mul = 1.f - lr * wd;
    denom_scale = (float)(1.0 / __builtin_sqrt(bc2));
  }
  bf16_t* pb = param_dt == DT_BF16 ? (bf16_t*)param_out : nullptr;
  float* pf = param_dt == DT_F32 ? (float*)param_out : nullptr;
  if (grad_dt == DT_BF16)
    hipLaunchKernelGGL(adamw_kernel<bf16_t>, dim3(ew_grid(n / 4)), dim3(EW_THREADS), 0, s, master,
                       (const bf16_t*)grad, m, v, pb, pf, b1, b2, eps, step_size, decay_mul,
                       denom_scale, hf, grad_scale, n);
  else
    hipLaunchKernelGGL(adamw_kernel<float>, dim3(ew_grid(n / 4)), dim3(EW_THREADS), 0, s, master,
                       (const float*)grad, m, v, pb, pf, b1, b2, eps, step_size, decay_mul,
                       denom_scale, hf, grad_scale, n);
  return 0;
}

int launch_adamw_mt(float* master, float* m, float* v, void* param_out, int param_dt,
                    const void* const* grads, const int64_t* offs, const int64_t* numels,
                    int ntens, int grad_dt, float lr, float b1, float b2, float eps, float wd,
                    int step, int mode, float grad_scale, const float* corr, float corr_lr,
                    hipStream_t s, const void* const* grads2, const float* gscale) {
  const double bc1 = 1.0 - __builtin_pow((double)b1, step);
  const double bc2 = 1.0 - __builtin_pow((double)b2, step);
  const int hf = mode == 0;
  const float step_size = hf ? (float)(lr * __builtin_sqrt(bc2) / bc1) : (float)(lr / bc1);
  const float decay_mul = 1.f - lr * wd;
  const float denom_scale = hf ? 1.f : (float)(1.0 / __builtin_sqrt(bc2));
  bf16_t* pb = param_dt == DT_BF16 ? (bf16_t*)param_out : nullptr;
  float* pf = param_dt == DT_F32 ? (float*)param_out : nullptr;
  const int esz = grad_dt == DT_BF16 ? 2 : 4;
  constexpr int64_t CHUNK = 8192;
  for (int g0 = 0; g0 < ntens; g0 += MT_MAX) {
    MTArgs a{};
    a.n = ntens - g0 < MT_MAX ? ntens - g0 : MT_MAX;
    a.start[0] = 0;
    for (int i = 0; i < a.n; ++i) {
      a.g[i] = grads[g0 + i];
      a.g2[i] = grads2 ? grads2[g0 + i] : nullptr;
      a.off[i] = offs[g0 + i];
      a.numel[i] = numels[g0 + i];
      a.start[i + 1] = a.start[i] + (numels[g0 + i] + 3) / 4 * 4;
      a.aligned[i] = (((uintptr_t)grads[g0 + i]) % (4 * esz) == 0) && (offs[g0 + i] % 4 == 0) &&
                     (((uintptr_t)a.g2[i]) % (4 * esz) == 0);
    }
    const int64_t total = a.start[a.n];
    if (total == 0) continue;
    const unsigned grid = (unsigned)((total + CHUNK - 1) / CHUNK);
    if (grad_dt == DT_BF16)
      hipLaunchKernelGGL(adamw_mt_kernel<bf16_t>, dim3(grid), dim3(EW_THREADS), 0, s, master, m, v,
                         pb, pf, a, CHUNK, b1, b2, eps, step_size, decay_mul, denom_scale, hf,
                         grad_scale, corr, corr_lr, gscale);
    else
      hipLaunchKernelGGL(adamw_mt_kernel<float>, dim3(grid), dim3(EW_THREADS), 0, s, master, m, v,
                         pb, pf, a, CHUNK, b1, b2, eps, step_size, decay_mul, denom_scale, hf,
                         grad_scale, corr, corr_lr, gscale);
  }
  return 0;
}

static constexpr int64_t kSumsqChunk = 16384;

int64_t sumsq_mt_blocks(const int64_t* numels, int ntens) {
  int64_t blocks = 0;
  for (int g0 = 0; g0 < ntens; g0 += MT_MAX) {
    const int n = ntens - g0 < MT_MAX ? ntens - g0 : MT_MAX;
    int64_t total = 0;
    for (int i = 0; i < n; ++i) total += (numels[g0 + i] + 3) / 4 * 4;
    blocks += (total + kSumsqChunk - 1) / kSumsqChunk;
  }
  return blocks;
}

int launch_clip_coef_mt(const void* const* grads, const void* const* grads2, const int64_t* numels,
                        int ntens, int grad_dt, float* partial, float max_norm, float* out,
                        hipStream_t s) {
  const int esz = grad_dt == DT_BF16 ? 2 : 4;
  int64_t base = 0;
  for (int g0 = 0; g0 < ntens; g0 += MT_MAX) {
    MTArgs a{};
    a.n = ntens - g0 < MT_MAX ? ntens - g0 : MT_MAX;
    a.start[0] = 0;
    for (int i = 0; i < a.n; ++i) {
      a.g[i] = grads[g0 + i];
      a.g2[i] = grads2 ? grads2[g0 + i] : nullptr;
      a.off[i] = 0;
      a.numel[i] = numels[g0 + i];
      a.start[i + 1] = a.start[i] + (numels[g0 + i] + 3) / 4 * 4;
      a.aligned[i] = (((uintptr_t)grads[g0 + i]) % (4 * esz) == 0) &&
                     (((uintptr_t)a.g2[i]) % (4 * esz) == 0);
    }
    const int64_t total = a.start[a.n];
    const unsigned grid = (unsigned)((total + kSumsqChunk - 1) / kSumsqChunk);
    if (grid == 0) continue;
    if (grad_dt == DT_BF16)
      hipLaunchKernelGGL(sumsq_mt_kernel<bf16_t>, dim3(grid), dim3(EW_THREADS), 0, s, a,
                         kSumsqChunk, partial + base);
    else
      hipLaunchKernelGGL(sumsq_mt_kernel<float>, dim3(grid), dim3(EW_THREADS), 0, s, a,
                         kSumsqChunk, partial + base);
    base += grid;
  }
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(EW_THREADS), 0, s, partial, (int)base,
                     max_norm, out);
  return 0;
}

int launch_block_sketch(const void* x, int x_dt, int64_t n, int dim, uint32_t ka, uint32_t kb,
                        float* out, hipStream_t s) {
  const int64_t blk = (n + dim - 1) / dim;
  if (x_dt == DT_BF16)
    hipLaunchKernelGGL(block_sketch_kernel<bf16_t>, dim3(dim), dim3(EW_THREADS), 0, s, (const bf16_t*)x, n, blk, ka, kb, out);
  else
    hipLaunchKernelGGL(block_sketch_kernel<float>, dim3(dim), dim3(EW_THREADS), 0, s, (const float*)x, n, blk, ka, kb, out);
  return 0;
}

int launch_update_stats(const void* a, const void* b, int dt, int64_t n, int dim, uint32_t ka,
                        uint32_t kb, float* out, hipStream_t s) {
  const int64_t blk = (n + dim - 1) / dim;
  if (dt == DT_BF16)
    hipLaunchKernelGGL(update_stats_kernel<bf16_t>, dim3(dim), dim3(EW_THREADS), 0, s,
                       (const bf16_t*)a, (const bf16_t*)b, n, blk, ka, kb, out);
  else
    hipLaunchKernelGGL(update_stats_kernel<float>, dim3(dim), dim3(EW_THREADS), 0, s,
                       (const float*)a, (const float*)b, n, blk, ka, kb, out);
  return 0;
}

}  // namespace bcfl
