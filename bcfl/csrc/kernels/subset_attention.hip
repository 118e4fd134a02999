// Pooled-row ("query subset") attention, forward + backward: ONE query row per sequence (the [CLS]
// row of BERT / ALBERT / DistilBERT, the last token of Llama) against all keys of its sequence.
//
// Why: a sequence classifier only reads one row of the last encoder layer (reference
// BertForSequenceClassification pooler), so that layer's attention, output
// projection, FFN and LayerNorms run on B rows instead of T (bcfl/models/*: pooled_rows_only).
// Its attention is B x S_max scores — far too small for the MFMA flash kernels — and as eager torch
// it was ~60 small kernels per step (gathers, einsums, softmax, a 15-op hash chain, their
// autograd) = the largest block of eager launches in the bench. Here: one workgroup per
// (sequence, kv head), 4 waves; lane = head-dim element (d = 64: one per lane; d = 128: two),
// keys split across the waves; scores / probabilities live in LDS (<= 8192 keys).
//
// Same math as bcfl/ops/functional.py::query_subset_attention and as the varlen flash kernels
// restricted to those queries, INCLUDING the dropout keep bits (element index
// (t * nh + h) * 8192 + key, one hash per 4 elements), so logits and gradients equal the full-layer
// computation. Backward: dk / dv rows are owned by exactly one thread across the query heads of a
// GQA group (read-modify-write, no atomics: deterministic); dq goes to the pooled row only; the
// caller zero-fills dqkv.
#include "common.h"
#include "kernels.h"

namespace bcfl {
namespace {

constexpr int SA_THREADS = 256;
constexpr int SA_WAVES = SA_THREADS / WAVE;
constexpr int SA_MAXK = 6144;  // keys per sequence (2 fp32 LDS rows of this size in the backward)
constexpr int SA_DROP_STRIDE = 8192;

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  v = is_max ? wave_max(v) : wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int i = 1; i < SA_WAVES; ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
  return r;
}

__device__ __forceinline__ bool sa_keep(uint32_t e, uint32_t p8, uint32_t ka, uint32_t kb) {
  return keep_elem(e, p8, ka, kb);
}

// q . row (bf16, HD = 32 / 64 / 128): lane owns elements lane (+64); full sum in every lane
template <int HD>
__device__ __forceinline__ float dot_row(const float (&q)[(HD + 63) / 64], const bf16_t* row, int lane) {
  float a = 0.f;
#pragma unroll
  for (int c = 0; c < (HD + 63) / 64; ++c) {
    const int d = lane + 64 * c;
    if (d < HD) a += q[c] * bf2f(row[d]);
  }
  return wave_sum(a);
}

// thread-per-key dot product: q (fp32, LDS broadcast) . row[0:HD] (bf16, 16-byte loads)
template <int HD>
__device__ __forceinline__ float dot_q_row(const float* __restrict__ qs, const bf16_t* row) {
  float a = 0.f;
#pragma unroll
  for (int c = 0; c < HD; c += 8) {
    float v[8];
    Vec8<bf16_t>::load(row + c, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) a += qs[c + e] * v[e];
  }
  return a;
}

template <int HD>
__global__ __launch_bounds__(SA_THREADS) void subset_attn_fwd_kernel(SubsetAttnParams p) {
  constexpr int NC = (HD + 63) / 64;
  __shared__ float sc[SA_MAXK];
  __shared__ float red[SA_WAVES];
  __shared__ float opart[SA_WAVES][HD];
  __shared__ float qs[HD];
  const int b = blockIdx.x, hk = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int start = p.cu[b];
  const int qrow = p.rows[b];
  // keys of the sequence (causal: up to and including the pooled row itself)
  const int L = p.causal ? qrow - start + 1 : p.cu[b + 1] - start;
  const int grp = p.nh / p.nkv;
  const int rs = (p.nh + 2 * p.nkv) * HD;
  const bf16_t* qkv = reinterpret_cast<const bf16_t*>(p.qkv);
  const bf16_t* kbase = qkv + (size_t)start * rs + p.nh * HD + hk * HD;
  const bf16_t* vbase = qkv + (size_t)start * rs + (p.nh + p.nkv) * HD + hk * HD;
  const float sdrop = p.p8 ? keep_scale(p.p8) : 1.f;
  for (int g = 0; g < grp; ++g) {
    const int h = hk * grp + g;
    for (int d = threadIdx.x; d < HD; d += SA_THREADS)
      qs[d] = bf2f(qkv[(size_t)qrow * rs + h * HD + d]) * p.scale;
    __syncthreads();
    float mx = -INFINITY;
    for (int j = threadIdx.x; j < L; j += SA_THREADS) {  // one key per thread
      const float s = dot_q_row<HD>(qs, kbase + (size_t)j * rs);
      sc[j] = s;
      mx = fmaxf(mx, s);
    }
    mx = block_reduce(mx, red, true);
    float sum = 0.f;
    for (int j = threadIdx.x; j < L; j += SA_THREADS) {
      const float e = __expf(sc[j] - mx);
      sc[j] = e;
      sum += e;
    }
    sum = block_reduce(sum, red, false);
    const float inv = 1.f / sum;
    const uint32_t erow = (uint32_t)(qrow * p.nh + h) * (uint32_t)SA_DROP_STRIDE;
    for (int j = threadIdx.x; j < L; j += SA_THREADS) {
      float pj = sc[j] * inv;
      if (p.p8) pj = sa_keep(erow + (uint32_t)j, p.p8, p.ka, p.kb) ? pj * sdrop : 0.f;
      sc[j] = pj;
    }
    __syncthreads();
    float o[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) o[c] = 0.f;
    for (int j = w; j < L; j += SA_WAVES) {
      const float pj = sc[j];
      const bf16_t* vr = vbase + (size_t)j * rs;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int d = lane + 64 * c;
        if (d < HD) o[c] += pj * bf2f(vr[d]);
      }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int d = lane + 64 * c;
      if (d < HD) opart[w][d] = o[c];
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int d = lane + 64 * c;
        if (d < HD) {
          float a = 0.f;
#pragma unroll
          for (int i = 0; i < SA_WAVES; ++i) a += opart[i][d];
          reinterpret_cast<bf16_t*>(p.out)[(size_t)b * p.nh * HD + h * HD + d] = f2bf(a);
        }
      }
      if (lane == 0) p.lse[(size_t)b * p.nh + h] = mx + logf(sum);
    }
    __syncthreads();
  }
}

template <int HD>
__global__ __launch_bounds__(SA_THREADS) void subset_attn_bwd_kernel(SubsetAttnBwdParams p) {
  constexpr int NC = (HD + 63) / 64;
  __shared__ float pr[SA_MAXK];   // P_j (softmax, before dropout)
  __shared__ float dpr[SA_MAXK];  // dP_j = keep_j c (dO . v_j)
  __shared__ float red[SA_WAVES];
  __shared__ float qpart[SA_WAVES][HD];
  __shared__ float qs[HD], dos[HD];
  const int b = blockIdx.x, hk = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int start = p.cu[b];
  const int qrow = p.rows[b];
  const int L = p.causal ? qrow - start + 1 : p.cu[b + 1] - start;
  const int grp = p.nh / p.nkv;
  const int rs = (p.nh + 2 * p.nkv) * HD;
  const bf16_t* qkv = reinterpret_cast<const bf16_t*>(p.qkv);
  bf16_t* dqkv = reinterpret_cast<bf16_t*>(p.dqkv);
  const int koff = p.nh * HD + hk * HD, voff = (p.nh + p.nkv) * HD + hk * HD;
  const float sdrop = p.p8 ? keep_scale(p.p8) : 1.f;
  for (int g = 0; g < grp; ++g) {
    const int h = hk * grp + g;
    float q[NC], dob[NC];
    float delta_part = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int d = lane + 64 * c;
      const bool in = d < HD;
      q[c] = in ? bf2f(qkv[(size_t)qrow * rs + h * HD + d]) * p.scale : 0.f;
      dob[c] = in ? bf2f(reinterpret_cast<const bf16_t*>(p.dout)[(size_t)b * p.nh * HD + h * HD + d]) : 0.f;
      const float ov = in ? bf2f(reinterpret_cast<const bf16_t*>(p.out)[(size_t)b * p.nh * HD + h * HD + d]) : 0.f;
      delta_part += dob[c] * ov;
    }
    const float delta = wave_sum(delta_part);  // dO . O = sum_j P_j dP_j (every wave has it)
    const float lse = p.lse[(size_t)b * p.nh + h];
    const uint32_t erow = (uint32_t)(qrow * p.nh + h) * (uint32_t)SA_DROP_STRIDE;
    if (w == 0) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int d = lane + 64 * c;
        if (d < HD) { qs[d] = q[c]; dos[d] = dob[c]; }
      }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < L; j += SA_THREADS) {  // one key per thread: s_j and dO . v_j
      const bf16_t* row = qkv + (size_t)(start + j) * rs;
      const float s = dot_q_row<HD>(qs, row + koff);
      const float dpv = dot_q_row<HD>(dos, row + voff);
      const bool keep = !p.p8 || sa_keep(erow + (uint32_t)j, p.p8, p.ka, p.kb);
      pr[j] = __expf(s - lse);
      dpr[j] = keep ? dpv * sdrop : 0.f;
    }
    __syncthreads();
    float dq[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) dq[c] = 0.f;
    for (int j = w; j < L; j += SA_WAVES) {
      const float pj = pr[j], dpj = dpr[j];
      const float ds = pj * (dpj - delta);                       // dL/ds_j (s = scale q.k)
      const bf16_t* row = qkv + (size_t)(start + j) * rs;
      bf16_t* drow = dqkv + (size_t)(start + j) * rs;
      const bool kept = !p.p8 || sa_keep(erow + (uint32_t)j, p.p8, p.ka, p.kb);
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int d = lane + 64 * c;
        if (d < HD) {
          dq[c] += ds * bf2f(row[koff + d]);
          float dk = ds * q[c];                                   // q already scaled
          float dv = kept ? pj * sdrop * dob[c] : 0.f;
          if (g > 0) {                                            // GQA: this thread owns the row
            dk += bf2f(drow[koff + d]);
            dv += bf2f(drow[voff + d]);
          }
          drow[koff + d] = f2bf(dk);
          drow[voff + d] = f2bf(dv);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int d = lane + 64 * c;
      if (d < HD) qpart[w][d] = dq[c];
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int d = lane + 64 * c;
        if (d < HD) {
          float a = 0.f;
#pragma unroll
          for (int i = 0; i < SA_WAVES; ++i) a += qpart[i][d];
          dqkv[(size_t)qrow * rs + h * HD + d] = f2bf(a * p.scale);
        }
      }
    }
    __syncthreads();
  }
}

template <int HD>
void sa_launch(const SubsetAttnParams& p, hipStream_t s) {
  hipLaunchKernelGGL(subset_attn_fwd_kernel<HD>, dim3(p.B, p.nkv), dim3(SA_THREADS), 0, s, p);
}
template <int HD>
void sa_launch_bwd(const SubsetAttnBwdParams& p, hipStream_t s) {
  hipLaunchKernelGGL(subset_attn_bwd_kernel<HD>, dim3(p.B, p.nkv), dim3(SA_THREADS), 0, s, p);
}

}  // namespace

int launch_subset_attn_fwd(const SubsetAttnParams& p, hipStream_t s) {
  if (p.nh % p.nkv || p.max_s > SA_MAXK) return -2;
  if (p.B == 0) return 0;
  switch (p.d) {
    case 32: sa_launch<32>(p, s); break;
    case 64: sa_launch<64>(p, s); break;
    case 128: sa_launch<128>(p, s); break;
    default: return -1;
  }
  return 0;
}

int launch_subset_attn_bwd(const SubsetAttnBwdParams& p, hipStream_t s) {
  if (p.nh % p.nkv || p.max_s > SA_MAXK) return -2;
  if (p.B == 0) return 0;
  switch (p.d) {
    case 32: sa_launch_bwd<32>(p, s); break;
    case 64: sa_launch_bwd<64>(p, s); break;
    case 128: sa_launch_bwd<128>(p, s); break;
    default: return -1;
  }
  return 0;
}

}  // namespace bcfl
