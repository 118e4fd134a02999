// K9: softmax cross-entropy for the classifier head: logits [B, C] (C = 2 /
// 3 / 40 / 41 in the reference scripts), labels [B].
//
//   xent_fwd    mean loss (fp32 scalar) AND the loss gradient (softmax - onehot) / B, in one
//               single-workgroup launch (the backward is then one multiply by dL/dloss)
//   xent_stats  evaluation: adds [correct, count, sum CE, sum CE / B] into a device fp64
//               accumulator (the reference test()'s metrics incl. its sum-of-batch-means loss,
//               src/Servercase/server_IID_IMDB.py:121-135) — one launch per eval batch instead
//               of the cast / argmax / compare / CE / reduce chain.
// One wave per row (lanes over classes), rows strided over the 4 waves, block sums through LDS in
// a fixed order: deterministic.
#include "common.h"
#include "kernels.h"

namespace bcfl {
namespace {

constexpr int XT = 256;
constexpr int XW = XT / WAVE;

template <typename T>
__device__ __forceinline__ void row_stats(const T* __restrict__ lg, int C, int lab, float& lse,
                                          float& xl, int& amax) {
  const int lane = threadIdx.x & 63;
  float mx = -INFINITY;
  int am = 0x7fffffff;
  for (int c = lane; c < C; c += WAVE) {
    const float v = ld<T>(lg, c);
    if (v > mx) { mx = v; am = c; }
  }
  // wave argmax (first index of the max, like torch.argmax)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > mx || (om == mx && oa < am)) { mx = om; am = oa; }
  }
  float s = 0.f;
  for (int c = lane; c < C; c += WAVE) s += __expf(ld<T>(lg, c) - mx);
  s = wave_sum(s);
  lse = mx + __logf(s);
  xl = ld<T>(lg, lab);
  amax = am;
}

template <typename T>
__global__ __launch_bounds__(XT) void xent_fwd_kernel(const T* __restrict__ logits,
                                                      const int* __restrict__ labels, int B, int C,
                                                      float* __restrict__ loss, T* __restrict__ grad) {
  __shared__ float part[XW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float acc = 0.f;
  const float invb = 1.f / (float)B;
  for (int r = w; r < B; r += XW) {
    const T* lg = logits + (size_t)r * C;
    const int lab = labels[r];
    float lse, xl;
    int am;
    row_stats<T>(lg, C, lab, lse, xl, am);
    acc += lse - xl;
    for (int c = lane; c < C; c += WAVE) {
      const float p = __expf(ld<T>(lg, c) - lse);
      st<T>(grad, (size_t)r * C + c, (p - (c == lab ? 1.f : 0.f)) * invb);
    }
  }
  if (lane == 0) part[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < XW; ++i) t += part[i];
    loss[0] = t * invb;
  }
}

template <typename T>
__global__ __launch_bounds__(XT) void xent_stats_kernel(const T* __restrict__ logits,
                                                        const int* __restrict__ labels, int B,
                                                        int C, double* __restrict__ acc4) {
  __shared__ float pc[XW], pl[XW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float correct = 0.f, ce = 0.f;
  for (int r = w; r < B; r += XW) {
    const T* lg = logits + (size_t)r * C;
    const int lab = labels[r];
    float lse, xl;
    int am;
    row_stats<T>(lg, C, lab, lse, xl, am);
    ce += lse - xl;
    correct += (am == lab) ? 1.f : 0.f;
  }
  if (lane == 0) { pc[w] = correct; pl[w] = ce; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double c = 0.0, l = 0.0;
#pragma unroll
    for (int i = 0; i < XW; ++i) { c += pc[i]; l += pl[i]; }
    acc4[0] += c;
    acc4[1] += (double)B;
    acc4[2] += l;
    acc4[3] += l / (double)B;
  }
}

}  // namespace

int launch_xent_fwd(const void* logits, const int* labels, int B, int C, float* loss, void* grad,
                    int dt, hipStream_t s) {
  if (B <= 0 || C <= 0) return -2;
  if (dt == DT_BF16)
    hipLaunchKernelGGL(xent_fwd_kernel<bf16_t>, dim3(1), dim3(XT), 0, s, (const bf16_t*)logits,
                       labels, B, C, loss, (bf16_t*)grad);
  else
    hipLaunchKernelGGL(xent_fwd_kernel<float>, dim3(1), dim3(XT), 0, s, (const float*)logits,
                       labels, B, C, loss, (float*)grad);
  return 0;
}

int launch_xent_stats(const void* logits, const int* labels, int B, int C, double* acc4, int dt,
                      hipStream_t s) {
  if (B <= 0) return 0;
  if (C <= 0) return -2;
  if (dt == DT_BF16)
    hipLaunchKernelGGL(xent_stats_kernel<bf16_t>, dim3(1), dim3(XT), 0, s, (const bf16_t*)logits,
                       labels, B, C, acc4);
  else
    hipLaunchKernelGGL(xent_stats_kernel<float>, dim3(1), dim3(XT), 0, s, (const float*)logits,
                       labels, B, C, acc4);
  return 0;
}

}  // namespace bcfl
