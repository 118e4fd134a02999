// Tall-skinny products of the LoRA adapters (SURVEY.md §2.6 / BASELINE config 5: Llama-3-8B with
// rank-16 adapters on q,k,v,o,gate,up,down). With M = 8k packed tokens the four low-rank products
// of a projection are
//
//   xa  = x A^T          [M, nr]  = X[M, K] . W[nr, K]^T          (forward)
//   gbs = g (s Bbd)      [M, nr]  = X[M, N] . W[nr, N]^T, W = s Bbd^T (backward, into dx's tail)
//   dA  = gbs^T x        [nr, K]  = P[M, nr]^T . X[M, K]          (adapter A gradient)
//   dB  = s g^T xa       [N, nr]  = (P[M, nr]^T . X[M, N])^T      (adapter B gradient)
//
// with nr = n * r <= 64. Each reads ONE big activation (x or g: 64-470 MB) once and a few hundred
// KB of adapter — HBM-bound, not MFMA-bound. A 256-column GEMM tile wastes 4-16x of its MFMA
// work on zero padding, and a library kernel reduces M = 8k in a handful of workgroups
// (16.9 % of config 5's kernel time on hipBLASLt, profiles/config5_kernel_stats_r3.md). Here:
//
//   skinny_xwt: one wave per (32 rows, K slice): X fragments straight from HBM into MFMA
//               operands (16-byte loads, 128-byte row segments per wave), the W fragments from
//               L2 (the adapter is tiny and shared by every wave); split-K fp32 partials.
//   skinny_ptx: the reduction runs over the ROW index of both operands, so both are staged
//               row-major through LDS and read back with ds_read_b64_tr_b16 (the hardware
//               transpose, cdna_hip_programming.md T10) as MFMA operands; one workgroup per
//               (64 columns, M slice), double-buffered tiles; split-M fp32 partials.
//   reduce:     the slices summed in a fixed order (deterministic), bf16 out, optional zero
//               columns (the tail-segment padding the fused LoRA GEMMs of gemm8.hip read).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "lds_dma.h"

namespace bcfl {
namespace {

__device__ __forceinline__ f32x4_t sk_mfma(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t ld_frag(const bf16_t* p) {
  return *reinterpret_cast<const bf16x8_t*>(p);
}


// ---- skinny_xwt --------------------------------------------------------------------------------
// part[s, m, c] = sum_{k in slice s} X[m, k] W[c, k],  c < 16 RB (rows of W >= R are clamped:
// their columns are computed and never stored by the reduce). Wave = 32 rows; block = 4 waves.
template <int RB>
__global__ __launch_bounds__(256) void skinny_xwt_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                         const bf16_t* __restrict__ W, int64_t ldw,
                                                         int M, int K, int R, int kc,
                                                         float* __restrict__ part) {
  constexpr int RP = 16 * RB;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int m0 = (blockIdx.x * 4 + wave) * 32;
  if (m0 >= M) return;  // wave-uniform; no LDS, no barrier in this kernel
  const int s = blockIdx.y;
  const int kb = s * kc;
  const int ke = min(K, kb + kc);
  const int r16 = lane & 15, g = lane >> 4;
  // operand rows (clamped: out-of-range rows read valid memory and are never stored)
  const bf16_t* xr[2];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) xr[rb] = X + (int64_t)min(m0 + rb * 16 + r16, M - 1) * ldx + 8 * g;
  const bf16_t* wr[RB];
#pragma unroll
  for (int cb = 0; cb < RB; ++cb) wr[cb] = W + (int64_t)min(cb * 16 + r16, R - 1) * ldw + 8 * g;

  f32x4_t acc[2][RB];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) acc[rb][cb] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // two 64-deep k steps per iteration: the next step's X and W fragments are in flight while
  // this step's MFMAs run (X from HBM, W from L2)
  struct Frag {
    bf16x8_t x[2][2], w[RB][2];
  };
  Frag fa, fb;
  auto load = [&](Frag& f, int k) {
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int h = 0; h < 2; ++h) f.x[rb][h] = ld_frag(xr[rb] + k + 32 * h);
#pragma unroll
    for (int cb = 0; cb < RB; ++cb)
#pragma unroll
      for (int h = 0; h < 2; ++h) f.w[cb][h] = ld_frag(wr[cb] + k + 32 * h);
  };
  auto step = [&](const Frag& f) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < RB; ++cb) acc[rb][cb] = sk_mfma(f.x[rb][h], f.w[cb][h], acc[rb][cb]);
  };
  int k = kb;
  if (k < ke) load(fa, k);
  for (; k + 64 < ke; k += 128) {
    load(fb, k + 64);
    step(fa);
    if (k + 128 < ke) load(fa, k + 128);
    step(fb);
  }
  if (k < ke) step(fa);

  // C tile: col = lane & 15, row = 4 (lane >> 4) + reg
  float* pp = part + (int64_t)s * M * RP;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + rb * 16 + 4 * g + r;
      if (m < M) {
#pragma unroll
        for (int cb = 0; cb < RB; ++cb) pp[(int64_t)m * RP + cb * 16 + r16] = acc[rb][cb][r];
      }
    }
}

// out[m, c] = c < R ? bf16(scale * sum_s part[s, m, c]) : 0   for c < Cz
__global__ __launch_bounds__(256) void skinny_reduce_rows_kernel(const float* __restrict__ part,
                                                                 int S, int M, int RP, int R, int Cz,
                                                                 float scale, bf16_t* __restrict__ out,
                                                                 int64_t ldo) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)M * Cz) return;
  const int m = (int)(i / Cz), c = (int)(i % Cz);
  float v = 0.f;
  if (c < R) {
    for (int s = 0; s < S; ++s) v += part[((int64_t)s * M + m) * RP + c];
    v *= scale;
  }
  out[(int64_t)m * ldo + c] = f2bf(v);
}

// ---- skinny_ptx --------------------------------------------------------------------------------
// part[s, c, n] = sum_{m in slice s} P[m, c] X[m, n] for c < 16 RB, n in the block's 64 columns.
// LDS images: [32 m rows][72] bf16 (144-byte rows: 16-byte aligned chunks for the staging writes,
// and the transposed reads of one 16-lane group (4 rows x 32 bytes) fall on disjoint banks).
constexpr int PTX_LD = 72;
constexpr int PTX_TILE = 32 * PTX_LD;  // elements per image

template <int RB>
__global__ __launch_bounds__(256) void skinny_ptx_kernel(const bf16_t* __restrict__ P, int64_t ldp,
                                                         const bf16_t* __restrict__ X, int64_t ldx,
                                                         int M, int N, int R, int mc,
                                                         float* __restrict__ part) {
  constexpr int RP = 16 * RB;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2][2][PTX_TILE];  // [buffer][X | P][tile]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int n0 = blockIdx.x * 64;
  const int s = blockIdx.y;
  const int mb = s * mc, me = min(M, mb + mc);
  // staging: thread t moves row t >> 3, 16-byte chunk t & 7 of the X tile (and of the P tile
  // while the chunk is inside its RP columns)
  const int srow = t >> 3, sch = t & 7;
  const bool p_on = sch * 8 < RP;
  const bool p_in = sch * 8 < R;  // chunks past the adapter's real columns stage zeros
  uint4 xv, pv;
  auto fetch = [&](int m) {
    const int mm = m + srow;
    const bool ok = mm < me;
    xv = ok ? *reinterpret_cast<const uint4*>(X + (int64_t)mm * ldx + n0 + sch * 8) : make_uint4(0, 0, 0, 0);
    if (p_on)
      pv = (ok && p_in) ? *reinterpret_cast<const uint4*>(P + (int64_t)mm * ldp + sch * 8)
                        : make_uint4(0, 0, 0, 0);
  };
  auto stage = [&](int b) {
    *reinterpret_cast<uint4*>(&lds[b][0][srow * PTX_LD + sch * 8]) = xv;
    if (p_on) *reinterpret_cast<uint4*>(&lds[b][1][srow * PTX_LD + sch * 8]) = pv;
  };
  // transposed-read lane addresses (T10): group g = lane >> 4 takes k-rows 8g + 4h + q,
  // lane 4q + p supplies row q's columns col0 + 4p .. + 3 and receives column col0 + (lane & 15)
  const int g = lane >> 4, q = (lane & 15) >> 2, p4 = (lane & 3) * 4;
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) bf16_t*)&lds[0][0][0];
  auto tr_addr = [&](int b, int img, int h, int col0) -> uint32_t {
    return base + 2u * (uint32_t)(((b * 2 + img) * PTX_TILE) + (8 * g + 4 * h + q) * PTX_LD + col0 + p4);
  };
  f32x4_t acc[RB];
#pragma unroll
  for (int cb = 0; cb < RB; ++cb) acc[cb] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  int b = 0;
  fetch(mb);
  stage(0);
  __syncthreads();
  for (int m = mb; m < me; m += 32) {
    const bool more = m + 32 < me;
    if (more) fetch(m + 32);  // global loads in flight under this tile's reads and MFMAs
    // B operand: X[k = m rows][n = 16 wave + lane]; A operands: P^T[r = 16 cb + lane][k = m rows]
    s16x4_t xlo = ds_tr_read<0>(tr_addr(b, 0, 0, 16 * wave));
    s16x4_t xhi = ds_tr_read<0>(tr_addr(b, 0, 1, 16 * wave));
    s16x4_t plo[RB], phi[RB];
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) {
      plo[cb] = ds_tr_read<0>(tr_addr(b, 1, 0, 16 * cb));
      phi[cb] = ds_tr_read<0>(tr_addr(b, 1, 1, 16 * cb));
    }
    lgk_wait<0>();
    reg_fence(xlo);
    reg_fence(xhi);
    const bf16x8_t bx = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(xlo, xhi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
    for (int cb = 0; cb < RB; ++cb) {
      reg_fence(plo[cb]);
      reg_fence(phi[cb]);
      const bf16x8_t ap = __builtin_bit_cast(bf16x8_t,
                                             __builtin_shufflevector(plo[cb], phi[cb], 0, 1, 2, 3, 4, 5, 6, 7));
      acc[cb] = sk_mfma(ap, bx, acc[cb]);
    }
    if (more) {
      stage(b ^ 1);  // the other buffer: its last readers finished before the previous barrier
      __syncthreads();
      b ^= 1;
    }
  }
  // C tile: col = n0 + 16 wave + (lane & 15), row c = 16 cb + 4 (lane >> 4) + reg
  float* pp = part + (int64_t)s * RP * N;
  const int n = n0 + 16 * wave + (lane & 15);
#pragma unroll
  for (int cb = 0; cb < RB; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) pp[(int64_t)(cb * 16 + 4 * g + r) * N + n] = acc[cb][r];
}

// out[c, n] = bf16(scale * sum_s part[s, c, n]) for c < R
__global__ __launch_bounds__(256) void skinny_reduce_cols_kernel(const float* __restrict__ part,
                                                                 int S, int RP, int R, int N,
                                                                 float scale, bf16_t* __restrict__ out,
                                                                 int64_t ldo) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)R * N) return;
  const int c = (int)(i / N), n = (int)(i % N);
  float v = 0.f;
  for (int s = 0; s < S; ++s) v += part[((int64_t)s * RP + c) * N + n];
  out[(int64_t)c * ldo + n] = f2bf(v * scale);
}

// LoRA dB: out[n, j] = bf16(scale * sum_s part[s, blk(n) r + j, n]), n fastest across threads
// (coalesced partial reads)
__global__ __launch_bounds__(256) void skinny_reduce_bdiag_kernel(const float* __restrict__ part,
                                                                  int S, int RP, int N, int r,
                                                                  int nblk, int4 lo, int hi4,
                                                                  float scale, bf16_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)r * N) return;
  const int j = (int)(i / N), n = (int)(i % N);
  const int bo[5] = {lo.x, lo.y, lo.z, lo.w, hi4};
  int b = 0;
#pragma unroll
  for (int q = 1; q < 4; ++q) b += (q < nblk && n >= bo[q]) ? 1 : 0;
  const int c = b * r + j;
  float v = 0.f;
  for (int s = 0; s < S; ++s) v += part[((int64_t)s * RP + c) * N + n];
  out[(int64_t)n * r + j] = f2bf(v * scale);
}

__global__ __launch_bounds__(256) void lora_pack_b_kernel(LoraPackParams p) {
  const int nr = p.nblk * p.r;
  const int64_t tot1 = (int64_t)p.N * p.k2, tot2 = (int64_t)nr * p.N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < tot1 + tot2;
       i += (int64_t)gridDim.x * 256) {
    int n, c;
    if (i < tot1) {
      n = (int)(i / p.k2);
      c = (int)(i % p.k2);
    } else {
      c = (int)((i - tot1) / p.N);
      n = (int)((i - tot1) % p.N);
    }
    float v = 0.f;
    if (c < nr) {
      const int b = c / p.r;
      if (n >= p.boff[b] && n < p.boff[b + 1])
        v = p.s * bf2f(reinterpret_cast<const bf16_t*>(p.B[b])[(int64_t)(n - p.boff[b]) * p.r + (c - b * p.r)]);
    }
    if (i < tot1) reinterpret_cast<bf16_t*>(p.bb)[i] = f2bf(v);
    else reinterpret_cast<bf16_t*>(p.bbt)[(int64_t)c * p.N + n] = f2bf(v);
  }
}

}  // namespace

int launch_lora_pack_b(const LoraPackParams& p, hipStream_t s) {
  if (p.nblk < 1 || p.nblk > 4 || p.r < 1 || p.nblk * p.r > p.k2 || p.boff[0] != 0 ||
      p.boff[p.nblk] != p.N)
    return -1;
  const int64_t tot = (int64_t)p.N * p.k2 + (int64_t)p.nblk * p.r * p.N;
  const int grid = (int)std::min<int64_t>((tot + 255) / 256, 4096);
  hipLaunchKernelGGL(lora_pack_b_kernel, dim3(grid), dim3(256), 0, s, p);
  return 0;
}

// grid-size targets (A/B: BCFL_SKINNY_XWT_WAVES, BCFL_SKINNY_PTX_WGS, BCFL_SKINNY_MIN_STEPS)
static int skinny_env(const char* name, int dflt) {
  const char* e = std::getenv(name);
  const int v = e ? std::atoi(e) : 0;
  return v > 0 ? v : dflt;
}

int skinny_xwt_splits(int M, int K, int* kc) {
  // ~2 slices per CU's worth of 32-row waves: at M = 8k, 256 row waves x S slices
  static const int target = skinny_env("BCFL_SKINNY_XWT_WAVES", 2048);
  static const int min_steps = skinny_env("BCFL_SKINNY_MIN_STEPS", 8);
  const int waves = (M + 31) / 32;
  int S = (target + waves - 1) / waves;
  const int maxS = K / (64 * min_steps) > 0 ? K / (64 * min_steps) : 1;  // >= min_steps k-steps
  if (S > maxS) S = maxS;
  if (S < 1) S = 1;
  int c = (K + S - 1) / S;
  c = (c + 63) / 64 * 64;
  *kc = c;
  return (K + c - 1) / c;
}

int launch_skinny_xwt(const SkinnyParams& p, hipStream_t s) {
  if (p.R < 1 || p.R > 64 || p.K % 64 || p.ldx % 8 || p.ldw % 8 || p.ldo % 8 || !p.part) return -1;
  const int RB = (p.R + 15) / 16;
  const dim3 grid((p.M + 127) / 128, p.S);
  switch (RB) {
    case 1: hipLaunchKernelGGL(skinny_xwt_kernel<1>, grid, dim3(256), 0, s, (const bf16_t*)p.X, p.ldx, (const bf16_t*)p.W, p.ldw, p.M, p.K, p.R, p.kc, p.part); break;
    case 2: hipLaunchKernelGGL(skinny_xwt_kernel<2>, grid, dim3(256), 0, s, (const bf16_t*)p.X, p.ldx, (const bf16_t*)p.W, p.ldw, p.M, p.K, p.R, p.kc, p.part); break;
    case 3: hipLaunchKernelGGL(skinny_xwt_kernel<3>, grid, dim3(256), 0, s, (const bf16_t*)p.X, p.ldx, (const bf16_t*)p.W, p.ldw, p.M, p.K, p.R, p.kc, p.part); break;
    default: hipLaunchKernelGGL(skinny_xwt_kernel<4>, grid, dim3(256), 0, s, (const bf16_t*)p.X, p.ldx, (const bf16_t*)p.W, p.ldw, p.M, p.K, p.R, p.kc, p.part); break;
  }
  const int64_t tot = (int64_t)p.M * p.Cz;
  hipLaunchKernelGGL(skinny_reduce_rows_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s,
                     p.part, p.S, p.M, 16 * RB, p.R, p.Cz, p.scale, (bf16_t*)p.out, p.ldo);
  return 0;
}

int skinny_ptx_splits(int M, int N, int* mc) {
  static const int target = skinny_env("BCFL_SKINNY_PTX_WGS", 1024);  // sweep: 512 470 us, 1024 425 us over the config-5 shapes (profiles/skinny_sweep_r4.txt)
  const int blocks = N / 64;
  int S = (target + blocks - 1) / blocks;
  const int maxS = M / 512 > 0 ? M / 512 : 1;  // >= 16 m-steps per slice
  if (S > maxS) S = maxS;
  if (S < 1) S = 1;
  int c = (M + S - 1) / S;
  c = (c + 31) / 32 * 32;
  *mc = c;
  return (M + c - 1) / c;
}

int launch_skinny_ptx(const SkinnyParams& p, hipStream_t s) {
  // here X is the big [M, N] operand, W the skinny [M, R] one (P), out [R, N]
  if (p.R < 1 || p.R > 64 || p.R % 8 || p.N % 64 || p.ldx % 8 || p.ldw % 8 || p.ldo % 8 || !p.part)
    return -1;
  const int RB = (p.R + 15) / 16;
  const dim3 grid(p.N / 64, p.S);
  switch (RB) {
    case 1: hipLaunchKernelGGL(skinny_ptx_kernel<1>, grid, dim3(256), 0, s, (const bf16_t*)p.W, p.ldw, (const bf16_t*)p.X, p.ldx, p.M, p.N, p.R, p.kc, p.part); break;
    case 2: hipLaunchKernelGGL(skinny_ptx_kernel<2>, grid, dim3(256), 0, s, (const bf16_t*)p.W, p.ldw, (const bf16_t*)p.X, p.ldx, p.M, p.N, p.R, p.kc, p.part); break;
    case 3: hipLaunchKernelGGL(skinny_ptx_kernel<3>, grid, dim3(256), 0, s, (const bf16_t*)p.W, p.ldw, (const bf16_t*)p.X, p.ldx, p.M, p.N, p.R, p.kc, p.part); break;
    default: hipLaunchKernelGGL(skinny_ptx_kernel<4>, grid, dim3(256), 0, s, (const bf16_t*)p.W, p.ldw, (const bf16_t*)p.X, p.ldx, p.M, p.N, p.R, p.kc, p.part); break;
  }
  if (p.bdr > 0) {  // LoRA dB: the diagonal blocks, transposed into [N, r]
    if (p.nblk < 1 || p.nblk > 4 || p.nblk * p.bdr != p.R || p.boff[p.nblk] != p.N) return -2;
    const int64_t tot = (int64_t)p.bdr * p.N;
    hipLaunchKernelGGL(skinny_reduce_bdiag_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s,
                       p.part, p.S, 16 * RB, p.N, p.bdr, p.nblk,
                       make_int4(p.boff[0], p.boff[1], p.boff[2], p.boff[3]), p.boff[4], p.scale,
                       (bf16_t*)p.out);
    return 0;
  }
  const int64_t tot = (int64_t)p.R * p.N;
  hipLaunchKernelGGL(skinny_reduce_cols_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s,
                     p.part, p.S, 16 * RB, p.R, p.N, p.scale, (bf16_t*)p.out, p.ldo);
  return 0;
}

}  // namespace bcfl
