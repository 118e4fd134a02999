// K9: weight-gradient GEMM  dW[N, K] = G[M, N]^T X[M, K]  on MFMA, split over the token dim M.
//
// Why a hand-written kernel: every Linear backward needs dW with the reduction running over the
// token dimension (M = T ~ 11k packed tokens for the bench batch) and a SMALL output (768 x 768 ..
// 3072 x 768 for BERT-base). hipBLASLt covers this shape with few, long-K tiles: measured 157-430
// TF/s (scripts/wgrad_variants.py; 248-622 TF/s even with both operands pre-transposed), i.e. the
// weight gradient was ~46 % of all GEMM time of a BERT train step. Here:
//   * the reduction is split into S chunks of Mc rows so the grid fills all 256 CUs
//     (~2 workgroups per CU), fp32 partials are reduced by a second, deterministic kernel;
//   * both operands are consumed in their natural row-major [M, *] layout: [64 x 128] tiles are
//     staged into LDS (16-byte-unit XOR swizzle, mfma_tiles.h) and turned into MFMA operands by
//     ds_read_b64_tr_b16 hardware-transposed reads — no transpose pass over G or X;
//   * global loads of step i+2 are in flight (two register sets) during the MFMAs of steps i and
//     i+1, one barrier per step (double-buffered LDS);
//   * optionally the bias gradient db = colsum(G) is fused in (the G fragments are already in
//     registers), replacing a separate full read of G;
//   * the workgroup -> (split, tile) map is XCD-aware: the 8 XCDs each own a contiguous range of
//     logical ids, so concurrently running tiles of one XCD share the same G/X rows in its L2.
//
// Tile: 128 (N) x 128 (K) per workgroup of 4 waves (2 x 2), each wave 64 x 64 = 2 x 2 MFMA
// 32x32x16 accumulators; 64 reduction rows per step (4 MFMA k-steps).
// Replaces the autograd wgrad of the reference's nn.Linear layers (HF BERT/ALBERT/DistilBERT/
// Llama dense layers, e.g. SURVEY.md §2.6 K1 "dense GEMMs").
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "mfma_tiles.h"

namespace bcfl {
namespace {

constexpr int BM = 64;    // reduction rows per pipeline step
constexpr int BT = 128;   // output tile edge (N and K)
constexpr int TPB = 256;  // threads per workgroup

typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;

// Buffer descriptor over rows [m_begin, m_end) of a row-major bf16 matrix: loads past m_end
// return zeros from the hardware range check (no branches, so no waits at divergent joins).
// Built from workgroup-uniform values only (readfirstlane'd) so it stays in SGPRs.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const bf16_t* base, int64_t ld,
                                                           int m_begin, int m_end) {
  const bf16_t* p = base + (int64_t)m_begin * ld;
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uint32_t nbytes = __builtin_amdgcn_readfirstlane((uint32_t)((int64_t)(m_end - m_begin) * ld * 2));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo),
                                           (short)0, (int)nbytes, 0x00020000);
}

// register staging of one [BM x BT] bf16 tile: 4 x 16 B per thread, 16 threads per 256-B row.
// Lane byte offset `voff` = (row0 * ld + c0 + unit * 8) * 2; the row step goes in soffset.
struct StageTile {
  u32x4_t v[4];
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int voff, int row_bytes, int step) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      v[i] = __builtin_amdgcn_raw_buffer_load_b128(r, voff, (step * BM + 16 * i) * row_bytes, 0);
  }
  __device__ __forceinline__ void store(bf16_t* dst) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = threadIdx.x + TPB * i;
      *reinterpret_cast<u32x4_t*>(dst + swz_off<BT>(idx >> 4, idx & 15)) = v[i];
    }
  }
};

template <bool BIAS>
__global__ __launch_bounds__(TPB) void wgrad_kernel(WgradParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);  // [2 stages][G tile | X tile]
  constexpr int TILE_E = BM * BT;
  constexpr int STG = 2 * TILE_E;

  const int tilesK = p.K / BT;
  const int tiles = (p.N / BT) * tilesK;
  const int nwg = gridDim.x, b = blockIdx.x;
  // hardware dispatches workgroup b to XCD b % 8: give each XCD a contiguous logical range
  const int L = (nwg & 7) ? b : (b & 7) * (nwg >> 3) + (b >> 3);
  const int s = L / tiles, tile = L - s * tiles;
  const int n0 = (tile / tilesK) * BT, k0 = (tile % tilesK) * BT;
  const int m_begin = s * p.Mc;
  const int m_end = min(p.M, m_begin + p.Mc);
  const int nsteps = m_end > m_begin ? (m_end - m_begin + BM - 1) / BM : 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wn = w >> 1, wk = w & 1;
  const int hh = lane >> 5;
  const bf16_t* G = reinterpret_cast<const bf16_t*>(p.G);
  const bf16_t* X = reinterpret_cast<const bf16_t*>(p.X);
  bf16_t* out = reinterpret_cast<bf16_t*>(p.out);

  f32x16_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();
  // fused bias gradient db[n] = sum_m G[m, n]: the waves of the k0 == 0 tiles with wk == 0 add up
  // the G fragments they already hold (lane: column n, 8 of the 16 rows of each k-step)
  const bool do_bias = BIAS && k0 == 0 && wk == 0;  // BIAS: compile-time, no cost otherwise
  float cs[2] = {0.f, 0.f};

  if (nsteps > 0) {  // workgroup-uniform
    // transposed-read lane offsets of this wave's two G column blocks (u = 2wn + i) and two X
    // column blocks (u = 2wk + j), low / high k-halves (same formula as TileOffsets::tr)
    int offg[2][2], offx[2][2];
    {
      const int g16 = (lane >> 4) & 1, q = (lane & 15) >> 2, pc = lane & 3;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int hi = 0; hi < 2; ++hi) {
          const int row = 4 * hh + q + 8 * hi;
          offg[i][hi] = swz_off<BT>(row, 4 * (2 * wn + i) + 2 * g16 + (pc >> 1)) + 4 * (pc & 1);
          offx[i][hi] = swz_off<BT>(row, 4 * (2 * wk + i) + 2 * g16 + (pc >> 1)) + 4 * (pc & 1);
        }
    }
    // Prefetch distance 2: register set r0/r1 alternate, so the global loads of step i+2 are in
    // flight through two full steps of MFMAs (a first-touch HBM/MALL miss outlasts one step).
    const __amdgpu_buffer_rsrc_t rg = rows_rsrc(G, p.ldg, m_begin, m_end);
    const __amdgpu_buffer_rsrc_t rx = rows_rsrc(X, p.ldx, m_begin, m_end);
    const int rbg = (int)p.ldg * 2, rbx = (int)p.ldx * 2;
    const int vg = (threadIdx.x >> 4) * rbg + (n0 + (threadIdx.x & 15) * 8) * 2;
    const int vx = (threadIdx.x >> 4) * rbx + (k0 + (threadIdx.x & 15) * 8) * 2;
    // Every load / store below is unconditional (waitcnt stays exact: the wait for set i+1 never
    // covers the just-issued set i+2); steps past the split read zeros from the range check, so
    // the step count is rounded up to even and the extra step adds nothing.
    StageTile ga0, xa0, ga1, xa1;
    ga0.load(rg, vg, rbg, 0);
    xa0.load(rx, vx, rbx, 0);
    ga1.load(rg, vg, rbg, 1);
    xa1.load(rx, vx, rbx, 1);
    ga0.store(lds);
    xa0.store(lds + TILE_E);
    __syncthreads();
    auto step = [&](int it, StageTile& gl, StageTile& xl, StageTile& gs, StageTile& xs) {
      // gl/xl: free set, receives step it+2; gs/xs: holds step it+1, stored after the MFMAs
      gl.load(rg, vg, rbg, it + 2);
      xl.load(rx, vx, rbx, it + 2);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch at the top of the step
      const bf16_t* Gs = lds + (it & 1) * STG;
      const bf16_t* Xs = Gs + TILE_E;
#pragma unroll
      for (int ks = 0; ks < BM / 16; ++ks) {
        // A operand: G^T rows (n) x 16 reduction rows; B operand: X columns (k) — the same
        // (permuted) k order on both sides, so the product is the plain sum over m.
        bf16x8_t a[2], bx[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          a[i] = tr_operand(Gs + 16 * ks * BT, offg[i][0], offg[i][1]);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bx[j] = tr_operand(Xs + 16 * ks * BT, offx[j][0], offx[j][1]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(a[i], bx[j], acc[i][j]);
        if (do_bias) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 8; ++e) cs[i] += (float)a[i][e];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      bf16_t* nx = lds + ((it + 1) & 1) * STG;
      gs.store(nx);
      xs.store(nx + TILE_E);
      __syncthreads();
    };
    for (int it = 0; it < nsteps; it += 2) {
      step(it, ga0, xa0, ga1, xa1);
      step(it + 1, ga1, xa1, ga0, xa0);
    }
  }

  if (do_bias) {  // lanes l and l + 32 hold the two k-halves of column n
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float t = cs[i] + __shfl_xor(cs[i], 32, 64);
      const int n = n0 + 64 * wn + 32 * i + (lane & 31);
      if (hh == 0) {
        if (p.S == 1)
          reinterpret_cast<bf16_t*>(p.dbias)[n] = f2bf(t);
        else
          p.dbias_part[(int64_t)s * p.N + n] = t;
      }
    }
  }
  // epilogue: accumulator column = lane & 31 -> k, rows acc_row -> n
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int kk = k0 + 64 * wk + 32 * j + (lane & 31);
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int n = n0 + 64 * wn + 32 * i + acc_row(reg, hh);
        if (p.S == 1)
          out[(int64_t)n * p.ldo + kk] = f2bf(acc[i][j][reg]);
        else
          p.part[((int64_t)s * p.N + n) * p.K + kk] = acc[i][j][reg];
      }
    }
}

// out[n, k] = bf16( sum_s part[s, n, k] ), fixed summation order (deterministic). The blocks
// past the main grid reduce the bias-gradient partials db[n] = bf16( sum_s dbias_part[s, n] ) in
// the same launch (one reduction kernel per weight gradient instead of two).
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int S,
                                                           int N, int K, bf16_t* __restrict__ out,
                                                           int64_t ldo, int main_blocks,
                                                           const float* __restrict__ bpart,
                                                           bf16_t* __restrict__ dbias, int SB) {
  if ((int)blockIdx.x >= main_blocks) {  // bias columns (block-uniform branch)
    const int n = (blockIdx.x - main_blocks) * 256 + threadIdx.x;
    if (n >= N) return;
    float a = 0.f;
    for (int s = 0; s < SB; ++s) a += bpart[(int64_t)s * N + n];
    dbias[n] = f2bf(a);
    return;
  }
  const int64_t NK = (int64_t)N * K;
  const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (e >= NK) return;
  float4 a = *reinterpret_cast<const float4*>(part + e);
  for (int s = 1; s < S; ++s) {
    const float4 x = *reinterpret_cast<const float4*>(part + (int64_t)s * NK + e);
    a.x += x.x;
    a.y += x.y;
    a.z += x.z;
    a.w += x.w;
  }
  const int64_t n = e / K, k = e - n * K;
  const float v[4] = {a.x, a.y, a.z, a.w};
  Vec4<bf16_t>::store(out + n * ldo + k, v);
}

}  // namespace

int launch_wgrad_reduce(const float* part, int S, int N, int K, void* out, int64_t ldo,
                        const float* bpart, void* dbias, hipStream_t s, int SB) {
  const int64_t n4 = (int64_t)N * K / 4;
  const int main_blocks = part ? (int)((n4 + 255) / 256) : 0;  // part == nullptr: bias only
  if (SB <= 0) SB = S;
  const int bias_blocks = bpart ? (N + 255) / 256 : 0;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)(main_blocks + bias_blocks)), dim3(256), 0,
                     s, part, S, N, K, reinterpret_cast<bf16_t*>(out), ldo, main_blocks, bpart,
                     reinterpret_cast<bf16_t*>(dbias), SB);
  return 0;
}

int wgrad_splits(int M, int N, int K, int* Mc) {
  if (N % BT || K % BT || M <= 0) return -1;
  const int tiles = (N / BT) * (K / BT);
  // 2 workgroups fit per CU (64 KiB LDS, 2 waves/SIMD): 512 resident on 256 CUs. Never exceed
  // one full residency round — a 2nd round of a few workgroups would double the kernel time.
  // BCFL_WGRAD_SLOTS lowers the target when concurrent client lanes already fill the GPU (fewer
  // splits = less fp32 partial traffic and a shorter reduce).
  static const int slots = [] {
    const char* e = std::getenv("BCFL_WGRAD_SLOTS");
    const int v = e ? std::atoi(e) : 512;
    return v > 0 ? v : 512;
  }();
  int S = slots / tiles;
  const int maxS = (M + 255) / 256;  // keep >= 4 pipeline steps per split
  if (S > maxS) S = maxS;
  if (S < 1) S = 1;
  int mc = (M + S - 1) / S;
  mc = (mc + BM - 1) / BM * BM;
  *Mc = mc;
  return (M + mc - 1) / mc;
}

int launch_wgrad(const WgradParams& p, hipStream_t s) {
  if (p.N % BT || p.K % BT || p.S < 1 || (p.S > 1 && !p.part)) return -1;
  const int tiles = (p.N / BT) * (p.K / BT);
  const size_t lds = (size_t)2 * 2 * BM * BT * sizeof(bf16_t);
  if (p.dbias_part)
    hipLaunchKernelGGL(wgrad_kernel<true>, dim3(tiles * p.S), dim3(TPB), lds, s, p);
  else
    hipLaunchKernelGGL(wgrad_kernel<false>, dim3(tiles * p.S), dim3(TPB), lds, s, p);
  if (p.S > 1) {
    const int64_t n4 = (int64_t)p.N * p.K / 4;
    const int main_blocks = (int)((n4 + 255) / 256);
    const int bias_blocks = p.dbias_part ? (p.N + 255) / 256 : 0;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)(main_blocks + bias_blocks)), dim3(256),
                       0, s, p.part, p.S, p.N, p.K, reinterpret_cast<bf16_t*>(p.out), p.ldo,
                       main_blocks, p.dbias_part, reinterpret_cast<bf16_t*>(p.dbias), p.S);
  }
  return 0;
}

}  // namespace bcfl
