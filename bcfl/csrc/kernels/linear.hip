// Dense-layer GEMMs with fused epilogues on MFMA:
//
//   forward  ("NT")  C[M, N] = A[M, K] · B[N, K]^T        A = activations x, B = weight W [out, in]
//   dgrad    ("NN")  C[M, N] = A[M, K] · B[K, N]          A = dY [M, out], B = W [out, in]
//
// Epilogues (fused into the kernel that produces the tile, so no extra pass over [M, N]):
//   EPI_STORE     C = acc
//   EPI_BIAS      C = acc + bias[n]                                 (QKV / pooler projections)
//   EPI_BIAS_ACT  aux = acc + bias[n] (pre-activation, saved for backward), C = act(aux)
//                 — HF BertIntermediate dense -> GELU (K6); replaces bias_act_fwd
//   EPI_DACT      C = acc * act'(aux[m, n])   — dgrad of the layer AFTER an activation: writes the
//                 gradient w.r.t. the pre-activation directly (replaces bias_act_bwd)
//
// Structure (same machinery as the K9 weight-gradient kernel, gemm.hip): 128 x 128 output tile
// per workgroup of 4 waves (2 x 2, each 64 x 64 = 2 x 2 v_mfma_f32_32x32x16_bf16 accumulators),
// 64-deep reduction steps; operand tiles are register-staged with buffer loads (prefetch distance
// 2: two register sets, global loads of step i+2 in flight under the MFMAs of steps i and i+1),
// stored to double-buffered LDS with a 16-byte-unit XOR swizzle, one barrier per step.
//   * K-contiguous operand tiles ([128 rows][64 k]: A always, B in NT) are read as MFMA operands
//     by row reads (lane = row, 8 consecutive k) — the swizzle makes them bank-conflict free;
//   * the NN weight tile ([64 k][128 n], W rows) is read by ds_read_b64_tr_b16 hardware
//     transposes (mfma_tiles.h tr_operand) — no transpose pass over W.
// Rows past M read zeros (buffer-resource range check) and are not stored; N must be a multiple
// of 128 and K of 64 (every BERT / ALBERT / DistilBERT / Llama projection); the host falls back
// to the library GEMM otherwise. The workgroup -> tile map is XCD-aware (bijective for any grid):
// each XCD walks a contiguous range of row-major tiles, so the A rows it streams stay in its L2.
#include <cstdlib>

#include "act.h"
#include "common.h"
#include "kernels.h"
#include "mfma_tiles.h"

namespace bcfl {
namespace {

constexpr int LK = 64;     // reduction step
constexpr int EP_LD = 72;  // epilogue slab row stride (floats): rows r and r + 4 on disjoint banks

typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc_l(const bf16_t* base, int64_t ld,
                                                             int r_begin, int r_end) {
  const bf16_t* p = base + (int64_t)r_begin * ld;
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int rows = r_end > r_begin ? r_end - r_begin : 0;
  const uint32_t nbytes = __builtin_amdgcn_readfirstlane((uint32_t)((int64_t)rows * ld * 2));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo),
                                           (short)0, (int)nbytes, 0x00020000);
}

// [ROWS][64 k] K-contiguous tile: 8 x 16 B units per row; load i of thread t covers row
// t/8 + i*T/8, unit t%8 (lane offsets: voff + i * row_step, the k step goes in soffset)
template <int ROWS, int T>
struct RowTile {
  static constexpr int U = ROWS * 8 / T;
  u32x4_t v[U];
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int voff, int row_step, int kbytes) {
#pragma unroll
    for (int i = 0; i < U; ++i)
      v[i] = __builtin_amdgcn_raw_buffer_load_b128(r, voff + i * row_step, kbytes, 0);
  }
  __device__ __forceinline__ void store(bf16_t* dst) const {
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int idx = threadIdx.x + T * i;
      *reinterpret_cast<u32x4_t*>(dst + swz_off<LK>(idx >> 3, idx & 7)) = v[i];
    }
  }
};

// [64 k][COLS n] N-contiguous tile (NN weight operand), kept as COLS/128 swizzled [64][128]
// sub-tiles. The hardware-transposed read hands lane-half hh the k-rows {4hh..4hh+3,
// 4hh+8..4hh+11} of each 16-row group, while the row-read A operand holds k = 8hh .. 8hh+7.
// Storing k-row 4c + q at LDS row 4 swap2(c) + q (swap2 exchanges the two bits of c, an
// involution) makes the transposed read deliver natural k order, so both MFMA operands agree on
// k — at zero cost (only the store row moves).
__device__ __forceinline__ int k_perm(int row) {
  const int c = (row >> 2) & 3;
  return (row & ~15) | ((((c & 1) << 1) | (c >> 1)) << 2) | (row & 3);
}
template <int COLS, int T>
struct ColTile {
  static constexpr int U = 64 * COLS / 8 / T;
  static_assert(T % 16 == 0 && T <= 1024 && COLS % 128 == 0, "ColTile geometry");
  u32x4_t v[U];
  // load i of thread t: row (t >> 4) + ((T/16) i mod 64), column 128 ((T i) >> 10) + 8 (t & 15):
  // a per-thread base plus a workgroup-uniform (scalar) term per i
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int vbase, int ldb_bytes, int kbytes) {
#pragma unroll
    for (int i = 0; i < U; ++i)
      v[i] = __builtin_amdgcn_raw_buffer_load_b128(
          r, vbase, kbytes + (((T / 16) * i) & 63) * ldb_bytes + ((T * i) >> 10) * 256, 0);
  }
  __device__ __forceinline__ void store(bf16_t* dst) const {
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int idx = threadIdx.x + T * i;
      *reinterpret_cast<u32x4_t*>(dst + (idx >> 10) * (64 * 128) +
                                  swz_off<128>(k_perm((idx >> 4) & 63), idx & 15)) = v[i];
    }
  }
};

// BM x BN output tile per workgroup of WGM x WGN waves; wave tile (BM/WGM) x (BN/WGN) built from
// 32 x 32 accumulators (I x J of them).
template <bool NN, int EPI, int ACT, int BM, int BN, int WGM, int WGN,
          bool PF2 = (BM * BN <= 128 * 128)>
__global__ __launch_bounds__(64 * WGM * WGN) void linear_kernel(LinearParams p) {
  constexpr int T = 64 * WGM * WGN;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int I = WTM / 32, J = WTN / 32;
  constexpr int A_E = BM * LK, B_E = BN * LK;
  constexpr int STG = A_E + B_E;
  static_assert(WTN == 64, "epilogue slab assumes 64-column wave tiles");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);  // [2 stages][A tile | B tile]

  const int tilesN = p.N / BN;
  const int tilesM = (p.M + BM - 1) / BM;
  const int nwg = tilesM * tilesN;
  const int b = blockIdx.x;
  // bijective XCD-aware remap: dispatch sends workgroup b to XCD b % 8
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = b & 7;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int m0 = (L / tilesN) * BM, n0 = (L % tilesN) * BN;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w / WGN, wn = w % WGN;
  const int hh = lane >> 5;
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.A);
  const bf16_t* B = reinterpret_cast<const bf16_t*>(p.B);
  const int nsteps = p.K / LK;

  f32x16_t acc[I][J];
#pragma unroll
  for (int i = 0; i < I; ++i)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[i][j] = zero16();

  // operand read offsets (elements, inside one stage's tile)
  int offa[4];  // A row reads: row WTM wm + (lane & 31) [+32 i], unit 2ks + hh
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) offa[ks] = swz_off<LK>(WTM * wm + (lane & 31), 2 * ks + hh);
  int offb[4];      // NT: B row reads (row = n)
  int offbt[J][2];  // NN: B transposed reads (32-column block u, low / high k-halves)
  if constexpr (!NN) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) offb[ks] = swz_off<LK>(WTN * wn + (lane & 31), 2 * ks + hh);
  } else {
    const int g16 = (lane >> 4) & 1, q = (lane & 15) >> 2, pc = lane & 3;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int u = WTN / 32 * wn + j;
#pragma unroll
      for (int hi = 0; hi < 2; ++hi) {
        const int row = 4 * hh + q + 8 * hi;
        offbt[j][hi] = (u >> 2) * (64 * 128) +
                       swz_off<128>(row, 4 * (u & 3) + 2 * g16 + (pc >> 1)) + 4 * (pc & 1);
      }
    }
  }

  const __amdgpu_buffer_rsrc_t ra = rows_rsrc_l(A, p.lda, m0, min(p.M, m0 + BM));
  const int va = (threadIdx.x >> 3) * (int)p.lda * 2 + (threadIdx.x & 7) * 16;
  const int ra_row = T / 8 * (int)p.lda * 2;
  using ATile = RowTile<BM, T>;
  using BTileT = typename std::conditional<NN, ColTile<BN, T>, RowTile<BN, T>>::type;
  __amdgpu_buffer_rsrc_t rb;
  int vb = 0, rb_row = 0, rb_step;
  if constexpr (!NN) {  // W rows n0 .. n0+BN-1, k contiguous
    rb = rows_rsrc_l(B, p.ldb, n0, n0 + BN);
    vb = (threadIdx.x >> 3) * (int)p.ldb * 2 + (threadIdx.x & 7) * 16;
    rb_row = T / 8 * (int)p.ldb * 2;
    rb_step = LK * 2;
  } else {              // W rows k (all K), columns n0 .. n0+BN-1
    rb = rows_rsrc_l(B, p.ldb, 0, p.K);
    vb = (threadIdx.x >> 4) * (int)p.ldb * 2 + (n0 + (threadIdx.x & 15) * 8) * 2;
    rb_row = (int)p.ldb * 2;
    rb_step = LK * (int)p.ldb * 2;
  }
  auto load_a = [&](ATile& t, int step) { t.load(ra, va, ra_row, step * LK * 2); };
  auto load_b = [&](BTileT& t, int step) {
    if constexpr (!NN) t.load(rb, vb, rb_row, step * rb_step);
    else t.load(rb, vb, rb_row, step * rb_step);
  };

  ATile a0;
  BTileT b0;
  load_a(a0, 0);
  load_b(b0, 0);
  a0.store(lds);
  b0.store(lds + A_E);

  auto compute = [&](int it) {
    const bf16_t* As = lds + (it & 1) * STG;
    const bf16_t* Bs = As + A_E;
#pragma unroll
    for (int ks = 0; ks < LK / 16; ++ks) {
      bf16x8_t fa[I], fb[J];
#pragma unroll
      for (int i = 0; i < I; ++i) fa[i] = lds_row8(As + offa[ks] + 32 * i * LK);
      if constexpr (!NN) {
#pragma unroll
        for (int j = 0; j < J; ++j) fb[j] = lds_row8(Bs + offb[ks] + 32 * j * LK);
      } else {
#pragma unroll
        for (int j = 0; j < J; ++j) fb[j] = tr_operand(Bs + 16 * ks * 128, offbt[j][0], offbt[j][1]);
      }
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j) acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
    }
  };
  int it = 0;
  if constexpr (PF2) {
    // prefetch distance 2: register sets alternate, the loads of step it+2 are issued at the top
    // of step it and stay in flight through the MFMAs of steps it and it+1
    ATile a1;
    BTileT b1;
    load_a(a1, 1);
    load_b(b1, 1);
    __syncthreads();
    auto step = [&](int i, ATile& al, BTileT& bl, ATile& as, BTileT& bs) {
      load_a(al, i + 2);
      load_b(bl, i + 2);
      __builtin_amdgcn_sched_barrier(0);
      compute(i);
      __builtin_amdgcn_sched_barrier(0);
      bf16_t* nx = lds + ((i + 1) & 1) * STG;
      as.store(nx);
      bs.store(nx + A_E);
      __syncthreads();
    };
    for (; it + 1 < nsteps; it += 2) {
      step(it, a0, b0, a1, b1);
      step(it + 1, a1, b1, a0, b0);
    }
    if (nsteps & 1) compute(it);  // the last (odd) step is already in LDS: no loads, no stores
  } else {
    // prefetch distance 1 (one register set; the 256 x 256 tile's accumulators need the
    // registers): step it+1 is loaded right after the barrier and lands under compute(it)
    load_a(a0, 1);
    load_b(b0, 1);
    __syncthreads();
    for (; it < nsteps; ++it) {
      compute(it);
      if (it + 1 < nsteps) {
        __builtin_amdgcn_sched_barrier(0);
        bf16_t* nx = lds + ((it + 1) & 1) * STG;
        a0.store(nx);
        b0.store(nx + A_E);
        __syncthreads();
        if (it + 2 < nsteps) {
          load_a(a0, it + 2);
          load_b(b0, it + 2);
        }
      }
    }
  }

  // ---- epilogue, staged through LDS so every global access is a 16-byte row segment, one
  // 32-row accumulator block (i) at a time:
  // (1) each wave parks its 32 x 64 fp32 block in its own LDS slab ([32][EP_LD]: the padded
  //     stride keeps the two lane-halves' rows on disjoint banks);
  // (2) lane -> (row (lane >> 3) + 8 r, 8 consecutive columns): bias / activation / act' math on
  //     8-wide vectors, 16-byte loads of aux and 16-byte stores of C (and aux), 128 B per row.
  float* ep = reinterpret_cast<float*>(smem) + w * (32 * EP_LD);
  bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
  bf16_t* aux = reinterpret_cast<bf16_t*>(p.aux);
  const bf16_t* bias = reinterpret_cast<const bf16_t*>(p.bias);
  const int cc = (lane & 7) * 8;
  const int n = n0 + WTN * wn + cc;
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_ACT) {
    if (bias) Vec8<bf16_t>::load(bias + n, bv);
  }
#pragma unroll
  for (int i = 0; i < I; ++i) {
    __syncthreads();  // operand tiles (i == 0) / the previous block's slab reads are done
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg)
        ep[acc_row(reg, hh) * EP_LD + 32 * j + (lane & 31)] = acc[i][j][reg];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rr = (lane >> 3) + 8 * r;
      const int m = m0 + WTM * wm + 32 * i + rr;
      if (m < p.M) {
        float v[8];
        Vec8<float>::load(ep + rr * EP_LD + cc, v);
        if constexpr (EPI == EPI_BIAS) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += bv[e];
        } else if constexpr (EPI == EPI_BIAS_ACT) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = bf2f(f2bf(v[e] + bv[e]));  // pre, as stored
          Vec8<bf16_t>::store(aux + (int64_t)m * p.ldaux + n, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = act_ft<ACT>(v[e]);
        } else if constexpr (EPI == EPI_DACT) {
          float a[8];
          Vec8<bf16_t>::load(aux + (int64_t)m * p.ldaux + n, a);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= act_dt<ACT>(a[e]);
        }
        Vec8<bf16_t>::store(C + (int64_t)m * p.ldc + n, v);
      }
    }
  }
}

// Persistent variant of the 128 x 128 kernel: a grid of at most 2 workgroups per CU walks the
// tiles (stride = grid size, a multiple of 8 so every tile keeps its XCD), and the first two
// reduction steps of the NEXT tile are loaded before the current tile's epilogue, so their
// latency hides behind the epilogue (with K = 768 a tile has only 12 steps; prologue and epilogue
// are a large share of it). Default for the 128 x 128 configuration (same-box A/B at the bench
// shapes: dgrad +4..9 %, GELU' dgrad +2..5 %, forward +0..4 %, fused bias+GELU forward unchanged;
// profiles/experiments_r2.md); BCFL_LINEAR_PERSIST=0 selects the one-tile-per-workgroup kernel.
template <bool NN, int EPI, int ACT>
__global__ __launch_bounds__(256) void linear_persist_kernel(LinearParams p) {
  constexpr int BM = 128, BN = 128, WGN = 2, T = 256;
  constexpr int WTM = 64, WTN = 64, I = 2, J = 2;
  constexpr int A_E = BM * LK, B_E = BN * LK, STG = A_E + B_E;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);

  const int tilesN = p.N / BN;
  const int tilesM = (p.M + BM - 1) / BM;
  const int nwg = tilesM * tilesN;
  const int G = gridDim.x;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  auto remap = [&](int t) {  // bijective XCD-aware map (t & 7 = this workgroup's XCD)
    const int xcd = t & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (t >> 3);
  };
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w / WGN, wn = w % WGN;
  const int hh = lane >> 5;
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.A);
  const bf16_t* B = reinterpret_cast<const bf16_t*>(p.B);
  const int nsteps = p.K / LK;

  int offa[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) offa[ks] = swz_off<LK>(WTM * wm + (lane & 31), 2 * ks + hh);
  int offb[4];
  int offbt[J][2];
  if constexpr (!NN) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) offb[ks] = swz_off<LK>(WTN * wn + (lane & 31), 2 * ks + hh);
  } else {
    const int g16 = (lane >> 4) & 1, q = (lane & 15) >> 2, pc = lane & 3;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int u = WTN / 32 * wn + j;
#pragma unroll
      for (int hi = 0; hi < 2; ++hi) {
        const int row = 4 * hh + q + 8 * hi;
        offbt[j][hi] = (u >> 2) * (64 * 128) +
                       swz_off<128>(row, 4 * (u & 3) + 2 * g16 + (pc >> 1)) + 4 * (pc & 1);
      }
    }
  }
  const int va = (threadIdx.x >> 3) * (int)p.lda * 2 + (threadIdx.x & 7) * 16;
  const int ra_row = T / 8 * (int)p.lda * 2;
  using ATile = RowTile<BM, T>;
  using BTileT = typename std::conditional<NN, ColTile<BN, T>, RowTile<BN, T>>::type;
  // per-tile operand sources (A rows m0.., B rows n0.. (NT) or columns n0.. (NN))
  struct Src {
    __amdgpu_buffer_rsrc_t ra, rb;
    int vb;
  };
  const int rb_row = NN ? (int)p.ldb * 2 : T / 8 * (int)p.ldb * 2;
  const int rb_step = NN ? LK * (int)p.ldb * 2 : LK * 2;
  const __amdgpu_buffer_rsrc_t rb_nn = rows_rsrc_l(B, p.ldb, 0, p.K);
  auto source = [&](int L) {
    Src sr;
    const int m0 = (L / tilesN) * BM, n0 = (L % tilesN) * BN;
    sr.ra = rows_rsrc_l(A, p.lda, m0, min(p.M, m0 + BM));
    if constexpr (!NN) {
      sr.rb = rows_rsrc_l(B, p.ldb, n0, n0 + BN);
      sr.vb = (threadIdx.x >> 3) * (int)p.ldb * 2 + (threadIdx.x & 7) * 16;
    } else {
      sr.rb = rb_nn;
      sr.vb = (threadIdx.x >> 4) * (int)p.ldb * 2 + (n0 + (threadIdx.x & 15) * 8) * 2;
    }
    return sr;
  };
  auto load_a = [&](ATile& t, const Src& sr, int step) { t.load(sr.ra, va, ra_row, step * LK * 2); };
  auto load_b = [&](BTileT& t, const Src& sr, int step) { t.load(sr.rb, sr.vb, rb_row, step * rb_step); };

  f32x16_t acc[I][J];
  auto compute = [&](int it) {
    const bf16_t* As = lds + (it & 1) * STG;
    const bf16_t* Bs = As + A_E;
#pragma unroll
    for (int ks = 0; ks < LK / 16; ++ks) {
      bf16x8_t fa[I], fb[J];
#pragma unroll
      for (int i = 0; i < I; ++i) fa[i] = lds_row8(As + offa[ks] + 32 * i * LK);
      if constexpr (!NN) {
#pragma unroll
        for (int j = 0; j < J; ++j) fb[j] = lds_row8(Bs + offb[ks] + 32 * j * LK);
      } else {
#pragma unroll
        for (int j = 0; j < J; ++j) fb[j] = tr_operand(Bs + 16 * ks * 128, offbt[j][0], offbt[j][1]);
      }
#pragma unroll
      for (int i = 0; i < I; ++i)
#pragma unroll
        for (int j = 0; j < J; ++j) acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
    }
  };

  int tile = blockIdx.x;
  int L = remap(tile);
  Src cur = source(L);
  ATile a0, a1;
  BTileT b0, b1;
  load_a(a0, cur, 0);
  load_b(b0, cur, 0);
  load_a(a1, cur, 1);
  load_b(b1, cur, 1);
  const bf16_t* bias = reinterpret_cast<const bf16_t*>(p.bias);
  bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
  bf16_t* aux = reinterpret_cast<bf16_t*>(p.aux);
  float* ep = reinterpret_cast<float*>(smem) + w * (32 * EP_LD);
  const int cc = (lane & 7) * 8;

  while (true) {  // workgroup-uniform trip count
    const int m0 = (L / tilesN) * BM, n0 = (L % tilesN) * BN;
#pragma unroll
    for (int i = 0; i < I; ++i)
#pragma unroll
      for (int j = 0; j < J; ++j) acc[i][j] = zero16();
    a0.store(lds);
    b0.store(lds + A_E);
    __syncthreads();
    auto step = [&](int it, ATile& al, BTileT& bl, ATile& as, BTileT& bs) {
      load_a(al, cur, it + 2);
      load_b(bl, cur, it + 2);
      __builtin_amdgcn_sched_barrier(0);
      compute(it);
      __builtin_amdgcn_sched_barrier(0);
      bf16_t* nx = lds + ((it + 1) & 1) * STG;
      as.store(nx);
      bs.store(nx + A_E);
      __syncthreads();
    };
    int it = 0;
    for (; it + 1 < nsteps; it += 2) {
      step(it, a0, b0, a1, b1);
      step(it + 1, a1, b1, a0, b0);
    }
    if (nsteps & 1) compute(it);
    // next tile's first two steps go in flight now, under this tile's epilogue
    const int next = tile + G;
    const bool more = next < nwg;
    int Ln = L;
    Src nsr = cur;
    if (more) {
      Ln = remap(next);
      nsr = source(Ln);
      load_a(a0, nsr, 0);
      load_b(b0, nsr, 0);
      load_a(a1, nsr, 1);
      load_b(b1, nsr, 1);
    }
    // ---- epilogue (as linear_kernel) ----
    const int n = n0 + WTN * wn + cc;
    float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_ACT) {
      if (bias) Vec8<bf16_t>::load(bias + n, bv);
    }
#pragma unroll
    for (int i = 0; i < I; ++i) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < J; ++j)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg)
          ep[acc_row(reg, hh) * EP_LD + 32 * j + (lane & 31)] = acc[i][j][reg];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (lane >> 3) + 8 * r;
        const int m = m0 + WTM * wm + 32 * i + rr;
        if (m < p.M) {
          float v[8];
          Vec8<float>::load(ep + rr * EP_LD + cc, v);
          if constexpr (EPI == EPI_BIAS) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += bv[e];
          } else if constexpr (EPI == EPI_BIAS_ACT) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = bf2f(f2bf(v[e] + bv[e]));
            Vec8<bf16_t>::store(aux + (int64_t)m * p.ldaux + n, v);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = act_ft<ACT>(v[e]);
          } else if constexpr (EPI == EPI_DACT) {
            float a[8];
            Vec8<bf16_t>::load(aux + (int64_t)m * p.ldaux + n, a);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= act_dt<ACT>(a[e]);
          }
          Vec8<bf16_t>::store(C + (int64_t)m * p.ldc + n, v);
        }
      }
    }
    if (!more) break;
    __syncthreads();  // every wave's slab reads are done before stage 0 is overwritten
    tile = next;
    L = Ln;
    cur = nsr;
  }
}

template <int BM, int BN, int WGM, int WGN>
constexpr size_t lin_lds() {
  const size_t stages = (size_t)2 * (BM + BN) * LK * sizeof(bf16_t);
  const size_t slab = (size_t)WGM * WGN * 32 * EP_LD * sizeof(float);
  return stages > slab ? stages : slab;
}

template <bool NN, int BM, int BN, int WGM, int WGN>
int launch_cfg(const LinearParams& p, hipStream_t s) {
  const int nwg = ((p.M + BM - 1) / BM) * (p.N / BN);
  constexpr size_t lds = lin_lds<BM, BN, WGM, WGN>();
  const dim3 grid(nwg), block(64 * WGM * WGN);
#define BCFL_LIN(E, A) \
  hipLaunchKernelGGL((linear_kernel<NN, E, A, BM, BN, WGM, WGN>), grid, block, lds, s, p)
  if (p.epi == EPI_STORE) {
    BCFL_LIN(EPI_STORE, 0);
  } else if (p.epi == EPI_BIAS) {
    BCFL_LIN(EPI_BIAS, 0);
  } else if (p.epi == EPI_BIAS_ACT || p.epi == EPI_DACT) {
    const bool fwd = p.epi == EPI_BIAS_ACT;
    switch (p.act) {
      case ACT_GELU: if (fwd) BCFL_LIN(EPI_BIAS_ACT, ACT_GELU); else BCFL_LIN(EPI_DACT, ACT_GELU); break;
      case ACT_GELU_TANH:
        if (fwd) BCFL_LIN(EPI_BIAS_ACT, ACT_GELU_TANH); else BCFL_LIN(EPI_DACT, ACT_GELU_TANH);
        break;
      case ACT_RELU: if (fwd) BCFL_LIN(EPI_BIAS_ACT, ACT_RELU); else BCFL_LIN(EPI_DACT, ACT_RELU); break;
      default: return -5;  // other activations: host uses the unfused path
    }
  } else {
    return -4;
  }
#undef BCFL_LIN
  return 0;
}

template <bool NN>
int launch_persist(const LinearParams& p, hipStream_t s) {
  const int nwg = ((p.M + 127) / 128) * (p.N / 128);
  const int slots = 512;  // 2 workgroups per CU x 256 CUs; a multiple of 8 (tile keeps its XCD)
  const int g = nwg < slots ? nwg : slots;
  constexpr size_t lds = lin_lds<128, 128, 2, 2>();
#define BCFL_LINP(E, A) \
  hipLaunchKernelGGL((linear_persist_kernel<NN, E, A>), dim3(g), dim3(256), lds, s, p)
  if (p.epi == EPI_STORE) {
    BCFL_LINP(EPI_STORE, 0);
  } else if (p.epi == EPI_BIAS) {
    BCFL_LINP(EPI_BIAS, 0);
  } else if (p.epi == EPI_BIAS_ACT || p.epi == EPI_DACT) {
    const bool fwd = p.epi == EPI_BIAS_ACT;
    switch (p.act) {
      case ACT_GELU: if (fwd) BCFL_LINP(EPI_BIAS_ACT, ACT_GELU); else BCFL_LINP(EPI_DACT, ACT_GELU); break;
      case ACT_GELU_TANH:
        if (fwd) BCFL_LINP(EPI_BIAS_ACT, ACT_GELU_TANH); else BCFL_LINP(EPI_DACT, ACT_GELU_TANH);
        break;
      case ACT_RELU: if (fwd) BCFL_LINP(EPI_BIAS_ACT, ACT_RELU); else BCFL_LINP(EPI_DACT, ACT_RELU); break;
      default: return -5;
    }
  } else {
    return -4;
  }
#undef BCFL_LINP
  return 0;
}

// The 8-phase LDS-DMA kernel (gemm8.hip) takes every shape it supports (N % 256, K % 128): it
// matches or beats hipBLASLt on the BERT projections (profiles/g8_v1_vs_hipblaslt.json); the
// register-staged kernels below remain for the other shapes. BCFL_G8=0 disables it.
template <bool NN>
int try_g8(const LinearParams& p, hipStream_t s) {
  static const bool on = [] {
    const char* e = std::getenv("BCFL_G8");
    return !(e && e[0] == '0');
  }();
  if (!on || p.tile >= 0) return 1;
  G8Params g{p.A, p.B, p.C, p.lda, p.ldb, p.ldc, p.M, p.N, p.K};
  g.b_col = NN ? 1 : 0;
  g.epi = p.epi;
  g.act = p.act;
  g.bias = p.bias;
  g.aux = p.aux;
  g.ldaux = p.ldaux;
  g.kc = p.K;
  g.bm = g8_auto_bm(p.M, p.N, 1);
  if (g8_supported(g) != 0) return 1;
  return launch_g8(g, s);
}

template <bool NN>
int launch_linear_t(const LinearParams& p, hipStream_t s) {
  if (p.M == 0 && p.N % 128 == 0) return 0;
  if (p.M > 0 && try_g8<NN>(p, s) == 0) return 0;
  if (p.epi == EPI_ACCUM) return -4;
  if (p.N % 128 || p.K % LK || p.M < 0 || p.K <= 0) return -1;
  if (p.lda % 8 || p.ldb % 8 || p.ldc % 8 || p.ldaux % 8) return -2;
  if ((p.epi == EPI_BIAS_ACT || p.epi == EPI_DACT) && (!p.aux || p.ldaux <= 0)) return -3;
  if (p.M == 0) return 0;
  // 256 x 256 tiles (8 waves, 128 x 64 per wave: 25 % fewer LDS reads per MFMA, half the
  // global->LDS traffic per FLOP) pay off on long reductions (K >= 2048: +30 % at 4096^3) when
  // the grid still covers the chip; at K = 768 the 128 x 128 tile is faster
  // (profiles/linear_gemm_vs_hipblaslt.md)
  int tile = p.tile;
  if (tile < 0) {
    const int64_t t256 = (int64_t)((p.M + 255) / 256) * (p.N / 256);
    tile = (p.N % 256 == 0 && p.K >= 2048 && t256 >= 240) ? 1 : 0;
  }
  if (tile == 1 && p.N % 256 == 0) return launch_cfg<NN, 256, 256, 2, 4>(p, s);
  static const bool persist = [] {
    const char* e = std::getenv("BCFL_LINEAR_PERSIST");
    return !(e && e[0] == '0');
  }();
  if (persist) return launch_persist<NN>(p, s);
  return launch_cfg<NN, 128, 128, 2, 2>(p, s);
}

}  // namespace

int launch_linear_nt(const LinearParams& p, hipStream_t s) { return launch_linear_t<false>(p, s); }
int launch_linear_nn(const LinearParams& p, hipStream_t s) { return launch_linear_t<true>(p, s); }

}  // namespace bcfl
