// g8: the dense-layer GEMMs of every BERT / ALBERT / DistilBERT / Llama projection on MFMA with an
// 8-phase, LDS-DMA (buffer_load ... lds) software pipeline (SURVEY.md §2.6 K3 / K5 / K6 / K7 and
// the K9 weight gradient; reference hot path: the HF BertSelfAttention / BertSelfOutput /
// BertIntermediate / BertOutput dense layers printed at
// src/Serverlesscase/serverless_cancer_classification_with_BioBERT.ipynb:526-569).
//
//   C[M, N] = sum_k A(m, k) B(k, n)     (+ fused epilogue)
//
// Operand storage (the "kind" of each operand, compile-time):
//   A ROW: A(m, k) = A[m * lda + k]  (activations x / dY)    A COL: A(m, k) = A[k * lda + m]  (G^T)
//   B ROW: B(k, n) = B[n * ldb + k]  (nn.Linear weight, fwd) B COL: B(k, n) = B[k * ldb + n]  (W in
//                                                              dgrad, X in the weight gradient)
// so forward = (ROW, ROW), input gradient = (ROW, COL), weight gradient = (COL, COL).
//
// Block tile BM x 256 (BM = 256 or 128), 64-deep K-tiles, 8 waves (2 M x 4 N). Each K-tile is
// staged as four half-tiles (A rows [0, BM/2) / [BM/2, BM), B cols [0, 128) / [128, 256)) in two
// LDS buffers (even / odd K-tile). A wave owns rows {a BM/2 + wr BM/4 + [0, BM/4)} and columns
// {b 128 + wc 32 + [0, 32)} for a, b in {0, 1}, i.e. one quadrant (a, b) per half-tile pair, so a
// K-tile is consumed in 4 phases:
//     phase 1: ds_read B_lo -> B0, A_lo -> A   MFMA quadrant (0, 0)
//     phase 2: ds_read B_hi -> B1              MFMA quadrant (0, 1)
//     phase 3: ds_read A_hi -> A               MFMA quadrant (1, 1)
//     phase 4: (registers only)                MFMA quadrant (1, 0)
// Each half-tile of a buffer is last read in a known phase (B_lo 1, A_lo 1, B_hi 2, A_hi 3), so it
// is re-staged with the K-tile two ahead as soon as the reads are retired: B_lo in phase 2 (its
// reads are retired by the lgkmcnt before phase 1's barrier), A_lo in 3, B_hi in 4, A_hi in the
// next tile's phase 1. One LDS-DMA half-tile is issued per phase and three stay in flight across
// barriers: the only vmcnt waits are the counted ones in phases 4 / 8 (never vmcnt(0) in the main
// loop) and the barriers are raw s_barrier (a __syncthreads() would drain the DMA queue).
// The two wave rows run staggered by one barrier (ping-pong): one group's MFMA cluster overlaps
// the other group's LDS reads and DMA issue. cdna_hip_programming.md §5 "The 256² 8-phase
// template" (rules T2-T5), re-derived here for three operand layouts.
//
// LDS images (one __shared__ array, 128 KiB at BM = 256), written lane-linearly by the DMA; the
// bank-conflict swizzles are applied on the per-lane SOURCE address and on the read address:
//   ROW half-tile [H rows][64 k], 128-B rows:  16-B chunk c of row r at chunk c ^ ((r >> 1) & 7)
//     -> the v_mfma_f32_16x16x32_bf16 operand read (lane: row l & 15, chunk 4s + (l >> 4),
//        ds_read_b128) hits 16 distinct bank slots in each of its four 16-lane groups;
//   COL half-tile [64 k][128 idx], 256-B rows: chunk c of k-row r at c ^ ((r & 3) << 2 | (r >> 2) & 3)
//     -> the operand is read with two ds_read_b64_tr_b16 hardware transposes (k = 8G..8G+3,
//        8G+4..8G+7 of lane group G), conflict-free per 32-lane half.
// Epilogues (EPI_*) are applied while the 256 x BN tile streams out through a per-wave LDS slab
// (16-byte row segments): bias, bias + activation (pre-activation saved), activation' (dgrad of
// the layer after an activation), accumulate into C (beta = 1), or fp32 split-K partials.
#include <cstdlib>

#include "act.h"
#include "common.h"
#include "kernels.h"
#include "lds_dma.h"

namespace bcfl {
namespace {

constexpr int T8 = 512;  // threads per workgroup (8 waves)
constexpr int BN8 = 256;

typedef __attribute__((ext_vector_type(8))) short g8_s16x8_t;

__device__ __forceinline__ f32x4_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// k-row image swizzle of a COL half-tile with 128 columns (16 chunks of 16 B per row)
__device__ __forceinline__ int colswz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

template <int BM, bool ACOL, bool BCOL, int EPI, int ACT>
struct G8 {
  static constexpr int HA = BM / 2, HB = BN8 / 2;   // half-tile extents (rows of A / cols of B)
  static constexpr int LA = HA / 64, LB = HB / 64;  // LDS-DMA instructions per thread per half-tile
  static constexpr int QM = HA / 2, QN = HB / 4;    // wave quadrant: QM rows x QN cols
  static constexpr int TI = QM / 16, TJ = QN / 16;  // 16 x 16 MFMA tiles per quadrant
  static constexpr int HBYTES_A = HA * 128, HBYTES_B = HB * 128;
  static constexpr int BUF = 2 * HBYTES_A + 2 * HBYTES_B;  // one K-tile (A + B)
  static constexpr int LDS = 2 * BUF;
  static constexpr int VMN = 2 * LB + LA;  // DMA instructions of the 3 half-tiles left in flight
  // reads per phase: ROW frag = 1 ds_read_b128, COL frag = 2 ds_read_b64_tr_b16
  static constexpr int RA0 = TI * 2 * (ACOL ? 2 : 1);
  static constexpr int RA = RA0 < 15 ? RA0 : 15;  // lgkmcnt is a 4-bit field
  static_assert(HA % 64 == 0 && TI >= 1 && TJ >= 1, "tile geometry");
  static_assert(!ACOL || HA == 128, "COL A operand needs 128-row half-tiles");
};

struct G8Lane {
  int lane, w, wr, wc;
};

// ---- one operand ----------------------------------------------------------------------------
// DMA: half-tile h of K-tile kt -> LDS byte base `dst`. ROW: idx = j*512 + tid -> row idx >> 3,
// LDS chunk idx & 7 holds source chunk (idx & 7) ^ ((row >> 1) & 7). COL (128 idx per k-row):
// k-row idx >> 4, LDS chunk idx & 15 holds source chunk (idx & 15) ^ colswz(k-row).
// TAIL: a second reduction segment (K-tiles kt >= kt0 come from another matrix of the same kind,
// e.g. the LoRA factors appended to the base projection's reduction: C = A B + A2 B2).
template <bool COL, int H, bool TAIL = false>
struct G8Op {
  static constexpr int L = H / 64;
  __amdgpu_buffer_rsrc_t rs;
  int voff[2][L];  // per half: per-thread source byte offsets (k-tile 0 of the segment)
  int kbytes;      // source bytes per K-tile
  // tail segment (TAIL): its operand is set up in place of the base segment's when the first
  // K-tile >= kt0 is issued (per operand the issue order is non-decreasing in K-tile: A_hi(t + 1),
  // A_lo(t + 2), A_hi(t + 2), ...), so it costs no extra VGPRs in the pipelined loop
  const bf16_t* base2;
  int64_t ld2;
  int i02, nv2, ke2, kt0, ktb, hoff2;
  int tid_;

  // ROW: base = rows [i0, i0 + n_rows) of a [*, ld] matrix, K range starts at k0 (elements);
  //      half-tile 1 starts `hoff` rows below half-tile 0 (H; the paired block's offset for the
  //      SwiGLU gate|up tiles)
  // COL: base = k-rows [k0, k_end) of a [*, ld] matrix, columns from i0
  __device__ __forceinline__ void init(const bf16_t* base, int64_t ld, int i0, int n_valid, int k0,
                                       int k_end, int tid, int hoff = H) {
    if constexpr (!COL) {
      rs = buf_rsrc(base, ((int64_t)i0 * ld + k0) * 2, (int64_t)n_valid * ld * 2 - (int64_t)k0 * 2);
      kbytes = 64 * 2;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < L; ++j) {
          const int idx = j * T8 + tid;
          const int r = (idx >> 3);
          const int c = (idx & 7) ^ ((r >> 1) & 7);
          voff[h][j] = (int)((int64_t)(h * hoff + r) * ld * 2) + c * 16;
        }
    } else {
      rs = buf_rsrc(base, (int64_t)k0 * ld * 2, (int64_t)(k_end - k0) * ld * 2);
      kbytes = (int)(64 * ld * 2);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < L; ++j) {
          const int idx = j * T8 + tid;
          const int r = idx >> 4;
          const int c = (idx & 15) ^ colswz(r);
          voff[h][j] = (int)((int64_t)r * ld * 2) + (i0 + h * H + c * 8) * 2;
        }
    }
    if constexpr (TAIL) ktb = 0;
  }
  // the tail segment: K-tiles [ktiles0, ...) read `base` from its k 0 (COL: k-rows [0, k_end),
  // rows past k_end zero-filled by the range check; ROW: zero-padded columns)
  __device__ __forceinline__ void init2(const bf16_t* base, int64_t ld, int i0, int n_valid,
                                        int k_end, int tid, int ktiles0, int hoff = H) {
    if constexpr (TAIL) {
      base2 = base;
      ld2 = ld;
      i02 = i0;
      nv2 = n_valid;
      ke2 = k_end;
      kt0 = ktiles0;
      tid_ = tid;
      hoff2 = hoff;
    }
  }
  // issue the DMA of half-tile h of K-tile kt into LDS byte offset dst (wave w's 1-KiB pieces)
  __device__ __forceinline__ void dma(char* smem, int dst, int h, int kt, int w) {
    if constexpr (TAIL) {
      if (kt >= kt0 && ktb == 0) {  // workgroup-uniform, once per tile
        init(base2, ld2, i02, nv2, 0, ke2, tid_, hoff2);
        ktb = kt0;
      }
      kt -= ktb;
    }
    // the K-tile offset goes into the per-lane offset (VGPR): the range check, which zero-fills
    // k-rows past the split end, covers it
    const int ko = kt * kbytes;
#pragma unroll
    for (int j = 0; j < L; ++j) dma16(rs, smem + dst + j * (T8 * 16) + w * 1024, voff[h][j] + ko);
  }
};

// read offsets of one operand's MFMA fragments inside a half-tile (bytes)
//   ROW: frag (16-row block at `base_idx`, k-step s): lane l -> row l & 15, chunk 4s + (l >> 4)
//   COL: frag (16-idx block u, k-step s): two transposed reads, k-rows 32s + 8G + q (+4)
struct G8RowRd {
  int off[2];
  __device__ __forceinline__ void init(int lane) {
    const int r = lane & 15;
#pragma unroll
    for (int s = 0; s < 2; ++s) off[s] = r * 128 + (((4 * s + (lane >> 4)) ^ ((r >> 1) & 7)) << 4);
  }
  __device__ __forceinline__ bf16x8_t frag(const char* half, int idx0, int s) const {
    return *reinterpret_cast<const bf16x8_t*>(half + idx0 * 128 + off[s]);
  }
};

// The transposed reads are inline asm (ds_tr_read, lds_dma.h): hipcc does not count asm loads, so
// every phase waits lgkmcnt(0) itself after its first barrier and then marks the fragments
// written (g8_fence) before the MFMAs may read them.
// Transposed-read fragments of a COL operand: one 32-bit LDS base address per (16-idx block u,
// k-half h) and lane; the buffer / half-tile / k-step offset is the instruction's immediate, so
// the whole main loop addresses LDS with NU x 2 base registers.
template <int NU>  // NU 16-idx blocks per quadrant
struct G8ColRd {
  uint32_t base[NU][2];
  __device__ __forceinline__ void init(uint32_t region, int lane, int u0) {
    const int G = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kr = 8 * G + q + 4 * h;
        const int chunk = 2 * (u0 + u) + (p >> 1);
        base[u][h] = region + kr * 256 + ((chunk ^ colswz(kr)) << 4) + (p & 1) * 8;
      }
  }
  // HALF: byte offset of the half-tile inside the operand's LDS region; S: k-step (32 k-rows)
  template <int HALF, int S>
  __device__ __forceinline__ bf16x8_t frag(int u) const {
    const s16x4_t lo = ds_tr_read<HALF + S * 32 * 256>(base[u][0]);
    const s16x4_t hi = ds_tr_read<HALF + S * 32 * 256>(base[u][1]);
    const g8_s16x8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8_t, v);
  }
};

template <int N>
__device__ __forceinline__ void g8_fence(bf16x8_t (&f)[N][2]) {
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s) asm volatile("" : "+v"(f[i][s]));
}

template <int BM, bool ACOL, bool BCOL, int EPI, int ACT, bool PERSIST, bool TAIL = false>
__global__ __launch_bounds__(T8) void g8_kernel(G8Params p) {
  using C = G8<BM, ACOL, BCOL, EPI, ACT>;
  constexpr int TI = C::TI, TJ = C::TJ, QM = C::QM, QN = C::QN, HA = C::HA, HB = C::HB;
  constexpr bool PAIR = EPI == EPI_SWIGLU;
  static_assert(!PAIR || !BCOL, "SwiGLU pairing: ROW B (forward) only");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // ---- tile / split assignment (XCD-aware: each XCD walks a contiguous range of tiles) -------
  // The hardware puts workgroup b on XCD b % 8; XCD x owns logical tiles [xbase, xbase + xcnt).
  // One-shot grids (grid = tiles x splits) take logical tile xbase + b / 8. PERSIST grids
  // (a multiple of 8 workgroups, one per CU) walk their XCD's range with stride grid / 8, and
  // issue the next tile's prologue DMA before the current tile's epilogue (separate epilogue
  // slab): the DMA latency and the workgroup relaunch leave the critical path.
  const int tilesN = p.N / BN8;
  const int tilesM = (p.M + BM - 1) / BM;
  const int ntile = tilesM * tilesN;
  const int nwg = ntile * p.splits;
  const int b = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = b & 7;
  const int xbase = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int xcnt = q8 + (xcd < r8 ? 1 : 0);
  const int jstep = PERSIST ? (int)(gridDim.x >> 3) : xcnt;
  int jt = b >> 3;
  if (jt >= xcnt) return;  // workgroup-uniform (PERSIST grids larger than an XCD's share)

  struct TileC {
    int m0, n0, split, kbeg, kend, nt;
  };
  auto coords = [&](int jj) {
    const int L = xbase + jj;
    const int tile = L / p.splits;
    TileC c;
    c.split = L - tile * p.splits;
    c.m0 = (tile / tilesN) * BM;
    // SwiGLU forward: output tile t covers gate columns [128 t, 128 t + 128) (B half 0) and the
    // same up columns (B half 1, `pair` rows further): each wave holds gate and up of its columns
    c.n0 = (tile % tilesN) * (PAIR ? HB : BN8);
    c.kbeg = c.split * p.kc;
    c.kend = min(p.K, c.kbeg + p.kc);
    c.nt = ((c.kend - c.kbeg + 127) / 128) * 2;  // K-tiles, even
    if constexpr (TAIL) c.nt += p.K2 / 64;        // + the tail segment's (K2 % 128 == 0)
    return c;
  };
  TileC cur = coords(jt);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;

  // ---- operands ---------------------------------------------------------------------------
  G8Op<ACOL, HA, TAIL> opA;
  G8Op<BCOL, HB, TAIL> opB;
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.A);
  const bf16_t* B = reinterpret_cast<const bf16_t*>(p.B);
  auto init_ops = [&](const TileC& c) {
    if constexpr (!ACOL) opA.init(A, p.lda, c.m0, min(BM, p.M - c.m0), c.kbeg, c.kend, tid);
    else opA.init(A, p.lda, c.m0, 0, c.kbeg, c.kend, tid);
    if constexpr (PAIR) opB.init(B, p.ldb, c.n0, p.pair + HB, c.kbeg, c.kend, tid, p.pair);
    else if constexpr (!BCOL) opB.init(B, p.ldb, c.n0, min(BN8, p.N - c.n0), c.kbeg, c.kend, tid);
    else opB.init(B, p.ldb, c.n0, 0, c.kbeg, c.kend, tid);
    if constexpr (TAIL) {  // splits == 1: the base segment is K-tiles [0, K / 64)
      static_assert(!ACOL, "tail segment: ROW A operand only");
      const int kt0 = p.K / 64;
      opA.init2(reinterpret_cast<const bf16_t*>(p.A2), p.lda2, c.m0, min(BM, p.M - c.m0), p.K2, tid, kt0);
      if constexpr (PAIR)
        opB.init2(reinterpret_cast<const bf16_t*>(p.B2), p.ldb2, c.n0, p.pair + HB, p.K2, tid, kt0, p.pair);
      else if constexpr (!BCOL)
        opB.init2(reinterpret_cast<const bf16_t*>(p.B2), p.ldb2, c.n0, min(BN8, p.N - c.n0), p.K2, tid, kt0);
      else
        opB.init2(reinterpret_cast<const bf16_t*>(p.B2), p.ldb2, c.n0, 0, p.K2rows, tid, kt0);
    }
  };
  init_ops(cur);

  // LDS byte offsets: buffer q, A half a / B half b
  // LDS: A region [buffer 0 half 0 | b0 h1 | b1 h0 | b1 h1], then the B region the same way
  // (every half-tile of one operand within 64 KiB of its region base: 16-bit ds offsets)
  auto a_half = [&](int q, int a) { return (2 * q + a) * C::HBYTES_A; };
  auto b_half = [&](int q, int bh) { return 4 * C::HBYTES_A + (2 * q + bh) * C::HBYTES_B; };

  const uint32_t lds32 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  // read-side lane offsets
  G8RowRd rowrd;
  rowrd.init(lane);
  G8ColRd<TI> colA;
  G8ColRd<TJ> colB;
  if constexpr (ACOL) colA.init(lds32, lane, wr * QM / 16);
  if constexpr (BCOL) colB.init(lds32 + 4 * C::HBYTES_A, lane, wc * QN / 16);

  f32x4_t acc[2][2][TI][TJ];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bb = 0; bb < 2; ++bb)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[a][bb][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  bf16x8_t fa[TI][2], fb0[TJ][2], fb1[TJ][2];
  // bias gradient (A COL): wave column wc sums A half (wc & 1), k-half (wc >> 1) of each K-tile
  bool rs_on = ACOL && p.rowsum != nullptr && cur.n0 == 0;  // workgroup-uniform
  f32x4_t rsacc[ACOL ? TI : 1];
#pragma unroll
  for (int i = 0; i < (ACOL ? TI : 1); ++i) rsacc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;

  auto readA = [&](auto qc, auto ac) {
    constexpr int q = decltype(qc)::value, a = decltype(ac)::value;
    constexpr int OFF = (2 * q + a) * C::HBYTES_A;  // = a_half(q, a)
    const char* hp = smem + OFF;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      if constexpr (!ACOL) {
        fa[i][0] = rowrd.frag(hp, wr * QM + 16 * i, 0);
        fa[i][1] = rowrd.frag(hp, wr * QM + 16 * i, 1);
      } else {
        fa[i][0] = colA.template frag<OFF, 0>(i);
        fa[i][1] = colA.template frag<OFF, 1>(i);
      }
    }
  };
  auto readB = [&](auto qc, auto bc, bf16x8_t (&fb)[TJ][2]) {
    constexpr int q = decltype(qc)::value, bh = decltype(bc)::value;
    constexpr int OFF = (2 * q + bh) * C::HBYTES_B;  // offset inside the B region
    const char* hp = smem + 4 * C::HBYTES_A + OFF;
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      if constexpr (!BCOL) {
        fb[j][0] = rowrd.frag(hp, wc * QN + 16 * j, 0);
        fb[j][1] = rowrd.frag(hp, wc * QN + 16 * j, 1);
      } else {
        fb[j][0] = colB.template frag<OFF, 0>(j);
        fb[j][1] = colB.template frag<OFF, 1>(j);
      }
    }
  };
  auto mma = [&](int a, int bh, const bf16x8_t (&fb)[TJ][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[a][bh][i][j] = mfma16(fa[i][s], fb[j][s], acc[a][bh][i][j]);
    if constexpr (ACOL) {
      if (rs_on && bh == 0 && a == (wc & 1)) {  // sum_k A(m, k) = (A . ones)(m, *)
        if (wc >> 1) {
#pragma unroll
          for (int i = 0; i < TI; ++i) rsacc[i] = mfma16(fa[i][1], ones, rsacc[i]);
        } else {
#pragma unroll
          for (int i = 0; i < TI; ++i) rsacc[i] = mfma16(fa[i][0], ones, rsacc[i]);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  // after a phase's first barrier: its LDS reads have landed (asm transposed reads are not
  // counted by the compiler, so wait explicitly and mark the fragments written)
  auto landed = [&](bf16x8_t (&fb)[TJ][2], bool a_read) {
    if constexpr (ACOL || BCOL) {
      lgk_wait<0>();
      if constexpr (BCOL) g8_fence(fb);
      if constexpr (ACOL) {
        if (a_read) g8_fence(fa);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // DMA issue helpers (half-tiles of buffer q with K-tile kt)
  auto dmaA = [&](int q, int a, int kt) { opA.dma(smem, a_half(q, a), a, kt, w); };
  auto dmaB = [&](int q, int bh, int kt) { opB.dma(smem, b_half(q, bh), bh, kt, w); };

  // ---- prologue: K-tile 0 (all four half-tiles) + K-tile 1 (B_lo, A_lo, B_hi) ---------------
  auto prologue = [&]() {
    dmaB(0, 0, 0);
    dmaA(0, 0, 0);
    dmaB(0, 1, 0);
    dmaA(0, 1, 0);
    dmaB(1, 0, 1);
    dmaA(1, 0, 1);
    dmaB(1, 1, 1);
  };
  prologue();
  vm_wait<C::VMN>();  // K-tile 0 landed (this wave's pieces) ...
  BCFL_BAR();           // ... and every wave's
  if (wr == 1) BCFL_BAR();  // stagger: the second wave row runs one barrier behind

  // one K-tile in buffer Q: 4 phases. `full`: issue the DMAs of the K-tiles two ahead.
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  auto ktile = [&](auto Qc, int t, bool full) {
    constexpr int Q = decltype(Qc)::value;
    using IQ = std::integral_constant<int, Q>;
    // phase 1: B_lo -> fb0, A_lo -> fa; DMA A_hi of the other buffer (K-tile t + 1)
    readB(IQ{}, I0{}, fb0);
    __builtin_amdgcn_sched_barrier(0);
    readA(IQ{}, I0{});
    if (Q == 0 || full) dmaA(1 - Q, 1, t + 1);
    lgk_wait<C::RA>();  // B_lo reads retired before the barrier (B_lo is re-staged in phase 2)
    BCFL_BAR();
    landed(fb0, true);
    mma(0, 0, fb0);
    BCFL_BAR();
    // phase 2: B_hi -> fb1; DMA B_lo (K-tile t + 2)
    readB(IQ{}, I1{}, fb1);
    if (full) dmaB(Q, 0, t + 2);
    BCFL_BAR();
    landed(fb1, false);
    mma(0, 1, fb1);
    BCFL_BAR();
    // phase 3: A_hi -> fa; DMA A_lo (t + 2)
    readA(IQ{}, I1{});
    if (full) dmaA(Q, 0, t + 2);
    BCFL_BAR();
    landed(fb1, true);
    mma(1, 1, fb1);
    BCFL_BAR();
    // phase 4: DMA B_hi (t + 2); retire everything but the last three half-tiles
    if (full) {
      dmaB(Q, 1, t + 2);
      vm_wait<C::VMN>();
    } else {
      vm_wait<0>();
    }
    BCFL_BAR();
    mma(1, 0, fb0);
    BCFL_BAR();
  };

  // ---- epilogue of tile c: per-wave LDS slab, 16-byte row segments --------------------------
  // (PERSIST: the slab sits past the operand buffers, which the next tile's prologue fills)
  constexpr int LDF = QN + 4;  // slab row stride (floats)
  float* slab = reinterpret_cast<float*>(smem + (PERSIST ? C::LDS : 0)) + w * (QM * LDF);
  constexpr int LPR = QN / 8;           // lanes per slab row
  constexpr int RPP = 64 / LPR;         // rows per pass
  const int rr0 = lane / LPR, cc = (lane % LPR) * 8;
  bf16_t* Cp = reinterpret_cast<bf16_t*>(p.C);
  bf16_t* aux = reinterpret_cast<bf16_t*>(p.aux);
  const bf16_t* bias = reinterpret_cast<const bf16_t*>(p.bias);
  // bias of the tile's columns, loaded before the next tile's prologue DMA is issued (a load
  // issued after it would make the compiler drain that DMA before the first bias use)
  float bvs[2][8];
  auto load_bias = [&](const TileC& c) {
#pragma unroll
    for (int bh = 0; bh < 2; ++bh) {
#pragma unroll
      for (int e = 0; e < 8; ++e) bvs[bh][e] = 0.f;
      if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_ACT) {
        if (bias) Vec8<bf16_t>::load(bias + c.n0 + bh * HB + wc * QN + cc, bvs[bh]);
      }
    }
  };
  auto epilogue = [&](const TileC& c) {
    if constexpr (ACOL) {
      if (rs_on && (lane & 15) == 0) {  // column 0 of each 16 x 16 row-sum tile
        float* rsp = p.rowsum + (int64_t)(2 * c.split + (wc >> 1)) * p.M;
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = c.m0 + (wc & 1) * HA + wr * QM + 16 * i + (lane >> 4) * 4 + r;
            if (m < p.M) rsp[m] = rsacc[i][r];
          }
      }
    }
    // accumulator quadrant (a, bh) -> the wave's slab; 8 consecutive columns of slab row rr back
    auto put = [&](int a, int bh) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            slab[(16 * i + (lane >> 4) * 4 + r) * LDF + 16 * j + (lane & 15)] = acc[a][bh][i][j][r];
    };
    auto get = [&](int rr, float (&v)[8]) {
      if constexpr (PERSIST) {
        // asm reads: the compiler would drain the next tile's DMA (vmcnt(0)) in front of a
        // C++ LDS read while it is in flight
        const uint32_t ad = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)(slab + rr * LDF + cc);
        f32x4_t lo, hi;
        asm volatile("ds_read_b128 %0, %1" : "=v"(lo) : "v"(ad) : "memory");
        asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(hi) : "v"(ad) : "memory");
        lgk_wait<0>();
        reg_fence(lo);
        reg_fence(hi);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = lo[e];
          v[4 + e] = hi[e];
        }
      } else {
        Vec8<float>::load(slab + rr * LDF + cc, v);
      }
    };
    if constexpr (PAIR) {
      // SwiGLU forward: the wave's gate (bh 0) and up (bh 1) quadrants cover the same columns
      constexpr int NP = QM / RPP;
      const int n = c.n0 + wc * QN + cc;  // gate column; the up column is pair + n
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        float gv[NP][8];
        put(a, 0);
#pragma unroll
        for (int ps = 0; ps < NP; ++ps) get(rr0 + ps * RPP, gv[ps]);
        put(a, 1);
#pragma unroll
        for (int ps = 0; ps < NP; ++ps) {
          const int rr = rr0 + ps * RPP;
          const int m = c.m0 + a * HA + wr * QM + rr;
          float u[8];
          get(rr, u);
          if (m < p.M) {
            float o[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {  // the projection as stored (bf16), then silu(g) u
              const float g = bf2f(f2bf(gv[ps][e]));
              u[e] = bf2f(f2bf(u[e]));
              gv[ps][e] = g;
              o[e] = g / (1.f + __expf(-g)) * u[e];
            }
            Vec8<bf16_t>::store(aux + (int64_t)m * p.ldaux + n, gv[ps]);
            Vec8<bf16_t>::store(aux + (int64_t)m * p.ldaux + p.pair + n, u);
            Vec8<bf16_t>::store(Cp + (int64_t)m * p.ldc + n, o);
          }
        }
      }
      return;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int bh = 0; bh < 2; ++bh) {
        put(a, bh);
        const int n = c.n0 + bh * HB + wc * QN + cc;
        const float* bv = bvs[bh];
#pragma unroll
        for (int ps = 0; ps < QM / RPP; ++ps) {
          const int rr = rr0 + ps * RPP;
          const int m = c.m0 + a * HA + wr * QM + rr;
          float v[8];
          get(rr, v);
          if (m < p.M) {
            if constexpr (EPI == EPI_PARTIAL) {
              float* dst = p.part + ((int64_t)c.split * p.M + m) * p.ldc + n;
              Vec8<float>::store(dst, v);
            } else {
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
                float av[8];
                Vec8<bf16_t>::load(aux + (int64_t)m * p.ldaux + n, av);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] *= act_dt<ACT>(av[e]);
              } else if constexpr (EPI == EPI_RESID) {  // residual stream add (Llama x + o)
                float rv[8];
                Vec8<bf16_t>::load(aux + (int64_t)m * p.ldaux + n, rv);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] += rv[e];
              } else if constexpr (EPI == EPI_SWIGLU_BWD) {  // dA -> (d gate, d up)
                float gg[8], uu[8], du[8];
                Vec8<bf16_t>::load(aux + (int64_t)m * p.ldaux + n, gg);
                Vec8<bf16_t>::load(aux + (int64_t)m * p.ldaux + p.pair + n, uu);
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                  const float d = bf2f(f2bf(v[e]));  // dA as the unfused path stores it
                  const float sg = 1.f / (1.f + __expf(-gg[e]));
                  du[e] = d * (gg[e] * sg);
                  v[e] = d * uu[e] * sg * (1.f + gg[e] * (1.f - sg));
                }
                Vec8<bf16_t>::store(Cp + (int64_t)m * p.ldc + p.pair + n, du);
              } else if constexpr (EPI == EPI_ACCUM) {
                float ov[8];
                Vec8<bf16_t>::load(Cp + (int64_t)m * p.ldc + n, ov);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] += ov[e];
              }
              Vec8<bf16_t>::store(Cp + (int64_t)m * p.ldc + n, v);
            }
          }
        }
      }
  };

  while (true) {
    const int iters = cur.nt >> 1;
    for (int it = 0; it < iters - 1; ++it) {
      ktile(I0{}, 2 * it, true);
      ktile(I1{}, 2 * it + 1, true);
    }
    // last pair: the even tile's phase 1 still issues the odd tile's A_hi; no further DMA
    ktile(I0{}, cur.nt - 2, false);
    ktile(I1{}, cur.nt - 1, false);
    if (wr == 0) BCFL_BAR();  // close the stagger
    lgk_wait<0>();
    if constexpr (!PERSIST) {
      __syncthreads();
      load_bias(cur);
      epilogue(cur);
      break;
    } else {
      const int jn = jt + jstep;
      const bool more = jn < xcnt;  // workgroup-uniform
      load_bias(cur);
      BCFL_BAR();  // every wave is done reading the operand buffers
      TileC nxt = cur;
      if (more) {  // next tile's prologue in flight under this tile's epilogue
        nxt = coords(jn);
        init_ops(nxt);
        prologue();
      }
      epilogue(cur);
      if (!more) break;
      jt = jn;
      cur = nxt;
      rs_on = ACOL && p.rowsum != nullptr && cur.n0 == 0;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j) acc[a][bb][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      if constexpr (ACOL) {
#pragma unroll
        for (int i = 0; i < TI; ++i) rsacc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
      vm_wait<0>();  // the next tile's K-tiles 0 / 1 (and this epilogue's stores) have landed
      BCFL_BAR();
      if (wr == 1) BCFL_BAR();  // re-open the stagger
    }
  }
}

// persistent grid (one workgroup per CU, BM = 128 only: 96 KiB of operand buffers + the 36 KiB
// epilogue slab) when the launch has more tiles than CUs; BCFL_G8_PERSIST=0/1 overrides.
// Measured: BERT shapes 0-5 % per GEMM (profiles/g8_persistent_r3.json), one-client round
// 0.0922 -> 0.0913 s, 8-lane round 0.5635 -> 0.5604 s (3 / 2 interleaved reps)
// (The round-3 overlap-test failure first blamed on it was the dy / dres aliasing race fixed in
// ops._BDALN: scripts/overlap_diag.py showed the same two gradients off with it on and off.)
bool g8_persist_default = true;
// block rows pinned by the runtime (0 = choose per launch, g8_auto_bm): client lanes that run
// concurrently share the chip, so the tile with the best per-FLOP efficiency (256 rows) wins over
// the one that fills a lone launch's waves (8-lane bench 0.573-0.575 vs 0.583-0.593 s/round,
// profiles/bench_r5_gemm_ab.json)
int g8_bm_pinned = 0;

template <int BM, bool ACOL, bool BCOL, bool PERSIST>
int g8_dispatch_t(const G8Params& p, hipStream_t s, int nwg) {
  constexpr int SLAB = T8 / 64 * G8<BM, ACOL, BCOL, 0, 0>::QM * (G8<BM, ACOL, BCOL, 0, 0>::QN + 4) * 4;
  constexpr size_t lds = G8<BM, ACOL, BCOL, 0, 0>::LDS + (PERSIST ? SLAB : 0);
  const dim3 grid(PERSIST ? 256 : nwg), block(T8);
#define G8_L(E, A) hipLaunchKernelGGL((g8_kernel<BM, ACOL, BCOL, E, A, PERSIST>), grid, block, lds, s, p)
  switch (p.epi) {
    case EPI_STORE: G8_L(EPI_STORE, 0); break;
    case EPI_BIAS: G8_L(EPI_BIAS, 0); break;
    case EPI_ACCUM: G8_L(EPI_ACCUM, 0); break;
    case EPI_PARTIAL: G8_L(EPI_PARTIAL, 0); break;
    case EPI_BIAS_ACT:
    case EPI_DACT: {
      const bool fwd = p.epi == EPI_BIAS_ACT;
      switch (p.act) {
        case ACT_GELU: if (fwd) G8_L(EPI_BIAS_ACT, ACT_GELU); else G8_L(EPI_DACT, ACT_GELU); break;
        case ACT_GELU_TANH:
          if (fwd) G8_L(EPI_BIAS_ACT, ACT_GELU_TANH); else G8_L(EPI_DACT, ACT_GELU_TANH);
          break;
        case ACT_RELU: if (fwd) G8_L(EPI_BIAS_ACT, ACT_RELU); else G8_L(EPI_DACT, ACT_RELU); break;
        default: return -5;
      }
      break;
    }
    default: return -4;
  }
#undef G8_L
  return 0;
}

// tail-segment launches (the LoRA base + low-rank products of _LoRALinear): EPI_STORE, and
// EPI_RESID for the forward projections that feed the residual stream (o_proj, down_proj)
template <int BM, bool BCOL, bool PERSIST>
int g8_dispatch_tail(const G8Params& p, hipStream_t s, int nwg) {
  constexpr int SLAB = T8 / 64 * G8<BM, false, BCOL, 0, 0>::QM * (G8<BM, false, BCOL, 0, 0>::QN + 4) * 4;
  constexpr size_t lds = G8<BM, false, BCOL, 0, 0>::LDS + (PERSIST ? SLAB : 0);
  const dim3 grid(PERSIST ? 256 : nwg), block(T8);
  if (p.epi == EPI_STORE)
    hipLaunchKernelGGL((g8_kernel<BM, false, BCOL, EPI_STORE, 0, PERSIST, true>), grid, block, lds, s, p);
  else if (p.epi == EPI_RESID && !BCOL)
    hipLaunchKernelGGL((g8_kernel<BM, false, false, EPI_RESID, 0, PERSIST, true>), grid, block, lds, s, p);
  else if (p.epi == EPI_SWIGLU && !BCOL)
    hipLaunchKernelGGL((g8_kernel<BM, false, false, EPI_SWIGLU, 0, PERSIST, true>), grid, block, lds, s, p);
  else if (p.epi == EPI_SWIGLU_BWD && BCOL)
    hipLaunchKernelGGL((g8_kernel<BM, false, true, EPI_SWIGLU_BWD, 0, PERSIST, true>), grid, block, lds, s, p);
  else
    return -4;
  return 0;
}

template <int BM, bool ACOL, bool BCOL>
int g8_dispatch(const G8Params& p, hipStream_t s) {
  const int nwg = ((p.M + BM - 1) / BM) * (p.N / BN8) * p.splits;
  bool persist = g8_persist_default;
  if (const char* e = std::getenv("BCFL_G8_PERSIST")) persist = e[0] == '1';
  if constexpr (!ACOL) {
    static const bool force_tail = [] {  // diagnostic: plain STORE GEMMs on the tail kernel
      const char* e = std::getenv("BCFL_G8_TAIL_FORCE");
      return e && e[0] == '1';
    }();
    if (p.K2 > 0 || (force_tail && p.epi == EPI_STORE && p.splits == 1)) {
      if constexpr (BM == 128) {
        if (persist && nwg > 256) return g8_dispatch_tail<BM, BCOL, true>(p, s, nwg);
      }
      return g8_dispatch_tail<BM, BCOL, false>(p, s, nwg);
    }
  }
  if constexpr (BM == 128) {
    if (persist && nwg > 256) return g8_dispatch_t<BM, ACOL, BCOL, true>(p, s, nwg);
  }
  return g8_dispatch_t<BM, ACOL, BCOL, false>(p, s, nwg);
}

}  // namespace

extern int g8_wgrad_slots_pinned;
void set_g8_persistent(bool on) { g8_persist_default = on; }
void set_g8_block_rows(int bm) { g8_bm_pinned = (bm == 128 || bm == 256) ? bm : 0; }
void set_wgrad_slots(int slots) { g8_wgrad_slots_pinned = slots > 0 ? slots : 0; }

// Weight gradient dW[N, K] = G[M, N]^T X[M, K] on the 8-phase kernel: A = G (transposed reads),
// B = X (transposed reads), reduction over the M tokens split into S slices so the grid covers
// about a quarter of the chip (64 tile slots: the rest stays free for the dgrad / attention
// kernels running concurrently on the compute stream or other client lanes, and fewer slices
// mean less fp32 partial traffic); fp32 slice partials are summed by
// the deterministic reduce kernel (gemm.hip), which also sums the bias-gradient partials the
// n-tile-0 workgroups produce in the main loop (G^T . ones on MFMA: no second pass over G).
// tile slots pinned by the runtime (0 = 64): a rank that trains ONE client lane uses 96 — with the
// caller-thread backward the one-client round drops 2.9 % against 64 (3 interleaved
// reps, profiles/host_issue_r6.json); with concurrent lanes the chip is full and 64 stays
int g8_wgrad_slots_pinned = 0;

int wgrad_g8_splits(int M, int N, int K, int* Mc, int slots_override) {
  if (N % BN8 || K % BN8 || N <= 0 || M <= 0) return 0;
  static const int slots_env = [] {
    const char* e = std::getenv("BCFL_G8_WGRAD_SLOTS");
    const int v = e ? std::atoi(e) : 0;  // round 5, 1-client round: 64 slots 0.0927 s, 128 0.0942, 256 0.0968
    return v > 0 ? v : 0;
  }();
  const int slots = slots_override > 0 ? slots_override
                    : slots_env > 0 ? slots_env
                    : g8_wgrad_slots_pinned > 0 ? g8_wgrad_slots_pinned : 64;
  const int tiles = (N / BN8) * (K / BN8);  // 256 x 256 output tiles of dW[N, K]
  int S = (slots + tiles - 1) / tiles;
  const int maxS = M / 1024 > 0 ? M / 1024 : 1;  // keep >= 16 K-tiles per slice
  if (S > maxS) S = maxS;
  if (S < 1) S = 1;
  int mc = (M + S - 1) / S;
  mc = (mc + 127) / 128 * 128;
  *Mc = mc;
  return (M + mc - 1) / mc;
}

int launch_wgrad_g8(const WgradParams& p, hipStream_t s) {
  if (p.N % BN8 || p.K % BN8 || p.S < 1 || (p.S > 1 && !p.part)) return -1;
  G8Params g{p.G, p.X, p.S > 1 ? nullptr : p.out, p.ldg, p.ldx, p.S > 1 ? (int64_t)p.K : p.ldo,
             p.N, p.K, p.M};
  g.a_col = 1;
  g.b_col = 1;
  g.bm = 256;
  g.splits = p.S;
  g.kc = p.Mc;
  g.epi = p.S > 1 ? EPI_PARTIAL : EPI_STORE;
  g.part = p.part;
  g.rowsum = p.dbias ? p.dbias_part : nullptr;  // bias gradient fused: 2 partial rows per split
  int rc = launch_g8(g, s);
  if (rc) return rc;
  const int SB = 2 * p.S;
  if (p.S > 1 || p.dbias)
    return launch_wgrad_reduce(p.S > 1 ? p.part : nullptr, p.S, p.N, p.K, p.out, p.ldo,
                               p.dbias ? p.dbias_part : nullptr, p.dbias, s, SB);
  return 0;
}

int wgrad_g8_bias_parts(int S) { return 2 * S; }

// Block-row choice: a launch takes ceil(tiles / 256 CUs) waves of tiles, a 128-row tile takes
// ~0.57 of a 256-row tile's time (measured 1.15x less efficient per FLOP). Pick the smaller
// predicted time: on the BERT shapes M = 7680 with N = 768 / 2304 this is 128 (90 -> 180 tiles,
// 270 -> 540), at M = 11264 and on 4096^3 it is 256 (profiles/g8_v1_vs_hipblaslt.json).
int g8_auto_bm(int M, int N, int splits) {
  // BCFL_G8_BM=128/256 pins the block rows (A/B runs: with several client lanes sharing the chip
  // the wave-count argument below no longer holds and the per-FLOP efficiency decides)
  static const int env_bm = [] {
    const char* e = std::getenv("BCFL_G8_BM");
    const int v = e ? std::atoi(e) : 0;
    return (v == 128 || v == 256) ? v : 0;
  }();
  if (env_bm) return env_bm;
  if (g8_bm_pinned) return g8_bm_pinned;
  const int64_t t256 = (int64_t)((M + 255) / 256) * (N / BN8) * splits;
  const int64_t t128 = (int64_t)((M + 127) / 128) * (N / BN8) * splits;
  const double c256 = (double)((t256 + 255) / 256) * 256.0;
  const double c128 = (double)((t128 + 255) / 256) * 128.0 * 1.15;
  return c128 < c256 ? 128 : 256;
}

int g8_supported(const G8Params& p) {
  if (p.M <= 0 || p.N <= 0 || p.K <= 0) return -1;
  if (p.N % BN8) return -1;
  if (p.bm != 128 && p.bm != 256 && p.bm > 0) return -1;
  if (p.a_col && p.bm != 256) return -1;
  // ROW operands read whole 128-deep K pairs: every split must cover a multiple of 128
  if ((!p.a_col || !p.b_col) && (p.K % 128 || p.kc % 128)) return -2;
  if (p.splits < 1 || p.kc <= 0 || (int64_t)p.kc * (p.splits - 1) >= p.K) return -3;
  if (p.lda % 8 || p.ldb % 8 || p.ldc % 8) return -2;
  if ((p.epi == EPI_BIAS_ACT || p.epi == EPI_DACT) && (!p.aux || p.ldaux % 8)) return -3;
  if (p.epi == EPI_PARTIAL && !p.part) return -3;
  if ((p.epi == EPI_SWIGLU || p.epi == EPI_SWIGLU_BWD) && p.K2 <= 0) return -4;  // LoRA path only
  if (p.K2 > 0) {  // tail segment: one split, ROW A2, K2 a whole number of K-tile pairs
    if (p.a_col || p.splits != 1 || p.K2 % 128 || !p.A2 || !p.B2 || p.lda2 % 8 || p.ldb2 % 8) return -3;
    const bool aux_ok = p.aux && p.ldaux % 8 == 0;
    const bool pair_ok = p.pair > 0 && p.pair % 128 == 0 && aux_ok;
    if (!(p.epi == EPI_STORE || (p.epi == EPI_RESID && !p.b_col && aux_ok) ||
          (p.epi == EPI_SWIGLU && !p.b_col && pair_ok && p.N == 2 * p.pair) ||
          (p.epi == EPI_SWIGLU_BWD && p.b_col && pair_ok && p.N == p.pair)))
      return -4;
    if (p.b_col && (p.K2rows <= 0 || p.K2rows > p.K2)) return -3;
  }
  return 0;
}

int launch_g8(const G8Params& p_in, hipStream_t s) {
  G8Params p = p_in;
  if (p.bm <= 0) p.bm = p.a_col ? 256 : g8_auto_bm(p.M, p.N, p.splits);
  const int rc = g8_supported(p);
  if (rc) return rc;
  if (p.bm == 256) {
    if (!p.a_col && !p.b_col) return g8_dispatch<256, false, false>(p, s);
    if (!p.a_col && p.b_col) return g8_dispatch<256, false, true>(p, s);
    if (p.a_col && p.b_col) return g8_dispatch<256, true, true>(p, s);
    return g8_dispatch<256, true, false>(p, s);
  }
  if (!p.a_col && !p.b_col) return g8_dispatch<128, false, false>(p, s);
  if (!p.a_col && p.b_col) return g8_dispatch<128, false, true>(p, s);
  return -1;
}

}  // namespace bcfl
