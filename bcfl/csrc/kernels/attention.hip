// K4: varlen flash attention forward + backward on MFMA (gfx950), bf16 in, fp32 accumulate.
//
// What it replaces: HF BERT 4.35 runs attention EAGER in the reference (matmul -> /8 -> +mask ->
// softmax -> dropout -> matmul on [32,12,512,512] padded scores). Here rows are
// packed (cu_seqlens), padding is never computed, the S x S matrix is never materialised, and the
// dropout mask is regenerated from a counter hash in the backward pass.
//
// Geometry (all kernels): workgroup = 4 waves (256 threads); each wave owns 32 rows of the
// "outer" dimension and the workgroup shares 64-row tiles of the "inner" dimension through LDS.
//   fwd  : wave = 32 queries; K/V tiles of 64 keys staged in LDS.
//   dq   : wave = 32 queries; recompute S, P and dP against K/V tiles; dQ += dS K.
//   dkdv : wave = 32 keys (K, V fragments stay in registers); Q/dO tiles of 64 queries staged in
//          LDS; dV += P^T dO, dK += dS^T Q accumulate in registers over every query (and every
//          query head of the GQA group) — no atomics, deterministic.
//
// Pipelining (cdna_hip_programming.md T14 "issue early / write late" + double-buffered LDS): the
// global loads of tile i+1 are issued into registers BEFORE the MFMAs of tile i, written to the
// other LDS buffer after them, and ONE barrier per tile publishes it.
//
// MFMA mapping (v_mfma_f32_32x32x16_bf16, cdna_hip_programming.md §3): the score tile is computed
// SWAPPED in fwd/dq (S^T = K Q^T: the query is the accumulator COLUMN = lane, so the softmax row
// statistics are lane-local plus one xor-32 shuffle), and the accumulator feeds the next MFMA
// directly as its B operand ("accumulator as operand", k-order 16s+8(j>>2)+4h+(j&3)). The A
// operand of that second product needs the other tensor column-wise: it is read with
// ds_read_b64_tr_b16 (hardware transpose, T10) from a row-major LDS tile.
// LDS tiles are unpadded and 16-B-unit XOR-swizzled so both row reads and transposed reads are
// bank-conflict-free (see swz()).
//
// Softmax VALU trims (d = 64 makes attention VALU-heavy): the softmax scale is folded into the
// exp2 FMA (max taken on raw scores), key masking runs only on tiles that straddle the sequence
// end / causal diagonal, and the O rescale is skipped unless some row's running max grew.
//
// Dropout keep bits: the forward evaluates the counter hash (bcfl/ops/rng.py layout, one hash per
// 4 scores) and also WRITES the decisions as a bitmask (1 bit per score, ~6 MB per BERT layer);
// the dq and dkdv kernels read those bits back — 2 VALU ops per score (bit-field extract to a
// 0 / -1 mask + AND) instead of re-hashing in each of them.
#include <math.h>

#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "lds_dma.h"
#include "mfma_tiles.h"

namespace bcfl {
namespace {

constexpr int NWAVE = 4;
constexpr int ROWS = 32;              // rows per wave
constexpr int BLK = NWAVE * ROWS;     // 128 outer rows per workgroup
constexpr int TILE = 64;              // inner tile
constexpr int DROP_STRIDE = 8192;     // dropout element index = (tq*nh + h)*8192 + key_pos
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
// forward: the running row max m is only raised (O and l rescaled) when a tile's max exceeds it
// by more than this (log2 units): P <= 2^8 then, harmless for bf16 P and fp32 sums, and the rescale
// leaves the tile loop after the first tile or two
constexpr float RESCALE_LOG2 = 8.f;

// raw v_exp_f32: softmax arguments are <= 0 and a flushed denormal result is harmless, so skip
// exp2f's denormal range-reduction (cmp + 2 cndmask + add + ldexp per element).
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// broadcast lane (quad base + E) of each 4-lane quad (DPP quad_perm, no LDS round trip)
template <int E>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, E | (E << 2) | (E << 4) | (E << 6), 0xf, 0xf, false);
}

// 0 or -1 (all ones) from bit `pos` of w: AND it into a float's bits to apply a keep decision
__device__ __forceinline__ float keep_and(float v, uint32_t w, int pos) {
  return __int_as_float(__float_as_int(v) & __builtin_amdgcn_sbfe((int)w, pos, 1));
}

// Register-staged loader of two [TILE x HD] row tiles (e.g. K and V) gathered from token rows
// tok0 + row0 .. of two sources; rows >= L are zero-filled (so masked V rows can never be NaN).
template <int HD>
struct Stage2 {
  static constexpr int CPR = HD / 8;             // 16-byte chunks per row
  static constexpr int N = TILE * CPR / 256;     // chunks per thread per tensor
  uint4 a[N], b[N];
  __device__ __forceinline__ void load(const bf16_t* sa, int rsa, const bf16_t* sb, int rsb,
                                       int tok0, int row0, int L) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int idx = threadIdx.x + 256 * i;
      const int rr = idx / CPR, c = idx % CPR;
      const int row = row0 + rr;
      if (row < L) {
        a[i] = *reinterpret_cast<const uint4*>(sa + (size_t)(tok0 + row) * rsa + c * 8);
        b[i] = *reinterpret_cast<const uint4*>(sb + (size_t)(tok0 + row) * rsb + c * 8);
      } else {
        a[i] = make_uint4(0, 0, 0, 0);
        b[i] = make_uint4(0, 0, 0, 0);
      }
    }
  }
  __device__ __forceinline__ void store(bf16_t* da, bf16_t* db) const {  // swizzled tiles
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int idx = threadIdx.x + 256 * i;
      const int o = swz_off<HD>(idx / CPR, idx % CPR);
      *reinterpret_cast<uint4*>(da + o) = a[i];
      *reinterpret_cast<uint4*>(db + o) = b[i];
    }
  }
};

// ------------------------------------------------------------------------------------------------
// Work order. A launch is (head, unit) with unit = (sequence b, 128-row block); with a schedule
// (attn_schedule, built on the host with the batch) units come longest-sequence first, so the
// dispatcher starts the long blocks at once and back-fills with short ones (LPT order). Without
// one, every (b, block < ceil(max_s / 128)) in batch order.
__device__ __forceinline__ void attn_unit(const int* sched, int u, int max_s, int& b, int& blk) {
  if (sched) {
    const int e = sched[u];
    b = e >> 12;
    blk = e & 4095;
  } else {
    const int nb = (max_s + BLK - 1) / BLK;
    b = u / nb;
    blk = u - b * nb;
  }
}

// the partner half-wave's value (lane l ^ 32) as v_permlane32_swap: returns {lo-half image,
// hi-half image}; max / sum of a lane and its partner is op(r[0], r[1]) on every lane
__device__ __forceinline__ float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ uint32_t xor32_get(uint32_t x, int hh) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return hh ? r[0] : r[1];
}

// bit of key j (0..31 inside its 32-key block) in a keep word (kernels.h)
__device__ __forceinline__ int attn_mbit(int j) { return 8 * (j & 3) + ((j >> 3) & 3) + 4 * ((j >> 2) & 1); }

// keep flags of 4 scores from one 32-bit hash (byte e decides score e): bit 7 of byte e of the
// result is set iff byte e >= p8. SWAR: (x | 0x80) - p7 keeps each byte >= 1 (no borrow across
// bytes) and has bit 7 set iff (x & 0x7f) >= p7; combined with x's own bit 7 by OR (p8 < 128)
// or AND (p8 >= 128).
template <int DROP>  // 1: p8 < 128, 2: p8 >= 128
__device__ __forceinline__ uint32_t keep_flags4(uint32_t x, uint32_t p7x4) {
  const uint32_t t = (x | 0x80808080u) - p7x4;
  return DROP == 2 ? (x & t) : (x | t);
}

// ------------------------------------------------------------------------------------------------
// Forward. K / V tiles arrive by LDS-DMA (buffer_load ... lds, one 1-KiB piece per wave
// instruction, rows past the sequence end zero-filled by the buffer range check) into a 2-deep
// ring: tile i + 1 is in flight while tile i is computed, with one counted wait and one barrier
// per tile and no VGPR staging. Per tile and wave (32 queries x 64 keys, 32 scores per lane):
//   * S^T = K Q^T on MFMA (8 x 32x32x16), the query on the lane;
//   * p = exp2(s * scale * log2e - m); the running max m is raised (with the O / l rescale) only
//     when a tile's max exceeds it by RESCALE_LOG2 — in practice on the first tile only;
//   * dropout: one 32-bit hash per 4 scores; the 4 keep decisions are made at once (SWAR byte
//     compare, keep_flags4), expanded by two v_perm_b32 into bf16-pair masks ANDed into the
//     packed P, and folded into the keep bitmask with one bit-field insert;
//   * keep words are staged in LDS (a 16-word ring per query) and flushed with coalesced stores
//     every 8 tiles and at the end — no stores inside the tile loop;
//   * O += P V on MFMA with the accumulator as the B operand, V read by ds_read_b64_tr_b16 (asm,
//     immediate offsets: the compiler would drain the DMA queue before the builtin form).
template <int HD>
struct FwdCfg {
  static constexpr int CPR = HD / 8;              // 16-B chunks per K / V row
  static constexpr int TBYTES = TILE * HD * 2;    // one K or V tile
  static constexpr int PW = TBYTES / 1024 / NWAVE;  // DMA pieces per wave per tensor
  static constexpr int STG = 2 * TBYTES;          // K | V
  static constexpr int MW = 16;                   // keep words staged per query (8 tiles)
  static constexpr int MWS = 20;                  // padded LDS row (16-B aligned, 2-way writes)
  static constexpr int LDS = 2 * STG + NWAVE * ROWS * MWS * 4;
  static_assert(PW >= 1, "tile geometry");
};

template <int HD, int WPE, int DROP>  // DROP: 0 none, 1 p8 < 128, 2 p8 >= 128
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void attn_fwd_kernel(AttnParams p) {
  using C = FwdCfg<HD>;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  int b, qb;
  attn_unit(p.sched, blockIdx.y, p.max_s, b, qb);
  const int h = blockIdx.x;
  const int tok0 = p.cu[b];
  const int L = p.cu[b + 1] - tok0;
  const int q0 = qb * BLK;
  if (q0 >= L) return;
  const int lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int qw0 = q0 + wid * ROWS;
  const bool active = qw0 < L;
  const int hk = h / (p.nh / p.nkv);
  const int rs = (p.nh + 2 * p.nkv) * HD;
  const bf16_t* qkv = reinterpret_cast<const bf16_t*>(p.qkv);
  const int kend = p.causal ? min(L, q0 + BLK) : L;
  const int ntiles = (kend + TILE - 1) / TILE;

  // ---- K / V tile DMA: one resource over this sequence's rows --------------------------------
  const __amdgpu_buffer_rsrc_t rsrc = buf_rsrc(qkv, (int64_t)tok0 * rs * 2, (int64_t)L * rs * 2);
  int voff[2][C::PW];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int colbase = (x == 0 ? p.nh + hk : p.nh + p.nkv + hk) * HD;
#pragma unroll
    for (int i = 0; i < C::PW; ++i) {
      const int c = 64 * (wid + NWAVE * i) + lane;  // LDS chunk of the tile this lane fills
      const int row = c / C::CPR;
      const int u = (c % C::CPR) ^ swz<HD>(row);    // source chunk (the swizzle is an involution)
      voff[x][i] = row * rs * 2 + (colbase + 8 * u) * 2;
    }
  }
  auto dma = [&](int st, int k0) {
    const int ko = k0 * rs * 2;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int i = 0; i < C::PW; ++i)
        dma16(rsrc, smem + st * C::STG + x * C::TBYTES + (wid + NWAVE * i) * 1024, voff[x][i] + ko);
  };
  dma(0, 0);

  bf16x8_t qf[HD / 16];
  {
    const int qi = min(qw0 + r, L - 1);
    const bf16_t* qrow = qkv + (size_t)(tok0 + qi) * rs + h * HD;
#pragma unroll
    for (int s = 0; s < HD / 16; ++s) qf[s] = *reinterpret_cast<const bf16x8_t*>(qrow + 16 * s + 8 * hh);
  }
  f32x16_t o[HD / 32];
#pragma unroll
  for (int u = 0; u < HD / 32; ++u) o[u] = zero16();
  float m = 0.f, l = 0.f;  // m: row max of the first tile in the scaled log2 domain
  const float sl2 = p.scale * LOG2E;
  const float sd = DROP ? keep_scale(p.p8) : 1.f;
  const int myq = qw0 + r;
  const uint32_t cnt0 = ((uint32_t)((tok0 + myq) * p.nh + h) * (uint32_t)DROP_STRIDE + 4u * hh) >> 2;
  const uint32_t p7x4 = (p.p8 & 0x7fu) * 0x01010101u;

  // keep-word staging: this wave's [32 queries][MWS] words
  uint32_t* mst = reinterpret_cast<uint32_t*>(smem + 2 * C::STG) + wid * ROWS * C::MWS;
  int mflushed = 0;  // first keep word not yet flushed (multiple of MW)
  auto flush = [&](int wend) {  // words [mflushed, wend) of the wave's rows -> global
    const int row = lane >> 1, half = lane & 1;
    const int q = qw0 + row;
    if (q < L) {
      uint32_t* g = p.mask + (size_t)((tok0 + q) * p.nh + h) * p.mask_w + mflushed;
      const uint32_t* sp = mst + row * C::MWS;
#pragma unroll
      for (int i = 0; i < C::MW / 2; ++i) {
        const int wdx = (C::MW / 2) * half + i;
        if (mflushed + wdx < wend) g[wdx] = sp[wdx];
      }
    }
    mflushed = wend;
  };

  TileOffsets<HD> to;
  to.init(lane);
  const uint32_t lds32 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  uint32_t rowb[HD / 16];    // row-read bases (K tile of stage 0)
#pragma unroll
  for (int s2 = 0; s2 < HD / 16; ++s2) rowb[s2] = lds32 + 2 * to.row[s2];
  uint32_t trb[HD / 32][2];  // transposed-read bases (V tile of stage 0)
#pragma unroll
  for (int u = 0; u < HD / 32; ++u)
#pragma unroll
    for (int hi = 0; hi < 2; ++hi) trb[u][hi] = lds32 + C::TBYTES + 2 * to.tr[u][hi];

  vm_wait<0>();
  // Q has landed: tell the compiler (its waitcnt pass would otherwise keep treating the Q loads
  // as outstanding inside the loop and count the in-flight DMAs down before every Q MFMA)
#pragma unroll
  for (int s2 = 0; s2 < HD / 16; ++s2) reg_fence(qf[s2]);
  BCFL_BAR();

  auto tile = [&](auto stc, int it) {
    constexpr int ST = decltype(stc)::value;
    const int k0 = it * TILE;
    if (it > 0) {
      vm_wait<0>();  // this wave's pieces of tile it have landed ...
      BCFL_BAR();    // ... and every wave's; every wave is done with tile it - 1's buffer
    }
    if (it + 1 < ntiles) dma(ST ^ 1, k0 + TILE);
    if (!active || (p.causal && k0 > qw0 + ROWS - 1)) return;
    // S^T = K Q^T: K fragments by asm row reads (immediate offsets), half t = 0 consumed while
    // half 1 is still in flight
    bf16x8_t kf[2][HD / 16];
    auto kread = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      constexpr int OFF = ST * C::STG + 32 * t * HD * 2;
#pragma unroll
      for (int s = 0; s < HD / 16; ++s) kf[t][s] = ds_row_read<OFF>(rowb[s]);
    };
    kread(std::integral_constant<int, 0>{});
    kread(std::integral_constant<int, 1>{});
    f32x16_t sacc[2];
    lgk_wait<HD / 16>();
#pragma unroll
    for (int s = 0; s < HD / 16; ++s) reg_fence(kf[0][s]);
    sacc[0] = zero16();
#pragma unroll
    for (int s = 0; s < HD / 16; ++s) sacc[0] = mfma32(kf[0][s], qf[s], sacc[0]);
    lgk_wait<0>();
#pragma unroll
    for (int s = 0; s < HD / 16; ++s) reg_fence(kf[1][s]);
    sacc[1] = zero16();
#pragma unroll
    for (int s = 0; s < HD / 16; ++s) sacc[1] = mfma32(kf[1][s], qf[s], sacc[1]);
    if ((k0 + TILE > L) || (p.causal && k0 + TILE - 1 > qw0)) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int key = k0 + 32 * t + acc_row(reg, hh);
          if (key >= L || (p.causal && key > myq)) sacc[t][reg] = -INFINITY;
        }
    }
    {
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) mx = fmaxf(mx, sacc[t][reg]);
      mx = xor32_max(mx) * sl2;
      if (it == 0) {
        m = mx;
      } else if (__any(mx > m + RESCALE_LOG2)) {  // wave-uniform, rare after the first tile
        const float mn = fmaxf(m, mx);
        const float alpha = fexp2(m - mn);
        l *= alpha;
#pragma unroll
        for (int u = 0; u < HD / 32; ++u)
#pragma unroll
          for (int reg = 0; reg < 16; ++reg) o[u][reg] *= alpha;
        m = mn;
      }
    }
    uint32_t pw[4][4];  // P as bf16 pairs: fragment ks = 2t + (g4 >> 1), word 2 (g4 & 1) + e / 2
    uint32_t bits[2];
    float ls;
    {
      ls = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        bits[t] = 0u;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          float pv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            pv[e] = fexp2(fmaf(sacc[t][4 * g4 + e], sl2, -m));
            ls += pv[e];
          }
          uint32_t w0 = pack2bf(pv[0], pv[1]), w1 = pack2bf(pv[2], pv[3]);
          if constexpr (DROP != 0) {
            const uint32_t cnt = (cnt0 + (uint32_t)((k0 >> 2) + 8 * t + 2 * g4)) & 0x3fffffffu;  // uint32 wrap of the element index
            const uint32_t f = keep_flags4<DROP>(hash32(cnt, p.ka, p.kb), p7x4);
            const uint32_t fs = f << 8;
            // v_perm_b32 selectors 8..11 replicate bits 15 / 31 of the low and high source
            // dwords: {fs, f} -> flag 0 = sel 10, flag 1 = sel 8, flag 2 = sel 11, flag 3 = sel 9
            w0 &= __builtin_amdgcn_perm(fs, f, 0x08080A0Au);
            w1 &= __builtin_amdgcn_perm(fs, f, 0x09090B0Bu);
            // flags (bits 7 + 8e) -> bits 8e + g4 of the keep word
            bits[t] |= (f >> (7 - g4)) & (0x01010101u << g4);
          }
          pw[2 * t + (g4 >> 1)][2 * (g4 & 1)] = w0;
          pw[2 * t + (g4 >> 1)][2 * (g4 & 1) + 1] = w1;
        }
      }
    }
    l += ls;
    if constexpr (DROP != 0) {  // publish this (query, 2 key blocks)'s decisions: half hh writes block hh
      const uint32_t mine = bits[hh] << (4 * hh), other = bits[hh ^ 1] << (4 * hh);
      const uint32_t word = mine | xor32_get(other, hh);
      mst[r * C::MWS + ((((k0 >> 5) + hh)) & (C::MW - 1))] = word;
    }
    // O += P V: V^T fragments by transposed reads of the stage's V tile
    bf16x8_t vf[HD / 32][4];
    auto vread = [&](auto ksc) {
      constexpr int ks = decltype(ksc)::value;
      constexpr int OFF = ST * C::STG + 16 * ks * HD * 2;
#pragma unroll
      for (int u = 0; u < HD / 32; ++u) {
        const s16x4_t lo = ds_tr_read<OFF>(trb[u][0]);
        const s16x4_t hi = ds_tr_read<OFF>(trb[u][1]);
        vf[u][ks] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
    };
    vread(std::integral_constant<int, 0>{});
    vread(std::integral_constant<int, 1>{});
    vread(std::integral_constant<int, 2>{});
    vread(std::integral_constant<int, 3>{});
    lgk_wait<0>();
#pragma unroll
    for (int u = 0; u < HD / 32; ++u)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) reg_fence(vf[u][ks]);
#pragma unroll
    for (int u = 0; u < HD / 32; ++u)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const uint4 w4 = make_uint4(pw[ks][0], pw[ks][1], pw[ks][2], pw[ks][3]);
        o[u] = mfma32(vf[u][ks], __builtin_bit_cast(bf16x8_t, w4), o[u]);
      }
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  int it = 0;
  for (; it + 1 < ntiles; it += 2) {
    tile(I0{}, it);
    tile(I1{}, it + 1);
    if (DROP && ((it + 2) & 7) == 0 && it + 2 < ntiles) flush(2 * (it + 2));
  }
  if (it < ntiles) tile(I0{}, it);
  if (DROP && active) flush(2 * ntiles);
  if (!active) return;
  l = xor32_sum(l);
  if (myq >= L) return;
  const float inv = sd / l;
  bf16_t* orow = reinterpret_cast<bf16_t*>(p.out) + (size_t)(tok0 + myq) * p.nh * HD + h * HD;
#pragma unroll
  for (int u = 0; u < HD / 32; ++u)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const float v[4] = {o[u][4 * g4] * inv, o[u][4 * g4 + 1] * inv, o[u][4 * g4 + 2] * inv,
                          o[u][4 * g4 + 3] * inv};
      Vec4<bf16_t>::store(orow + 32 * u + 8 * g4 + 4 * hh, v);
    }
  if (hh == 0) p.lse[(size_t)(tok0 + myq) * p.nh + h] = (m + log2f(l)) * LN2;
}

// ------------------------------------------------------------------------------------------------
// delta[t, h] = sum_d dO * O
template <int HD>
__global__ __launch_bounds__(256) void attn_delta_kernel(const bf16_t* __restrict__ dout,
                                                        const bf16_t* __restrict__ out,
                                                        float* __restrict__ delta, int64_t rows) {
  constexpr int LPR = HD / 8;  // lanes per (t, h) row
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t row = gid / LPR;
  const int c = gid % LPR;
  float a = 0.f;
  if (row < rows) {
    const uint4 x = *reinterpret_cast<const uint4*>(dout + row * HD + c * 8);
    const uint4 y = *reinterpret_cast<const uint4*>(out + row * HD + c * 8);
    const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      a += __uint_as_float(xs[k] << 16) * __uint_as_float(ys[k] << 16) +
           __uint_as_float(xs[k] & 0xffff0000u) * __uint_as_float(ys[k] & 0xffff0000u);
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  if (row < rows && c == 0) delta[row] = a;
}

// ------------------------------------------------------------------------------------------------
template <int HD, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void attn_bwd_dq_kernel(AttnBwdParams p) {
  constexpr int STG = 2 * TILE * HD;  // K tile (row reads for S^T, transposed for dQ) | V tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);

  int b, qb;
  attn_unit(p.sched_q, blockIdx.y, p.max_s, b, qb);
  const int h = blockIdx.x;
  const int tok0 = p.cu[b];
  const int L = p.cu[b + 1] - tok0;
  const int q0 = qb * BLK;
  if (q0 >= L) return;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int qw0 = q0 + wid * ROWS;
  const bool active = qw0 < L;
  const int hk = h / (p.nh / p.nkv);
  const int rs = (p.nh + 2 * p.nkv) * HD;
  const bf16_t* qkv = reinterpret_cast<const bf16_t*>(p.qkv);
  const bf16_t* dout = reinterpret_cast<const bf16_t*>(p.dout);
  const bf16_t* ksrc = qkv + p.nh * HD + hk * HD;
  const bf16_t* vsrc = qkv + (p.nh + p.nkv) * HD + hk * HD;
  const int myq = qw0 + r;
  const int qi = min(myq, L - 1);
  const int kend = p.causal ? min(L, q0 + BLK) : L;
  const int ntiles = (kend + TILE - 1) / TILE;

  Stage2<HD> stg;
  stg.load(ksrc, rs, vsrc, rs, tok0, 0, L);

  bf16x8_t qf[HD / 16], df[HD / 16];
  {
    const bf16_t* qrow = qkv + (size_t)(tok0 + qi) * rs + h * HD;
    const bf16_t* drow_ = dout + (size_t)(tok0 + qi) * p.nh * HD + h * HD;
#pragma unroll
    for (int s = 0; s < HD / 16; ++s) {
      qf[s] = *reinterpret_cast<const bf16x8_t*>(qrow + 16 * s + 8 * hh);
      df[s] = *reinterpret_cast<const bf16x8_t*>(drow_ + 16 * s + 8 * hh);
    }
  }
  // dropout's 1/(1-p) is folded into P (lse shifted by log2 sd) and delta (divided by sd):
  // dS = P sd (keep dP - delta / sd) — no per-element scale multiply.
  const float sd = p.p8 ? keep_scale(p.p8) : 1.f;
  const float lse2 = p.lse[(size_t)(tok0 + qi) * p.nh + h] * LOG2E - log2f(sd);
  const float dlt = p.delta[(size_t)(tok0 + qi) * p.nh + h] / sd;
  f32x16_t dq[HD / 32];
#pragma unroll
  for (int u = 0; u < HD / 32; ++u) dq[u] = zero16();
  const float sl2 = p.scale * LOG2E;
  const uint32_t* mrow = p.mask + (size_t)((tok0 + qi) * p.nh + h) * p.mask_w;

  TileOffsets<HD> to;
  to.init(lane);
  stg.store(lds, lds + TILE * HD);
  __syncthreads();

  for (int it = 0; it < ntiles; ++it) {
    const int k0 = it * TILE;
    const bool more = it + 1 < ntiles;
    if (more) stg.load(ksrc, rs, vsrc, rs, tok0, k0 + TILE, L);
    uint2 kw2 = make_uint2(0u, 0u);
    if (p.p8) kw2 = *reinterpret_cast<const uint2*>(mrow + (k0 >> 5));
    const bf16_t* Ks = lds + (it & 1) * STG;
    const bf16_t* Vs = Ks + TILE * HD;
    if (active && !(p.causal && k0 > qw0 + ROWS - 1)) {
      f32x16_t sacc[2], pacc[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        sacc[t] = zero16();
        pacc[t] = zero16();
#pragma unroll
        for (int s = 0; s < HD / 16; ++s) {
          sacc[t] = mfma32(lds_row8(Ks + 32 * t * HD + to.row[s]), qf[s], sacc[t]);
          pacc[t] = mfma32(lds_row8(Vs + 32 * t * HD + to.row[s]), df[s], pacc[t]);
        }
      }
      const bool need_mask = (k0 + TILE > L) || (p.causal && k0 + TILE - 1 > qw0);
      bf16x8_t dsf[4];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const uint32_t wk = (t ? kw2.y : kw2.x) >> (4 * hh);
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          float pv = fexp2(fmaf(sacc[t][reg], sl2, -lse2));
          if (need_mask) {
            const int key = k0 + 32 * t + acc_row(reg, hh);
            if (key >= L || (p.causal && key > myq)) pv = 0.f;
          }
          float dp = pacc[t][reg];
          if (p.p8) dp = keep_and(dp, wk, 8 * (reg & 3) + (reg >> 2));  // key 8 (reg >> 2) + 4 hh + (reg & 3)
          dsf[2 * t + (reg >> 3)][reg & 7] = (__bf16)(pv * (dp - dlt));
        }
      }
#pragma unroll
      for (int u = 0; u < HD / 32; ++u)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          dq[u] = mfma32(tr_operand(Ks + 16 * ks * HD, to.tr[u][0], to.tr[u][1]), dsf[ks], dq[u]);
    }
    if (more) {
      bf16_t* nk = lds + ((it + 1) & 1) * STG;
      stg.store(nk, nk + TILE * HD);
    }
    __syncthreads();
  }
  if (!active || myq >= L) return;
  bf16_t* dst = reinterpret_cast<bf16_t*>(p.dqkv) + (size_t)(tok0 + myq) * rs + h * HD;
#pragma unroll
  for (int u = 0; u < HD / 32; ++u)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const float v[4] = {dq[u][4 * g4] * p.scale, dq[u][4 * g4 + 1] * p.scale,
                          dq[u][4 * g4 + 2] * p.scale, dq[u][4 * g4 + 3] * p.scale};
      Vec4<bf16_t>::store(dst + 32 * u + 8 * g4 + 4 * hh, v);
    }
}

// ------------------------------------------------------------------------------------------------
template <int HD, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void attn_bwd_dkdv_kernel(AttnBwdParams p) {
  // Q | dO | lse, delta (fp32 = 2 bf16 slots) | keep words [4 waves][64 queries] (uint32)
  constexpr int STG = 2 * TILE * HD + 2 * TILE * 2 + NWAVE * TILE * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);

  int b, kb;
  attn_unit(p.sched_k, blockIdx.y, p.max_s, b, kb);
  const int hk = blockIdx.x;
  const int tok0 = p.cu[b];
  const int L = p.cu[b + 1] - tok0;
  const int kb0 = kb * BLK;
  if (kb0 >= L) return;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int kw0 = kb0 + wid * ROWS;
  const bool active = kw0 < L;
  const int rs = (p.nh + 2 * p.nkv) * HD;
  const int grp = p.nh / p.nkv;
  const bf16_t* qkv = reinterpret_cast<const bf16_t*>(p.qkv);
  const bf16_t* dout = reinterpret_cast<const bf16_t*>(p.dout);
  const int koff = p.nh * HD + hk * HD;
  const int voff = (p.nh + p.nkv) * HD + hk * HD;
  const int mykey = kw0 + r;
  const int ki = min(mykey, L - 1);
  const int mbit = attn_mbit(r);  // my key's bit in a keep word
  const int qstart = p.causal ? (kb0 / TILE) * TILE : 0;
  const int nqt = (L - qstart + TILE - 1) / TILE;  // q tiles per head
  const int ntiles = nqt * grp;

  // dropout scale folded into the staged lse / delta exactly as in the dq kernel
  const float sd = p.p8 ? keep_scale(p.p8) : 1.f;
  const float lsd = log2f(sd), isd = 1.f / sd;
  Stage2<HD> stg;
  float ls_r = 0.f, dl_r = 0.f;  // lse / delta of row threadIdx.x (threads < TILE)
  uint32_t mk_r = 0u;            // keep word: wave (threadIdx.x >> 6)'s key block, query tid & 63
  auto issue = [&](int it) {
    const int hq = hk * grp + it / nqt;
    const int q0 = qstart + (it % nqt) * TILE;
    stg.load(qkv + hq * HD, rs, dout + hq * HD, p.nh * HD, tok0, q0, L);
    if (threadIdx.x < TILE) {
      const int q = q0 + threadIdx.x;
      ls_r = q < L ? p.lse[(size_t)(tok0 + q) * p.nh + hq] * LOG2E - lsd : 0.f;
      dl_r = q < L ? p.delta[(size_t)(tok0 + q) * p.nh + hq] * isd : 0.f;
    }
    if (p.p8) {
      const int q = q0 + (threadIdx.x & 63);
      mk_r = q < L ? p.mask[(size_t)((tok0 + q) * p.nh + hq) * p.mask_w + (kb0 >> 5) + (threadIdx.x >> 6)]
                   : 0u;
    }
  };
  auto commit = [&](int buf) {
    bf16_t* Qs = lds + buf * STG;
    bf16_t* Ds = Qs + TILE * HD;
    stg.store(Qs, Ds);
    float* fs = reinterpret_cast<float*>(Ds + TILE * HD);
    if (threadIdx.x < TILE) {
      fs[threadIdx.x] = ls_r;
      fs[TILE + threadIdx.x] = dl_r;
    }
    reinterpret_cast<uint32_t*>(fs + 2 * TILE)[threadIdx.x] = mk_r;
  };
  issue(0);

  bf16x8_t kf[HD / 16], vf[HD / 16];
  {
    const bf16_t* base = qkv + (size_t)(tok0 + ki) * rs;
#pragma unroll
    for (int s = 0; s < HD / 16; ++s) {
      kf[s] = *reinterpret_cast<const bf16x8_t*>(base + koff + 16 * s + 8 * hh);
      vf[s] = *reinterpret_cast<const bf16x8_t*>(base + voff + 16 * s + 8 * hh);
    }
  }
  f32x16_t dk[HD / 32], dv[HD / 32];
#pragma unroll
  for (int u = 0; u < HD / 32; ++u) { dk[u] = zero16(); dv[u] = zero16(); }
  const float sl2 = p.scale * LOG2E;

  TileOffsets<HD> to;
  to.init(lane);
  commit(0);
  __syncthreads();

  for (int it = 0; it < ntiles; ++it) {
    const int hq = hk * grp + it / nqt;
    const int q0 = qstart + (it % nqt) * TILE;
    const bool more = it + 1 < ntiles;
    if (more) issue(it + 1);
    const bf16_t* Qs = lds + (it & 1) * STG;
    const bf16_t* Ds = Qs + TILE * HD;
    const float* lse_s = reinterpret_cast<const float*>(Ds + TILE * HD);
    const float* dl_s = lse_s + TILE;
    // keep words of this wave's 32 keys (bit r = my key) for the tile's 64 queries
    const uint32_t* mk_s = reinterpret_cast<const uint32_t*>(lse_s + 2 * TILE) + wid * TILE;
    if (active) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int qt0 = q0 + 32 * t;
        if (p.causal && qt0 + 31 < kw0) continue;  // every query of the subtile precedes my keys
        if (qt0 >= L) continue;
        f32x16_t sacc = zero16(), pacc = zero16();
#pragma unroll
        for (int s = 0; s < HD / 16; ++s) {
          sacc = mfma32(lds_row8(Qs + 32 * t * HD + to.row[s]), kf[s], sacc);
          pacc = mfma32(lds_row8(Ds + 32 * t * HD + to.row[s]), vf[s], pacc);
        }
        const bool need_mask = (qt0 + 32 > L) || (p.causal && qt0 < kw0 + ROWS);
        bf16x8_t pf[2], dsf[2];
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int ql = 32 * t + 8 * g4 + 4 * hh;  // 4 consecutive queries
          const float4 ls4 = *reinterpret_cast<const float4*>(lse_s + ql);
          const float4 dl4 = *reinterpret_cast<const float4*>(dl_s + ql);
          const float lsv[4] = {ls4.x, ls4.y, ls4.z, ls4.w}, dlv[4] = {dl4.x, dl4.y, dl4.z, dl4.w};
          uint4 m4 = make_uint4(0u, 0u, 0u, 0u);
          if (p.p8) m4 = *reinterpret_cast<const uint4*>(mk_s + ql);
          const uint32_t mw[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int reg = 4 * g4 + e;
            const int q = q0 + ql + e;
            float pv = fexp2(fmaf(sacc[reg], sl2, -lsv[e]));  // = P / (1 - p)
            if (need_mask && (q >= L || (p.causal && mykey > q))) pv = 0.f;
            float pd = pv, dp = pacc[reg];
            if (p.p8) {
              const int km = __builtin_amdgcn_sbfe((int)mw[e], mbit, 1);
              pd = __int_as_float(__float_as_int(pv) & km);
              dp = __int_as_float(__float_as_int(dp) & km);
            }
            pf[reg >> 3][reg & 7] = (__bf16)pd;
            dsf[reg >> 3][reg & 7] = (__bf16)(pv * (dp - dlv[e]));
          }
        }
#pragma unroll
        for (int u = 0; u < HD / 32; ++u)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const int kb = (32 * t + 16 * s2) * HD;
            dv[u] = mfma32(tr_operand(Ds + kb, to.tr[u][0], to.tr[u][1]), pf[s2], dv[u]);
            dk[u] = mfma32(tr_operand(Qs + kb, to.tr[u][0], to.tr[u][1]), dsf[s2], dk[u]);
          }
      }
    }
    if (more) commit((it + 1) & 1);
    __syncthreads();
  }
  if (!active || mykey >= L) return;
  bf16_t* drow = reinterpret_cast<bf16_t*>(p.dqkv) + (size_t)(tok0 + mykey) * rs;
#pragma unroll
  for (int u = 0; u < HD / 32; ++u)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const float kv[4] = {dk[u][4 * g4] * p.scale, dk[u][4 * g4 + 1] * p.scale,
                           dk[u][4 * g4 + 2] * p.scale, dk[u][4 * g4 + 3] * p.scale};
      const float vv[4] = {dv[u][4 * g4], dv[u][4 * g4 + 1], dv[u][4 * g4 + 2], dv[u][4 * g4 + 3]};
      Vec4<bf16_t>::store(drow + koff + 32 * u + 8 * g4 + 4 * hh, kv);
      Vec4<bf16_t>::store(drow + voff + 32 * u + 8 * g4 + 4 * hh, vv);
    }
}

}  // namespace

// "F,Q,K" minimum waves per SIMD of the fwd / dq / dkdv kernels (each 1 or 3; scripts/attn_time.py)
struct AttnOcc { int f = 3, q = 1, k = 1; };  // measured: fwd 73.8 -> 70.6 us; dq, dkdv slower at 3
const AttnOcc& attn_occupancy() {
  static const AttnOcc o = [] {
    AttnOcc a;
    if (const char* e = std::getenv("BCFL_ATTN_WPE")) std::sscanf(e, "%d,%d,%d", &a.f, &a.q, &a.k);
    return a;
  }();
  return o;
}

int attn_units(int n_units, int B, int max_s) {
  return n_units > 0 ? n_units : B * ((max_s + BLK - 1) / BLK);
}

template <int HD, int WPE>
void fwd_launch(const AttnParams& p, dim3 grid, size_t lds, hipStream_t s) {
  if (p.p8 == 0)
    hipLaunchKernelGGL((attn_fwd_kernel<HD, WPE, 0>), grid, dim3(256), lds, s, p);
  else if (p.p8 < 128)
    hipLaunchKernelGGL((attn_fwd_kernel<HD, WPE, 1>), grid, dim3(256), lds, s, p);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<HD, WPE, 2>), grid, dim3(256), lds, s, p);
}

template <int HD>
void fwd_hd(const AttnParams& p, hipStream_t s) {
  dim3 grid(p.nh, attn_units(p.sched ? p.n_units : 0, p.B, p.max_s));
  const size_t lds = FwdCfg<HD>::LDS;
  if (HD <= 64 && attn_occupancy().f == 3)  // d = 128 spills at 168 registers: 2 waves / SIMD
    fwd_launch<HD, 3>(p, grid, lds, s);
  else
    fwd_launch<HD, 1>(p, grid, lds, s);
}

template <int HD>
void bwd_hd(const AttnBwdParams& p, hipStream_t s) {
  const int64_t rows = (int64_t)p.T * p.nh;
  const int nu = attn_units(p.sched_q ? p.n_units : 0, p.B, p.max_s);
  dim3 gq(p.nh, nu);
  dim3 gk(p.nkv, nu);
  const bf16_t* dout = reinterpret_cast<const bf16_t*>(p.dout);
  const bf16_t* out = reinterpret_cast<const bf16_t*>(p.out);
  hipLaunchKernelGGL(attn_delta_kernel<HD>, dim3((unsigned)((rows * (HD / 8) + 255) / 256)),
                     dim3(256), 0, s, dout, out, p.delta, rows);
  const AttnOcc& o = attn_occupancy();
  const size_t lq = (size_t)2 * 2 * TILE * HD * 2;
  if (o.q == 3)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, 3>), gq, dim3(256), lq, s, p);
  else
    hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, 1>), gq, dim3(256), lq, s, p);
  const size_t lk = (size_t)2 * (2 * TILE * HD + 2 * TILE * 2 + NWAVE * TILE * 2) * 2;
  if (o.k == 3)
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HD, 3>), gk, dim3(256), lk, s, p);
  else
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HD, 1>), gk, dim3(256), lk, s, p);
}

int attn_dropmask_words(int max_s) {
  // >= one word per 32 keys and >= the 4 key blocks of the last dkdv workgroup; power of two
  const int need = 4 * ((max_s + BLK - 1) / BLK);
  int w = 4;
  while (w < need) w <<= 1;
  return w;
}

int launch_attn_fwd(const AttnParams& p, hipStream_t s) {
  if (p.nh % p.nkv) return -2;
  if (p.p8 && (!p.mask || p.mask_w < attn_dropmask_words(p.max_s))) return -3;
  switch (p.d) {
    case 32: fwd_hd<32>(p, s); break;
    case 64: fwd_hd<64>(p, s); break;
    case 128: fwd_hd<128>(p, s); break;
    default: return -1;
  }
  return 0;
}

int launch_attn_bwd(const AttnBwdParams& p, hipStream_t s) {
  if (p.nh % p.nkv) return -2;
  if (p.p8 && (!p.mask || p.mask_w < attn_dropmask_words(p.max_s))) return -3;
  switch (p.d) {
    case 32: bwd_hd<32>(p, s); break;
    case 64: bwd_hd<64>(p, s); break;
    case 128: bwd_hd<128>(p, s); break;
    default: return -1;
  }
  return 0;
}

}  // namespace bcfl
