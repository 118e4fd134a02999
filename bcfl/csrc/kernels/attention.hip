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
// the dq and dkdv kernels read those bits back instead of re-hashing in each of them — dkdv with
// 2 VALU ops per score (bit-field extract to a 0 / -1 mask + AND), dq with 1.5 (a byte-spread
// word, v_cvt_f32_ubyte to 0.f / 1.f, the multiply folded into a packed fma).
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

// byte B of x as a float (v_cvt_f32_ubyte{B}: one full-rate op; the compiler's own lowering of
// (float)((x >> 8B) & 0xff) re-derives the bits with extra shifts when x is a masked word)
template <int B>
__device__ __forceinline__ float cvt_ubyte(uint32_t x) {
  float r;
  if constexpr (B == 0) asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(r) : "v"(x));
  if constexpr (B == 1) asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(r) : "v"(x));
  if constexpr (B == 2) asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(r) : "v"(x));
  if constexpr (B == 3) asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(r) : "v"(x));
  return r;
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
      // exponent arguments and the row sum in packed fp32 (v_pk_fma_f32 / v_pk_add_f32: two
      // scores per VALU op), the exp itself per score
      const f32x2_t sl2v = {sl2, sl2}, nmv = {-m, -m};
      f32x2_t lsv = {0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        bits[t] = 0u;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          float pv[4];
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const f32x2_t s2 = {sacc[t][4 * g4 + e], sacc[t][4 * g4 + e + 1]};
            const f32x2_t a2 = __builtin_elementwise_fma(s2, sl2v, nmv);
            pv[e] = fexp2(a2.x);
            pv[e + 1] = fexp2(a2.y);
            lsv += f32x2_t{pv[e], pv[e + 1]};
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
      ls = lsv.x + lsv.y;
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
// Backward prep: per (token, head) row, the two row constants of the backward in the form the
// kernels consume them (dropout's 1/(1-p) = sd folded in: dS = P sd (keep dP - delta / sd)):
//   rc[0][row] = lse * log2(e) - log2(sd)   so  P sd = exp2(s * scale * log2(e) - rc0)
//   rc[1][row] = sum_d dO * O / sd
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_prep_kernel(const bf16_t* __restrict__ dout,
                                                           const bf16_t* __restrict__ out,
                                                           const float* __restrict__ lse,
                                                           float* __restrict__ rc, int64_t rows,
                                                           float lsd, float isd) {
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
  if (row < rows && c == 0) {
    rc[row] = fmaf(lse[row], LOG2E, -lsd);
    rc[rows + row] = a * isd;
  }
}

// ------------------------------------------------------------------------------------------------
// dQ. Same K / V LDS-DMA ring as the forward. Per tile and wave (32 queries x 64 keys), for each
// 32-key half: S^T = K Q^T and dP^T = V dO^T on MFMA (K, V row fragments by asm reads), then
// dS = P sd (keep dP - delta / sd) from the prepped row constants and the forward's keep words
// (prefetched one tile ahead into registers, issued before the tile's DMA so the compiler's wait
// for them never counts the DMA down); finally dQ += dS K with K^T fragments by transposed reads.
template <int HD, int WPE, int DROP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void attn_bwd_dq_kernel(AttnBwdParams p) {
  using C = FwdCfg<HD>;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  int b, qb;
  attn_unit(p.sched_q, blockIdx.y, p.max_s, b, qb);
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
  const bf16_t* dout = reinterpret_cast<const bf16_t*>(p.dout);
  const int myq = qw0 + r;
  const int qi = min(myq, L - 1);
  const int kend = p.causal ? min(L, q0 + BLK) : L;
  const int ntiles = (kend + TILE - 1) / TILE;

  const __amdgpu_buffer_rsrc_t rsrc = buf_rsrc(qkv, (int64_t)tok0 * rs * 2, (int64_t)L * rs * 2);
  int voff[2][C::PW];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int colbase = (x == 0 ? p.nh + hk : p.nh + p.nkv + hk) * HD;
#pragma unroll
    for (int i = 0; i < C::PW; ++i) {
      const int c = 64 * (wid + NWAVE * i) + lane;
      const int row = c / C::CPR;
      const int u = (c % C::CPR) ^ swz<HD>(row);
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
  // keep words of this lane's query row: 2 per 64-key tile, prefetched a tile ahead
  const uint32_t* mrow = p.mask + (size_t)((tok0 + qi) * p.nh + h) * p.mask_w;
  u32x2_t kwn = {0u, 0u};
  if constexpr (DROP != 0) kwn = *reinterpret_cast<const u32x2_t*>(mrow);
  dma(0, 0);

  bf16x8_t qf[HD / 16], df[HD / 16];
  {
    const bf16_t* qrow = qkv + (size_t)(tok0 + qi) * rs + h * HD;
    const bf16_t* drow_ = dout + (size_t)(tok0 + qi) * p.nh * HD + h * HD;
#pragma unroll
    for (int s2 = 0; s2 < HD / 16; ++s2) {
      qf[s2] = *reinterpret_cast<const bf16x8_t*>(qrow + 16 * s2 + 8 * hh);
      df[s2] = *reinterpret_cast<const bf16x8_t*>(drow_ + 16 * s2 + 8 * hh);
    }
  }
  const size_t rrow = (size_t)(tok0 + qi) * p.nh + h;
  const float lse2 = p.delta[rrow];
  const float dlt = p.delta[(size_t)p.T * p.nh + rrow];
  f32x16_t dq[HD / 32];
#pragma unroll
  for (int u = 0; u < HD / 32; ++u) dq[u] = zero16();
  const float sl2 = p.scale * LOG2E;
  const f32x2_t sl2v = {sl2, sl2}, nlv = {-lse2, -lse2}, ndv = {-dlt, -dlt};

  TileOffsets<HD> to;
  to.init(lane);
  const uint32_t lds32 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  uint32_t rowb[HD / 16];
#pragma unroll
  for (int s2 = 0; s2 < HD / 16; ++s2) rowb[s2] = lds32 + 2 * to.row[s2];
  uint32_t trb[HD / 32][2];  // K^T reads (K tile of stage 0)
#pragma unroll
  for (int u = 0; u < HD / 32; ++u)
#pragma unroll
    for (int hi = 0; hi < 2; ++hi) trb[u][hi] = lds32 + 2 * to.tr[u][hi];

  vm_wait<0>();
#pragma unroll
  for (int s2 = 0; s2 < HD / 16; ++s2) {
    reg_fence(qf[s2]);
    reg_fence(df[s2]);
  }
  BCFL_BAR();

  auto tile = [&](auto stc, int it) {
    constexpr int ST = decltype(stc)::value;
    const int k0 = it * TILE;
    if (it > 0) {
      vm_wait<0>();
      BCFL_BAR();
    }
    u32x2_t kw = kwn;
    reg_fence(kw);
    if constexpr (DROP != 0) {
      if (it + 1 < ntiles) kwn = *reinterpret_cast<const u32x2_t*>(mrow + ((k0 + TILE) >> 5));
    }
    if (it + 1 < ntiles) dma(ST ^ 1, k0 + TILE);
    if (!active || (p.causal && k0 > qw0 + ROWS - 1)) return;
    const bool need_mask = (k0 + TILE > L) || (p.causal && k0 + TILE - 1 > qw0);
    uint32_t dsw[4][4];  // dS as bf16 pairs, fragment ks = 2t + (reg >> 3)
    auto half = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      bf16x8_t kf[HD / 16], vf[HD / 16];
#pragma unroll
      for (int s2 = 0; s2 < HD / 16; ++s2) kf[s2] = ds_row_read<ST * C::STG + 32 * t * HD * 2>(rowb[s2]);
#pragma unroll
      for (int s2 = 0; s2 < HD / 16; ++s2) vf[s2] = ds_row_read<ST * C::STG + C::TBYTES + 32 * t * HD * 2>(rowb[s2]);
      lgk_wait<HD / 16>();
#pragma unroll
      for (int s2 = 0; s2 < HD / 16; ++s2) reg_fence(kf[s2]);
      f32x16_t sacc = zero16(), pacc = zero16();
#pragma unroll
      for (int s2 = 0; s2 < HD / 16; ++s2) sacc = mfma32(kf[s2], qf[s2], sacc);
      lgk_wait<0>();
#pragma unroll
      for (int s2 = 0; s2 < HD / 16; ++s2) reg_fence(vf[s2]);
#pragma unroll
      for (int s2 = 0; s2 < HD / 16; ++s2) pacc = mfma32(vf[s2], df[s2], pacc);
      const uint32_t wk = (t ? kw[1] : kw[0]) >> (4 * hh);
      if (need_mask) {
#pragma unroll
        for (int rg = 0; rg < 16; ++rg) {
          const int key = k0 + 32 * t + acc_row(rg, hh);
          if (key >= L || (p.causal && key > myq)) sacc[rg] = -INFINITY;
        }
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // accumulator rows 4g + e hold keep bit 8e + g of the word (key 8 g + 4 hh + e): one
        // shift + and leaves byte e = that bit, v_cvt_f32_ubyte{e} turns it into 0.f / 1.f, and
        // the multiply rides in the packed fma dp * keep - delta (1.5 VALU ops per score for
        // dropout instead of 2)
        uint32_t kb = 0x01010101u;
        if constexpr (DROP != 0) kb = (wk >> g) & 0x01010101u;
        const f32x2_t k01 = {cvt_ubyte<0>(kb), cvt_ubyte<1>(kb)};
        const f32x2_t k23 = {cvt_ubyte<2>(kb), cvt_ubyte<3>(kb)};
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const int reg = 4 * g + e;
          // score pairs in packed fp32 (v_pk_fma / v_pk_mul), the exp per score
          const f32x2_t a2 = __builtin_elementwise_fma(f32x2_t{sacc[reg], sacc[reg + 1]}, sl2v, nlv);
          const f32x2_t dp = {pacc[reg], pacc[reg + 1]};
          const f32x2_t kd = DROP != 0 ? __builtin_elementwise_fma(dp, e ? k23 : k01, ndv) : dp + ndv;
          const f32x2_t ds = f32x2_t{fexp2(a2.x), fexp2(a2.y)} * kd;
          dsw[2 * t + (reg >> 3)][(reg & 7) >> 1] = pack2bf(ds.x, ds.y);
        }
      }
    };
    half(std::integral_constant<int, 0>{});
    half(std::integral_constant<int, 1>{});
    // dQ += dS K: K^T fragments (k = key) by transposed reads of the stage's K tile
    bf16x8_t kt[HD / 32][4];
    auto kread = [&](auto ksc) {
      constexpr int ks = decltype(ksc)::value;
      constexpr int OFF = ST * C::STG + 16 * ks * HD * 2;
#pragma unroll
      for (int u = 0; u < HD / 32; ++u) {
        const s16x4_t lo = ds_tr_read<OFF>(trb[u][0]);
        const s16x4_t hi = ds_tr_read<OFF>(trb[u][1]);
        kt[u][ks] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
    };
    kread(std::integral_constant<int, 0>{});
    kread(std::integral_constant<int, 1>{});
    kread(std::integral_constant<int, 2>{});
    kread(std::integral_constant<int, 3>{});
    lgk_wait<0>();
#pragma unroll
    for (int u = 0; u < HD / 32; ++u)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) reg_fence(kt[u][ks]);
#pragma unroll
    for (int u = 0; u < HD / 32; ++u)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const uint4 w4 = make_uint4(dsw[ks][0], dsw[ks][1], dsw[ks][2], dsw[ks][3]);
        dq[u] = mfma32(kt[u][ks], __builtin_bit_cast(bf16x8_t, w4), dq[u]);
      }
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  int it = 0;
  for (; it + 1 < ntiles; it += 2) {
    tile(I0{}, it);
    tile(I1{}, it + 1);
  }
  if (it < ntiles) tile(I0{}, it);
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
// dK, dV. A wave owns 32 keys (K, V fragments and the dK^T / dV^T accumulators in registers) and
// the workgroup sweeps every query tile of every query head of its GQA group. Per tile the LDS
// ring stage holds, all by LDS-DMA: the Q and dO tiles (16-B pieces), the 64 prepped row
// constants (4-B pieces: wave 0 rc0, wave 1 rc1) and each wave's 64 keep words (4-B pieces).
template <int HD>
struct DkdvCfg {
  static constexpr int CPR = HD / 8;
  static constexpr int TBYTES = TILE * HD * 2;
  static constexpr int PW = TBYTES / 1024 / NWAVE;
  // [stage 0 | stage 1 small arrays (rc0 256 B, rc1 256 B, keep words 1 KiB)] then
  // [stage 0 Q | dO][stage 1 Q | dO]: every immediate LDS offset stays below 64 KiB at d = 128
  static constexpr int SMALL = 512 + NWAVE * 256;
  static constexpr int L0 = 0, DL0 = 256, M0 = 512;
  static constexpr int TB = 2 * SMALL;
  static constexpr int LDS = TB + 4 * TBYTES;
  static constexpr int small(int st) { return st * SMALL; }
  static constexpr int q(int st) { return TB + st * 2 * TBYTES; }
  static constexpr int d(int st) { return TB + st * 2 * TBYTES + TBYTES; }
};

__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t rs, char* lds_base, int voff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds_base,
                                           4, voff, 0, 0, 0);
#endif
}

template <int OFF>
__device__ __forceinline__ f32x4_t ds_read_f4(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field is 16 bits");
  f32x4_t v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}

template <int HD, int WPE, int DROP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void attn_bwd_dkdv_kernel(AttnBwdParams p) {
  using C = DkdvCfg<HD>;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  int b, kb;
  attn_unit(p.sched_k, blockIdx.y, p.max_s, b, kb);
  const int hk = blockIdx.x;
  const int tok0 = p.cu[b];
  const int L = p.cu[b + 1] - tok0;
  const int kb0 = kb * BLK;
  if (kb0 >= L) return;
  const int lane = threadIdx.x & 63, r = lane & 31, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kw0 = kb0 + wid * ROWS;
  const bool active = kw0 < L;
  const int rs = (p.nh + 2 * p.nkv) * HD;
  const int ds_ = p.nh * HD;  // dO row stride
  const int grp = p.nh / p.nkv;
  const bf16_t* qkv = reinterpret_cast<const bf16_t*>(p.qkv);
  const bf16_t* dout = reinterpret_cast<const bf16_t*>(p.dout);
  const int koff = p.nh * HD + hk * HD;
  const int voff_ = (p.nh + p.nkv) * HD + hk * HD;
  const int mykey = kw0 + r;
  const int ki = min(mykey, L - 1);
  const int mbit = attn_mbit(r);  // my key's bit in a keep word
  const int qstart = p.causal ? (kb0 / TILE) * TILE : 0;
  const int nqt = (L - qstart + TILE - 1) / TILE;  // q tiles per head
  const int ntiles = nqt * grp;

  // ---- per-tile LDS-DMA sources --------------------------------------------------------------
  const __amdgpu_buffer_rsrc_t rq = buf_rsrc(qkv, (int64_t)tok0 * rs * 2, (int64_t)L * rs * 2);
  const __amdgpu_buffer_rsrc_t rd = buf_rsrc(dout, (int64_t)tok0 * ds_ * 2, (int64_t)L * ds_ * 2);
  const __amdgpu_buffer_rsrc_t rc = buf_rsrc(p.delta, (int64_t)tok0 * p.nh * 4,
                                             (int64_t)((size_t)p.T * p.nh + (size_t)L * p.nh) * 4);
  const __amdgpu_buffer_rsrc_t rm =
      buf_rsrc(p.mask, (int64_t)tok0 * p.nh * p.mask_w * 4, (int64_t)L * p.nh * p.mask_w * 4);
  int qv[C::PW], dv[C::PW];
#pragma unroll
  for (int i = 0; i < C::PW; ++i) {
    const int c = 64 * (wid + NWAVE * i) + lane;
    const int row = c / C::CPR;
    const int u = (c % C::CPR) ^ swz<HD>(row);
    qv[i] = row * rs * 2 + 16 * u;
    dv[i] = row * ds_ * 2 + 16 * u;
  }
  // rc1 rows of this sequence start T*nh floats after rc0's: only rows < L are in range for rc0
  // (the resource's end bounds rc1), so rc0 reads past L land in rc0 of later sequences — rows
  // >= L are masked out of every product below, whatever they hold
  const int lv = lane * p.nh * 4;
  const int mv = lane * p.nh * p.mask_w * 4 + ((kb0 >> 5) + wid) * 4;
  auto dma = [&](int st, int it2) {
    const int hq = hk * grp + it2 / nqt;
    const int q0 = qstart + (it2 % nqt) * TILE;
#pragma unroll
    for (int i = 0; i < C::PW; ++i) {
      dma16(rq, smem + C::q(st) + (wid + NWAVE * i) * 1024, qv[i] + q0 * rs * 2 + hq * HD * 2);
      dma16(rd, smem + C::d(st) + (wid + NWAVE * i) * 1024, dv[i] + q0 * ds_ * 2 + hq * HD * 2);
    }
    char* sm = smem + C::small(st);
    const int rowc = (q0 * p.nh + hq) * 4;
    if (wid == 0) dma4(rc, sm + C::L0, lv + rowc);
    if (wid == 1) dma4(rc, sm + C::DL0, lv + rowc + p.T * p.nh * 4);
    if constexpr (DROP != 0) dma4(rm, sm + C::M0 + wid * 256, mv + (q0 * p.nh + hq) * p.mask_w * 4);
  };
  dma(0, 0);

  bf16x8_t kf[HD / 16], vf[HD / 16];
  {
    const bf16_t* base = qkv + (size_t)(tok0 + ki) * rs;
#pragma unroll
    for (int s2 = 0; s2 < HD / 16; ++s2) {
      kf[s2] = *reinterpret_cast<const bf16x8_t*>(base + koff + 16 * s2 + 8 * hh);
      vf[s2] = *reinterpret_cast<const bf16x8_t*>(base + voff_ + 16 * s2 + 8 * hh);
    }
  }
  f32x16_t dk[HD / 32], dv2[HD / 32];
#pragma unroll
  for (int u = 0; u < HD / 32; ++u) { dk[u] = zero16(); dv2[u] = zero16(); }
  const float sl2 = p.scale * LOG2E;

  TileOffsets<HD> to;
  to.init(lane);
  const uint32_t lds32 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  uint32_t rowb[HD / 16];
#pragma unroll
  for (int s2 = 0; s2 < HD / 16; ++s2) rowb[s2] = lds32 + 2 * to.row[s2];
  uint32_t trb[HD / 32][2];
#pragma unroll
  for (int u = 0; u < HD / 32; ++u)
#pragma unroll
    for (int hi = 0; hi < 2; ++hi) trb[u][hi] = lds32 + 2 * to.tr[u][hi];
  // row-constant / keep-word reads: 4 consecutive queries 8 g4 + 4 hh (+ 32 t) of the tile
  const uint32_t cb = lds32 + 16 * hh;
  const uint32_t mb = lds32 + wid * 256 + 16 * hh;

  vm_wait<0>();
#pragma unroll
  for (int s2 = 0; s2 < HD / 16; ++s2) {
    reg_fence(kf[s2]);
    reg_fence(vf[s2]);
  }
  BCFL_BAR();

  auto tile = [&](auto stc, int it2) {
    constexpr int ST = decltype(stc)::value;
    const int q0 = qstart + (it2 % nqt) * TILE;
    if (it2 > 0) {
      vm_wait<0>();
      BCFL_BAR();
    }
    if (it2 + 1 < ntiles) dma(ST ^ 1, it2 + 1);
    if (!active) return;
    auto half = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      const int qt0 = q0 + 32 * t;
      if (p.causal && qt0 + 31 < kw0) return;  // every query of the subtile precedes my keys
      if (qt0 >= L) return;
      bf16x8_t qr[HD / 16], dr[HD / 16];
#pragma unroll
      for (int s2 = 0; s2 < HD / 16; ++s2) qr[s2] = ds_row_read<C::q(ST) + 32 * t * HD * 2>(rowb[s2]);
#pragma unroll
      for (int s2 = 0; s2 < HD / 16; ++s2) dr[s2] = ds_row_read<C::d(ST) + 32 * t * HD * 2>(rowb[s2]);
      f32x4_t lc[4], dc[4];
      u32x4_t mw[4];
      static_for<4>([&](auto gc) {
        constexpr int g4 = decltype(gc)::value;
        lc[g4] = ds_read_f4<C::small(ST) + C::L0 + (32 * t + 8 * g4) * 4>(cb);
        dc[g4] = ds_read_f4<C::small(ST) + C::DL0 + (32 * t + 8 * g4) * 4>(cb);
        if constexpr (DROP != 0)
          mw[g4] = __builtin_bit_cast(u32x4_t, ds_read_f4<C::small(ST) + C::M0 + (32 * t + 8 * g4) * 4>(mb));
      });
      lgk_wait<0>();
#pragma unroll
      for (int s2 = 0; s2 < HD / 16; ++s2) {
        reg_fence(qr[s2]);
        reg_fence(dr[s2]);
      }
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        reg_fence(lc[g4]);
        reg_fence(dc[g4]);
        if constexpr (DROP != 0) reg_fence(mw[g4]);
      }
      f32x16_t sacc = zero16(), pacc = zero16();
#pragma unroll
      for (int s2 = 0; s2 < HD / 16; ++s2) {
        sacc = mfma32(qr[s2], kf[s2], sacc);
        pacc = mfma32(dr[s2], vf[s2], pacc);
      }
      if ((qt0 + 32 > L) || (p.causal && qt0 < kw0 + ROWS)) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int q = qt0 + acc_row(reg, hh);
          if (q >= L || (p.causal && mykey > q)) sacc[reg] = -INFINITY;
        }
      }
      uint32_t pw[2][4], dw[2][4];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        float pd[4], dsv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int reg = 4 * g4 + e;
          const float pv = fexp2(fmaf(sacc[reg], sl2, -lc[g4][e]));  // = P sd
          float pdv = pv, dp = pacc[reg];
          if constexpr (DROP != 0) {
            const int km = __builtin_amdgcn_sbfe((int)mw[g4][e], mbit, 1);
            pdv = __int_as_float(__float_as_int(pv) & km);
            dp = __int_as_float(__float_as_int(dp) & km);
          }
          pd[e] = pdv;
          dsv[e] = pv * (dp - dc[g4][e]);
        }
        pw[g4 >> 1][2 * (g4 & 1)] = pack2bf(pd[0], pd[1]);
        pw[g4 >> 1][2 * (g4 & 1) + 1] = pack2bf(pd[2], pd[3]);
        dw[g4 >> 1][2 * (g4 & 1)] = pack2bf(dsv[0], dsv[1]);
        dw[g4 >> 1][2 * (g4 & 1) + 1] = pack2bf(dsv[2], dsv[3]);
      }
      // dV^T += dO^T P, dK^T += Q^T dS: dO^T / Q^T fragments by transposed reads
      bf16x8_t dt[HD / 32][2], qt[HD / 32][2];
      auto trd = [&](auto s2c) {
        constexpr int s2 = decltype(s2c)::value;
        constexpr int KB = (32 * t + 16 * s2) * HD * 2;
#pragma unroll
        for (int u = 0; u < HD / 32; ++u) {
          const s16x4_t a0 = ds_tr_read<C::d(ST) + KB>(trb[u][0]);
          const s16x4_t a1 = ds_tr_read<C::d(ST) + KB>(trb[u][1]);
          dt[u][s2] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
          const s16x4_t b0 = ds_tr_read<C::q(ST) + KB>(trb[u][0]);
          const s16x4_t b1 = ds_tr_read<C::q(ST) + KB>(trb[u][1]);
          qt[u][s2] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7));
        }
      };
      trd(std::integral_constant<int, 0>{});
      trd(std::integral_constant<int, 1>{});
      lgk_wait<0>();
#pragma unroll
      for (int u = 0; u < HD / 32; ++u)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          reg_fence(dt[u][s2]);
          reg_fence(qt[u][s2]);
        }
#pragma unroll
      for (int u = 0; u < HD / 32; ++u)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const uint4 a = make_uint4(pw[s2][0], pw[s2][1], pw[s2][2], pw[s2][3]);
          const uint4 c2 = make_uint4(dw[s2][0], dw[s2][1], dw[s2][2], dw[s2][3]);
          dv2[u] = mfma32(dt[u][s2], __builtin_bit_cast(bf16x8_t, a), dv2[u]);
          dk[u] = mfma32(qt[u][s2], __builtin_bit_cast(bf16x8_t, c2), dk[u]);
        }
    };
    half(std::integral_constant<int, 0>{});
    half(std::integral_constant<int, 1>{});
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  int it = 0;
  for (; it + 1 < ntiles; it += 2) {
    tile(I0{}, it);
    tile(I1{}, it + 1);
  }
  if (it < ntiles) tile(I0{}, it);
  if (!active || mykey >= L) return;
  bf16_t* drow = reinterpret_cast<bf16_t*>(p.dqkv) + (size_t)(tok0 + mykey) * rs;
#pragma unroll
  for (int u = 0; u < HD / 32; ++u)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const float kv[4] = {dk[u][4 * g4] * p.scale, dk[u][4 * g4 + 1] * p.scale,
                           dk[u][4 * g4 + 2] * p.scale, dk[u][4 * g4 + 3] * p.scale};
      const float vv[4] = {dv2[u][4 * g4], dv2[u][4 * g4 + 1], dv2[u][4 * g4 + 2], dv2[u][4 * g4 + 3]};
      Vec4<bf16_t>::store(drow + koff + 32 * u + 8 * g4 + 4 * hh, kv);
      Vec4<bf16_t>::store(drow + voff_ + 32 * u + 8 * g4 + 4 * hh, vv);
    }
}

}  // namespace

// "F,Q,K" minimum waves per SIMD of the fwd / dq / dkdv kernels (each 1 or 3; scripts/attn_time.py)
struct AttnOcc { int f = 3, q = 1, k = 1; };  // minimum waves / SIMD: 3 = at most 168 registers (d <= 64)
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

template <int HD, int DROP>
void bwd_launch(const AttnBwdParams& p, hipStream_t s) {
  const int nu = attn_units(p.sched_q ? p.n_units : 0, p.B, p.max_s);
  const AttnOcc& o = attn_occupancy();
  if (HD <= 64 && o.q == 3)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, 3, DROP>), dim3(p.nh, nu), dim3(256), FwdCfg<HD>::LDS, s, p);
  else
    hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, 1, DROP>), dim3(p.nh, nu), dim3(256), FwdCfg<HD>::LDS, s, p);
  if (HD <= 64 && o.k == 3)
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HD, 3, DROP>), dim3(p.nkv, nu), dim3(256), DkdvCfg<HD>::LDS, s, p);
  else
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HD, 1, DROP>), dim3(p.nkv, nu), dim3(256), DkdvCfg<HD>::LDS, s, p);
}

template <int HD>
void bwd_hd(const AttnBwdParams& p, hipStream_t s) {
  const int64_t rows = (int64_t)p.T * p.nh;
  const float sd = p.p8 ? 256.0f / (256.0f - (float)p.p8) : 1.f;
  hipLaunchKernelGGL(attn_bwd_prep_kernel<HD>, dim3((unsigned)((rows * (HD / 8) + 255) / 256)),
                     dim3(256), 0, s, reinterpret_cast<const bf16_t*>(p.dout),
                     reinterpret_cast<const bf16_t*>(p.out), p.lse, p.delta, rows, log2f(sd), 1.f / sd);
  if (p.p8)
    bwd_launch<HD, 1>(p, s);
  else
    bwd_launch<HD, 0>(p, s);
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
