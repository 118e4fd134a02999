// Shared MFMA / LDS tile helpers for bcfl's gfx950 matrix-core kernels (attention.hip, gemm.hip).
//
// v_mfma_f32_32x32x16_bf16 operand layout (cdna_hip_programming.md §3): lane l holds row (l & 31)
// of A (or column of B) and k = 8(l >> 5) + j, j = 0..7; the 16 accumulator registers of lane l
// hold column (l & 31), rows acc_row(reg, l >> 5).
#pragma once
#include "common.h"

namespace bcfl {
namespace {

typedef __attribute__((ext_vector_type(8))) short s16x8_t;

__device__ __forceinline__ f32x16_t mfma32(const bf16x8_t& a, const bf16x8_t& b, const f32x16_t& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t lds_row8(const bf16_t* p) {
  return *reinterpret_cast<const bf16x8_t*>(p);
}

__device__ __forceinline__ s16x4_t tr4(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p));
}

// ---- LDS tile layout -----------------------------------------------------------------------
// Every staged tile is [TILE rows][HD] bf16 with NO padding; 16-byte units of a row are XOR-
// swizzled: element (row, col) lives at row*HD + ((col/8) ^ swz(row))*8 + col%8. One layout serves
// both access kinds (MI355X_MICROARCH.md §LDS bank rules):
//   * row reads (ds_read_b128, lane = row, 16-lane groups {0-3,12-15,20-27}/{4-11,16-19,28-31}):
//     the 16 rows of a group land on 16 distinct 16-B slots of the 256-B bank row;
//   * transposed reads (ds_read_b64_tr_b16, 32-lane halves read 4 consecutive rows x 64 B): the
//     4 rows land on disjoint quarters of the bank row.
// The padded strides this replaces were conflict-free for one kind only (2-way on the other).
// swz(row) depends on row bits 0..3 only, so it is invariant under the multiple-of-16 row offsets
// the loops add: all lane-dependent addressing is precomputed once (TileOffsets).
template <int HD>
__device__ __forceinline__ int swz(int row) {
  if constexpr (HD == 32) {
    return (row >> 2) & 3;
  } else if constexpr (HD == 64) {
    const int a = (row >> 1) & 7;
    return ((a & 1) << 2) | (((a >> 2) & 1) << 1) | ((a >> 1) & 1);
  } else {
    return ((row & 3) << 2) | ((row >> 2) & 3);
  }
}
template <int HD>
__device__ __forceinline__ int swz_off(int row, int unit) {
  return row * HD + ((unit ^ swz<HD>(row)) << 3);
}

template <int HD>
struct TileOffsets {
  // row reads: MFMA operand of row (lane & 31) [+32t], k-unit 2s + hh
  int row[HD / 16];
  // transposed reads (A operand of the second product, X[k][col] for k = kb + {0..3, 8..11}):
  // per 16-lane group g, rows kb + 4hh + ((lane & 15) >> 2) [+8 for the high half], columns
  // 32u + 16(g & 1) + 4(lane & 3); the multiple-of-16 part of kb is added by the caller.
  int tr[HD / 32][2];
  __device__ __forceinline__ void init(int lane) {
    const int r = lane & 31, hh = lane >> 5;
#pragma unroll
    for (int s = 0; s < HD / 16; ++s) row[s] = swz_off<HD>(r, 2 * s + hh);
    const int g = (lane >> 4) & 1, q = (lane & 15) >> 2, pc = lane & 3;
#pragma unroll
    for (int u = 0; u < HD / 32; ++u)
#pragma unroll
      for (int hi = 0; hi < 2; ++hi)
        tr[u][hi] = swz_off<HD>(4 * hh + q + 8 * hi, 4 * u + 2 * g + (pc >> 1)) + 4 * (pc & 1);
  }
};

__device__ __forceinline__ bf16x8_t tr_operand(const bf16_t* tile, int off_lo, int off_hi) {
  const s16x4_t lo = tr4(tile + off_lo);
  const s16x4_t hi = tr4(tile + off_hi);
  const s16x8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, v);
}

__device__ __forceinline__ f32x16_t zero16() {
  f32x16_t z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// row offset inside a 32x32 accumulator: reg -> row (reg&3) + 8(reg>>2) + 4h
__device__ __forceinline__ int acc_row(int reg, int hh) { return (reg & 3) + 8 * (reg >> 2) + 4 * hh; }

}  // namespace
}  // namespace bcfl
