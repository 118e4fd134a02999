// LDS-DMA and hand-counted synchronisation helpers shared by the pipelined MFMA kernels
// (gemm8.hip, attention.hip).
//
//   * buf_rsrc(): a raw buffer resource over [base + off, + nbytes): buffer loads past the end
//     return zeros (the hardware range check), which is how ragged tiles are zero-filled;
//   * dma16(): one buffer_load_dwordx4 ... lds — 16 B per lane straight into LDS at
//     (wave-uniform base) + 16 * lane, no VGPR round trip;
//   * vm_wait<N>() / lgk_wait<N>(): counted waits (asm: the compiler does not see the DMA's LDS
//     writes nor the asm LDS reads below, so the kernels place these themselves);
//   * ds_tr_read<OFF>() / ds_row_read<OFF>(): ds_read_b64_tr_b16 / ds_read_b128 with a 16-bit
//     immediate offset, as inline asm — for LDS reads it can see, the compiler's waitcnt pass
//     puts vmcnt waits (a drain of the DMA queue, including tiles still in flight for later use)
//     in front of the read's consumer whenever a DMA is outstanding;
//   * BCFL_BAR(): a raw s_barrier fenced against compiler reordering (a __syncthreads() would also
//     drain the DMA queue).
#pragma once
#include <type_traits>

#include "common.h"

namespace bcfl {
namespace {

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, int64_t byte_off,
                                                          int64_t nbytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base) + (uint64_t)byte_off;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  int64_t nb = nbytes < 0 ? 0 : nbytes;
  if (nb > 0x7fffffff) nb = 0x7fffffff;
  const uint32_t n = __builtin_amdgcn_readfirstlane((uint32_t)nb);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo),
                                           (short)0, (int)n, 0x00020000);
}

// 16 B per lane from (rsrc, voff) into LDS at lds_base + 16 * lane. The range check covers voff
// only (not soffset), so tile offsets go into voff. Device pass only: the host pass cannot
// type-check the builtin, and a failed host-side instantiation silently drops the launch stub.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds_base, int voff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds_base,
                                           16, voff, 0, 0, 0);
#endif
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void lgk_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
}

template <int OFF>
__device__ __forceinline__ s16x4_t ds_tr_read(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field is 16 bits");
  s16x4_t v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}

template <int OFF>
__device__ __forceinline__ bf16x8_t ds_row_read(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field is 16 bits");
  bf16x8_t v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}

// an asm-produced register is "written" here: keeps its consumers after the preceding wait
template <typename T>
__device__ __forceinline__ void reg_fence(T& v) {
  asm volatile("" : "+v"(v));
}

// f(std::integral_constant<int, I>{}) for I = 0 .. N-1: loop indices that must be compile-time
// (immediate LDS offsets)
template <int I, int N>
struct StaticFor {
  template <class F>
  __device__ __forceinline__ static void run(F& f) {
    f(std::integral_constant<int, I>{});
    StaticFor<I + 1, N>::run(f);
  }
};
template <int N>
struct StaticFor<N, N> {
  template <class F>
  __device__ __forceinline__ static void run(F&) {}
};
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  StaticFor<0, N>::run(f);
}

#define BCFL_BAR()                                \
  do {                                            \
    __builtin_amdgcn_sched_barrier(0);            \
    asm volatile("s_barrier" ::: "memory");       \
    __builtin_amdgcn_sched_barrier(0);            \
  } while (0)

}  // namespace
}  // namespace bcfl
