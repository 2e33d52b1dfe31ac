// dladmm_common.h -- device helpers shared by the fused and the per-layer D-LADMM kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "../../include/dladmm.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace dladmm {


enum { EM_V1 = 0, EM_VVAR = 1, EM_LASSO = 2 };   // E-step form
// parameter broadcast class; PK_S1 = scalar params plus a per-layer step s1 on W Var (V5)
enum { PK_SCALAR = 0, PK_ROW = 1, PK_ELEM = 2, PK_S1 = 3 };

constexpr int kWaves = 4;
constexpr int kTileCols = 16 * kWaves;  // batch columns per workgroup
constexpr int kFrag = 256;              // floats per packed 16x16 fragment (1 KiB)

// literal relu(x - th) - relu(-1.0*x - th) (main_lena.py:52-53); NaN propagates like torch relu
__device__ __forceinline__ float relu_(float v) { return (v <= 0.0f) ? 0.0f : v; }
__device__ __forceinline__ float shrink(float x, float th) {
  return relu_(x - th) - relu_(-x - th);
}

// Two-VALU-op form for a wave-uniform threshold: x + sg * clamp(x, -|th|, |th|), sg = -1 for
// th >= 0 and +1 for th < 0 (fma by +-1 is a single exact add/sub).
//  * th >= 0: bit-identical to the literal form (x > th: fl(x - th) both ways; x < -th:
//    -fl(-x - th) = fl(x + th); otherwise +0);
//  * th < 0 (both relus open): identical for |x| >= |th|; for |x| < |th| it returns 2x where
//    the literal form rounds fl(fl(x - th) - fl(-x - th)) -- within one ulp of |th|.
// No per-element branch: a uniform branch per row splits the unrolled body and costs spills.
struct ShrinkP { float ath, sg; };
__device__ __forceinline__ ShrinkP shrink_params(float th) {
  return ShrinkP{fabsf(th), th >= 0.0f ? -1.0f : 1.0f};
}
__device__ __forceinline__ float shrink_u(float x, ShrinkP p) {
  return __builtin_fmaf(p.sg, __builtin_amdgcn_fmed3f(x, -p.ath, p.ath), x);
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_bf16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// LDS-DMA of one 1 KiB fragment: lane l copies 16 B from sbase + voff to ldst + 16 l.
// sbase and ldst are wave-uniform.  Written as inline asm on purpose: when the compiler sees an
// LDS-DMA (the __builtin_amdgcn_global_load_lds form) in a loop it stops counting LDS reads and
// emits lgkmcnt(0) before every fragment use, which collapses the fragment read-ahead to one
// step.  The hardware counts LDS-DMA on vmcnt only; ring_barrier() waits for it explicitly.
// M0 is compiler-reserved, so it is saved and restored inside the same statement.
__device__ __forceinline__ void glds16(const float* sbase, uint32_t voff, f32x4* ldst) {
  unsigned keep;
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ldst);
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(dst)
      : "memory");
}

#ifndef DLADMM_DMA4
#define DLADMM_DMA4 1  // weight chunk DMA: 4 consecutive fragments per wave with one M0 setup
#endif
// Four consecutive 1 KiB fragments (sbase + 0..3 KiB -> ldst + 0..3 KiB) by LDS-DMA with one
// M0 setup: the instruction offset advances the global source and the LDS destination alike
// (tools/probe/ldsdma_offset.hip).
__device__ __forceinline__ void glds16x4(const float* sbase, uint32_t voff, const void* ldst) {
  unsigned keep;
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ldst);
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "global_load_lds_dwordx4 %1, %2 offset:1024\n\t"
      "global_load_lds_dwordx4 %1, %2 offset:2048\n\t"
      "global_load_lds_dwordx4 %1, %2 offset:3072\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(dst)
      : "memory");
}

// 4-byte variant: lane i's dword lands at ldst + 4 i (64 lanes = 256 consecutive bytes).
__device__ __forceinline__ void glds4(const float* sbase, uint32_t voff, void* ldst) {
  unsigned keep;
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ldst);
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(dst)
      : "memory");
}

// Counted form of ring_barrier(): this wave's VM operations except the newest N are complete
// (the LDS-DMAs that must have landed), its LDS reads are complete, then the barrier.
template <int N>
__device__ __forceinline__ void ring_barrier_n() {
  static_assert(N == 0 || N == 4 || N == 8, "counts used by the slice loop");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ring_barrier() that lets this wave's newest N VM operations stay in flight: correct when at
// least N operations were issued after the awaited LDS-DMA (VM operations complete in issue
// order for vmcnt; counting fewer than were issued only waits longer).
template <int N>
__device__ __forceinline__ void ring_barrier_cnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// All waves: own LDS-DMA + LDS reads complete, then workgroup barrier.  One opaque statement,
// so the compiler can neither hoist ring reads above it nor sink earlier ones below it.
#ifndef DLADMM_SYNC_MODE
#define DLADMM_SYNC_MODE 0  // experiment knob: 1 = no vmcnt wait, 2 = no barrier (WRONG results)
#endif
__device__ __forceinline__ void ring_barrier() {
#if DLADMM_SYNC_MODE == 0
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#elif DLADMM_SYNC_MODE == 1
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
}

// Pin a value to the accumulation register file (AGPR).  The MFMA operands Z and Var live
// there for the whole forward (MFMA srcA/srcB may be AGPRs on gfx950), leaving the 256 arch
// VGPRs for E, L, fragments and epilogue temporaries.
__device__ __forceinline__ void pin_agpr(float& x) { asm("" : "+a"(x)); }

// Compile-time loop: fn(std::integral_constant<int, 0..N-1>) in order.  The unrolled GEMM
// phases are written with it (not #pragma unroll) so every step's body is specialised in the
// front end -- dead epilogue branches never reach the optimiser.
template <typename Fn, int... Is>
__device__ __forceinline__ void static_for_impl(Fn&& fn, std::integer_sequence<int, Is...>) {
  (fn(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void static_for(Fn&& fn) {
  static_for_impl(fn, std::make_integer_sequence<int, N>{});
}

// sum over the 4 lane groups that share a batch column (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ float col_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// sum over the 16 lanes of a DPP row (l & ~15 .. +15: the 16 batch columns of one MFMA C/D row
// group), every lane of the row receiving it: four v_add_f32 with DPP operands (xor 1, xor 2,
// the half-row mirror, the row mirror) -- no LDS round trip, no address registers.  The order
// is fixed, and the two lanes that combine a pair of partial sums add them in the same order.
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

using rsrc_t = __amdgpu_buffer_rsrc_t;
constexpr uint32_t kOOB = 0x80000000u;  // lane offset that is out of range for every buffer

// raw buffer resource; accesses at byte offsets >= bytes are dropped (stores) / read 0 (loads)
__device__ __forceinline__ rsrc_t mkrsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float bload(rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
__device__ __forceinline__ void bstore(rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)off, 0, 0);
}
// store with a wave-uniform row offset in soffset: no per-lane address arithmetic
__device__ __forceinline__ void bstore_s(rsrc_t r, uint32_t voff, uint32_t soff, float v) {
#ifdef DLADMM_ABLATE_NOSTORE  // timing experiment only: drop the store, keep the value live
  asm volatile("" ::"v"(v));
#else
#ifndef DLADMM_STORE_AUX
// cache-policy bits of the fused kernel's output stores: 2 = nt (streaming: the outputs are
// never re-read by the kernel), 2.5 % faster than the default policy (sc1: 5 % slower)
#define DLADMM_STORE_AUX 2
#endif
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)voff, (int)soff,
                                        DLADMM_STORE_AUX);
#endif
}
typedef const __attribute__((address_space(4))) float* cfloat_p;  // scalar-loaded

// Byte offset walker over the rows 16b + 4g + r of a [rows][ld] matrix, one block at a time.
// The running offset is made opaque after every step so the compiler cannot precompute (and
// keep live) one offset register per row of the unrolled layer body.
struct Walk {
  uint32_t cur, ld4;
  __device__ __forceinline__ uint32_t at(int r) const { return cur + (uint32_t)r * ld4; }
  __device__ __forceinline__ void next() {
    cur += 16u * ld4;
    asm volatile("" : "+v"(cur));
  }
};

// Uniform (SGPR) byte offset of rows 16b + r of a [rows][ld] matrix, one block at a time; the
// lane's own 4g row and column live in the buffer instruction's voffset.
struct SWalk {
  uint32_t cur, ld4;
  __device__ __forceinline__ uint32_t at(int r) const { return cur + (uint32_t)r * ld4; }
  __device__ __forceinline__ void next() {
    // readfirstlane: the value is uniform, but the uniformity analysis may not prove it after
    // divergent regions (per-row table loads), and the asm below needs an SGPR
    cur = __builtin_amdgcn_readfirstlane(cur + 16u * ld4);
    asm volatile("" : "+s"(cur));
  }
  __device__ __forceinline__ void reset() {
    cur = 0u;
    asm volatile("" : "+s"(cur));
  }
};

}  // namespace dladmm
