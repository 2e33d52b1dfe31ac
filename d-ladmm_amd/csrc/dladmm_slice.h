// dladmm_slice.h -- the per-layer "slice GEMM" main loop shared by the per-layer forward kernels
// (dladmm_layered.hip) and the backward kernels (dladmm_backward.hip).
//
// One workgroup of NW waves owns 16*NW batch columns and SB 16-row output blocks starting at
// block ib0; wave w owns 16 columns and keeps the SB 16x16 accumulators (4*SB registers) in the
// C/D layout of v_mfma_f32_16x16x4_f32 (lane l: column l&15, rows 16b + 4(l>>4) + r).
//   acc[i] += sum_kb  Wp-fragment(kb, ib0+i) * S[16kb + 4g + q][col]
// The contraction runs as a RUNTIME loop over k-blocks of 16: the B operand (4 rows of S, this
// lane's column) is LDS-DMA'd by each wave for itself two k-blocks ahead (one ds_read_b128 per
// k-block), the A operands (packed fragments, k-major order [KB][MBp]) stream through a
// double-buffered LDS ring by LDS-DMA, shared by the NW waves.  Each output block is ONE accumulation chain in k order starting from
// zero, so every caller computing the same product with the same packing gets the same bits
// (the backward recomputes A*Z_k and W_k*Var_k bit-identically to the forward).
#pragma once

#include "dladmm_common.h"

namespace dladmm {

constexpr int kSliceCF = 16;  // fragments per ring chunk (16 KiB)

// LDS of a slice kernel: the weight ring (2 chunks) followed by the B-operand ring (NSB k-blocks
// of NW KiB).  One __shared__ array per kernel, so the compiler sees a single LDS object.
template <int NW, int NSB>
constexpr int slice_lds_f4() { return 2 * kSliceCF * 64 + NSB * NW * 64; }

// ring: __shared__ f32x4[slice_lds_f4<NW, NSB>()] of the calling kernel.  Ends with a ring
// barrier (the speculative prefetches have landed), so the ring may be reused by a second call.
//
// The B operand (4 rows of S, the lane's column) is LDS-DMA'd by the wave itself, NSB - 1
// k-blocks ahead: 4 dword DMAs per wave and k-block, instruction i bringing rows 4i + (l & 3)
// of columns (l >> 2) in the order the MFMA lane (column l & 15, rows 4(l >> 4) + q) reads them
// back with one ds_read_b128.  Rows past Krows are clamped to the last row (the packed weights
// are zero there, so they add exactly 0) and columns past B to column 0 (discarded outputs).
// Every VM operation of the loop is an LDS-DMA issued here, so the waits are exact counts: a
// freshly issued prefetch is never drained by a barrier or a register copy.
template <int NW, int SB, int NSB = 3>
__device__ __forceinline__ void slice_gemm(f32x4* ring, const float* Wp, int MBp, int ib0, int KB,
                                           const float* S, int64_t ldS, int Krows, int64_t B,
                                           f32x4 (&acc)[SB]) {
  constexpr int CF = kSliceCF;
  constexpr int NCI = SB / CF;       // chunks per k-block
  constexpr int D = 2;               // fragment read-ahead
  constexpr int NBUF = D + 2;        // a step consumes a PAIR of fragments: D + 2 in rotation
  constexpr int WPW = CF / NW;       // weight DMAs per wave and chunk
  static_assert(SB % CF == 0, "slice must be whole chunks");
  static_assert(CF % NW == 0 && WPW == 4, "4 weight DMAs per wave and chunk (vmcnt counts)");
  static_assert(NSB == 2 || NSB == 3, "B ring depth");
  static_assert(NCI <= 2, "vmcnt counts below assume at most 2 chunks per k-block");
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  f32x4* bring = ring + 2 * CF * 64;

  auto chunk_src = [&](int kb, int c) -> const float* {
    return Wp + ((int64_t)kb * MBp + ib0 + c * CF) * kFrag;
  };
  auto issue = [&](const float* src, int slot) {
    uint64_t sb = (uint64_t)src;
    asm volatile("" : "+s"(sb));
    const float* base = (const float*)sb;
    f32x4* dst = ring + slot * (CF * 64);
#if DLADMM_DMA4
    // wave w: the chunk's fragments 4w .. 4w+3 (contiguous 4 KiB), one M0 setup
    glds16x4(base + 4 * w * kFrag, lane * 16, dst + 4 * w * 64);
#else
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      const int f = i * NW + w;
      glds16(base + f * kFrag, lane * 16, dst + f * 64);
    }
#endif
  };
  // B DMA lanes: column (l >> 2) of this wave's 16, row offset (l & 3) within each group of 4
  const int64_t colD = (int64_t)blockIdx.x * (16 * NW) + w * 16 + (lane >> 2);
  const uint32_t colDo = (uint32_t)(colD < B ? colD : 0);
  const int rq = lane & 3;
  auto issue_b = [&](int kb, int slot) {
    uint64_t sb = (uint64_t)(S + (int64_t)(16 * kb) * ldS);
    asm volatile("" : "+s"(sb));
    const int rmax = Krows - 1 - 16 * kb;  // >= 0 for every k-block of the contraction
    char* dst = reinterpret_cast<char*>(bring + (slot * NW + w) * 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * i + rq < rmax ? 4 * i + rq : rmax;
      glds4((const float*)sb, (uint32_t)(((int64_t)r * ldS + colDo) * 4), dst + 256 * i);
    }
  };

#pragma unroll
  for (int i = 0; i < SB; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(chunk_src(0, 0), 0);
  issue_b(0, 0);
  if constexpr (NSB == 3) issue_b(KB > 1 ? 1 : 0, 1);
  f32x4 fr[NBUF];
  int chunk_id = 0;  // running chunk index (slot = chunk_id & 1)

  for (int kb = 0; kb < KB; ++kb) {
    f32x4 bcur;
    static_for<NCI>([&](auto C_) {
      constexpr int c = decltype(C_)::value;
      const int slot = chunk_id & 1;
      // VM operations issued after the one awaited (NSB 3): one chunk per k-block -> the B
      // prefetch issued after this chunk's weights; two -> none at c = 0 (the weights of
      // (kb, 0) were issued last), the B prefetch at c = 1.  NSB 2: the awaited DMA is the
      // newest.
      ring_barrier_n<(NSB == 3 && (NCI == 1 || c == 1)) ? 4 : 0>();
      {  // prefetch the next chunk (past the end: re-read chunk 0, never consumed)
        const int nc = c + 1 < NCI ? c + 1 : 0;
        const int nkb = c + 1 < NCI ? kb : (kb + 1 < KB ? kb + 1 : 0);
        issue(chunk_src(nkb, nc), slot ^ 1);
      }
      if constexpr (c == 0) {
        // NSB 3: B(kb+2) right after the next chunk's weights (slot (kb+2) % 3 was last read
        // at kb - 1, before this barrier)
        if constexpr (NSB == 3) issue_b(kb + 2 < KB ? kb + 2 : 0, (kb + 2) % 3);
        bcur = bring[((kb % NSB) * NW + w) * 64 + lane];
      }
      // NSB 2: B(kb+1) after the last chunk's weights, into the slot read at kb - 1
      if constexpr (NSB == 2 && c == NCI - 1) issue_b(kb + 1 < KB ? kb + 1 : 0, (kb + 1) % 2);
      const f32x4* rs = ring + slot * (CF * 64);
      static_for<D>([&](auto Dd) {
        constexpr int d = decltype(Dd)::value;
        fr[d % NBUF] = rs[d * 64 + lane];
      });
      // pairs of output blocks: 8 MFMAs alternating two independent accumulators
      static_for<CF / 2>([&](auto P_) {
        constexpr int p = decltype(P_)::value;
        constexpr int f0 = 2 * p, f1 = 2 * p + 1;
        if constexpr (f0 + D < CF) fr[(f0 + D) % NBUF] = rs[(f0 + D) * 64 + lane];
        if constexpr (f1 + D < CF) fr[(f1 + D) % NBUF] = rs[(f1 + D) * 64 + lane];
        const f32x4 w0 = fr[f0 % NBUF], w1 = fr[f1 % NBUF];
        f32x4& a0 = acc[c * CF + f0];
        f32x4& a1 = acc[c * CF + f1];
        a0 = mfma4(w0.x, bcur.x, a0);
        a1 = mfma4(w1.x, bcur.x, a1);
        a0 = mfma4(w0.y, bcur.y, a0);
        a1 = mfma4(w1.y, bcur.y, a1);
        a0 = mfma4(w0.z, bcur.z, a0);
        a1 = mfma4(w1.z, bcur.z, a1);
        a0 = mfma4(w0.w, bcur.w, a0);
        a1 = mfma4(w1.w, bcur.w, a1);
        __builtin_amdgcn_sched_barrier(0);
      });
      ++chunk_id;
    });
  }
  ring_barrier();  // drain the speculative prefetches before the ring is reused / the WG exits
}

}  // namespace dladmm

#ifndef DLADMM_BVIEW_AUX
#define DLADMM_BVIEW_AUX 0  // cache-policy bits of the backward epilogue stores (experiment)
#endif

namespace dladmm {

// A [rows][ld] fp32 matrix seen by one lane of a slice epilogue in the C/D layout (lane: column
// col, rows 16b + 4g + r): a raw buffer resource (NULL or out-of-range rows / columns read 0,
// stores are dropped) plus the lane's voffset; a row's uniform part goes in soffset, so an access
// costs no per-lane address arithmetic.  Requires rows * ld * 4 < 2^31 (checked on the host).
struct BView {
  rsrc_t r;
  uint32_t vo, ld4;
  __device__ __forceinline__ float ld(uint32_t row_u) const {
    return __builtin_bit_cast(float,
                              __builtin_amdgcn_raw_buffer_load_b32(r, (int)vo, (int)(row_u * ld4), 0));
  }
  __device__ __forceinline__ void st(uint32_t row_u, float v) const {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)vo,
                                          (int)(row_u * ld4), DLADMM_BVIEW_AUX);
  }
};
__device__ __forceinline__ BView make_view(const float* p, int rows, int64_t ld, int g,
                                           int64_t col, bool cv) {
  BView v;
  v.r = mkrsrc(p, p ? (uint32_t)((int64_t)rows * ld * 4) : 0u);
  v.vo = cv ? (uint32_t)(((int64_t)4 * g * ld + col) * 4) : kOOB;
  v.ld4 = (uint32_t)(ld * 4);
  return v;
}

}  // namespace dladmm
