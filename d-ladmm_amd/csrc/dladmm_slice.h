// dladmm_slice.h -- the per-layer "slice GEMM" main loop shared by the per-layer forward kernels
// (dladmm_layered.hip) and the backward kernels (dladmm_backward.hip).
//
// One workgroup of NW waves owns 16*NW batch columns and SB 16-row output blocks starting at
// block ib0; wave w owns 16 columns and keeps the SB 16x16 accumulators (4*SB registers) in the
// C/D layout of v_mfma_f32_16x16x4_f32 (lane l: column l&15, rows 16b + 4(l>>4) + r).
//   acc[i] += sum_kb  Wp-fragment(kb, ib0+i) * S[16kb + 4g + q][col]
// The contraction runs as a RUNTIME loop over k-blocks of 16: the B operand (4 rows of S, this
// lane's column) is loaded straight from HBM two k-blocks ahead, the A operands (packed
// fragments, k-major order [KB][MBp]) stream through a double-buffered LDS ring by LDS-DMA,
// shared by the NW waves.  Each output block is ONE accumulation chain in k order starting from
// zero, so every caller computing the same product with the same packing gets the same bits
// (the backward recomputes A*Z_k and W_k*Var_k bit-identically to the forward).
#pragma once

#include "dladmm_common.h"

namespace dladmm {

constexpr int kSliceCF = 16;  // fragments per ring chunk (16 KiB)

// B operand of one k-block for this lane: rows 16kb + 4g + q (q = 0..3) of column col of
// S[Krows][ld]; rows >= Krows (padding) and invalid columns read 0.  Branch-free: the address is
// clamped, the value selected.
__device__ __forceinline__ f32x4 load_bfrag(const float* S, int64_t ld, int Krows, int kb, int g,
                                            int64_t colc, bool cv) {
  f32x4 v;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = 16 * kb + 4 * g + q;
    const bool ok = cv && row < Krows;
    const float x = S[(int64_t)(ok ? row : 0) * ld + colc];
    v[q] = ok ? x : 0.0f;
  }
  return v;
}

// ring: __shared__ f32x4[2 * kSliceCF * 64] of the calling kernel.  Ends with a ring barrier (the
// speculative prefetch has landed), so the ring may be reused by a second call.
template <int NW, int SB>
__device__ __forceinline__ void slice_gemm(f32x4* ring, const float* Wp, int MBp, int ib0, int KB,
                                           const float* S, int64_t ldS, int Krows, int64_t colc,
                                           bool cv, f32x4 (&acc)[SB]) {
  constexpr int CF = kSliceCF;
  constexpr int NCI = SB / CF;       // chunks per k-block
  constexpr int D = 2;               // fragment read-ahead
  constexpr int NBUF = D + 2;        // a step consumes a PAIR of fragments: D + 2 in rotation
  static_assert(SB % CF == 0, "slice must be whole chunks");
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;

  auto chunk_src = [&](int kb, int c) -> const float* {
    return Wp + ((int64_t)kb * MBp + ib0 + c * CF) * kFrag;
  };
  auto issue = [&](const float* src, int slot) {
    uint64_t sb = (uint64_t)src;
    asm volatile("" : "+s"(sb));
    const float* base = (const float*)sb;
    f32x4* dst = ring + slot * (CF * 64);
#pragma unroll
    for (int i = 0; i < (CF + NW - 1) / NW; ++i) {
      const int f = i * NW + w;
      if (CF % NW == 0 || f < CF) glds16(base + f * kFrag, lane * 16, dst + f * 64);
    }
  };

#pragma unroll
  for (int i = 0; i < SB; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(chunk_src(0, 0), 0);
  f32x4 bn1 = load_bfrag(S, ldS, Krows, 0, g, colc, cv);
  f32x4 bn2 = load_bfrag(S, ldS, Krows, 1, g, colc, cv);
  f32x4 fr[NBUF];
  int chunk_id = 0;  // running chunk index (slot = chunk_id & 1)

  for (int kb = 0; kb < KB; ++kb) {
    const f32x4 bcur = bn1;
    bn1 = bn2;
    bn2 = load_bfrag(S, ldS, Krows, kb + 2, g, colc, cv);
    static_for<NCI>([&](auto C_) {
      constexpr int c = decltype(C_)::value;
      const int slot = chunk_id & 1;
      ring_barrier();
      {  // prefetch the next chunk (past the end: re-read chunk 0, never consumed)
        const int nc = c + 1 < NCI ? c + 1 : 0;
        const int nkb = c + 1 < NCI ? kb : (kb + 1 < KB ? kb + 1 : 0);
        issue(chunk_src(nkb, nc), slot ^ 1);
      }
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
  ring_barrier();  // drain the speculative prefetch before the ring is reused / the WG exits
}

}  // namespace dladmm

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
                                          (int)(row_u * ld4), 0);
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
