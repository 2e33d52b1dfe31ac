// dladmm_fused_x3_kernel.h -- MI355X (gfx950) fused K-layer D-LADMM forward whose fp32 GEMMs run
// on the f16 matrix cores (DLADMM_PREC_F32_SPLIT).  The kernel template; dladmm_fused_x3.hip
// instantiates the inference form, dladmm_fused_x3_savep.hip the training form that also stores
// P_k = A Z_k (fwd_desc.P) for the backward -- two translation units that compile in parallel.
//
// Same contract and the same one-launch, register-resident design as dladmm_fused.hip (the
// whole K-layer loop of DLADMMNet.forward -- main_lena.py:57-98, main_syn_l1l1_scalar.py:80-127,
// main_syn_lasso_scalar.py:65-114 -- in one kernel; state in registers in the MFMA C/D layout;
// every elementwise update in fp32 in the reference's operation order).  What changes is how
// each fp32 product M * S (M = -W_k or A, S = Var or Z) is formed:
//
//   * both operands are scaled by powers of two (M per tensor, by the pack kernel; S per batch
//     column) so that their magnitudes sit at the top of the f16 range, then split exactly as
//     x = hi + lo with hi = f16(x), lo = f16(x - hi): hi + lo carries 22 significant bits;
//   * M S = Mhi Shi + Mhi Slo + Mlo Shi, three v_mfma_f32_16x16x32_f16 per 16 x 16 x 32 block,
//     accumulated in fp32 (each product of two f16 is exact in fp32); the dropped Mlo Slo term
//     is 2^-22 of the product; the result is scaled back by one exact power-of-two multiply.
//   The error is that of an fp32 GEMM (measured: tools/probe/f16mfma.hip, 2.3e-7 vs 3.2e-7
//   norm-relative for the native fp32 MFMA chain, vs fp64), at 3 x 16 cycles per 16 x 16 x 32
//   block instead of 8 x 32 cycles for v_mfma_f32_16x16x4_f32.
//
// Geometry: one workgroup = 4 waves = 64 batch columns, wave w owns 16 columns; lane l holds
// column l & 15 and rows 16 b + 4 (l >> 4) + r of every state block b.  A 16 x 16 x 32 k-step
// s contracts rows 32 s .. 32 s + 31 = state blocks 2 s and 2 s + 1, i.e. exactly the lane's
// registers [2s][0..3] and [2s+1][0..3]: the packed weight fragments carry the matching k order,
// so the accumulator of one GEMM (after the epilogue) is the B operand of the next with no lane
// movement.
//
// Registers.  The split operands live in AGPRs (MFMA srcB may be an AGPR): Vpk (Var, B operand
// of G1, KS1 k-steps) and Zpk (Z_k, B operand of G2, KS2 k-steps).  fp32 Z is NOT kept across a
// layer: G1's epilogue writes Z_k (output, or workspace in lean mode) and splits it into Zpk
// right away, with a provisional column scale (the previous layer's column max + kHead bits of
// headroom); G1(k+1)'s epilogue gets Z_k back through the LDS ring (buffer LDS-DMA of 1 KiB
// blocks issued with the weight chunks, so the ring barrier's counted vmcnt covers them: a
// register load would make its wait drain every older output store).  If a column of Z_k
// outgrew the provisional scale (checked exactly at the end of G1), the wave re-reads Z_k and
// re-splits it with the exact scale (rare: first layer).  fp32 Var is kept (it is not an
// output) and split with its exact column scale at the start of G1.
//
// Weight stream: -W_k and A, packed as [step][hi|lo][64 lanes] f16x8 fragments (1 KiB each, 2
// per k-step), stream through a 4-slot LDS ring of 16 KiB chunks by LDS-DMA (three chunks in
// flight); the ring barrier waits with a counted vmcnt that leaves every younger VM operation
// (stores, Z re-reads, the next chunks' DMA) in flight.
#pragma once

#include "dladmm_common.h"
#include "dladmm_internal.h"

#ifndef X3_ABL
#define X3_ABL 0  // timing experiments only (tools/x3_ablate.py), every bit gives WRONG results:
                  // 1 no weight DMA, 2 no epilogue work, 4 no output stores, 8 no operand splits,
                  // 16 no MFMAs, 32 no Z re-read DMA, 64 no fragment LDS reads, 128 ring barriers
                  // do not wait for the DMA (vmcnt(63)), 256 no s_barrier, 512 no lgkmcnt(0)
                  // drain at the ring barrier, 1024 every store to one 1 KiB block (L2-resident),
                  // 2048 each store instruction writes 1 KiB contiguous (same bytes)
#endif
#ifndef X3_OFF
#define X3_OFF 0  // A/B knob: 1 immediate tile stores, 2 Z_{k-1} block read at the chunk start,
                  // 4 X rows read at the block start (the earlier schedules; correct results)
#endif
#ifndef X3_BAR2
#define X3_BAR2 0  // one ring barrier per two chunks (each refills two slots)
#endif
#ifndef X3_DMA_LATE
#define X3_DMA_LATE 0  // A/B build: a barrier step's DMA group issued after its MFMAs (the ring
                       // windows then count one step less)
#endif
#ifndef X3_SDLY
#define X3_SDLY 2  // deferred tile stores: steps between the read-back and the store
#endif
#ifndef X3_STAMP
#define X3_STAMP 0  // diagnostic build: per-wave cycle sums of the passes and ring barriers
#endif
#ifndef X3_SGB
#define X3_SGB 0  // >0: interleave that many non-MFMA instructions between a step's 3 MFMAs
#endif
#ifndef X3_SGM
#define X3_SGM 0x386  // instruction classes of those fillers (VALU | SALU | DS)
#endif

namespace dladmm {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

namespace x3 {

constexpr int kSlots = 4;  // LDS ring slots
constexpr int kHead = 12;  // provisional-scale headroom (bits) of the in-epilogue Z split

__device__ __forceinline__ f32x4 mfma(const f16x8& a, const f16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

struct BOp {
  f16x8 hi, lo;
};

// x = v * sc (exact: sc is a power of two) -> hi = f16(x), lo = f16(x - hi), each one RNE
// rounding (fma(v, sc, 0) / fma(v, sc, -hi) lower to v_fma_mix{lo,hi}_f16)
__device__ __forceinline__ void split4(const float (&v)[4], float sc, f16x8& hi, f16x8& lo,
                                       int o) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const _Float16 h = (_Float16)__builtin_fmaf(v[j], sc, 0.0f);
    hi[o + j] = h;
    lo[o + j] = (_Float16)__builtin_fmaf(v[j], sc, -(float)h);
  }
}
__device__ __forceinline__ BOp split8(const float (&a)[4], const float (&b)[4], float sc) {
  BOp r;
  if constexpr (X3_ABL & 8) {
    for (int j = 0; j < 4; ++j) {
      r.hi[j] = (_Float16)a[j]; r.hi[4 + j] = (_Float16)b[j]; r.lo = r.hi;
    }
    return r;
  }
  split4(a, sc, r.hi, r.lo, 0);
  split4(b, sc, r.hi, r.lo, 4);
  return r;
}

__device__ __forceinline__ void pin_agpr_b(BOp& b) {
  asm("" : "+a"(b.hi));
  asm("" : "+a"(b.lo));
}

// the 4 lane groups holding one batch column (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ float col_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}

// column scale exponent: mx * 2^s in [2^14, 2^15) (f16 max 65504), clamped so that 2^s and the
// combined inverse 2^-(s + sw) stay representable
__device__ __forceinline__ int scale_exp(float mx, int sw, int head) {
  int s = 15 - head - __builtin_amdgcn_frexp_expf(mx);
  const int hi = 149 - sw < 126 ? 149 - sw : 126;
  s = s < -126 ? -126 : s;
  return s > hi ? hi : s;
}
__device__ __forceinline__ float exp2i(int e) { return __builtin_amdgcn_ldexpf(1.0f, e); }

// LDS-DMA through a buffer resource, lane l: 16 B from voff + soff to LDS at ldst + 16 l.
// Out-of-range lanes (kOOB: padded columns) read 0, so padded columns stay exactly zero.  M0 is
// compiler-reserved: saved and restored in the statement.
__device__ __forceinline__ void blds16(i32x4 r, uint32_t voff, uint32_t soff, const void* ldst) {
  unsigned keep;
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ldst);
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(soff), "s"(dst)
      : "memory");
}
// Store cache policy of the output tiles. Measured on the d=15 headline (tools/x3_ablate.py,
// profiles/r02_x3_ablations.md): default policy 2.58 ms, sc0 2.59, nt 2.72, nt|sc1 2.73. The
// fp32 kernels keep DLADMM_STORE_AUX (nt); here the full-line dwordx4 stores merge in L2 anyway.
#ifndef X3_STORE_AUX
#define X3_STORE_AUX 0
#endif
__device__ __forceinline__ void bstore4(rsrc_t r, uint32_t voff, uint32_t soff, f32x4 v) {
  if constexpr (!(X3_ABL & 4))
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), r, (int)voff, (int)soff,
                                           X3_STORE_AUX);
}
// m = max(m, |v|) in one v_max_f32 (fmaxf would canonicalise both inputs first)
__device__ __forceinline__ float amax(float m, float v) {
  float r;
  asm("v_max_f32_e64 %0, %1, |%2|" : "=v"(r) : "v"(m), "v"(v));
  return r;
}
// m = max(m, |u|, |v|) in one v_max3_f32
__device__ __forceinline__ float amax2(float m, float u, float v) {
  float r;
  asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(m), "v"(u), "v"(v));
  return r;
}
__device__ __forceinline__ i32x4 mk_rsrc4(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
  r[3] = 0x00020000;
  return r;
}

// Chunk geometry.  The stream is the GEMM sequence A (prologue), -W_0, A, -W_1, ..., each ST
// steps = NCH chunks of SPC steps.  A G1 chunk also carries, per wave, the NZB blocks of Z_{k-1}
// (1 KiB each: 16 rows x the wave's 16 columns) that the epilogues of that chunk's steps read;
// the block of the last G1 block's epilogue (run after the pass) rides on the next G2 chunk 0.
template <int NB, int KS1, int SPC>
struct ZChunks {
  static constexpr int NZB = SPC / KS1;  // Z blocks per G1 chunk
  // Z block carried in slot q of G1 chunk c (-1: none)
  static constexpr int g1_block(int c, int q) {
    const int b = c * NZB - 1 + q;
    return (b >= 0 && b < NB) ? b : -1;
  }
  static constexpr int g1_blocks(int c) {
    int n = 0;
    for (int q = 0; q < NZB; ++q) n += g1_block(c, q) >= 0 ? 1 : 0;
    return n;
  }
};

// Static VM-operation windows of the ring barriers.  The barrier of chunk ch sits at position
// SPC-D of the chunk and waits for chunk ch+1 (weights + Z blocks), whose DMA group was issued
// at the barrier 3 chunks earlier; younger: the bodies of the 3*SPC steps since and the DMA
// groups of chunks ch+2, ch+3.  Counted: what every step body issues unconditionally (the
// epilogue stores) and the DMA instructions (Z blocks at one x4 instruction each; a tile
// that loads them by dword issues more, which only waits longer).  A step or chunk of the
// other pass type (the window reaching across a pass boundary) counts with that pass's
// schedule; the unrolled tails between passes only add younger operations.
template <int MB, int NB, int KS1, int KS2, int SPC, bool SAVEP = false, int PF = 0>
struct Win {
  using Z = ZChunks<NB, KS1, SPC>;
  static constexpr int ST = NB * KS1;
  static constexpr int NCH = ST / SPC;
  static constexpr int DMA = (2 * SPC + 3) / 4;  // weight DMA instructions per chunk and wave
  static constexpr int row_step(int r, int KS) { return (r * KS) / 4; }
  static constexpr int rows_at(int s, int KS) {
    int c = 0;
    for (int r = 0; r < 4; ++r) c += row_step(r, KS) == s ? 1 : 0;
    return c;
  }
  // Deferred tile stores: the staging tile of a finished block is read back (ds_read_b128) after
  // its last row and stored X3_SDLY steps later, so neither the read nor the store waits on LDS
  // latency.  Tile i (G2: E, L, T) is read at step s3 + 1 + i and stored at rd + X3_SDLY, steps
  // of the block whose steps ran the rows; a store past the block's last step runs in the next
  // block (or the pass tail).  Shapes too small for that flush at the last row.
  static constexpr int s3(int KS) { return row_step(3, KS); }
  static constexpr bool defer(int KS, int tiles) {
    return !(X3_OFF & 1) && s3(KS) + tiles < KS && X3_SDLY + tiles - 1 < KS;
  }
  static constexpr int st_step(int KS, int i) { return s3(KS) + 1 + i + X3_SDLY; }
  static constexpr int stores_at(int ib, int s, int KS, int tiles) {
    if (!defer(KS, tiles)) return (ib == 0 || s != s3(KS)) ? 0 : tiles;
    int n = 0;
    for (int i = 0; i < tiles; ++i) {
      const int ss = st_step(KS, i);
      if (ss < KS) n += (ib >= 1 && s == ss) ? 1 : 0;
      else n += (ib >= 2 && s == ss - KS) ? 1 : 0;
    }
    return n;
  }
  // G1 step body: the Z tile store (one dwordx4 per lane)
  static constexpr int ops1(int t) { return stores_at(t / KS1, t % KS1, KS1, 1); }
  // G2 step body: the E, L, T tile stores (+ SAVEP: one P dword store per epilogue row, block
  // ib - 1's rows running in block ib's steps; + PF: V1's per-element beta loads of block
  // ib + 1, PF per row at the row steps of block ib)
  static constexpr int ops2(int t) {
    return stores_at(t / KS2, t % KS2, KS2, 3) +
           ((SAVEP && t / KS2 >= 1) ? rows_at(t % KS2, KS2) : 0) +
           ((PF && t / KS2 + 1 < MB) ? PF * rows_at(t % KS2, KS2) : 0);
  }
  // DMA group of chunk c (c >= NCH: chunk c - NCH of the other pass)
  static constexpr int group(int c, bool g1) {
    if (c >= NCH) return group(c - NCH, !g1);
    if (g1) return DMA + Z::g1_blocks(c);
    return DMA + (c == 0 ? 1 : 0);  // G2 chunk 0 carries the last G1 block's Z
  }
  template <int T, bool G1>
  static constexpr int win() {
    const int ch = T / SPC;
    int n = group(ch + 2, G1) + group(ch + 3, G1);
    for (int u = T - 3 * SPC + (X3_DMA_LATE ? 1 : 0); u < T; ++u) {
      if (u >= 0) n += G1 ? ops1(u) : ops2(u);
      else if (ST + u >= 0) n += G1 ? ops2(ST + u) : ops1(ST + u);
    }
    return n < 63 ? n : 63;
  }
  // X3_BAR2: a barrier every other chunk (odd ch) waits for chunks ch+1 and ch+2, issued (in
  // that order) at the barrier two chunks earlier; younger: the bodies of the 2*SPC steps since
  template <int T, bool G1>
  static constexpr int win2() {
    int n = 0;
    for (int u = T - 2 * SPC; u < T; ++u) {
      if (u >= 0) n += G1 ? ops1(u) : ops2(u);
      else if (ST + u >= 0) n += G1 ? ops2(ST + u) : ops1(ST + u);
    }
    return n < 63 ? n : 63;
  }
};

}  // namespace x3

// LQ: the fused objective's fit term is 0.5 (X - A Z)^2 (LASSO) instead of |X - A Z| -- a
// compile-time choice, so each element accumulates only the term the call reduces
template <int MP, int NP, int EMODE, int PKIND, bool LQ, bool SAVEP>
__global__ __launch_bounds__(256, 1) void fused_x3_kernel(const FusedArgs a) {
  using namespace x3;
  constexpr int MB = MP / 16, NB = NP / 16, KS1 = MP / 32, KS2 = NP / 32;
  constexpr int ST = NB * KS1;  // k-steps of either GEMM
  static_assert(ST == MB * KS2, "both GEMMs have MP*NP/512 steps");
  static_assert(MB % 2 == 0 && NB % 2 == 0, "k-steps cover two 16-row blocks");
  constexpr int SPC = ST < 8 ? ST : 8;  // steps per ring chunk
  static_assert(SPC >= 2 && ST % SPC == 0 && SPC % KS1 == 0, "chunking");
  constexpr int NCH = ST / SPC;
  // the DMA group issued at a barrier targets the chunk 4 ahead: it must lie in this pass or the
  // next (the Z blocks a G1 chunk carries are only complete one pass ahead)
  static_assert(NCH >= kSlots, "at least kSlots chunks per pass");
  static_assert(!X3_BAR2 || (kSlots == 4 && NCH % 2 == 0), "paired barriers: 4 slots, even NCH");
#ifndef X3_ROT
#define X3_ROT 4
#endif
  constexpr int R = ST % X3_ROT == 0 ? X3_ROT : 2;  // fragment register rotation; divides ST, so
                                                    // every pass starts at rotation 0
  constexpr int D = R - 1;                // fragment read-ahead (steps)
  static_assert(ST % R == 0 && SPC >= D + 1, "rotation");
  using ZC = ZChunks<NB, KS1, SPC>;
  constexpr int NZB = ZC::NZB;
  constexpr int FPC = 2 * SPC;                 // 1 KiB weight fragments per chunk
  constexpr int SLOT_F4 = (FPC + kWaves * NZB) * 64;  // + each wave's Z blocks
  constexpr int RING_F4 = kSlots * SLOT_F4;
  constexpr int X_F4 = kWaves * MB * 64;
  constexpr int STG_F4 = kWaves * 4 * 64;  // per wave 4 output tiles of 16 x 16 floats
  static_assert(FPC == 16, "DMA issue: 4 fragments per wave and chunk");
  static_assert((RING_F4 + X_F4 + STG_F4) * 16 <= 160 * 1024, "LDS budget");
  static_assert(PKIND == PK_SCALAR || PKIND == PK_S1 || (PKIND == PK_ELEM && EMODE == EM_V1),
                "x3 path: scalar-parameter variants and V1's per-sample betas");
  constexpr bool kElem = PKIND == PK_ELEM;
  using W = Win<MB, NB, KS1, KS2, SPC, SAVEP, kElem ? 3 : 0>;
  __shared__ f32x4 smem[RING_F4 + X_F4 + STG_F4];
  f32x4* ring = smem;
  f32x4* xs = smem + RING_F4;  // xs[w][b][lane] = X rows 16b+4g+0..3 of this lane's column

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 15, g = lane >> 4;
  const int64_t col = (int64_t)blockIdx.x * kTileCols + w * 16 + j;
  const bool cv = col < a.B;
  const int m = a.m, n = a.n, K = a.K;
  const bool lossz = a.loss_kind != 0;
  auto lane_off = [&](int64_t ld) -> uint32_t {
    return cv ? (uint32_t)((col + (int64_t)(4 * g) * ld) * 4) : kOOB;
  };

  float Er[MB][4], Lr[MB][4], Vr[MB][4];
  BOp Vpk[KS1], Zpk[KS2];
  float regsum = 0.f, fit = 0.f;

  // ---------------------------------------------------------------- Z_{k-1} delivery
  // Block b of the Z matrix the next G1 chunks need (set per pass): rows 16b + (l >> 2), the
  // wave's columns c0 + 4 (l & 3) .. +3 -> LDS [16 rows][16 columns], 64 B rows.  The C ABI
  // routes a batch that is not a multiple of 4, or unaligned rows, to the fp32 kernel, so a
  // lane's 4 columns are all valid or all padding.
  const int64_t c0 = (int64_t)blockIdx.x * kTileCols + w * 16;
  auto off4 = [&](int64_t ld) -> uint32_t {  // lane offset of the 16-B-per-lane form
    const int64_t c4 = c0 + 4 * (lane & 3);
    return c4 < a.B ? (uint32_t)(((lane >> 2) * ld + c4) * 4) : kOOB;
  };
  struct ZSrc { i32x4 r; uint32_t v4; uint32_t ld4; };
  auto zsrc = [&](const float* p, int64_t ld) -> ZSrc {
    return ZSrc{mk_rsrc4(p, (uint32_t)(n * ld * 4)), off4(ld), (uint32_t)(ld * 4)};
  };
  ZSrc zd;  // source of the Z blocks the DMA groups issued during the current pass carry
  auto zdma = [&](int b, const f32x4* dst) {
    if constexpr (!(X3_ABL & 32)) blds16(zd.r, zd.v4, (uint32_t)(16 * b) * zd.ld4, dst);
  };
  // this wave's Z region of a ring slot: [NZB][1 KiB]
  auto zreg = [&](int slot, int q) -> f32x4* {
    return ring + slot * SLOT_F4 + (FPC + w * NZB + q) * 64;
  };
  // rows 4g + 0..3 of the lane's column from a Z block in LDS
  auto zread = [&](const f32x4* blk, float (&v)[4]) {
    const float* f = reinterpret_cast<const float*>(blk);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = f[(4 * g + r) * 16 + j];
  };

  // ---------------------------------------------------------------- output stores
  // An epilogue row writes its value into this wave's 16 x 16 staging tile (LDS, ds_write_b32);
  // once a block's 4 rows are done the tile goes out as ONE buffer_store_dwordx4 per lane (lane
  // l: row l >> 2, columns 4 (l & 3) .. +3 of the wave's 16): 4x fewer store instructions than
  // a dword per row (the store path is per-instruction bound).  Tiles whose rows are not
  // 16-B aligned (or a batch not a multiple of 4) run on the fp32 kernel (C ABI plan).
  f32x4* stg = smem + RING_F4 + X_F4 + w * 4 * 64;
  auto stage = [&](int tile, int r, float v) {
    reinterpret_cast<float*>(stg + tile * 64)[(4 * g + r) * 16 + j] = v;
  };
  // the finished tile -> rows 16b.. of the matrix (voff4: lane offset, soff: the block's rows)
  // v = the tile as read back (lane: its row segment)
  auto flush_v = [&](int tile, rsrc_t rs, uint32_t voff4, uint32_t soff, f32x4 v) {
    if constexpr (X3_ABL & 1024) {
      bstore4(rs, (uint32_t)(lane * 16), 0u, v);
      return;
    }
    if constexpr (X3_ABL & 2048) {  // same bytes, each wave-instruction 1 KiB contiguous
      const uint32_t b = soff / (uint32_t)(64 * a.ldo);
      const uint32_t nb = tile == 0 ? NB : MB;
      bstore4(rs, (uint32_t)(lane * 16), ((blockIdx.x * kWaves + w) * nb + b) * 1024u, v);
      return;
    }
    bstore4(rs, voff4, soff, v);
  };
  auto flush = [&](int tile, rsrc_t rs, uint32_t voff4, uint32_t soff) {
    flush_v(tile, rs, voff4, soff, stg[tile * 64 + lane]);
  };
  // deferred stores (Win::stores_at): the tile read back one step after the block's last row
  f32x4 pst[3];
  uint32_t pso = 0u;

  // ---------------------------------------------------------------- weight stream
  // GEMM gi: 0 = prologue A, 2k+1 = -W_k, 2k+2 = A; past the last GEMM, A again as filler.
  const int64_t wl = (int64_t)ST * 2 * kFrag;  // floats per packed tensor: ST x (hi, lo) KiB
  auto gsrc = [&](int gi) -> const float* {
    const int kk = gi >> 1;
    return ((gi & 1) && kk < K) ? a.Wp + (int64_t)(kk * a.wstep) * wl : a.Ap;
  };
  auto chunk_src = [&](int gi, int ch) -> const float* {
    uint64_t sb = (uint64_t)gsrc(gi + ch / NCH);
    asm volatile("" : "+s"(sb));
    return (const float*)sb + (int64_t)(ch % NCH) * FPC * kFrag;
  };
  // DMA group of chunk CH (relative to the pass: CH >= NCH = the next pass) into `slot`
  auto issue = [&](auto G1_, auto CH_, int gi, int slot) {
    constexpr bool G1 = decltype(G1_)::value;
    constexpr int CH = decltype(CH_)::value;
    const float* base = chunk_src(gi, CH);
    f32x4* dst = ring + slot * SLOT_F4;
    // wave w: fragments 4w .. 4w+3
    if constexpr (!(X3_ABL & 1)) glds16x4(base + 4 * w * kFrag, lane * 16, dst + 4 * w * 64);
    constexpr bool tg1 = (CH < NCH) == G1;  // the target chunk is a G1 chunk
    constexpr int tc = CH < NCH ? CH : CH - NCH;
    if constexpr (tg1) {
      static_for<NZB>([&](auto Q_) {
        constexpr int q = decltype(Q_)::value;
        if constexpr (ZC::g1_block(tc, q) >= 0) zdma(ZC::g1_block(tc, q), zreg(slot, q));
      });
    } else if constexpr (tc == 0 && G1) {
      zdma(NB - 1, zreg(slot, 0));  // the last G1 block, for the tail after the pass
    }
  };
  auto slot_add = [](int s, int d) -> int { s += d; return s >= kSlots ? s - kSlots : s; };
  int cur = 0;
  auto frag = [&](int slot, int f) -> f16x8 {
    if constexpr (X3_ABL & 64) {
      f16x8 v = {};
      v[0] = (_Float16)(float)(slot * 16 + f);
      return v;
    }
    return __builtin_bit_cast(f16x8, ring[slot * SLOT_F4 + f * 64 + lane]);
  };

  // ---------------------------------------------------------------- parameters
  struct LayerP { float b1n, b2, b3, ss2, ss2b, s1; ShrinkP the, thz; };
  auto layer_params = [&](int k) -> LayerP {
    LayerP p{};
    const int kk = k < 0 ? 0 : k;
    const int kn = k < 0 ? 0 : (k + 1 < K ? k + 1 : k);
    cfloat_p sp = (cfloat_p)a.scal + kk * DLADMM_NSCALAR;
    p.b2 = sp[DLADMM_P_BETA2];
    p.b3 = sp[DLADMM_P_BETA3];
    p.ss2 = sp[DLADMM_P_SS2];
    p.ss2b = sp[DLADMM_P_SS2B];
    p.the = shrink_params(sp[DLADMM_P_THETA_E]);
    p.thz = shrink_params(sp[DLADMM_P_THETA_Z]);
    if constexpr (PKIND == PK_S1) p.s1 = sp[DLADMM_P_S1];
    p.b1n = ((cfloat_p)a.scal)[kn * DLADMM_NSCALAR + DLADMM_P_BETA1];
    return p;
  };
  // weight scale exponents (pack kernel): wexp[0] = A, wexp[1 + k] = -W_k (shared: wexp[1])
  const int sw_a = __builtin_amdgcn_readfirstlane(a.wexp[0]);
  auto sw_w = [&](int k) -> int {
    return __builtin_amdgcn_readfirstlane(a.wexp[1 + (a.wstep ? k : 0)]);
  };

  // ---------------------------------------------------------------- initial state
  const uint32_t oz0 = lane_off(a.ldz0), oo = lane_off(a.ldo), ozw = lane_off(a.ldzw);
  const uint32_t ozw4 = off4(a.ldzw);
  float zmx = 0.f;        // lane max of |Z_k| of the layer being formed
  float zmx_prev;         // column max of Z_{k-1} (Z0 first), exact
  int zexp;               // scale exponent the current Zpk was split with
  {
    const rsrc_t re = mkrsrc(a.E0, (uint32_t)(m * a.lde0 * 4));
    const rsrc_t rl = mkrsrc(a.L0, (uint32_t)(m * a.ldl0 * 4));
    const rsrc_t rx = mkrsrc(a.X, (uint32_t)(m * a.ldx * 4));
    const uint32_t oe = lane_off(a.lde0), ol = lane_off(a.ldl0), ox = lane_off(a.ldx);
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      f32x4 xv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        xv[r] = bload(rx, ox + (uint32_t)((16 * b + r) * a.ldx * 4));
        Er[b][r] = bload(re, oe + (uint32_t)((16 * b + r) * a.lde0 * 4));
        Lr[b][r] = bload(rl, ol + (uint32_t)((16 * b + r) * a.ldl0 * 4));
      }
      xs[(w * MB + b) * 64 + lane] = xv;  // read back only by this wave
      __builtin_amdgcn_sched_barrier(0);
    }
    // Z0: exact column max, then re-read and split (no fp32 copy of Z0 stays live)
    const rsrc_t rz = mkrsrc(a.Z0, (uint32_t)(n * a.ldz0 * 4));
    float mx = 0.f;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        mx = fmaxf(mx, fabsf(bload(rz, oz0 + (uint32_t)((16 * b + r) * a.ldz0 * 4))));
      if (b % 4 == 3) __builtin_amdgcn_sched_barrier(0);  // at most 16 loads in flight
    }
    zmx_prev = col_max(mx);
    zexp = scale_exp(zmx_prev, sw_a, 0);
    const float sc = exp2i(zexp);
#pragma unroll
    for (int s = 0; s < KS2; ++s) {
      float va[4], vb[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        va[r] = bload(rz, oz0 + (uint32_t)((32 * s + r) * a.ldz0 * 4));
        vb[r] = bload(rz, oz0 + (uint32_t)((32 * s + 16 + r) * a.ldz0 * 4));
      }
      Zpk[s] = split8(va, vb, sc);
      pin_agpr_b(Zpk[s]);
      if (s % 2 == 1) __builtin_amdgcn_sched_barrier(0);
    }
  }

  const uint32_t mbytes = (uint32_t)(m * a.ldo * 4);
  const uint32_t oo4 = off4(a.ldo);
  SWalk zw{0u, (uint32_t)(a.ldo * 4)}, mw{0u, (uint32_t)(a.ldo * 4)};

  // ---------------------------------------------------------------- epilogues
  // G1 block b, row r of layer k: Z = S(Z_{k-1} + s1 * q, theta_z) with q = -W_k Var (the packed
  // weights are negated), main_lena.py:86 / main_syn_l1l1_scalar_tied.py:114
  float zn[2][4];        // fp32 Z_k of the current block pair, split into Zpk when complete
  float zo[NZB][4];      // Z_{k-1} of the blocks whose epilogues run in the current chunk
  // acc = the chain's raw sum; qs = 2^-(sW + sVar) (times s1 for V5): acc * qs is exactly the
  // reference's fc(Var) (s1 * fc(Var)) up to the GEMM's rounding, so the fma is one rounding of
  // Z_{k-1} - fc(Var) like the reference's subtraction
  auto epi1_row = [&](const LayerP& P, int b, int r, float zp, float acc, float qs) {
    if constexpr (X3_ABL & 2) {  // keep the MFMA chain alive
      zn[b & 1][r] = acc;
      asm volatile("" ::"v"(acc));
      return;
    }
    float u;
    if constexpr (PKIND == PK_S1) u = zp + acc * qs;
    else u = __builtin_fmaf(acc, qs, zp);
    const float z = shrink_u(u, P.thz);
    zn[b & 1][r] = z;
    stage(0, r, z);
    regsum += fabsf(z);
    if (r & 1) zmx = amax2(zmx, zn[b & 1][(r - 1) & 3], z);  // rows in pairs: one v_max3
    // materialise the running sums here: left alone, the scheduler sinks both serial chains
    // below the pass and keeps every row's z live (spills)
    asm volatile("" : "+v"(regsum), "+v"(zmx));
  };
  // G2 block b, row r of layer k (Pv = A Z_k, x = X).  pro: T0 = A Z0 + E0 - X, Var_0.
  struct OutR { rsrc_t e, l, t, p; };
  auto flush2 = [&](const OutR& O, uint32_t soff) {
    flush(1, O.e, oo4, soff);
    flush(2, O.l, oo4, soff);
    flush(3, O.t, oo4, soff);
  };
  float vmx = 0.f, vpend = 0.f;
  // V1 (PK_ELEM): the per-sample betas of the G2 rows -- beta1_k (the L update, main_lena.py:89),
  // beta2_k (the E-step, :87) and beta1_{k+1} (the next Var, :85) of block b, row r -- loaded two
  // blocks ahead of their epilogue row into a 3-block ring of registers (pf_block below)
  float pb[kElem ? 3 : 1][3][4];
  auto epi2_row = [&](const LayerP& P, bool pro, int b, int r, float Pv, float x, const OutR& O) {
    // SAVEP: A Z_k for the backward, the product exactly as the updates below consume it (a
    // dword store per row: the staging tiles carry E, L, T); mw still at block b's rows here
    if constexpr (SAVEP) bstore_s(O.p, oo, mw.at(r), Pv);
    if constexpr (X3_ABL & 2) {
      Vr[b][r] = Pv;
      pin_agpr(Vr[b][r]);
      asm volatile("" ::"v"(Pv));
      return;
    }
    const float l0 = Lr[b][r];
    const float e0 = Er[b][r];
    float b2 = P.b2, b3 = P.b3, b1n = P.b1n;
    if constexpr (kElem) {
      b3 = pb[b % 3][0][r];
      b2 = pb[b % 3][1][r];
      b1n = pb[b % 3][2][r];
    }
    float e;
    if constexpr (EMODE == EM_V1) {
      e = shrink_u((x - Pv) - b2 * l0, P.the);                       // main_lena.py:87
    } else if constexpr (EMODE == EM_VVAR) {
      const float vv = l0 + P.b2 * ((Pv + e0) - x);                  // scalar :114
      e = shrink_u(e0 - P.ss2 * vv, P.the);                          // scalar :115
    } else {
      e = P.ss2 * (x - Pv) - P.ss2b * l0;                            // lasso :102-103
    }
    e = pro ? e0 : e;
    const float t = (Pv + e) - x;                                    // main_lena.py:88
    float l = l0 + b3 * t;                                           // main_lena.py:89
    l = pro ? l0 : l;
    Er[b][r] = e;
    Lr[b][r] = l;
    stage(1, r, e);
    stage(2, r, l);
    stage(3, r, t);
    const float res = x - Pv;
    if constexpr (LQ) fit = __builtin_fmaf(res, res, fit);
    else fit += fabsf(res);
    const float v = l + b1n * t;                                     // main_lena.py:85
    if (r & 1) vmx = amax2(vmx, vpend, v);  // rows in pairs: one v_max3
    else vpend = v;
    asm volatile("" : "+v"(fit), "+v"(vmx));
    Vr[b][r] = v;
    pin_agpr(Vr[b][r]);  // AGPRs: Vr, Zpk (G2) / Vpk, Zpk (G1); VGPRs: E, L, fragments
  };
  auto flush_loss = [&](int k) {
    if (lossz && k >= 0) {
      const float rs = col_sum(regsum);
      const float fs = LQ ? 0.5f * col_sum(fit) : col_sum(fit);
      if (g == 0) {
        const int64_t c = (int64_t)blockIdx.x * kTileCols + w * 16 + j;
        a.lossp[(int64_t)(2 * k + 0) * a.ldl + c] = rs;
        a.lossp[(int64_t)(2 * k + 1) * a.ldl + c] = fs;
      }
    }
    regsum = 0.f;
    fit = 0.f;
  };

  // ---------------------------------------------------------------- ring steps
  // Step t of a GEMM pass: head = read-ahead of step t+D's two fragments (at chunk position
  // SPC-D: ring barrier, DMA group of chunk ch+4 into the freed slot, first fragments of the
  // next chunk), then the step body (epilogue rows / operand splits), then 3 MFMAs.
  f16x8 frh[R], frl[R];
#if X3_STAMP
  // diagnostic build: per-wave cycle sums (cdna_hip_programming.md, In-kernel stamps); read
  // their shares only, never this build's run time
  auto stamp = []() -> uint64_t {
    uint64_t v;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
    return v;
  };
  uint64_t st_vm = 0, st_bar = 0, st_g1 = 0, st_g2 = 0, st_mid = 0;
  const uint64_t st_0 = stamp();
#endif
  auto step_head = [&](auto G1_, auto T_, int gi) {
    constexpr bool G1 = decltype(G1_)::value;
    constexpr int t = decltype(T_)::value;
    constexpr int c = t % SPC, ch = t / SPC;
    constexpr int tn = t + D;
    if constexpr (c + D < SPC) {
      frh[tn % R] = frag(cur, 2 * (c + D));
      frl[tn % R] = frag(cur, 2 * (c + D) + 1);
    } else {
      // every wave has read all of chunk ch (its last fragments D steps ago, its Z blocks at
      // the chunk's first step)
      // X3_BAR2: barriers at odd chunks only, each refilling two slots
      constexpr bool BAR = !X3_BAR2 || ch % 2 == 1;
      constexpr int WN = (X3_ABL & 128) ? 63
                         : X3_BAR2     ? W::template win2<t, G1>()
                                       : W::template win<t, G1>();
      if constexpr (c + D == SPC && BAR) {
        if constexpr (X3_ABL & 256) {
          if constexpr (X3_ABL & 512) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WN) : "memory");
          else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(WN) : "memory");
        } else {
#if X3_STAMP
          __builtin_amdgcn_sched_barrier(0);
          const uint64_t t0 = stamp();
          asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(WN) : "memory");
          const uint64_t t1 = stamp();
          asm volatile("s_barrier" ::: "memory");
          const uint64_t t2 = stamp();
          __builtin_amdgcn_sched_barrier(0);
          st_vm += t1 - t0;
          st_bar += t2 - t1;
#else
          ring_barrier_cnt<WN>();
#endif
        }
        if constexpr (X3_BAR2) {
          // slots of chunks ch-1 and ch are free: chunks ch+3, ch+4
          issue(G1_, std::integral_constant<int, ch + 3>{}, gi, slot_add(cur, kSlots - 1));
          issue(G1_, std::integral_constant<int, ch + 4>{}, gi, cur);
        } else if constexpr (!X3_DMA_LATE) {
          issue(G1_, std::integral_constant<int, ch + kSlots>{}, gi, cur);
        }
      }
      const int nx = slot_add(cur, 1);
      frh[tn % R] = frag(nx, 2 * (c + D - SPC));
      frl[tn % R] = frag(nx, 2 * (c + D - SPC) + 1);
    }
  };
  auto step_tail = [&](auto T_, auto G1_, int gi) {
    constexpr int t = decltype(T_)::value;
    if constexpr (X3_DMA_LATE && !X3_BAR2 && t % SPC + D == SPC) {
      // the barrier step's DMA group, after its MFMAs (the barrier in its head freed slot cur)
      __builtin_amdgcn_sched_barrier(0);
      issue(G1_, std::integral_constant<int, t / SPC + kSlots>{}, gi, cur);
    }
#if X3_SGB
    // MFMA, X3_SGB fillers, MFMA, X3_SGB fillers, MFMA, rest (filler classes: X3_SGM)
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(X3_SGM, X3_SGB, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(X3_SGM, X3_SGB, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#endif
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (t % SPC == SPC - 1) cur = slot_add(cur, 1);
  };
  auto mfma3 = [&](int tr, const BOp& bop, f32x4 acc) -> f32x4 {
    if constexpr (X3_ABL & 16) {
      acc[0] += (float)frh[tr][0] + (float)bop.hi[0] + (float)bop.lo[1] + (float)frl[tr][2];
      return acc;
    }
    acc = mfma(frh[tr], bop.hi, acc);
    acc = mfma(frh[tr], bop.lo, acc);
    return mfma(frl[tr], bop.hi, acc);
  };

  // prime the ring: chunks 0..3 of the prologue GEMM (its following G1(0) chunks carry Z0)
  zd = zsrc(a.Z0, a.ldz0);
  static_for<kSlots>([&](auto C_) { issue(std::false_type{}, C_, 0, decltype(C_)::value); });
  ring_barrier_cnt<0>();
#pragma unroll
  for (int t = 0; t < D; ++t) {
    frh[t] = frag(0, 2 * t);
    frl[t] = frag(0, 2 * t + 1);
  }

  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

  // ---------------------------------------------------------------- G1(k): -W_k Var -> Z_k
  // Block ib's epilogue runs in block ib+1's steps (row r at step (r*KS1)/4) on the Z_{k-1}
  // block its chunk carried; Zpk[s] is split once blocks 2s, 2s+1 are complete; block 0's steps
  // split Var into Vpk.  The last block's epilogue runs after the MFMAs.
  constexpr int S31 = W::s3(KS1), S32 = W::s3(KS2);
  constexpr bool DF1 = W::defer(KS1, 1), DF2 = W::defer(KS2, 3);
  constexpr bool ZE = !(X3_OFF & 2) && NZB == 1 && S31 < SPC - 1;  // G1: Z_{k-1} read early
  constexpr bool XE = !(X3_OFF & 4) && S32 + 1 < KS2;  // G2: X rows read after the last use
  auto g1_pass = [&](int k, const LayerP& P, rsrc_t rzo, uint32_t vzo4, uint32_t vzo, float vsc,
                     float qs, float zsc) {
    const int gi = 2 * k + 1;
    zw.reset();
    SWalk zs = zw;
    f32x4 qp = zero4;
    static_for<NB>([&](auto IB_) {
      constexpr int ib = decltype(IB_)::value;
      f32x4 acc = zero4;
      static_for<KS1>([&](auto S_) {
        constexpr int s = decltype(S_)::value;
        constexpr int t = ib * KS1 + s;
        // first step of a chunk: its Z_{k-1} blocks -> registers (before the slot is reused);
        // with one Z block per chunk (ZE) that read runs one step early, below
        if constexpr (!ZE && t % SPC == 0) {
          static_for<NZB>([&](auto Q_) {
            constexpr int q = decltype(Q_)::value;
            if constexpr (ZC::g1_block(t / SPC, q) >= 0) zread(zreg(cur, q), zo[q]);
          });
        }
        step_head(std::true_type{}, std::integral_constant<int, t>{}, gi);
        if constexpr (ib == 0) {
          Vpk[s] = split8(Vr[2 * s], Vr[2 * s + 1], vsc);
          pin_agpr_b(Vpk[s]);
        } else {
          static_for<4>([&](auto R_) {
            constexpr int r = decltype(R_)::value;
            if constexpr (W::row_step(r, KS1) == s) {
              constexpr int q = (ib - 1) + 1 - (t / SPC) * NZB;  // Z block slot in this chunk
              epi1_row(P, ib - 1, r, zo[q][r], qp[r], qs);
              if constexpr (r == 3 && !DF1) {
                flush(0, rzo, vzo4, zs.at(0));
                zs.next();
              }
            }
          });
          if constexpr (DF1) {
            constexpr int ss = W::st_step(KS1, 0);
            if constexpr (ss < KS1 ? s == ss : (ib >= 2 && s == ss - KS1))
              flush_v(0, rzo, vzo4, pso, pst[0]);
            if constexpr (s == S31 + 1) {
              pso = zs.at(0);
              zs.next();
              pst[0] = stg[lane];
            }
          }
          // blocks 2s', 2s'+1 complete (the odd block's last row ran at this step or before)
          if constexpr (((ib - 1) & 1) && s == KS1 - 1) {
            constexpr int sp = (ib - 1) / 2;
            Zpk[sp] = split8(zn[0], zn[1], zsc);
            pin_agpr_b(Zpk[sp]);
          }
        }
        // ZE: the next chunk's Z_{k-1} block (slot cur+1, landed at this chunk's barrier), read
        // at this chunk's last step -- after the last row that used zo -- so the next chunk's
        // first row does not wait on LDS latency
        if constexpr (ZE && t % SPC == SPC - 1 && t / SPC + 1 < NCH) {
          if constexpr (ZC::g1_block(t / SPC + 1, 0) >= 0) zread(zreg(slot_add(cur, 1), 0), zo[0]);
        }
        acc = mfma3(t % R, Vpk[s], acc);
        step_tail(std::integral_constant<int, t>{}, std::true_type{}, gi);
      });
      qp = acc;
    });
    // tail: block NB-2's deferred store (if it wrapped), block NB-1 (its Z_{k-1} block rode on
    // the next G2 chunk 0, now slot cur)
    if constexpr (DF1 && W::st_step(KS1, 0) >= KS1) flush_v(0, rzo, vzo4, pso, pst[0]);
    float zl[4];
    zread(zreg(cur, 0), zl);
#pragma unroll
    for (int r = 0; r < 4; ++r) epi1_row(P, NB - 1, r, zl[r], qp[r], qs);
    flush(0, rzo, vzo4, zs.at(0));
    Zpk[KS2 - 1] = split8(zn[0], zn[1], zsc);
    pin_agpr_b(Zpk[KS2 - 1]);
  };

  // ---------------------------------------------------------------- G2(k): A Z_k -> E, L, T, Var
  // V1: per-element beta views of the pass, lane offset (rows 4g.. of the lane's column; padded
  // columns and rows past m read 0 through the buffer range)
  const uint32_t vb = lane_off(a.ldb);
  rsrc_t rb1 = mkrsrc(nullptr, 0u), rb2 = rb1, rbn = rb1;
  // row offsets walk in program order (one SGPR pair, advanced per block): precomputed per
  // (block, row) they were hoisted into ~64 SGPRs and spilled
  SWalk bw{0u, (uint32_t)(a.ldb * 4)};
  auto pf_row = [&](auto B_, auto R_) {
    constexpr int bb = decltype(B_)::value, rr = decltype(R_)::value;
    if constexpr (kElem) {
      const int so = (int)bw.at(rr);
      pb[bb % 3][0][rr] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb1, (int)vb, so, 0));
      pb[bb % 3][1][rr] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb2, (int)vb, so, 0));
      pb[bb % 3][2][rr] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rbn, (int)vb, so, 0));
      if constexpr (rr == 3) bw.next();
    }
  };
  auto g2_pass = [&](auto PRO_, int k, const LayerP& P, const OutR& O, float zinv) {
    constexpr bool PRO = decltype(PRO_)::value;
    const int gi = 2 * k + 2;
    mw.reset();
    f32x4 qp = zero4;
    f32x4 xv;
    if constexpr (kElem) {
      // beta1_k, beta2_k, beta1_{k+1} (the prologue: beta1_0 for Var_0 only), from the device
      // tables by scalar loads; then block 0's rows, ahead of the pass
      typedef const float* const __attribute__((address_space(4)))* ctab_p;
      const ctab_p t1 = (ctab_p)a.b1t, t2 = (ctab_p)a.b2t;
      const uint32_t eb = (uint32_t)(m * a.ldb * 4);
      const int kn = k + 1;
      rb1 = mkrsrc(PRO ? nullptr : t1[k < 0 ? 0 : k], PRO ? 0u : eb);
      rb2 = mkrsrc(PRO ? nullptr : t2[k < 0 ? 0 : k], PRO ? 0u : eb);
      rbn = mkrsrc(kn < K ? t1[kn] : nullptr, kn < K ? eb : 0u);
      bw.reset();
      static_for<4>([&](auto R_) { pf_row(std::integral_constant<int, 0>{}, R_); });
    }
    static_for<MB>([&](auto IB_) {
      constexpr int ib = decltype(IB_)::value;
      f32x4 acc = zero4;
      if constexpr (!XE && ib > 0) xv = xs[(w * MB + ib - 1) * 64 + lane];
      static_for<KS2>([&](auto S_) {
        constexpr int s = decltype(S_)::value;
        constexpr int t = ib * KS2 + s;
        step_head(std::false_type{}, std::integral_constant<int, t>{}, gi);
        // V1: block ib + 1's betas, one row per epilogue-row step (two blocks ahead of use)
        if constexpr (kElem && ib + 1 < MB) {
          static_for<4>([&](auto R_) {
            if constexpr (W::row_step(decltype(R_)::value, KS2) == s)
              pf_row(std::integral_constant<int, ib + 1>{}, R_);
          });
        }
        // XE: X rows of block ib (for its epilogue rows in block ib+1's steps / the tail), read
        // once block ib-1's last row has used xv
        if constexpr (XE && s == (ib == 0 ? 0 : S32 + 1)) xv = xs[(w * MB + ib) * 64 + lane];
        if constexpr (ib > 0) {
          static_for<4>([&](auto R_) {
            constexpr int r = decltype(R_)::value;
            if constexpr (W::row_step(r, KS2) == s) {
              epi2_row(P, PRO, ib - 1, r, qp[r] * zinv, xv[r], O);
              if constexpr (r == 3 && !DF2) {
                flush2(O, mw.at(0));
                mw.next();
              }
            }
          });
          if constexpr (DF2) {
            // tile i (E, L, T): read back at step S32 + 1 + i, stored X3_SDLY steps later
            static_for<3>([&](auto I_) {
              constexpr int i = decltype(I_)::value;
              constexpr int ss = W::st_step(KS2, i);
              if constexpr (ss < KS2 ? s == ss : (ib >= 2 && s == ss - KS2))
                flush_v(1 + i, i == 0 ? O.e : (i == 1 ? O.l : O.t), oo4, pso, pst[i]);
              if constexpr (s == S32 + 1 + i) {
                if constexpr (i == 0) {
                  pso = mw.at(0);
                  mw.next();
                }
                pst[i] = stg[(1 + i) * 64 + lane];
              }
            });
          }
        }
        acc = mfma3(t % R, Zpk[s], acc);
        step_tail(std::integral_constant<int, t>{}, std::false_type{}, gi);
      });
      qp = acc;
    });
    // block MB-2's stores that wrapped past the pass
    if constexpr (DF2) {
      static_for<3>([&](auto I_) {
        constexpr int i = decltype(I_)::value;
        if constexpr (W::st_step(KS2, i) >= KS2)
          flush_v(1 + i, i == 0 ? O.e : (i == 1 ? O.l : O.t), oo4, pso, pst[i]);
      });
    }
    if constexpr (!XE) xv = xs[(w * MB + MB - 1) * 64 + lane];
#pragma unroll
    for (int r = 0; r < 4; ++r) epi2_row(P, PRO, MB - 1, r, qp[r] * zinv, xv[r], O);
    flush2(O, mw.at(0));
  };

  // ---------------------------------------------------------------- prologue + K layers
  const rsrc_t none = mkrsrc(nullptr, 0u);
  {
    const LayerP P0 = layer_params(-1);
    const OutR O0{none, none,
                  mkrsrc(a.keep_all ? a.To : nullptr, (a.keep_all && a.To) ? mbytes : 0u), none};
    g2_pass(std::true_type{}, -1, P0, O0, exp2i(-(zexp + sw_a)));
  }
  flush_loss(-1);
  for (int k = 0; k < K; ++k) {
    const bool last = k == K - 1;
    const LayerP P = layer_params(k);
    const int swk = sw_w(k);
    // Var_k (from G2(k-1) / the prologue): exact column scale for this layer's weight
    const int vexp = scale_exp(col_max(vmx), swk, 0);
    vmx = 0.f;
    // Z_{k-1} -- the DMA source of this pass's groups (G1(k) chunks, G2(k) chunk 0) -- is set
    // (previous pass); Z_k goes to the output (keep_all or last layer) or the lean workspace
    const bool zout = a.keep_all || last;
    const int64_t ldzo = zout ? a.ldo : a.ldzw;
    float* zop = zout ? a.Zo + (int64_t)(a.keep_all ? k : 0) * n * a.ldo
                      : a.Zw + (int64_t)(k & 1) * n * a.ldzw;
    const rsrc_t rzo = mkrsrc(zop, (uint32_t)(n * ldzo * 4));
    const uint32_t vzo = zout ? oo : ozw;
    const uint32_t vzo4 = zout ? oo4 : ozw4;
    zw = SWalk{0u, (uint32_t)(ldzo * 4)};
    // provisional scale of Z_k's split: the column max of Z_{k-1} with kHead bits of headroom
    const int zexp_p = scale_exp(zmx_prev, sw_a, kHead);
    zmx = 0.f;
    const float qs = (PKIND == PK_S1 ? P.s1 : 1.0f) * exp2i(-(vexp + swk));
#if X3_STAMP
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t ta = stamp();
    __builtin_amdgcn_sched_barrier(0);
#endif
    g1_pass(k, P, rzo, vzo4, vzo, exp2i(vexp), qs, exp2i(zexp_p));
#if X3_STAMP
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t tb = stamp();
    __builtin_amdgcn_sched_barrier(0);
    st_g1 += tb - ta;
#endif
    // the groups issued during G2(k) carry Z_k for G1(k+1)
    zd = zsrc(zop, ldzo);
    // exact column max of Z_k; re-split if a column outgrew the provisional scale
    const float zm = col_max(zmx);
    zmx_prev = zm;
    zexp = zexp_p;
    if (__any(zm * exp2i(zexp_p) >= 65504.0f)) {  // wave-uniform; rare (first layer)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's Z_k stores
      zexp = scale_exp(zm, sw_a, 0);
      const float sc = exp2i(zexp);
      SWalk rw{0u, (uint32_t)(ldzo * 4)};
#pragma unroll
      for (int s = 0; s < KS2; ++s) {
        float va[4], vb[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          va[r] = bload(rzo, vzo + rw.at(32 * s + r));
          vb[r] = bload(rzo, vzo + rw.at(32 * s + 16 + r));
        }
        Zpk[s] = split8(va, vb, sc);
        pin_agpr_b(Zpk[s]);
        if (s % 2 == 1) __builtin_amdgcn_sched_barrier(0);
      }
    }
    const bool st = a.keep_all || last;
    const int ko = a.keep_all ? k : 0;
    const OutR O{mkrsrc(a.Eo + (int64_t)ko * m * a.ldo, st ? mbytes : 0u),
                 mkrsrc(a.Lo + (int64_t)ko * m * a.ldo, st ? mbytes : 0u),
                 mkrsrc(a.To ? a.To + (int64_t)(a.keep_all ? k + 1 : 0) * m * a.ldo : nullptr,
                        (a.To && st) ? mbytes : 0u),
                 mkrsrc(SAVEP && a.Po && a.keep_all ? a.Po + (int64_t)k * m * a.ldo : nullptr,
                        SAVEP && a.Po && a.keep_all ? mbytes : 0u)};
#if X3_STAMP
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t tc = stamp();
    __builtin_amdgcn_sched_barrier(0);
    st_mid += tc - tb;
#endif
    g2_pass(std::false_type{}, k, P, O, exp2i(-(zexp + sw_a)));
#if X3_STAMP
    __builtin_amdgcn_sched_barrier(0);
    st_g2 += stamp() - tc;
    __builtin_amdgcn_sched_barrier(0);
#endif
    flush_loss(k);
  }
  // drain: the ring's last LDS-DMAs must land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if X3_STAMP
  const uint64_t st_end = stamp();
  if (a.dbg && lane < 8) {  // vector stores: lane i writes sum i
    const uint64_t v[8] = {st_end - st_0, st_g1, st_g2, st_mid, st_vm, st_bar, 0, 0};
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x = lane == i ? v[i] : x;
    a.dbg[((int64_t)blockIdx.x * kWaves + w) * 8 + lane] = x;
  }
#endif
}

template <int MP, int NP, int EM, int PK, bool SAVEP>
hipError_t launch_x3(const FusedArgs& a, int grid, hipStream_t s) {
  if (a.loss_kind == DLADMM_LOSS_LASSO)
    hipLaunchKernelGGL((fused_x3_kernel<MP, NP, EM, PK, true, SAVEP>), dim3(grid), dim3(256), 0,
                       s, a);
  else
    hipLaunchKernelGGL((fused_x3_kernel<MP, NP, EM, PK, false, SAVEP>), dim3(grid), dim3(256), 0,
                       s, a);
  return hipGetLastError();
}

template <int MP, int NP, bool SAVEP>
hipError_t dispatch_x3_variant(int variant, const FusedArgs& a, int grid, hipStream_t s) {
  switch (variant) {
    case DLADMM_V4_SCALAR: return launch_x3<MP, NP, EM_VVAR, PK_SCALAR, SAVEP>(a, grid, s);
    case DLADMM_V5_TIED: return launch_x3<MP, NP, EM_VVAR, PK_S1, SAVEP>(a, grid, s);
    case DLADMM_V6_LASSO: return launch_x3<MP, NP, EM_LASSO, PK_SCALAR, SAVEP>(a, grid, s);
    case DLADMM_V1_LENA: return launch_x3<MP, NP, EM_V1, PK_ELEM, SAVEP>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

// Shapes 1 and 2 only: shape 0 (32 x 32) has fewer than kSlots chunks per pass; the C ABI
// runs those problems on shape 1 (zero padding is exact).
template <bool SAVEP>
hipError_t launch_x3_shape(int shape, int variant, const FusedArgs& a, int grid, hipStream_t s) {
  switch (shape) {
    case 1: return dispatch_x3_variant<kShapeMP[1], kShapeNP[1], SAVEP>(variant, a, grid, s);
    case 2: return dispatch_x3_variant<kShapeMP[2], kShapeNP[2], SAVEP>(variant, a, grid, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace dladmm
