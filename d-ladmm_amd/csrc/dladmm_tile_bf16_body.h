// dladmm_tile_bf16_body.h -- one output tile of the bf16 mode's per-layer products (BASELINE
// config 5), shared by the one-phase kernel (dladmm_tile_bf16.hip: a launch = one layer product
// over the whole batch) and the two-phase kernel (dladmm_tile_bf16_pair.hip: a launch = one
// product for each of two column halves that are one phase apart).  Design notes: the header of
// dladmm_tile_bf16.hip.
#pragma once

#include "dladmm_common.h"
#include "dladmm_internal.h"
#include "dladmm_layer_epi.h"

#ifndef DLADMM_TILE_DPOS
#define DLADMM_TILE_DPOS 2  // where a stage's LDS-DMA pieces issue (A/B, same results): 0 half
                            // beside the second half's fragment reads, half between the MFMA
                            // halves; 1 all between the halves; 2 one after each group of 4 MFMAs
                            // (2: 7.04-7.08 vs 7.09-7.11 ms per config-5 forward, r05_tile_dpos.json)
#endif
#ifndef DLADMM_TILE_EXP
#define DLADMM_TILE_EXP 0  // experiment bits (WRONG results): 1 no in-loop DMA, 2 no MFMA,
                           // 4 no epilogue
#endif

namespace dladmm {

// Tile geometry by workgroup width NW (8 waves: 256 columns, 4: 128 columns).  Every wave owns
// 128 rows x 64 columns; a stage is one k-block of the tile's 16 A and NW/2*4 B fragments, each
// wave LDS-DMAs FPW of them; the ring holds NST stages and the barrier's counted vmcnt keeps the
// NST - 2 stages issued after the awaited one in flight.
template <int NW>
struct TileG {
  static constexpr int NWC = NW / 2;                // wave columns (2 wave rows)
  static constexpr int CBT = 4 * NWC;               // column blocks per tile
  static constexpr int SF = kTileBlocks + CBT;      // fragments per stage
  static constexpr int FPW = SF / NW;               // fragments per wave per stage
  static constexpr int NST = NW == 8 ? 4 : 3;       // ring stages (128 KiB / 72 KiB)
  static constexpr int VMC = FPW * (NST - 2);       // younger DMA pieces at the barrier
  static constexpr int H1 = FPW / 2;                // pieces issued before the first MFMA half
  static_assert(SF % NW == 0 && FPW % 2 == 0, "even share of every stage per wave");
  static_assert(NST * SF * 1024 <= (NW == 8 ? 160 : 80) * 1024, "LDS: 1 (8 waves) / 2 per CU");
};
constexpr int kWaveRB = 8, kWaveCB = 4;  // blocks per wave: 128 rows x 64 columns
static_assert(2 * kWaveRB == kTileBlocks, "2 wave rows");

// One output tile (row tile `by`, column tile `bx`) of one layer product, main loop and fused
// epilogue.  `ring` is the workgroup's LDS ring (TileG<NW>::NST stages of SF fragments).
template <int EMODE, int PKIND, int PH, int NW>
__device__ __forceinline__ void tile_body(const LayerArgs& a, f32x4* ring, int bx, int by) {
  using G = TileG<NW>;
  constexpr int SF = G::SF, FPW = G::FPW, NST = G::NST;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w / G::NWC, wc = w % G::NWC;
  const int g = lane >> 4;
  const int ib0 = by * kTileBlocks;  // first output row block of the tile
  const int cb0 = bx * G::CBT;       // first column block
  const int KB = a.KB;

  // piece q (0..FPW-1) of wave w is stage fragment f = FPW w + q: f < 16 the weights' row block
  // ib0 + f, else the state's column block cb0 + f - 16 (wave-uniform either way)
  auto issue = [&](int kb, int slot, int q) {
    const int f = FPW * w + q;
    const float* src = f < kTileBlocks
        ? a.Wp + ((int64_t)kb * a.MBp + ib0 + f) * kFrag
        : a.S + ((int64_t)kb * a.nbp + cb0 + f - kTileBlocks) * kFrag;
    uint64_t sb = (uint64_t)src;
    asm volatile("" : "+s"(sb));
    glds16((const float*)sb, lane * 16, ring + (slot * SF + f) * 64);
  };

  f32x4 acc[kWaveRB][kWaveCB];
#pragma unroll
  for (int i = 0; i < kWaveRB; ++i)
#pragma unroll
    for (int j = 0; j < kWaveCB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: stages 0 .. NST-2 (past the end: re-read k-block 0, never consumed)
#pragma unroll
  for (int st = 0; st < NST - 1; ++st)
#pragma unroll
    for (int q = 0; q < FPW; ++q) issue(KB > st ? st : 0, st, q);
  int slot = 0;                 // ring slot of stage kb
  int nslot = NST - 1;          // slot of stage kb + NST - 1 (= the slot of stage kb - 1)
  for (int kb = 0; kb < KB; ++kb) {
    // this wave's pieces of stage kb have landed (those of the NST-2 younger stages may still
    // be in flight), every wave is past its reads of stage kb-1; then the barrier publishes
    // stage kb to all waves and frees the slot of stage kb-1
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(G::VMC) : "memory");
    const int nkb = kb + NST - 1 < KB ? kb + NST - 1 : 0;
    const bf16x8* st = reinterpret_cast<const bf16x8*>(ring + slot * SF * 64);
    // two halves of 4 row blocks x 4 column blocks (16 MFMAs each); the second half's A
    // fragments are read before the first half's MFMAs, the next stage's DMA pieces are spread
    // over the two halves
    bf16x8 bfr[kWaveCB], a0[4], a1[4];
#pragma unroll
    for (int j = 0; j < kWaveCB; ++j) bfr[j] = st[(kTileBlocks + kWaveCB * wc + j) * 64 + lane];
#pragma unroll
    for (int i = 0; i < 4; ++i) a0[i] = st[(kWaveRB * wr + i) * 64 + lane];
    if (!(DLADMM_TILE_EXP & 1) && DLADMM_TILE_DPOS == 0) {
#pragma unroll
      for (int q = 0; q < G::H1; ++q) issue(nkb, nslot, q);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) a1[i] = st[(kWaveRB * wr + 4 + i) * 64 + lane];
    if (DLADMM_TILE_EXP & 2) continue;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < kWaveCB; ++j) acc[i][j] = mfma_bf16(a0[i], bfr[j], acc[i][j]);
      if constexpr (!(DLADMM_TILE_EXP & 1) && DLADMM_TILE_DPOS == 2) {
        // pieces q = i, i + 4, ... after MFMA group i (FPW <= 8 pieces over 8 groups)
        if (i < FPW) {
          __builtin_amdgcn_sched_barrier(0);
          issue(nkb, nslot, i);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if (!(DLADMM_TILE_EXP & 1) && DLADMM_TILE_DPOS < 2) {
#pragma unroll
      for (int q = DLADMM_TILE_DPOS == 0 ? G::H1 : 0; q < FPW; ++q) issue(nkb, nslot, q);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < kWaveCB; ++j) acc[4 + i][j] = mfma_bf16(a1[i], bfr[j], acc[4 + i][j]);
      if constexpr (!(DLADMM_TILE_EXP & 1) && DLADMM_TILE_DPOS == 2) {
        if (4 + i < FPW) {
          __builtin_amdgcn_sched_barrier(0);
          issue(nkb, nslot, 4 + i);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    slot = slot + 1 == NST ? 0 : slot + 1;
    nslot = nslot + 1 == NST ? 0 : nslot + 1;
  }
  // drain the speculative stages before the workgroup's LDS can be handed to another
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if (DLADMM_TILE_EXP & 4) {
    float t = 0.f;  // keep every accumulator live
#pragma unroll
    for (int i = 0; i < kWaveRB; ++i)
#pragma unroll
      for (int j = 0; j < kWaveCB; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 12345.f) a.lossp[0] = t;
    return;
  }

  // ---------------------------------------------------------------- epilogue
  const LayerEpi<EMODE, PKIND, PH> epi(a);
  float lsum[kWaveCB];
#pragma unroll
  for (int j = 0; j < kWaveCB; ++j) lsum[j] = 0.f;
  char* pb = (char*)a.Pb;
  // Units of JB column blocks of one row block, software-pipelined: the loads of unit u + D are
  // issued before unit u computes and stores (a load cannot be moved above a store it may
  // alias, so this order is what keeps D units of loads in flight behind the stores).
  using In = typename LayerEpi<EMODE, PKIND, PH>::In;
  constexpr int JB = PH == 0 ? 4 : 2;           // column blocks per unit
  constexpr int NU = kWaveRB * (kWaveCB / JB);  // units per wave
  constexpr int D = (PH == 0 && PKIND != PK_ROW) ? 2 : 1;  // units of loads in flight
  In buf[D + 1][JB][4];
  auto load_unit = [&](auto U_) {
    constexpr int u = decltype(U_)::value;
    constexpr int i = u / (kWaveCB / JB), j0 = (u % (kWaveCB / JB)) * JB;
    const int ib = ib0 + kWaveRB * wr + i;
#pragma unroll
    for (int jj = 0; jj < JB; ++jj) {
      const int64_t col = (int64_t)(cb0 + kWaveCB * wc + j0 + jj) * 16 + (lane & 15);
      const bool cv = col < a.B;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        buf[u % (D + 1)][jj][r] = epi.load(16 * ib + 4 * g + r, cv, cv ? col : 0);
    }
  };
  static_for<D>([&](auto U_) {
    if constexpr (decltype(U_)::value < NU) load_unit(U_);
  });
  static_for<NU>([&](auto U_) {
    constexpr int u = decltype(U_)::value;
    if constexpr (u + D < NU) load_unit(std::integral_constant<int, u + D>{});
    constexpr int i = u / (kWaveCB / JB), j0 = (u % (kWaveCB / JB)) * JB;
    const int ib = ib0 + kWaveRB * wr + i;  // global row block
    const int kbo = ib >> 1;                // k-block of the packed output
    const bool pst = pb != nullptr && kbo < a.pb_kb;
#pragma unroll
    for (int jj = 0; jj < JB; ++jj) {
      const int j = j0 + jj;
      const int cb = cb0 + kWaveCB * wc + j;
      const int64_t col = (int64_t)cb * 16 + (lane & 15);
      const bool cv = col < a.B;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        v[r] = epi.finish(16 * ib + 4 * g + r, col, cv, buf[u % (D + 1)][jj][r], acc[i][j][r],
                          lsum[j]);
      if (pst) {
        // rows 16ib + 4g + r sit in k-block ib/2 at k 16(ib&1) + 4g + r: lane group
        // 2(ib&1) + g/2, elements 4(g&1) .. +3 of the 8 -> one 8-byte store
        uint32_t lo = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[0]) |
                      ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[1]) << 16);
        uint32_t hi = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[2]) |
                      ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[3]) << 16);
        const int L = (lane & 15) + 16 * (2 * (ib & 1) + (g >> 1));
        const int64_t off = (((int64_t)kbo * a.nbp + cb) * 64 + L) * 16 + 8 * (g & 1);
        *reinterpret_cast<uint2*>(pb + off) = make_uint2(lo, hi);
      }
    }
  });
  if (a.lossp && a.k >= 0 && !(PH == 2)) {
    // per-column partial over this wave's 128 rows: slot 2 * tile row + wr
#pragma unroll
    for (int j = 0; j < kWaveCB; ++j) {
      const float s = col_sum(lsum[j]);
      if (g == 0) {
        const float v = (PH == 1 && epi.lasso) ? 0.5f * s : s;
        const int64_t col = (int64_t)(cb0 + kWaveCB * wc + j) * 16 + lane;
        a.lossp[(int64_t)(2 * a.k + (PH == 0 ? 0 : 1)) * a.nslots +
                (int64_t)(2 * by + wr) * a.ldl + col] = v;
      }
    }
  }
}

}  // namespace dladmm
