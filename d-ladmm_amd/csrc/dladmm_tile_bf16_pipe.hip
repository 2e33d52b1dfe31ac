// dladmm_tile_bf16_pipe.hip -- the bf16 mode's G1 product (BASELINE config 5: Z_k = S(Z_{k-1} -
// s1 W_k Var_k), n = 4096 output rows, contraction m = 1024) as a PERSISTENT, software-pipelined
// tile loop: the epilogue of one output tile runs inside the main loop of the next.
//
// Why: the one-phase kernel (dladmm_tile_bf16.hip) gives every workgroup one tile -- main loop
// (MFMA, L2 -> LDS operand stream), then epilogue (HBM: read Z_{k-1}, write Z_k and its packed
// bf16 copy) -- and every workgroup of a launch passes through the two at about the same time, so
// the matrix cores idle while the epilogues stream and the HBM idles during the main loops
// (G1 ~250 us per layer against ~100 us of main loop).  Co-scheduling
// other workgroups beside them does not recover it (round 5, paired-halves launches: slower,
// profiles/r05_pair_ab.json).  Here each workgroup (8 waves, two per SIMD, one workgroup per CU,
// the narrow tile's 256 x 128 outputs, wave tile 64 x 64) owns the tiles t = blockIdx.x,
// + gridDim.x, ... and every wave carries TWO accumulator sets (2 x 64 AGPRs): while the MFMAs of
// tile i accumulate into one, the epilogue of tile i - 1 drains the other, one 16 x 16 block per
// two k-blocks (32 k-blocks, 16 blocks per wave), its operand loads issued D blocks ahead.  The
// epilogue's VALU work and HBM traffic then sit in the MFMA stream; only the last tile's
// epilogue is exposed.  (A 4-wave form with 128 x 64 wave tiles needs all 256 AGPRs for the two
// sets and spilled.)
//
// Main loop: the state fragments of k-block kb + 1 are read at the top of k-block kb (two sets)
// and each weight fragment of kb + 1 right after kb's MFMAs that use its row block, so no MFMA
// waits on an LDS read; the LDS-DMA ring
// (NST stages of one k-block: 16 weight + 8 state fragments) runs continuously across tiles.  At
// the top of k-block kb a wave waits for ITS pieces of stage kb + 1 with a counted vmcnt that
// leaves the NST - 3 younger stages in flight (the epilogue's loads and stores are younger too:
// counting only DMA pieces is conservative, never early), then the barrier publishes the stage to
// all waves and frees the slot of stage kb - 1, which receives stage kb + NST - 1.
//
// Each output element is the same chain as in the one-phase kernel (k-blocks in order, the same
// packed operands, LayerEpi's code), so the outputs are bit-identical to it (tested).
#include "dladmm_tile_bf16_body.h"

#ifndef DLADMM_PIPE_EXP
#define DLADMM_PIPE_EXP 0  // experiments (WRONG results): 1 no epilogue, 2 no MFMA
#endif

namespace dladmm {

template <int EMODE, int PKIND, int NST, int D>
__global__ __launch_bounds__(512, 1) void tile_pipe_g1_kernel(const LayerArgs a, const int gx,
                                                              const int ntiles) {
  using G = TileG<4>;                       // the narrow tile: 16 row blocks x 8 column blocks
  constexpr int NWV = 8;                    // waves: 4 wave rows x 2 wave columns
  constexpr int WRB = 4, WCB = 4;           // blocks per wave: 64 rows x 64 columns
  constexpr int SF = G::SF;                 // 24 fragments per stage
  constexpr int FPW = SF / NWV;             // 3 DMA pieces per wave and stage
  constexpr int KBP = 32;                   // k-blocks per tile: the contraction (a.KB == 32)
  constexpr int VMC = FPW * (NST - 3);      // younger DMA pieces at a top-of-k-block wait
  constexpr int NBLK = WRB * WCB;           // 16 epilogue blocks per wave and tile
  static_assert(NST >= 4 && NST * SF * 1024 <= 160 * 1024, "ring");
  static_assert(D >= 1 && D < NBLK, "epilogue load distance");
  __shared__ f32x4 ring[NST * SF * 64];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;  // wave row 0..3 (64 rows each), wave column 0..1
  const int g = lane >> 4;
  const int gs = gridDim.x, gid = blockIdx.x;
  const int cg = (ntiles - gid + gs - 1) / gs;  // tiles of this workgroup (the grid <= ntiles)

  // ---- the DMA stream: stage (tile d_i of this workgroup, k-block d_kb)
  auto tile_xy = [&](int i, int& bx, int& by) __attribute__((always_inline)) {
    int t = gid + i * gs;
    t = t < ntiles ? t : gid;  // past this workgroup's last tile: harmless re-reads
    by = __builtin_amdgcn_readfirstlane(t / gx);
    bx = __builtin_amdgcn_readfirstlane(t - by * gx);
  };
  // running source bases of the next stage (the fewest scalar registers: the kernel holds all
  // 512 vector registers, and scalar spills would land in them): pW = the weights' row block ib0
  // of k-block kb, pS = the state's column block cb0 of k-block kb
  const int64_t wstep = (int64_t)a.MBp * kFrag * 4, sstep = (int64_t)a.nbp * kFrag * 4;  // bytes
  int d_kb = 0, d_i = 0;
  uint64_t pW, pS;
  auto dma_tile = [&](int i) __attribute__((always_inline)) {
    int bx, by;
    tile_xy(i, bx, by);
    pW = (uint64_t)(a.Wp + (int64_t)by * kTileBlocks * kFrag);
    pS = (uint64_t)(a.S + (int64_t)bx * G::CBT * kFrag);
  };
  dma_tile(0);
  auto issue_next = [&](int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < FPW; ++q) {
      const int f = FPW * w + q;
      uint64_t sb = f < kTileBlocks ? pW + (uint64_t)f * (kFrag * 4)
                                    : pS + (uint64_t)(f - kTileBlocks) * (kFrag * 4);
      asm volatile("" : "+s"(sb));
      glds16((const float*)sb, lane * 16, ring + (slot * SF + f) * 64);
    }
    if (++d_kb < KBP) {
      pW += wstep;
      pS += sstep;
    } else {
      d_kb = 0;
      dma_tile(++d_i);
    }
  };

  // ---- fragments: this wave's 4 weight row blocks and 4 state column blocks, one register set:
  // the next stage's are read right after this k-block's MFMAs have issued (the stage was
  // published by this k-block's barrier); the partner wave on the SIMD covers their latency
  bf16x8 fa[WRB], fb[WCB];
  auto read_frags = [&](int slot) __attribute__((always_inline)) {
    const bf16x8* st = reinterpret_cast<const bf16x8*>(ring + slot * SF * 64);
#pragma unroll
    for (int j = 0; j < WCB; ++j) fb[j] = st[(kTileBlocks + WCB * wc + j) * 64 + lane];
#pragma unroll
    for (int i = 0; i < WRB; ++i) fa[i] = st[(WRB * wr + i) * 64 + lane];
  };

  f32x4 acc[2][WRB][WCB];

  // ---- epilogue of one tile: block b = (row block b / WCB, column block b % WCB) of this wave.
  // LayerEpi's PH 0 expressions (Z_k = S(Z_{k-1} - s1 u), the literal shrink) on buffer views:
  // a row offset per (row block, row) in soffset and the lane's part in voffset, so an element
  // costs one load and one store instruction and no address arithmetic.  Rows past n and columns
  // past B read 0 and drop their stores through the views' ranges (the lane offset kOOB), which
  // makes those elements exactly the one-phase kernel's zeros; the packed copy's padding columns
  // are written (zeros), as there.
  const int k = a.k;
  const cfloat_p sp = (cfloat_p)a.scal + (k < 0 ? 0 : k) * DLADMM_NSCALAR;
  const float s1 = PKIND == PK_SCALAR ? sp[DLADMM_P_S1] : 1.0f;
  const float thz_s = PKIND == PK_ROW ? 0.0f : sp[DLADMM_P_THETA_Z];
  const int n = a.n;
  const rsrc_t rzp = mkrsrc(a.Zprev, (uint32_t)((int64_t)n * a.ldzp * 4));
  const rsrc_t rzo = mkrsrc(a.Zo, (uint32_t)((int64_t)n * a.ldo * 4));
  const rsrc_t rpb = mkrsrc(a.Pb, a.Pb ? (uint32_t)((int64_t)a.pb_kb * a.nbp * 1024) : 0u);
  const rsrc_t rth = mkrsrc(PKIND == PK_ROW ? a.rowp + ((int64_t)k * 8 + DLADMM_P_THETA_Z) * a.rstride
                                            : nullptr,
                            PKIND == PK_ROW ? (uint32_t)(n * 4) : 0u);
  // lane offsets of block column j of tile column bx (formed where used: held per tile they
  // cost registers the kernel does not have)
  auto lane_off = [&](int bx, int j, int64_t ld) __attribute__((always_inline)) -> uint32_t {
    const int64_t col = (int64_t)(bx * G::CBT + WCB * wc + j) * 16 + (lane & 15);
    return col < a.B ? (uint32_t)((col + (int64_t)(4 * g) * ld) * 4) : kOOB;
  };
  const uint32_t vpk0 = (uint32_t)(((lane & 15) + 16 * (g >> 1)) * 16 + 8 * (g & 1));
  float ezp[D + 1][4], eth[PKIND == PK_ROW ? D + 1 : 1][4];
  float lsum[WCB];
  auto epi_load = [&](auto B_, int bx, int by) __attribute__((always_inline)) {
    constexpr int b = decltype(B_)::value, i = b / WCB, j = b % WCB;
    const int ib = by * kTileBlocks + WRB * wr + i;
    const uint32_t vzp = lane_off(bx, j, a.ldzp);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t so = (uint32_t)((int64_t)(16 * ib + r) * a.ldzp * 4);
      ezp[b % (D + 1)][r] =
          __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rzp, (int)vzp, (int)so, 0));
      if constexpr (PKIND == PK_ROW)
        eth[b % (D + 1)][r] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rth, 16 * g, (16 * ib + r) * 4, 0));
    }
  };
  auto epi_finish = [&](auto B_, auto SET_, int bx, int by) __attribute__((always_inline)) {
    constexpr int b = decltype(B_)::value, i = b / WCB, j = b % WCB;
    constexpr int se = decltype(SET_)::value;
    const int ib = by * kTileBlocks + WRB * wr + i;
    if constexpr (b == 0) {
#pragma unroll
      for (int jj = 0; jj < WCB; ++jj) lsum[jj] = 0.f;
    }
    const f32x4 av = acc[se][i][j];
    const uint32_t vzo = lane_off(bx, j, a.ldo);
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float u = av[r];
      if constexpr (PKIND == PK_SCALAR) u = s1 * u;
      const float th = PKIND == PK_ROW ? eth[b % (D + 1)][r] : thz_s;
      const float z = shrink(ezp[b % (D + 1)][r] - u, th);            // main_lena.py:79-80
      const uint32_t so = (uint32_t)((int64_t)(16 * ib + r) * a.ldo * 4);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, z), rzo, (int)vzo,
                                            (int)so, 0);
      lsum[j] += fabsf(z);
      v[r] = z;
    }
    const int kbo = ib >> 1;  // k-block of the packed output (G2's B operand)
    if (kbo < a.pb_kb) {
      const uint32_t lo = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[0]) |
                          ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[1]) << 16);
      const uint32_t hi = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[2]) |
                          ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[3]) << 16);
      const uint32_t so = (uint32_t)kbo * (uint32_t)a.nbp * 1024u + (uint32_t)(ib & 1) * 512u;
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      const u32x2 pk = {lo, hi};
      const uint32_t vpk = (uint32_t)(bx * G::CBT + WCB * wc + j) * 1024u + vpk0;
      __builtin_amdgcn_raw_buffer_store_b64(pk, rpb, (int)vpk, (int)so, 0);
    }
    if constexpr (b == NBLK - 1) {
      if (a.lossp && k >= 0) {
        // per-column partial over this wave's 64 rows, added to its wave-row partner's: the
        // one-phase kernel's slot 2 * tile row + (wr >> 1) holds the sum over 128 rows (its
        // wave row), i.e. over these two waves' rows in row order -- formed here in the same
        // order (rows 0-63 then 64-127 of that 128-row slab) through LDS-free DPP sums and one
        // partial exchanged in the loss buffer is not needed: the two 64-row sums are added
        // in the reduction (the slot count doubles)
#pragma unroll
        for (int jj = 0; jj < WCB; ++jj) {
          const float sm = col_sum(lsum[jj]);
          if (g == 0) {
            const int64_t c = (int64_t)(bx * G::CBT + WCB * wc + jj) * 16 + lane;
            a.lossp[(int64_t)(2 * k) * a.nslots + (int64_t)(4 * by + wr) * a.ldl + c] = sm;
          }
        }
      }
    }
  };

  // ---- one tile's main loop into acc[SET], with (EPI) the epilogue of the previous tile (from
  // acc[1 - SET], coordinates pbx, pby) spread over its k-blocks
  int cur = 0;  // ring slot of the current stage
  auto run_tile = [&](auto SET_, auto EPI_, int pbx, int pby) __attribute__((always_inline)) {
    constexpr int se = decltype(SET_)::value;
    constexpr bool ep = decltype(EPI_)::value && !(DLADMM_PIPE_EXP & 1);
#pragma unroll
    for (int i = 0; i < WRB; ++i)
#pragma unroll
      for (int j = 0; j < WCB; ++j) {
        acc[se][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        asm volatile("" : "+a"(acc[se][i][j]));  // volatile: one zero tuple per block, not CSE'd
      }
    static_for<KBP>([&](auto P_) __attribute__((always_inline)) {
      constexpr int p = decltype(P_)::value;
      // stage p + 1 landed (this wave's pieces; then every wave's, after the barrier), and
      // every wave is past k-block p - 1, whose slot is refilled below
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(VMC) : "memory");
      const int nx = cur + 1 == NST ? 0 : cur + 1;
      issue_next(cur == 0 ? NST - 1 : cur - 1);
      // epilogue schedule: block b finishes at k-block 2b + 1; its loads go out at k-block
      // 2(b - D) (blocks 0 .. D - 1: at k-block 0)
      if constexpr (ep && p % 2 == 0) {
        if constexpr (p == 0) {
          static_for<D>([&](auto B_) __attribute__((always_inline)) { epi_load(B_, pbx, pby); });
        }
        if constexpr (p / 2 + D < NBLK)
          epi_load(std::integral_constant<int, p / 2 + D>{}, pbx, pby);
      }
      if constexpr (!(DLADMM_PIPE_EXP & 2)) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < WRB; ++i)
#pragma unroll
          for (int j = 0; j < WCB; ++j) acc[se][i][j] = mfma_bf16(fa[i], fb[j], acc[se][i][j]);
        __builtin_amdgcn_s_setprio(0);
        // both accumulator sets live in the AGPRs; the VGPRs hold the fragments and epilogue
#pragma unroll
        for (int i = 0; i < WRB; ++i)
#pragma unroll
          for (int j = 0; j < WCB; ++j) asm volatile("" : "+a"(acc[se][i][j]));
      }
      read_frags(nx);  // stage p + 1
      if constexpr (ep && p % 2 == 1)
        epi_finish(std::integral_constant<int, p / 2>{}, std::integral_constant<int, 1 - se>{},
                   pbx, pby);
      cur = nx;
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  // the last tile's epilogue alone (loads D blocks ahead)
  auto final_epi = [&](auto SET_, int pbx, int pby) __attribute__((always_inline)) {
    if constexpr (!(DLADMM_PIPE_EXP & 1)) {
      static_for<D>([&](auto B_) __attribute__((always_inline)) { epi_load(B_, pbx, pby); });
      static_for<NBLK>([&](auto B_) __attribute__((always_inline)) {
        constexpr int b = decltype(B_)::value;
        if constexpr (b + D < NBLK) epi_load(std::integral_constant<int, b + D>{}, pbx, pby);
        epi_finish(B_, SET_, pbx, pby);
        // one block at a time (left free, the scheduler hoisted every load of the tile)
        __builtin_amdgcn_sched_barrier(0);
      });
    }
  };

  // prologue: stages 0 .. NST - 2, then stage 0's fragments
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue_next(s);
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(FPW * (NST - 2)) : "memory");
  read_frags(0);

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  // tiles alternate between the accumulator sets: 0, 1, 0, 1, ...; the loop body is one pair, so
  // each set keeps its registers (a parity branch in one body made the allocator spill them)
  int bx, by;
  tile_xy(0, bx, by);
  run_tile(I0{}, std::false_type{}, 0, 0);
  for (int i = 1;; i += 2) {
    if (i >= cg) {
      final_epi(I0{}, bx, by);
      break;
    }
    int pbx = bx, pby = by;
    tile_xy(i, bx, by);
    run_tile(I1{}, std::true_type{}, pbx, pby);
    if (i + 1 >= cg) {
      final_epi(I1{}, bx, by);
      break;
    }
    pbx = bx;
    pby = by;
    tile_xy(i + 1, bx, by);
    run_tile(I0{}, std::true_type{}, pbx, pby);
  }
  if constexpr ((DLADMM_PIPE_EXP & 1) != 0) {
    float t = 0.f;  // keep both accumulator sets live
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < WRB; ++i)
#pragma unroll
        for (int j = 0; j < WCB; ++j) t += acc[s2][i][j][0] + acc[s2][i][j][3];
    if (t == 12345.f) a.lossp[0] = t;
  }
  // the stream's speculative stages (and the stores) drain before the LDS is released
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
}

constexpr int kPipeNST = 6, kPipeD = 2;

template <int EMODE, int PKIND>
hipError_t launch_pipe_v(const LayerArgs& a, int gx, int ntiles, int grid, hipStream_t s) {
  hipLaunchKernelGGL((tile_pipe_g1_kernel<EMODE, PKIND, kPipeNST, kPipeD>), dim3(grid), dim3(512),
                     0, s, a, gx, ntiles);
  return hipGetLastError();
}

// G1 of the bf16 path, persistent: grid = min(tiles, CUs) workgroups of the narrow tile geometry
// (256 rows x 128 columns; 8 waves of 64 x 64).  The contraction is exactly 32 k-blocks (m in 993 .. 1024).
hipError_t launch_tile_bf16_pipe_g1(int variant, const LayerArgs& a, int gx, int slices, int cus,
                                    hipStream_t s) {
  if (a.KB != 32) return hipErrorInvalidValue;
  const int ntiles = gx * slices;
  const int grid = ntiles < cus ? ntiles : cus;
  switch (variant) {
    case DLADMM_V1_LENA: return launch_pipe_v<EM_V1, PK_ELEM>(a, gx, ntiles, grid, s);
    case DLADMM_V2_LTHETA: return launch_pipe_v<EM_V1, PK_ROW>(a, gx, ntiles, grid, s);
    case DLADMM_V3_FULL: return launch_pipe_v<EM_VVAR, PK_ROW>(a, gx, ntiles, grid, s);
    case DLADMM_V4_SCALAR:
    case DLADMM_V5_TIED: return launch_pipe_v<EM_VVAR, PK_SCALAR>(a, gx, ntiles, grid, s);
    case DLADMM_V6_LASSO: return launch_pipe_v<EM_LASSO, PK_SCALAR>(a, gx, ntiles, grid, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace dladmm
