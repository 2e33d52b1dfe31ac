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

#ifndef DLADMM_PIPE_ZPOL
#define DLADMM_PIPE_ZPOL 0  // cache policy of the Z_k / packed stores (experiment: 2 nt, 16 sc1)
#endif
#ifndef DLADMM_PIPE_EXP
#define DLADMM_PIPE_EXP 0  // experiments (WRONG results): 1 no epilogue, 2 no MFMA; through
                           // zero-size views (instructions kept, no bytes): 4 the Z stores, 8 the
                           // Z_{k-1} loads, 16 the packed stores
#endif

namespace dladmm {

// Static VM-operation schedule of one tile (32 k-blocks = positions t) for the counted waits.
// Position t issues, in order: this wave's FPW DMA pieces of stage t + NST - 1 (at its top), the
// epilogue loads of even t (t = 0: blocks 0 .. D - 1 first; then block t / 2 + D), and at odd t,
// after the MFMAs, the stores of block (t - 1) / 2 (the packed copy; for odd blocks the 4 Z_k rows
// of the block and of its even neighbour; at t = 31 the 4 loss partials).  Every one of them is issued unconditionally (out-of-range ones
// are dropped by their buffer view), so the counts are exact; operations of the previous tile
// are not counted (fewer counted = a longer wait, never an early one).  L = loads per block.
template <int D, int L, int FPW, int NST>
struct PipeSched {
  static constexpr int NB = 16, T = 32;
  static constexpr int loads_at(int t) {
    if (t < 0 || t % 2) return 0;
    return (t == 0 ? L * D : 0) + (t / 2 + D < NB ? L : 0);
  }
  // stores of block c: its packed copy; odd c also the Z_k rows of c - 1 and c (a 128-B line is
  // the row segments of two column blocks: both halves leave together); the last its loss partials
  static constexpr int st_blk(int c) {
    return (c % 2 ? ((DLADMM_PIPE_EXP & 32) ? 3 : 9) : 1) + (c == NB - 1 ? 4 : 0);
  }
  static constexpr int stores_at(int t) { return (t >= 0 && t % 2) ? st_blk(t / 2) : 0; }
  static constexpr int E(int t, bool epi) { return epi ? loads_at(t) + stores_at(t) : 0; }
  // top of position t: this wave's pieces of stage t + 1 went out at the top of t - (NST - 2)
  static constexpr int vmc(int t, bool epi) {
    int n = E(t - (NST - 2), epi);
    for (int u = t - (NST - 3); u < t; ++u) n += FPW + E(u, epi);
    return n;
  }
  // before the stores of block b (t = 2 b + 1): operations issued after block b's loads
  static constexpr int wfin(int b) {
    const int tb = b < D ? 0 : 2 * (b - D), t = 2 * b + 1;
    int n = b < D ? L * (D - 1 - b) + (D < NB ? L : 0) : 0;
    for (int u = tb + 1; u < t; ++u) n += FPW + E(u, true);
    return n + FPW;
  }
  // the last tile's epilogue alone: loads of blocks 0 .. D - 1, then per block b: the loads of
  // block b + D, the wait, the stores
  static constexpr int wfinal(int b) {
    int n = 0;
    for (int c = b + 1; c <= b + D && c < NB; ++c) n += L;
    for (int c = b - D > 0 ? b - D : 0; c < b; ++c) n += st_blk(c);
    return n;
  }
  static constexpr bool ok() {
    for (int t = 0; t < T; ++t)
      if (vmc(t, true) > 63 || vmc(t, false) > 63) return false;
    for (int b = 0; b < NB; ++b)
      if (wfin(b) > 63 || wfinal(b) > 63) return false;
    return true;
  }
};

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
// buffer resource words (the layout __builtin_amdgcn_make_buffer_rsrc builds in mkrsrc), for
// loads issued by inline asm: the compiler neither counts nor waits for them -- every use is
// behind an explicit counted wait (PipeSched), so the ring's waits stay exact
__device__ __forceinline__ u32x4_t rsrc_words(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  return u32x4_t{(uint32_t)a, (uint32_t)(a >> 32) & 0xffffu, bytes, 0x00020000u};
}
// one dword per lane of a buffer view straight into LDS (lane i's at ldst + 4 i; out-of-range
// lanes write 0): the epilogue's operand stream holds no registers while in flight
__device__ __forceinline__ void asm_bload_lds(u32x4_t r, uint32_t voff, uint32_t soff, float* ldst) {
  unsigned keep;
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ldst);
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
      "buffer_load_dword %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(soff), "s"(dst)
      : "memory");
}

template <int EMODE, int PKIND, int NST, int D>
__global__ __launch_bounds__(512, 1) void tile_pipe_g1_kernel(const LayerArgs a, const int gx,
                                                              const int ntiles) {
  using G = TileG<4>;                       // the narrow tile: 16 row blocks x 8 column blocks
  constexpr int NWV = 8;                    // waves: 4 wave rows x 2 wave columns
  constexpr int WRB = 4, WCB = 4;           // blocks per wave: 64 rows x 64 columns
  constexpr int SF = G::SF;                 // 24 fragments per stage
  constexpr int FPW = SF / NWV;             // 3 DMA pieces per wave and stage
  constexpr int KBP = 32;                   // k-blocks per tile: the contraction (a.KB == 32)
  constexpr int NBLK = WRB * WCB;           // 16 epilogue blocks per wave and tile
  using Sch = PipeSched<D, 4, FPW, NST>;
  static_assert(NBLK == Sch::NB && Sch::ok(), "vmcnt counts");
  static_assert(WCB % 2 == 0, "block parity = column parity (PipeSched::st_blk)");
  static_assert(PKIND != PK_ROW, "per-row thresholds: the one-phase kernel");
  // epilogue operands in flight: D + 1 blocks of 4 rows per wave, landed by LDS-DMA (block b + D's
  // loads go out before block b has been read)
  __shared__ float estage[NWV][D + 1][4][64];
  static_assert((NST * SF * 64 * 16 + NWV * (D + 1) * 4 * 64 * 4) <= 160 * 1024, "LDS");
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
  const float thz_s = sp[DLADMM_P_THETA_Z];
  const int n = a.n;
  const u32x4_t rzp = rsrc_words(a.Zprev, (DLADMM_PIPE_EXP & 8) ? 0u : (uint32_t)((int64_t)n * a.ldzp * 4));
  const rsrc_t rzo = mkrsrc(a.Zo, (DLADMM_PIPE_EXP & 4) ? 0u : (uint32_t)((int64_t)n * a.ldo * 4));
  const rsrc_t rpb = mkrsrc(a.Pb, (a.Pb && !(DLADMM_PIPE_EXP & 16)) ? (uint32_t)((int64_t)a.pb_kb * a.nbp * 1024) : 0u);
  // loss partials [2K][nslots] (null: a zero-size view, the stores are dropped)
  const rsrc_t rls = mkrsrc(a.lossp, a.lossp && k >= 0 ? (uint32_t)((int64_t)2 * a.K * a.nslots * 4) : 0u);
  // lane offsets of block column j of tile column bx (formed where used: held per tile they
  // cost registers the kernel does not have)
  auto lane_off = [&](int bx, int j, int64_t ld) __attribute__((always_inline)) -> uint32_t {
    const int64_t col = (int64_t)(bx * G::CBT + WCB * wc + j) * 16 + (lane & 15);
    return col < a.B ? (uint32_t)((col + (int64_t)(4 * g) * ld) * 4) : kOOB;
  };
  const uint32_t vpk0 = (uint32_t)(((lane & 15) + 16 * (g >> 1)) * 16 + 8 * (g & 1));
  float lsum[WCB];
  auto epi_load = [&](auto B_, int bx, int by) __attribute__((always_inline)) {
    constexpr int b = decltype(B_)::value, i = b / WCB, j = b % WCB;
    const int ib = by * kTileBlocks + WRB * wr + i;
    const uint32_t vzp = lane_off(bx, j, a.ldzp);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t so = (uint32_t)((int64_t)(16 * ib + r) * a.ldzp * 4);
      asm_bload_lds(rzp, vzp, so, &estage[w][b % (D + 1)][r][0]);
    }
  };
  // the finish of block b in three parts, so the main loop can interleave its rows with the
  // MFMAs of the next tile: begin (wait for the block's operands, read them and the block's
  // accumulators), row r (Z_k = S(Z_{k-1} - s1 u) and its store), end (the packed copy and, for
  // the last block, the loss partials)
  float ez[4], v[4], zh[4];
  f32x4 av;
  auto fin_begin = [&](auto B_, auto SET_, auto W_) __attribute__((always_inline)) {
    constexpr int b = decltype(B_)::value, i = b / WCB, j = b % WCB;
    constexpr int se = decltype(SET_)::value;
    // this block's operands have landed in LDS: W = the operations issued after them
    // (PipeSched); the "memory" clobber keeps the LDS reads below the wait
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(decltype(W_)::value) : "memory");
#pragma unroll
    for (int r = 0; r < 4; ++r) ez[r] = estage[w][b % (D + 1)][r][lane];
    if constexpr (b == 0) {
#pragma unroll
      for (int jj = 0; jj < WCB; ++jj) lsum[jj] = 0.f;
    }
    av = acc[se][i][j];
  };
  auto fin_row = [&](auto B_, int r, int bx, int by) __attribute__((always_inline)) {
    constexpr int b = decltype(B_)::value, i = b / WCB, j = b % WCB;
    const int ib = by * kTileBlocks + WRB * wr + i;
    float u = av[r];
    if constexpr (PKIND == PK_SCALAR) u = s1 * u;
    const float z = shrink(ez[r] - u, thz_s);                       // main_lena.py:79-80
    // Z_k rows leave in pairs of column blocks (j even held until j + 1), so the two 64-B halves
    // of each 128-B line reach the L2 back to back (measured: no change against one block at a
    // time, profiles/r05_pipe_ab.json)
    if constexpr (DLADMM_PIPE_EXP & 32) {
      // timing probe (WRONG values): the pair's 2 KiB as two 16-B-per-lane stores of whole
      // 128-B row segments, 8 rows each
      if constexpr (j % 2 == 1) {
        if (r == 3) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int row = 8 * q + (lane >> 3);
            const uint32_t so = (uint32_t)((int64_t)(16 * ib + row) * a.ldo * 4);
            const int64_t col = (int64_t)(bx * G::CBT + WCB * wc + j - 1) * 16 + 4 * (lane & 7);
            const uint32_t vo = col < a.B ? (uint32_t)(col * 4) : kOOB;
            const u32x4_t d4 = {__builtin_bit_cast(uint32_t, z), __builtin_bit_cast(uint32_t, zh[0]),
                                __builtin_bit_cast(uint32_t, zh[1]), __builtin_bit_cast(uint32_t, zh[2])};
            __builtin_amdgcn_raw_buffer_store_b128(d4, rzo, (int)vo, (int)so, DLADMM_PIPE_ZPOL);
          }
        }
      } else {
        zh[r] = z;
      }
    } else if constexpr (j % 2 == 0) {
      zh[r] = z;
    } else {
      const uint32_t so = (uint32_t)((int64_t)(16 * ib + r) * a.ldo * 4);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, zh[r]), rzo,
                                            (int)lane_off(bx, j - 1, a.ldo), (int)so, DLADMM_PIPE_ZPOL);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, z), rzo,
                                            (int)lane_off(bx, j, a.ldo), (int)so, DLADMM_PIPE_ZPOL);
    }
    lsum[j] += fabsf(z);
    v[r] = z;
  };
  auto fin_end = [&](auto B_, int bx, int by) __attribute__((always_inline)) {
    constexpr int b = decltype(B_)::value, i = b / WCB, j = b % WCB;
    const int ib = by * kTileBlocks + WRB * wr + i;
    // the packed copy (G2's B operand): k-block ib / 2 (past pb_kb: beyond the view, dropped)
    const int kbo = ib >> 1;
    {
      const uint32_t lo = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[0]) |
                          ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[1]) << 16);
      const uint32_t hi = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[2]) |
                          ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[3]) << 16);
      const uint32_t so = (uint32_t)kbo * (uint32_t)a.nbp * 1024u + (uint32_t)(ib & 1) * 512u;
      const u32x2_t pk = {lo, hi};
      const uint32_t vpk = (uint32_t)(bx * G::CBT + WCB * wc + j) * 1024u + vpk0;
      __builtin_amdgcn_raw_buffer_store_b64(pk, rpb, (int)vpk, (int)so, DLADMM_PIPE_ZPOL);
    }
    if constexpr (b == NBLK - 1) {
      // per-column partial over this wave's 64 rows (slot 4 * tile row + wave row: two per
      // 128-row slot of the one-phase kernel, so the fused sums equal its within fp32 rounding);
      // lanes 16 .. 63 drop theirs through the view
#pragma unroll
      for (int jj = 0; jj < WCB; ++jj) {
        const float sm = col_sum(lsum[jj]);
        const uint32_t vo = g == 0 ? (uint32_t)(((bx * G::CBT + WCB * wc + jj) * 16 + lane) * 4) : kOOB;
        const uint32_t so = (uint32_t)(((int64_t)(2 * k) * a.nslots + (int64_t)(4 * by + wr) * a.ldl) * 4);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, sm), rls, (int)vo, (int)so, 0);
      }
    }
  };
  auto epi_finish = [&](auto B_, auto SET_, auto W_, int bx, int by) __attribute__((always_inline)) {
    fin_begin(B_, SET_, W_);
#pragma unroll
    for (int r = 0; r < 4; ++r) fin_row(B_, r, bx, by);
    fin_end(B_, bx, by);
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
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(Sch::vmc(p, ep)) : "memory");
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
      // odd k-blocks finish block (p - 1) / 2 of the previous tile: its rows go between the
      // MFMA groups (row block i of this tile, then epilogue row i), so the epilogue's VALU
      // work and stores issue in the MFMAs' shadow instead of after them
      using BF = std::integral_constant<int, p / 2>;
      constexpr bool fin = ep && p % 2 == 1;
      if constexpr (fin)
        fin_begin(BF{}, std::integral_constant<int, 1 - se>{},
                  std::integral_constant<int, Sch::wfin(p / 2)>{});
#pragma unroll
      for (int i = 0; i < WRB; ++i) {
        if constexpr (!(DLADMM_PIPE_EXP & 2)) {
#pragma unroll
          for (int j = 0; j < WCB; ++j) acc[se][i][j] = mfma_bf16(fa[i], fb[j], acc[se][i][j]);
        }
        if constexpr (fin) fin_row(BF{}, i, pbx, pby);
      }
      // both accumulator sets live in the AGPRs; the VGPRs hold the fragments and epilogue
#pragma unroll
      for (int i = 0; i < WRB; ++i)
#pragma unroll
        for (int j = 0; j < WCB; ++j) asm volatile("" : "+a"(acc[se][i][j]));
      read_frags(nx);  // stage p + 1
      if constexpr (fin) fin_end(BF{}, pbx, pby);
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
        epi_finish(B_, SET_, std::integral_constant<int, Sch::wfinal(b)>{}, pbx, pby);
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

constexpr int kPipeNST = 5, kPipeD = 3;

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
    case DLADMM_V4_SCALAR:
    case DLADMM_V5_TIED: return launch_pipe_v<EM_VVAR, PK_SCALAR>(a, gx, ntiles, grid, s);
    case DLADMM_V6_LASSO: return launch_pipe_v<EM_LASSO, PK_SCALAR>(a, gx, ntiles, grid, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace dladmm
