// dladmm_fused_kernel.h -- MI355X (gfx950 / CDNA4) fused K-layer D-LADMM forward (the kernel
// template; dladmm_fused.hip instantiates the inference form, dladmm_fused_savep.hip the
// training form that also stores A Z_k -- two translation units so they compile in parallel).
//
// Replaces the Python loop of DLADMMNet.forward (main_lena.py:57-98,
// main_syn_l1l1_scalar.py:80-127, main_syn_lasso_scalar.py:65-114 and the other variants
// listed in include/dladmm.h) with ONE persistent-state kernel per forward.
//
// Design (DESIGN.md has the full derivation):
//  * one workgroup = 4 waves = a tile of 64 batch columns; wave w owns columns 16w..16w+15;
//  * the whole per-column state -- Z (n), E, L and Var (m each) -- stays in registers for all K
//    layers, laid out exactly like the C/D fragment of v_mfma_f32_16x16x4_f32: lane l holds
//    column (l & 15) and feature rows 16*b + 4*(l >> 4) + r, r = 0..3; X sits in LDS;
//  * with that layout the accumulator of one GEMM IS the B operand of the next: W_k*Var lands
//    in Z's layout, A*Z lands in E/L/T's layout, and every shrink / AXPY of the reference is
//    lane-local -- no LDS transpose, no HBM round trip for the state;
//  * two output blocks are computed together (two independent MFMA chains, so neither waits
//    on the MFMA's dependent-issue latency and no partial sums need combining); W_k is packed
//    as -W_k so the Z update is one add (V5 multiplies by its step ss1[k] first).  The chains start at zero: starting them at Z or
//    -X (saving that add) accumulates every rounding at the state's magnitude and measurably
//    loses accuracy against the reference on cancelling residuals;
//  * W_k and A are pre-packed (pack_frags_kernel) into paired fragment order (1 KiB per 16x16
//    fragment = what one wave's lanes need for 4 MFMAs) and streamed from L2/MALL by
//    LDS-DMA into a 3-slot LDS ring shared by the 4 waves (one chunk read, one landed, one in
//    flight), so the next chunk's first fragments are read ahead before the current one ends;
//  * each pair's epilogue (shrink, E/L/T/Var updates, HBM stores, objective partial sums) is
//    cut into its 8 rows and spread over the MFMA steps of the next pair.
// Elementwise arithmetic is compiled with -ffp-contract=off; a uniform-threshold shrink uses
// the clamp form x -+ med3(x, -|th|, |th|), which equals the reference's two-relu form for
// th >= 0 bit for bit (common.h).

#pragma once

#include "dladmm_common.h"
#include "dladmm_internal.h"

#ifndef DLADMM_ABLATE
#define DLADMM_ABLATE 0  // timing experiments only, see tools/ablate.py
#endif
#ifndef DLADMM_ABL_AUX
#define DLADMM_ABL_AUX 0
#endif
#ifndef DLADMM_STAMP
#define DLADMM_STAMP 0  // diagnostic build: per-wave cycle sums of the passes and ring barriers
#endif
#ifndef DLADMM_SLOTS
#define DLADMM_SLOTS 4  // weight ring slots (chunks in flight: slots - 1); the per-row kinds
                        // (their parameter tables take 24 KiB of LDS) use at most 4
#endif
#ifndef DLADMM_CNT
#define DLADMM_CNT 1  // ring barriers of every variant wait with counted vmcnt (else only V1)
#endif
#ifndef DLADMM_CHUNK
#define DLADMM_CHUNK 16
#endif
#ifndef DLADMM_DMA_LATE
#define DLADMM_DMA_LATE 0  // ring LDS-DMA group issued after the barrier step's MFMAs instead of
                           // beside its fragment reads (A/B; the ring windows count accordingly)
#endif
#ifndef DLADMM_VR_AGPR
#define DLADMM_VR_AGPR 1  // Var pinned to AGPRs (0: the compiler places it; A/B experiment)
#endif

#ifndef DLADMM_G2_CHAINS
// accumulation chains per output of A Z_k: the k sub-steps x, z of every 16-k block run on one
// accumulator and y, w on a second, summed once per output block.  An f32 MFMA is a bitwise fma
// chain (MI355X_MICROARCH.md), so one chain over n = 512 k rounds 512 times in sequence; two
// halve each chain.  A Z_k feeds T_{k+1} = (A Z_k + E_k) - X, a small residual, whose error the
// dual L_k accumulates: measured over the GPU parity suite the median error against fp64 fell
// from 1.2x to 1.0x the reference CPU fp32's (profiles/r03_parity.json) for 0.6 % of kernel time.
#define DLADMM_G2_CHAINS 2
#endif

namespace dladmm {

template <int MP, int NP, int EMODE, int PKIND>
struct Fused {
  static constexpr int MB = MP / 16;
  static constexpr int NB = NP / 16;
  static constexpr int GF = MB * NB;                // fragments per GEMM
  static constexpr int CF = GF < DLADMM_CHUNK ? GF : DLADMM_CHUNK;  // fragments per ring chunk
  static constexpr int NCH = GF / CF;               // chunks per GEMM
  static constexpr int TAB = ((6 * MP + NP + 63) / 64) * 64;  // per-row param table (floats,
                                                              // whole 64-entry DMA pieces)
  static constexpr int SLOTS = (PKIND == PK_ROW && DLADMM_SLOTS > 4) ? 4 : DLADMM_SLOTS;
  static constexpr int RING_F4 = SLOTS * CF * 64;  // ring slots of CF fragments
  static_assert(SLOTS >= 3, "the ring needs one slot being read, one landed, one in flight");
  static constexpr int TAB_F4 = (PKIND == PK_ROW) ? (3 * TAB) / 4 : 0;  // 3 layer buffers
  static constexpr int X_F4 = kWaves * MB * 64;     // the tile's X, resident in LDS
  static_assert(MB % 2 == 0 && NB % 2 == 0, "output blocks are processed in pairs");
  static_assert(GF % CF == 0 && CF % 2 == 0, "chunking");
  static_assert(TAB % 4 == 0, "table alignment");
  static_assert((RING_F4 + X_F4 + TAB_F4) * 16 <= 160 * 1024, "LDS budget");
};

// pending epilogue row i (0..7: block half i/4, row i%4) runs at step (i * SP) / 8 of a pair of
// SP steps
constexpr bool rows_at(int step, int SP, int i) { return (i * SP) / 8 == step; }

// Static VM-operation windows of the ring barriers (V1 / PK_ELEM: its 24 beta loads per G2 pair
// would otherwise be drained by the vmcnt(0) of the next barrier, one chunk after issue).  A
// barrier at step s (the last step of a chunk of SPC steps) waits for the chunk DMA issued at
// the previous barrier step s - SPC; every store and beta load issued in the bodies of steps
// s - SPC .. s - 1 (the barrier step's own body follows its head) is newer.  Counted: the
// stores of the epilogue rows (always issued; out-of-range ones go to 0-record buffers) and the
// beta prefetch at each G2 pair start.  Not counted (conditional): the per-column objective
// stores -- counting too few only waits longer.  Other variants return 0 (plain vmcnt(0)).
template <int MB, int NB, int CF, int PKIND, bool SAVEP>
struct WinCount {
  static constexpr int ST2 = SAVEP ? 4 : 3;  // stores of a G2 row: E, L, T (+ P)
  static constexpr int SPC = CF / 2;  // steps per chunk
  static constexpr int rows_in(int step, int SP) {
    int c = 0;
    for (int i = 0; i < 8; ++i) c += ((i * SP) / 8 == step) ? 1 : 0;
    return c;
  }
  // VM operations issued in the body of step t of a G1 / G2 pass
  static constexpr int ops1(int t) {
    return rows_in(t % MB, MB) * (t / MB == 0 ? ST2 : 1);  // pair 0 runs G2 rows (E, L, T)
  }
  // step of the pair that issues beta-prefetch part `part` (3 loads)
  static constexpr int part_step(int part) { return (part * NB) / 16; }
  static constexpr int parts_at(int kb) {
    int c = 0;
    for (int q = 0; q < 8; ++q) c += part_step(q) == kb ? 1 : 0;
    return c;
  }
  static constexpr int ops2(int t, bool pro) {
    const int p = t / NB, kb = t % NB;
    constexpr int pf = PKIND == PK_ELEM ? 3 : 0;  // beta loads per prefetch part
    if (p == 0) return (pro ? 0 : rows_in(kb, NB)) + pf * parts_at(kb);  // G1 rows + prefetch
    return (ST2 + pf) * rows_in(kb, NB);  // G2 rows (E, L, T stores) + a prefetch part each
  }
  static constexpr int T1 = (NB / 2) * MB, T2 = (MB / 2) * NB;  // steps of a G1 / G2 pass
  // With S slots the awaited chunk's DMA was issued S-2 barriers back: the bodies of the
  // (S-2)*SPC steps since and the DMA groups of the S-3 chunks issued after it are newer.  A
  // step before the pass counts with the previous pass's schedule (the smaller of the two
  // possible previous passes before G1; nothing before the prologue).
  static constexpr int SLOTS = (PKIND == PK_ROW && DLADMM_SLOTS > 4) ? 4 : DLADMM_SLOTS;
  static constexpr int WSTEPS = (SLOTS - 2) * SPC;
  // DMA_LATE: the awaited group was issued after its step's body, so that body is older
  static constexpr int W0 = DLADMM_DMA_LATE ? 1 : 0;
  static constexpr int DMAG = (SLOTS - 3) * ((CF + 3) / 4);
  template <int S>
  static constexpr int g1() {
    if constexpr ((PKIND != PK_ELEM && !DLADMM_CNT) || S % SPC != SPC - 1) return 0;
    int n = DMAG;
    for (int t = S - WSTEPS + W0; t < S; ++t) {
      if (t >= 0) n += ops1(t);
      else if (T2 + t >= 0) {
        const int a = ops2(T2 + t, true), b = ops2(T2 + t, false);
        n += a < b ? a : b;
      }
    }
    return n < 63 ? n : 63;
  }
  template <int S, bool PRO>
  static constexpr int g2() {
    if constexpr ((PKIND != PK_ELEM && !DLADMM_CNT) || S % SPC != SPC - 1) return 0;
    int n = DMAG;
    for (int t = S - WSTEPS + W0; t < S; ++t) {
      if (t >= 0) n += ops2(t, PRO);
      else if (!PRO && T1 + t >= 0) n += ops1(T1 + t);
    }
    return n < 63 ? n : 63;
  }
};

// SAVEP: also store P_k = A Z_k (a.Po) for the backward's BK1 (training forwards only: the
// fourth store per G2 element costs the inference path about 1.5 %)
template <int MP, int NP, int EMODE, int PKIND, bool SAVEP>
__global__ __launch_bounds__(256, 1) void fused_kernel(const FusedArgs a) {
  using F = Fused<MP, NP, EMODE, PKIND>;
  constexpr int MB = F::MB, NB = F::NB, CF = F::CF, NCH = F::NCH, TAB = F::TAB;
  using Win = WinCount<MB, NB, CF, PKIND, SAVEP>;
  __shared__ f32x4 smem[F::RING_F4 + F::X_F4 + F::TAB_F4];
  f32x4* ring = smem;
  f32x4* xs = smem + F::RING_F4;  // xs[w][b][lane] = X rows 16b+4g+0..3 of this lane's column
  float* tab = reinterpret_cast<float*>(smem + F::RING_F4 + F::X_F4);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 15, g = lane >> 4;
  const int64_t col = (int64_t)blockIdx.x * kTileCols + w * 16 + j;
  const bool cv = col < a.B;
  const int m = a.m, n = a.n, K = a.K;
  const bool lossz = a.loss_kind != 0;
  const bool lasso = __builtin_amdgcn_readfirstlane(a.loss_kind) == DLADMM_LOSS_LASSO;

  // per-lane byte offset of (row 4g, column col) in a [rows][ld] fp32 matrix; kOOB for padding
  auto lane_off = [&](int64_t ld) -> uint32_t {
    return cv ? (uint32_t)((col + (int64_t)(4 * g) * ld) * 4) : kOOB;
  };

  // V1 never reads E after the prologue (its E-step has no E term), so E is not state there:
  // the prologue's E0 arrives through the per-element prefetch instead (b2's slot).
  constexpr bool kEState = !(EMODE == EM_V1 && PKIND == PK_ELEM);
  float Zr[NB][4], Er[MB][4], Lr[MB][4], Vr[MB][4];
  // PK_ELEM: betas (b3, b2, b1 of k+1) of the pending G2 pair.  One buffer: the slot of row
  // (h, r) is reloaded for the pair being computed right after that row's epilogue read it.
  float pb[2][3][4];
  float regsum = 0.f, fit1 = 0.f, fit2 = 0.f;

  // ---------------------------------------------------------------- ring (LDS-DMA) stream
  // The stream is the GEMM sequence A (prologue), W_0, A, W_1, A, ..., W_{K-1}, A, then A again
  // as harmless filler.  GEMM gi: 0 = prologue A, 2k+1 = W_k, 2k+2 = A.
  const int64_t wl = (int64_t)F::GF * kFrag;  // floats per packed W_k
  auto gsrc = [&](int gi) -> const float* {
    const int kk = gi >> 1;
    return ((gi & 1) && kk < K) ? a.Wp + (int64_t)(kk * a.wstep) * wl : a.Ap;
  };
  // source of chunk ch (may run past the GEMM) of GEMM gi
  // The GEMM base goes through an opaque statement before the chunk offset is added: otherwise
  // the compiler precomputes the (loop-invariant) address of every chunk of A and keeps them
  // all live in SGPRs.
  auto chunk_src = [&](int gi, int ch) -> const float* {
    uint64_t sb = (uint64_t)gsrc(gi + ch / NCH);
    asm volatile("" : "+s"(sb));
    return (const float*)sb + (ch % NCH) * CF * kFrag;
  };
  auto issue = [&](const float* base, int slot) {
    f32x4* dst = ring + slot * (CF * 64);
#if DLADMM_ABLATE & 1  // timing experiment: no weight stream (WRONG results)
    if (base != a.Ap) return;
#endif
    if constexpr (DLADMM_DMA4 && CF % 16 == 0) {
      // wave w: fragments 16i + 4w .. +3, one M0 setup per 4 KiB
#pragma unroll
      for (int i = 0; i < CF / 16; ++i)
        glds16x4(base + (16 * i + 4 * w) * kFrag, lane * 16, dst + (16 * i + 4 * w) * 64);
    } else {
#pragma unroll
      for (int i = 0; i < (CF + 3) / 4; ++i) {
        const int f = i * 4 + w;
        if (CF % 4 == 0 || f < CF) glds16(base + f * kFrag, lane * 16, dst + f * 64);
      }
    }
  };
  auto slot_add = [](int s, int d) -> int {
    s += d;
    return s >= F::SLOTS ? s - F::SLOTS : s;
  };
  int cur = 0;  // ring slot of the chunk being consumed
  auto frag = [&](int slot, int fc) -> f32x4 { return ring[(slot * CF + fc) * 64 + lane]; };

  // ---------------------------------------------------------------- parameters
  // per-row params of layer k -> tab[buf], by LDS-DMA (each wave fills 64 consecutive entries
  // per piece; no register round trip).  Rows past m (n for theta_z) read the last valid row:
  // the padded rows' state is exactly zero whatever finite parameter they see.  Readers are
  // ring barriers away (their vmcnt(0) covers the DMA).
  auto row_tab_load = [&](int k, int buf) {
    if constexpr (PKIND == PK_ROW) {
      static_assert(TAB % 64 == 0, "whole wave pieces");  // entries past 6 MP + NP: padding
      float* t = tab + buf * TAB;
      const float* src = a.rowp + (int64_t)k * 8 * a.rstride;
#pragma unroll
      for (int j = 0; j < (TAB + 255) / 256; ++j) {
        if (256 * j + 64 * w < TAB) {  // wave-uniform
          const int i = 256 * j + 64 * w + lane;
          const int slot = i < 6 * MP ? i / MP : 6;
          const int row = i < 6 * MP ? i % MP : i - 6 * MP;
          const int lim = slot == 6 ? n : m;
          const int rowc = row < lim ? row : lim - 1;
          glds4(src, (uint32_t)(((int64_t)slot * a.rstride + rowc) * 4), t + 256 * j + 64 * w);
        }
      }
    }
  };
  // uniform per-layer scalars (s_load).  k = -1 (prologue) reads layer 0; b1n = beta1 of the
  // layer whose Var the G2 epilogue of layer k produces (k+1, clamped).
  struct LayerP { float b1n, b2, b3, ss2, ss2b, s1; ShrinkP the, thz; };
  auto layer_params = [&](int k) -> LayerP {
    LayerP p{};
    if constexpr (PKIND != PK_ROW) {
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
    }
    return p;
  };
  // value of param `slot` for (layer k, block b, reg r) of the per-row table
  auto rowp = [&](int k, int slot, int b, int r) -> float {
    const int off = (slot == DLADMM_P_THETA_Z) ? 6 * MP : slot * MP;
    return tab[(k % 3) * TAB + off + 16 * b + 4 * g + r];
  };

  // ---------------------------------------------------------------- initial state
  {
    const rsrc_t rz = mkrsrc(a.Z0, (uint32_t)(n * a.ldz0 * 4));
    const rsrc_t re = mkrsrc(a.E0, (uint32_t)(m * a.lde0 * 4));
    const rsrc_t rl = mkrsrc(a.L0, (uint32_t)(m * a.ldl0 * 4));
    const uint32_t oz = lane_off(a.ldz0), oe = lane_off(a.lde0),
                   ol = lane_off(a.ldl0), ox = lane_off(a.ldx);
    const rsrc_t rx = mkrsrc(a.X, (uint32_t)(m * a.ldx * 4));
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        Zr[b][r] = bload(rz, oz + (uint32_t)((16 * b + r) * a.ldz0 * 4));
        pin_agpr(Zr[b][r]);
      }
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      f32x4 xv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        xv[r] = bload(rx, ox + (uint32_t)((16 * b + r) * a.ldx * 4));
        if constexpr (kEState) Er[b][r] = bload(re, oe + (uint32_t)((16 * b + r) * a.lde0 * 4));
        Lr[b][r] = bload(rl, ol + (uint32_t)((16 * b + r) * a.ldl0 * 4));
        Vr[b][r] = 0.0f;
        if constexpr (DLADMM_VR_AGPR) pin_agpr(Vr[b][r]);
      }
      xs[(w * MB + b) * 64 + lane] = xv;  // read back only by this wave (no barrier needed)
    }
  }
  row_tab_load(0, 0);

  const uint32_t vo = lane_off(a.ldo);  // output lane offset (voffset of every store)
  const uint32_t vb = lane_off(a.ldb);  // per-element beta lane offset
  const uint32_t zbytes = (uint32_t)(n * a.ldo * 4), mbytes = (uint32_t)(m * a.ldo * 4);
  SWalk zw{0u, (uint32_t)(a.ldo * 4)}, mw{0u, (uint32_t)(a.ldo * 4)};
  SWalk bw{0u, (uint32_t)(a.ldb * 4)};

#if DLADMM_ABLATE & 16
  float abq[4][4];
  const int64_t c4 = (int64_t)blockIdx.x * kTileCols + w * 16 + 4 * (lane & 3);
  const uint32_t vo4 = c4 < a.B ? (uint32_t)(((lane >> 2) * a.ldo + c4) * 4) : kOOB;
  auto st4 = [&](rsrc_t r, uint32_t soff, const float (&v)[4]) {
    const f32x4 x = {v[0], v[1], v[2], v[3]};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(int __attribute__((ext_vector_type(4))), x),
                                           r, (int)vo4, (int)soff, DLADMM_ABL_AUX);
  };
#endif
  // ---------------------------------------------------------------- per-row epilogues
  // G1 block b, row r of layer k: Z = S(Z - s1*(W_k Var), theta_z)  main_lena.py:86 / tied :114
  // (q = -W_k Var: the chain ran on the negated packed weights, so Z + s1*q is the reference's
  // Z - ss1*fc(Var) operation for operation; s1 = 1 outside V5)
  auto epi1_row = [&](const LayerP& P, rsrc_t rzo, int k, int b, int r, const f32x4& q) {
#if DLADMM_ABLATE & 2  // timing experiment: no epilogue work (WRONG results)
    Zr[b][r] = q[r]; pin_agpr(Zr[b][r]); return;
#endif
    const float u = (PKIND == PK_S1) ? Zr[b][r] + P.s1 * q[r] : Zr[b][r] + q[r];
    float z;
    if constexpr (PKIND == PK_ROW) {
      // per-row theta in the clamp form as for the scalar kinds (common.h): for theta < 0 it
      // gives Z = 2U exactly where both relus are open, so the backward's masks read off the
      // saved Z_k (|Z| < 2|theta|) are exact -- the literal form can round U within an ulp of
      // -|theta| to Z = -2|theta| and drop a term there
      z = shrink_u(u, shrink_params(rowp(k, DLADMM_P_THETA_Z, b, r)));
    } else {
      z = shrink_u(u, P.thz);
    }
    Zr[b][r] = z;
    pin_agpr(Zr[b][r]);
#if DLADMM_ABLATE & 16  // timing experiment: one dwordx4 store per block, same bytes (WRONG data)
    abq[0][r] = z;
    if (r == 3) st4(rzo, zw.at(0), abq[0]);
#else
    bstore_s(rzo, vo, zw.at(r), z);
#endif
    // no column mask: padded columns hold exactly zero state (X = Z0 = E0 = L0 = 0)
    regsum += fabsf(z);
    if (r == 3) zw.next();
  };
  // G2 block b, row r of layer k (q = A Z_k, xv = X rows).  For the prologue (pro: k = -1) E and
  // L stay E0, L0 and T0 = A Z0 + E0 - X (main_lena.py:70) falls out of the same expression;
  // its E/L stores go to 0-record buffers.  pro is a compile-time constant except in the rows
  // of the prologue's last pair, which run inside G1(0).  h = block half of the pair (PK_ELEM).
  // The reference's operation order is kept throughout.
  struct OutR { rsrc_t e, l, t, p; };
  auto epi2_row = [&](const LayerP& P, const OutR& O, int k, bool pro, int b, int h, int r,
                      const f32x4& q, const f32x4& xv) {
#if DLADMM_ABLATE & 2
    Vr[b][r] = q[r]; pin_agpr(Vr[b][r]); return;
#endif
    const int kp = k < 0 ? 0 : k;
    const float Pv = q[r], x = xv[r];
    const float l0 = Lr[b][r];
    const float e0 = kEState ? Er[b][r] : pb[h][1][r];  // V1: E0 in b2's slot (pro rows only)
    float b2 = P.b2, b3 = P.b3, b1n = P.b1n;
    if constexpr (PKIND == PK_ELEM) {
      b3 = pb[h][0][r];
      b2 = pb[h][1][r];
      b1n = pb[h][2][r];
    } else if constexpr (PKIND == PK_ROW) {
      b2 = rowp(kp, DLADMM_P_BETA2, b, r);
      b3 = rowp(kp, DLADMM_P_BETA3, b, r);
      b1n = rowp(k + 1, DLADMM_P_BETA1, b, r);
    }
    float e;
    if constexpr (EMODE == EM_V1) {
      // E = S(X - A Z - b2*L, theta_e)                      main_lena.py:87
      const float u = (x - Pv) - b2 * l0;
      if constexpr (PKIND == PK_ROW) e = shrink(u, rowp(kp, DLADMM_P_THETA_E, b, r));
      else e = shrink_u(u, P.the);
    } else if constexpr (EMODE == EM_VVAR) {
      // VVar = L + b2*(A Z + E - X); E = S(E - ss2*VVar)    main_syn_l1l1_scalar.py:114-115
      if constexpr (PKIND == PK_ROW) {
        const float vv = l0 + b2 * ((Pv + e0) - x);
        e = shrink(e0 - rowp(kp, DLADMM_P_SS2, b, r) * vv, rowp(kp, DLADMM_P_THETA_E, b, r));
      } else {
        const float vv = l0 + b2 * ((Pv + e0) - x);
        e = shrink_u(e0 - P.ss2 * vv, P.the);
      }
    } else {
      // E = ss2_1*(X - A Z) - ss2_2*L                       main_syn_lasso_scalar.py:102-103
      e = P.ss2 * (x - Pv) - P.ss2b * l0;
    }
    e = pro ? e0 : e;
    const float t = (Pv + e) - x;                            // main_lena.py:70 / :88
    float l = l0 + b3 * t;                                   // main_lena.py:89 / scalar :118
    l = pro ? l0 : l;
    if constexpr (kEState) Er[b][r] = e;
    Lr[b][r] = l;
#if DLADMM_ABLATE & 16
    abq[1][r] = e; abq[2][r] = l; abq[3][r] = t;
    if (r == 3) {
      st4(O.e, mw.at(0), abq[1]);
      st4(O.l, mw.at(0), abq[2]);
      st4(O.t, mw.at(0), abq[3]);
    }
#else
    const uint32_t so = mw.at(r);
    bstore_s(O.e, vo, so, e);
    bstore_s(O.l, vo, so, l);
    bstore_s(O.t, vo, so, t);
#endif
    if constexpr (SAVEP) bstore_s(O.p, vo, so, Pv);  // A Z_k for the backward (none: prologue)
    const float res = x - Pv;
    fit1 += fabsf(res);                                      // |X - A Z|
    fit2 = __builtin_fmaf(res, res, fit2);                   // (X - A Z)^2
    // Var of the next layer: L + b1*T  (main_lena.py:85); unused after the last layer
    Vr[b][r] = l + b1n * t;
    if constexpr (DLADMM_VR_AGPR) pin_agpr(Vr[b][r]);
    if (r == 3) mw.next();
  };
  // per-column objective of layer k (k < 0: just reset the prologue's sums): the column's
  // rows are spread over the 4 lane groups
  auto flush_loss = [&](int k) {
    if (lossz && k >= 0) {
      const float rs = col_sum(regsum);
      const float fs = lasso ? 0.5f * col_sum(fit2) : col_sum(fit1);
      if (g == 0) {
        const int64_t c = (int64_t)blockIdx.x * kTileCols + w * 16 + j;
        a.lossp[(int64_t)(2 * k + 0) * a.ldl + c] = rs;
        a.lossp[(int64_t)(2 * k + 1) * a.ldl + c] = fs;
      }
    }
    regsum = 0.f;
    fit1 = 0.f;
    fit2 = 0.f;
  };
  // PK_ELEM: start the loads of the betas the G2 epilogue of (k, pair p) will need: b3, b2 and
  // the next layer's b1.  The prologue (k = -1) loads E0 into b2's slot and b1 of layer 0.
  const uint32_t ve = lane_off(a.lde0);
  SWalk ew{0u, (uint32_t)(a.lde0 * 4)};
  // Part `part` (0..7: block half h = part / 4, row r = part % 4) of the beta prefetch for the
  // pair being computed: right after the pending pair's row `part` consumed its slot (G2 pairs
  // p > 0), or spread over the first half of pair 0's steps (step (part * NB) / 16).
  // V1: the layer's beta pointers (b1 of layer k and k + 1, b2 of k), read from the device tables
  // once per G2 pass by SCALAR loads: a generic-pointer table read compiles to vector loads whose
  // waits drain every VM operation in flight (the weight DMA and the counted stores) -- 1.5 ms
  // per forward at the headline shape.
  const float* bp1 = nullptr;
  const float* bp2 = nullptr;
  const float* bpn = nullptr;
  auto beta_ptrs = [&](int k) {
    if constexpr (PKIND == PK_ELEM) {
      typedef const float* const __attribute__((address_space(4)))* ctab_p;
      const ctab_p t1 = (ctab_p)a.b1t, t2 = (ctab_p)a.b2t;
      const int kk = k < 0 ? 0 : k, kn = k + 1 < K ? k + 1 : kk;
      bp1 = t1[kk];
      bp2 = t2[kk];
      bpn = t1[kn];
    }
  };
  auto prefetch_part = [&](int k, bool pro, auto PART_) {
    constexpr int part = decltype(PART_)::value, h = part / 4, r = part % 4;
#if DLADMM_ABLATE & 8  // timing experiment: no per-element beta loads (WRONG results)
    if constexpr (PKIND == PK_ELEM) {
      pb[h][0][r] = 1.f; pb[h][1][r] = 0.5f; pb[h][2][r] = 1.f;
      return;
    }
#endif
    if constexpr (PKIND == PK_ELEM) {
      const uint32_t eb = (uint32_t)(m * a.ldb * 4);
      const rsrc_t r1 = mkrsrc(pro ? nullptr : bp1, pro ? 0u : eb);
      const rsrc_t r2 = pro ? mkrsrc(a.E0, (uint32_t)(m * a.lde0 * 4)) : mkrsrc(bp2, eb);
      const rsrc_t rn = mkrsrc(k + 1 < K ? bpn : nullptr, k + 1 < K ? eb : 0u);
      const uint32_t so = bw.at(r);
      pb[h][0][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r1, (int)vb, (int)so, 0));
      pb[h][1][r] = pro ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r2, (int)ve, (int)ew.at(r), 0))
                        : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r2, (int)vb, (int)so, 0));
      pb[h][2][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rn, (int)vb, (int)so, 0));
      if constexpr (r == 3) {
        bw.next();
        if (pro) ew.next();
      }
    }
  };

  // ---------------------------------------------------------------- one MFMA step
  // Step s of GEMM gi (compile-time s, runtime gi): fragments 2s, 2s+1 of the GEMM's stream.
  // Order inside a step: read ahead the next step's two fragments (at a chunk's last step:
  // ring barrier, next chunk's first fragments, LDS-DMA of the chunk after it), then the
  // epilogue rows scheduled here, then 8 MFMAs on two independent chains; a sched_barrier
  // pins that order.  fr[] rotates over 4 registers (2 steps x 2 fragments).
  f32x4 fr[4];
  // WIN = VM operations (stores, V1 beta loads) definitely issued since the awaited chunk's DMA
  // (WinCount): they stay in flight across the barrier
#if DLADMM_STAMP
  // diagnostic build: per-wave cycle sums (read the shares, not this build's run time)
  auto stamp = []() -> uint64_t {
    uint64_t v;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
    return v;
  };
  uint64_t st_vm = 0, st_bar = 0, st_g1 = 0, st_g2 = 0;
  const uint64_t st_0 = stamp();
#endif
  auto step_head = [&](auto S_, int gi, auto WIN_) {
    constexpr int s = decltype(S_)::value;
    constexpr int WIN = decltype(WIN_)::value;
    constexpr int fi = 2 * s, fc = fi % CF, ch = fi / CF;
    if constexpr (fc + 2 < CF) {
      fr[(fi + 2) % 4] = frag(cur, fc + 2);
      fr[(fi + 3) % 4] = frag(cur, fc + 3);
    } else {
      // chunk ch+1 landed for every wave; every wave is done with chunk ch-1
#if DLADMM_STAMP
      __builtin_amdgcn_sched_barrier(0);
      const uint64_t t0 = stamp();
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(WIN) : "memory");
      const uint64_t t1 = stamp();
      asm volatile("s_barrier" ::: "memory");
      const uint64_t t2 = stamp();
      __builtin_amdgcn_sched_barrier(0);
      st_vm += t1 - t0;
      st_bar += t2 - t1;
#else
      if constexpr (WIN > 0) ring_barrier_cnt<WIN>();
      else ring_barrier();
#endif
      if constexpr (!DLADMM_DMA_LATE)
        issue(chunk_src(gi, ch + F::SLOTS - 1), slot_add(cur, F::SLOTS - 1));
      const int nx = slot_add(cur, 1);
      fr[(fi + 2) % 4] = frag(nx, 0);
      fr[(fi + 3) % 4] = frag(nx, 1);
    }
  };
  auto step_tail = [&](auto S_, int gi) {
    constexpr int s = decltype(S_)::value;
    constexpr int fi = 2 * s, fc = fi % CF, ch = fi / CF;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (fc + 2 >= CF) {
      if constexpr (DLADMM_DMA_LATE) {
        // after the step's MFMAs (an LDS-DMA instruction issues cheaper among MFMAs than beside
        // ds_reads, MI355X_MICROARCH.md); the barrier at this step's head freed the slot
        issue(chunk_src(gi, ch + F::SLOTS - 1), slot_add(cur, F::SLOTS - 1));
        __builtin_amdgcn_sched_barrier(0);
      }
      cur = slot_add(cur, 1);
    }
  };

  // prime the ring: the first SLOTS - 1 chunks, then the first step's fragments
#pragma unroll
  for (int c = 0; c < F::SLOTS - 1; ++c) issue(chunk_src(0, c), c);
  ring_barrier();
  fr[0] = frag(0, 0);
  fr[1] = frag(0, 1);

  // ---------------------------------------------------------------- the GEMM passes
  f32x4 qa = {0.f, 0.f, 0.f, 0.f}, qb = {0.f, 0.f, 0.f, 0.f};  // pending pair accumulators
  f32x4 xa, xb;  // X rows of the pending G2 pair
  auto load_x = [&](int p) {
    xa = xs[(w * MB + 2 * p) * 64 + lane];
    xb = xs[(w * MB + 2 * p + 1) * 64 + lane];
  };
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

  // G1(k): -s1 W_k Var, chains of blocks (2p, 2p+1) over jb = 0..MB-1.  Pair 0 runs the
  // rows of the last G2 pair of layer k-1 (Pp, Op; the prologue's when k = 0).
  auto g1_pass = [&](int k, const LayerP& P, rsrc_t rzo, const LayerP& Pp, const OutR& Op) {
    const int gi = 2 * k + 1;
    zw.reset();
    // layer k+1's row table -> buffer (k+1)%3.  Its previous content (layer k-2) was last
    // read in G1(k-1)'s deferred epilogue, several ring barriers ago.
    if (k + 1 < K) row_tab_load(k + 1, (k + 1) % 3);
    static_for<NB / 2>([&](auto P_) {
      constexpr int p = decltype(P_)::value;
      f32x4 ca = zero4, cb = zero4;
      if constexpr (p == 0) load_x(MB / 2 - 1);
      static_for<MB>([&](auto J_) {
        constexpr int jb = decltype(J_)::value;
        constexpr int s = p * MB + jb;
        step_head(std::integral_constant<int, s>{}, gi,
                  std::integral_constant<int, Win::template g1<s>()>{});
        static_for<8>([&](auto I_) {
          constexpr int i = decltype(I_)::value;
          constexpr int h = i / 4, r = i % 4;
          if constexpr (rows_at(jb, MB, i)) {
            if constexpr (p == 0) {
              epi2_row(Pp, Op, k - 1, k == 0, MB - 2 + h, h, r, h ? qb : qa, h ? xb : xa);
              if constexpr (i == 7) flush_loss(k - 1);
            } else {
              epi1_row(P, rzo, k, 2 * p - 2 + h, r, h ? qb : qa);
            }
          }
        });
        const f32x4 wa = fr[(2 * s) % 4], wb = fr[(2 * s + 1) % 4];
        ca = mfma4(wa.x, Vr[jb][0], ca);
        cb = mfma4(wb.x, Vr[jb][0], cb);
        ca = mfma4(wa.y, Vr[jb][1], ca);
        cb = mfma4(wb.y, Vr[jb][1], cb);
        ca = mfma4(wa.z, Vr[jb][2], ca);
        cb = mfma4(wb.z, Vr[jb][2], cb);
        ca = mfma4(wa.w, Vr[jb][3], ca);
        cb = mfma4(wb.w, Vr[jb][3], cb);
        step_tail(std::integral_constant<int, s>{}, gi);
      });
      qa = ca;
      qb = cb;
    });
  };
  // G2(k): A Z_k, chains of blocks (2p, 2p+1) over kb = 0..NB-1.  Pair 0 runs the rows of
  // G1(k)'s last pair (none in the prologue); pair p > 0 runs those of pair p-1.
  auto g2_pass = [&](auto PRO_, int k, const LayerP& P, const OutR& O, rsrc_t rzo) {
    constexpr bool PRO = decltype(PRO_)::value;
    const int gi = 2 * k + 2;
    mw.reset();
    bw.reset();
    if constexpr (PRO) ew.reset();
    beta_ptrs(k);
    static_for<MB / 2>([&](auto P_) {
      constexpr int p = decltype(P_)::value;
      f32x4 ca = zero4, cb = zero4;
#if DLADMM_G2_CHAINS == 2
      f32x4 ca2 = zero4, cb2 = zero4;  // second accumulation chain (k sub-steps y, w)
#endif
      if constexpr (p > 0) load_x(p - 1);
      static_for<NB>([&](auto K_) {
        constexpr int kb = decltype(K_)::value;
        constexpr int s = p * NB + kb;
        step_head(std::integral_constant<int, s>{}, gi,
                  std::integral_constant<int, Win::template g2<s, PRO>()>{});
        if constexpr (p == 0) {
          static_for<8>([&](auto PT_) {
            constexpr int part = decltype(PT_)::value;
            if constexpr (Win::part_step(part) == kb) prefetch_part(k, PRO, PT_);
          });
        }
        static_for<8>([&](auto I_) {
          constexpr int i = decltype(I_)::value;
          constexpr int h = i / 4, r = i % 4;
          if constexpr (rows_at(kb, NB, i)) {
            if constexpr (p == 0) {
              if constexpr (!PRO) epi1_row(P, rzo, k, NB - 2 + h, r, h ? qb : qa);
            } else {
              epi2_row(P, O, k, PRO, 2 * p - 2 + h, h, r, h ? qb : qa, h ? xb : xa);
              prefetch_part(k, PRO, I_);  // this row's beta slot, for pair p
            }
          }
        });
        const f32x4 wa = fr[(2 * s) % 4], wb = fr[(2 * s + 1) % 4];
#if DLADMM_G2_CHAINS == 2
        ca = mfma4(wa.x, Zr[kb][0], ca);
        cb = mfma4(wb.x, Zr[kb][0], cb);
        ca2 = mfma4(wa.y, Zr[kb][1], ca2);
        cb2 = mfma4(wb.y, Zr[kb][1], cb2);
        ca = mfma4(wa.z, Zr[kb][2], ca);
        cb = mfma4(wb.z, Zr[kb][2], cb);
        ca2 = mfma4(wa.w, Zr[kb][3], ca2);
        cb2 = mfma4(wb.w, Zr[kb][3], cb2);
#else
        ca = mfma4(wa.x, Zr[kb][0], ca);
        cb = mfma4(wb.x, Zr[kb][0], cb);
        ca = mfma4(wa.y, Zr[kb][1], ca);
        cb = mfma4(wb.y, Zr[kb][1], cb);
        ca = mfma4(wa.z, Zr[kb][2], ca);
        cb = mfma4(wb.z, Zr[kb][2], cb);
        ca = mfma4(wa.w, Zr[kb][3], ca);
        cb = mfma4(wb.w, Zr[kb][3], cb);
#endif
        step_tail(std::integral_constant<int, s>{}, gi);
      });
#if DLADMM_G2_CHAINS == 2
      qa = ca + ca2;
      qb = cb + cb2;
#else
      qa = ca;
      qb = cb;
#endif
    });
  };

  // ---------------------------------------------------------------- prologue + K layers
  // G2(-1) [A Z0 - X -> T0, Var_0], then per layer G1(k) [Z_k], G2(k) [E_k, L_k, T_k+1, Var_k+1]
  const rsrc_t none = mkrsrc(nullptr, 0u);
  LayerP Pp = layer_params(-1);
  OutR Op{none, none,
          mkrsrc(a.keep_all ? a.To : nullptr, (a.keep_all && a.To) ? mbytes : 0u), none};
  g2_pass(std::true_type{}, -1, Pp, Op, none);
  for (int k = 0; k < K; ++k) {
    const bool st = a.keep_all || k == K - 1;
    const int ko = a.keep_all ? k : 0;
    const LayerP P = layer_params(k);
    // outputs of layer k; num_records 0 = not stored
    const rsrc_t rzo = mkrsrc(a.Zo + (int64_t)ko * n * a.ldo, st ? zbytes : 0u);
#if DLADMM_STAMP
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t ta = stamp();
    __builtin_amdgcn_sched_barrier(0);
#endif
    g1_pass(k, P, rzo, Pp, Op);
#if DLADMM_STAMP
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t tb = stamp();
    __builtin_amdgcn_sched_barrier(0);
    st_g1 += tb - ta;
#endif
    const OutR O{mkrsrc(a.Eo + (int64_t)ko * m * a.ldo, st ? mbytes : 0u),
                 mkrsrc(a.Lo + (int64_t)ko * m * a.ldo, st ? mbytes : 0u),
                 mkrsrc(a.To ? a.To + (int64_t)(a.keep_all ? k + 1 : 0) * m * a.ldo : nullptr,
                        (a.To && st) ? mbytes : 0u),
                 mkrsrc(SAVEP && a.Po && a.keep_all ? a.Po + (int64_t)k * m * a.ldo : nullptr,
                        SAVEP && a.Po && a.keep_all ? mbytes : 0u)};
    g2_pass(std::false_type{}, k, P, O, rzo);
#if DLADMM_STAMP
    __builtin_amdgcn_sched_barrier(0);
    st_g2 += stamp() - tb;
    __builtin_amdgcn_sched_barrier(0);
#endif
    Pp = P;
    Op = O;
  }
  // epilogue of the last G2 pair of layer K-1
  load_x(MB / 2 - 1);
#pragma unroll
  for (int i = 0; i < 8; ++i)
    epi2_row(Pp, Op, K - 1, false, MB - 2 + i / 4, i / 4, i % 4, i < 4 ? qa : qb,
             i < 4 ? xa : xb);
  flush_loss(K - 1);
  // drain: the ring's last LDS-DMA must land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if DLADMM_STAMP
  const uint64_t st_end = stamp();
  if (a.dbg && lane < 8) {  // vector stores: lane i writes sum i
    const uint64_t v[8] = {st_end - st_0, st_g1, st_g2, 0, st_vm, st_bar, 0, 0};
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x = lane == i ? v[i] : x;
    a.dbg[((int64_t)blockIdx.x * kWaves + w) * 8 + lane] = x;
  }
#endif
}


template <int MP, int NP, int EM, int PK, bool SAVEP>
hipError_t launch_fused(const FusedArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((fused_kernel<MP, NP, EM, PK, SAVEP>), dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace dladmm
