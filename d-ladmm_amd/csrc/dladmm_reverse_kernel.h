// dladmm_reverse_kernel.h -- MI355X (gfx950 / CDNA4) backward of the K-layer D-LADMM forward as ONE
// reverse sweep: the vector-Jacobian product torch autograd forms
// for total_loss.backward() (main_syn_l1l1_scalar.py:298, main_syn_lasso_scalar.py:285) through
// DLADMMNet.forward, for the scalar-parameter variants V4 / V6 after a training forward of the
// fused kernel (which saved P_k = A Z_k, fwd_desc.P).
//
// The per-layer backward (dladmm_backward.hip, phases 4 / 5 / 6) runs a layer as two GEMM
// launches whose adjoints round-trip through HBM.  This kernel has the forward's structure
// (dladmm_fused_kernel.h) instead:
//  * one workgroup = 4 waves = 64 batch columns, wave w owns 16.  The adjoint state -- of Z
//    (n rows) and the partial adjoint of L_{k-1} (m rows) -- and gP (m rows) stay in registers
//    for all K layers, in the C/D layout of v_mfma_f32_16x16x4_f32 (lane l: column l & 15, rows
//    16 b + 4 (l >> 4) + r); X sits in LDS.  The adjoint of E_{k-1} (V4 only; V6's E-step has
//    no E term) round-trips through the workspace rows after Var_k's, read one block ahead with
//    the saved state: in registers it would push the kernel past the 512-register budget;
//  * per layer k = K-1 .. 0, two products shaped exactly like the forward's two:
//      G1'(k)  R    = A^T gP_k     rows n, contraction m  (B operand gP_k, registers)
//      G2'(k)  gVar = M_k^T gU_k   rows m, contraction n  (B operand gU_k, registers)
//    with M_k = -s1 W_k.  A^T and every M_k^T are packed once per call in the forward's paired
//    fragment order and stream through the same 4-slot LDS-DMA ring.  Each output block is one
//    fma chain over the contraction in k order -- the order of the slice kernels -- so R and
//    gVar are the per-layer backward's bit for bit;
//  * G1'(k)'s epilogue is BK2(k) (phase 5): gU_k = adjoint of Z_{k-1}, with S'(U_k) from the
//    saved Z_k (for theta_z < 0 too: the forward's shrink is monotone, |Z| < 2|theta| exactly
//    where both relus are open).  G2'(k)'s is BK3(k) + BK1(k-1) on the saved P_{k-1} (phase 6).
//    Same expressions in the same order as those phases (the elementwise adjoints, gU and Var
//    are the per-layer sweep's values; only the sign of a zero may differ, where that sweep
//    adds a zero upstream cotangent);
//  * each output pair's epilogue rows are spread over the MFMA steps of the next pair; their
//    operands from the saved forward state (Z_k for BK2; P, E, L, T for BK1) are loaded one pair
//    ahead and stay in flight across the ring barriers (counted vmcnt, RevWin);
//  * the epilogues write gU_k and Var_k of every layer to the workspace; the weight gradient
//    gW_k = -s1 gU_k Var_k^T runs afterwards as split-K GEMMs (wgrad_kernel).  Parameter partials
//    go per (layer, slot, wave) to a buffer summed in fp64 in a fixed order.
#pragma once
// Instantiated per E-step form and shape by dladmm_reverse_{v1,vvar,lasso}[_small].hip (one
// translation unit each: the unrolled K-pass bodies take minutes per instantiation); the
// dispatch is dladmm_reverse.hip.
#include "dladmm_common.h"
#include "dladmm_internal.h"

#ifndef REV_ABL
#define REV_ABL 0  // timing / register-pressure experiments only (WRONG results): 1 no prologue
                   // rows, 2 no G2' rows, 4 no G1' rows, 8 no Z_k loads, 16 no gU stores, 32 no
                   // G2' operand loads, 64 no Var / adjoint-of-E stores; through a null buffer
                   // view (instructions kept, no memory traffic): 128 the adjoint of E (loads and
                   // stores), 256 X, 512 P, 1024 E, 2048 L; one dwordx4 per G2' block instead of
                   // a dword per row (fragment order; measured slower, profiles/r05_rev_x4.json):
                   // 4096 X, 8192 P, 16384 the adjoint of E
#endif

#ifndef REV_LOAD_AUX
#define REV_LOAD_AUX 2  // cache policy of the epilogue operand loads: nt (read once; 7.42 vs
                        // 7.50 ms backward with the default policy, profiles/r04_rev_loadaux_ab.json)
#endif
#ifndef REV_SLOTS
#define REV_SLOTS 4  // weight-ring slots (6 fit the LDS at 256 x 512 beside the AL tables)
#endif
#ifndef REV_CF
#define REV_CF 16    // fragments per ring chunk (a ring barrier every REV_CF / 2 MFMA steps)
#endif
#ifndef REV_DEEP
#define REV_DEEP 0   // 1: operands two pairs / one pair ahead (needs REV_SLOTS 6); measured no
                     // faster (7.58 vs 7.53 ms backward, profiles/r04_rev_deep_ab.json)
#endif

namespace dladmm {

template <int MP, int NP>
struct Rev {
  static constexpr int MB = MP / 16;
  static constexpr int NB = NP / 16;
  static constexpr int GF = MB * NB;                       // fragments per product
  static constexpr int CF = GF < REV_CF ? GF : REV_CF;     // fragments per ring chunk
  static constexpr int NCH = GF / CF;                      // chunks per product
  static constexpr int SLOTS = REV_SLOTS;                  // ring slots (SLOTS - 1 in flight)
  static constexpr int RING_F4 = SLOTS * CF * 64;
  static constexpr int AL_F4 = kWaves * MB * 64;           // partial adjoints of L, in LDS
  static_assert(MB % 2 == 0 && NB % 2 == 0, "output blocks are processed in pairs");
  static_assert(GF % CF == 0 && CF % 2 == 0, "chunking");
  static_assert((RING_F4 + AL_F4) * 16 <= 160 * 1024, "LDS budget");
};

// epilogue row i (0..7: block half i / 4, row i % 4) of a pair runs at step (i * SP) / 8 of the
// next pair's SP steps; part q of the np operand-load parts of a pass's first pair runs at step
// (q * SP) / (2 np) (the first half of the pair)
constexpr bool rev_rows_at(int step, int SP, int i) { return (i * SP) / 8 == step; }
constexpr int rev_part_step(int q, int SP, int np) { return (q * SP) / (2 * np); }

// VM operations (buffer stores and loads) each step's body issues, for the counted vmcnt of the
// ring barriers (the scheme of the forward's WinCount).  With SLOTS slots a barrier waits for
// the chunk DMA issued SLOTS - 2 barriers back; the bodies of the (SLOTS - 2) * SPC steps since
// and the SLOTS - 3 chunk DMA groups issued in between are newer and stay in flight.
// Operand loads run one block (G2') / one pair (G1') ahead, or with DEEP one pair / two pairs:
// ST1: the VM stores of one G1' row (gU; ROWP: theta_z's per-row partial).
//   G1' pass, pair 0: rows of the previous G2' pass's last pair (ST2 stores; not DEEP: the first
//     block's rows also load the second block's LD2 operands; none in the first pass) + the LD1
//     loads (Z_k, GZ: its cotangent) of pair 0 (DEEP: pairs 0 and 1) as parts; pair p > 0:
//     rows of pair p - 1 (gU store + the LD1 loads of pair p, DEEP: p + 1 while it exists).
//   G2' pass, pair 0: rows of G1''s last pair (gU store) + the LD2 loads of block 0's rows
//     (DEEP: blocks 0 and 1) as parts; pair p > 0: rows of pair p - 1 (ST2 stores + the LD2
//     loads of the next block, DEEP: of block 2p + h).
// ST2 / LD2: the VM stores / loads of one G2' row (reverse_kernel: Var, V4's adjoint of E, V1's
// beta gradients; P, L, T, X, E and V4's adjoint of E, V1's betas, the E / L / T cotangents).
// The parameter-partial stores of the pass boundaries are not counted (fewer counted = a
// longer wait only).
template <int MB, int NB, int CF, int SLOTS, int ST1, int ST2, int LD2, int LD1, bool DEEP>
struct RevWin {
  static constexpr int SPC = CF / 2;            // steps per chunk
  static constexpr int WSTEPS = (SLOTS - 2) * SPC;
  static constexpr int DMAG = (CF + 3) / 4;     // VM operations of one chunk DMA per wave
  static constexpr int T1 = (NB / 2) * MB, T2 = (MB / 2) * NB;  // steps of a G1' / G2' pass
  // first-pair load parts (G1': pair 1 exists when NB > 2)
  static constexpr int NP1 = (DEEP && NB / 2 > 1) ? 16 : 8, NP2 = DEEP ? 8 : 4;
  static constexpr int rows_in(int step, int SP) {
    int c = 0;
    for (int i = 0; i < 8; ++i) c += rev_rows_at(step, SP, i) ? 1 : 0;
    return c;
  }
  static constexpr int rows_h(int step, int SP, int h) {
    int c = 0;
    for (int i = 4 * h; i < 4 * h + 4; ++i) c += rev_rows_at(step, SP, i) ? 1 : 0;
    return c;
  }
  static constexpr int parts_at(int step, int SP, int np) {
    int c = 0;
    for (int q = 0; q < np; ++q) c += rev_part_step(q, SP, np) == step ? 1 : 0;
    return c;
  }
  static constexpr int ops1(int t, bool first) {
    const int p = t / MB, s = t % MB;
    if (p == 0) {
      const int prev = first ? 0 : DEEP ? ST2 * rows_in(s, MB)
                                        : (ST2 + LD2) * rows_h(s, MB, 0) + ST2 * rows_h(s, MB, 1);
      return prev + LD1 * parts_at(s, MB, NP1);
    }
    const bool loads = !DEEP || p + 1 < NB / 2;
    return (ST1 + (loads ? LD1 : 0)) * rows_in(s, MB);
  }
  static constexpr int ops2(int t) {
    const int p = t / NB, s = t % NB;
    if (p == 0) return ST1 * rows_in(s, NB) + LD2 * parts_at(s, NB, NP2);
    return (ST2 + LD2) * rows_in(s, NB);
  }
  template <int S, bool FIRST>
  static constexpr int g1() {
    if constexpr (S % SPC != SPC - 1) return 0;
    int n = DMAG * (SLOTS - 3);
    for (int t = S - WSTEPS; t < S; ++t) {
      if (t >= 0) n += ops1(t, FIRST);
      else if (!FIRST && T2 + t >= 0) n += ops2(T2 + t);  // the first pass follows a drain
    }
    return n < 63 ? n : 63;
  }
  template <int S>
  static constexpr int g2() {
    if constexpr (S % SPC != SPC - 1) return 0;
    int n = DMAG * (SLOTS - 3);
    for (int t = S - WSTEPS; t < S; ++t) {
      if (t >= 0) n += ops2(t);
      else if (T1 + t >= 0) n += ops1(T1 + t, true);  // the smaller of the two G1' forms
    }
    return n < 63 ? n : 63;
  }
};

// GZ: per-layer output cotangents of Z (a loss built from the returned Z_k with torch ops, as
// the reference's training loops do): one more load per G1' element, added where the per-layer
// BK2 adds it ((adjoint + gZ_k) + A^T gP).  COT: cotangents of E_k, L_k, T_{k+1} (main_lena.py:
// 221-228 reads E and L): three more loads per G2' element, added where the per-layer BK1 adds
// them.  EMODE EM_V1: V1 (main_lena.py:57-98), per-sample betas (m, B) -- their values and
// gradients are per-element operands of the G2' rows; beta1's gradient sums BK1's term (one G2'
// pass) and BK3's (the next), so it goes through HBM between the two passes as in the per-layer
// sweep.  ROWP: V2 / V3 (main_syn_l1l1_ltheta.py, main_syn_l1l1_full.py), per-row parameters:
// their values are per-row operands (a row-table load whose 16 lanes of a row share the address)
// and their gradients per-row partials -- the 16 columns of a wave summed (col16_sum) and written
// per (layer, slot, row, wave) exactly as the per-layer kernels write them, then reduced in fp64
// in a fixed order.
template <int MP, int NP, int EMODE, bool GZ, bool COT, bool ROWP>
__global__ __launch_bounds__(256, 1) void reverse_kernel(const RevArgs a) {
  using F = Rev<MP, NP>;
  constexpr int MB = F::MB, NB = F::NB, CF = F::CF, NCH = F::NCH;
  constexpr bool kAE = EMODE == EM_VVAR;             // the adjoint of E is state (workspace rows)
  constexpr bool kV1 = EMODE == EM_V1 && !ROWP;      // V1: per-sample betas
  constexpr bool kSC = !kV1 && !ROWP;                // scalar parameters (V4 / V5 / V6)
  // operands of one G2' row (pv slots): saved state, X, the partial adjoint of L (LDS), then the
  // variant's own and the cotangents
  constexpr int S_P = 0, S_L = 1, S_T = 2, S_X = 3, S_AL = 4;
  constexpr int S_E = 5, S_AE = 6;                              // V3 / V4 / V5
  constexpr int S_B1K = 5, S_B1J = 6, S_B2J = 7, S_GB1 = 8;     // V1
  constexpr int S_R = kAE ? 7 : 5;                              // ROWP: per-row parameters
  constexpr int S_RB1K = S_R, S_RB1J = S_R + 1, S_RB2J = S_R + 2, S_RTHE = S_R + 3;
  constexpr int S_RB3J = S_R + 4, S_RSS2J = S_R + 5;            // ROWP with the VVar E-step
  constexpr int NR = ROWP ? (kAE ? 6 : 4) : 0;
  constexpr int S_C = kV1 ? 9 : (kAE ? 7 : 5) + NR;
  constexpr int S_GE = S_C, S_GL = S_C + 1, S_GT = S_C + 2;     // COT
  constexpr int NS = S_C + (COT ? 3 : 0);
  // per-row parameter gradient slots a G2' row stores (BK3's beta1 of layer k; BK1's of layer
  // k - 1): V2 beta3 (= beta1's L term), beta2, theta_e; V3 also ss2
  constexpr int NRS = ROWP ? (kAE ? 5 : 4) : 0;
  constexpr int LD2 = 3 + (kAE ? 2 : 0) + (kV1 ? 4 : 0) + NR + (COT ? 3 : 0);
  constexpr int ST2 = 1 + (kAE ? 1 : 0) + (kV1 ? 3 : 0) + NRS;
  constexpr int LD1 = 1 + (GZ ? 1 : 0) + (ROWP ? 1 : 0);
  // DEEP: operands two pairs (G1') / one pair (G2') ahead instead of one pair / one block --
  // a second register set for them, where the registers allow (the ring's 5 chunks in flight
  // let the counted barriers keep them in flight)
  constexpr bool DEEP = REV_DEEP && 4 * NS + (GZ ? 16 : 8) <= 36;
  constexpr int PV = DEEP ? 2 : 1;   // operand register sets
  constexpr int ST1 = ROWP ? 2 : 1;
  using Win = RevWin<MB, NB, CF, F::SLOTS, ST1, ST2, LD2, LD1, DEEP>;
  __shared__ f32x4 smem[F::RING_F4 + F::AL_F4];
  f32x4* ring = smem;
  // als[w][b][lane][r]: partial adjoint of L_{k-1} at rows 16b+4g+r of this lane's column, from
  // one G2' pass to the next (read back only by this wave)
  float* als = reinterpret_cast<float*>(smem + F::RING_F4);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int64_t col = (int64_t)blockIdx.x * kTileCols + w * 16 + (lane & 15);
  const bool cv = col < a.B;
  const int m = a.m, K = a.K;
  const int cg = blockIdx.x * kWaves + w;  // column group (wave) index of the partials
  const uint32_t lqm = __builtin_amdgcn_readfirstlane(a.loss_kind) == DLADMM_LOSS_LASSO ? ~0u : 0u;
  const int64_t ldo = a.ldo, ml = (int64_t)m * ldo, zl = (int64_t)a.n * ldo;
  auto lane_off = [&](int64_t ld, bool ok) -> uint32_t {
    return ok ? (uint32_t)((col + (int64_t)(4 * g) * ld) * 4) : kOOB;
  };
  const uint32_t vo = lane_off(ldo, cv);          // saved forward state
  const uint32_t vx = lane_off(a.ldx, cv);        // X
  const uint32_t vw = lane_off(a.ldw, col < a.Bw);  // gU / Var workspaces (padding: zeros)
  const rsrc_t none = mkrsrc(nullptr, 0u);
  // buffer view of a wave-uniform (pointer, size) formed by runtime selects: readfirstlane keeps
  // both in SGPRs (otherwise a select lands in VGPRs and every access becomes a waterfall loop)
  auto urs = [](const float* p, uint32_t bytes) -> rsrc_t {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return mkrsrc((const float*)(((uint64_t)hi << 32) | lo), __builtin_amdgcn_readfirstlane(bytes));
  };
  // the call's pointer table, read by SCALAR loads (a generic-pointer read becomes vector loads
  // whose waits drain the weight DMA)
  typedef const float* const __attribute__((address_space(4)))* ctab_p;
  const ctab_p tab = (ctab_p)a.ptab;
  auto tptr = [&](int t, int k) -> const float* { return tab[rev_tab_at(t, K, k)]; };

  // adjoint state: of Z (AZ; gU once G1' formed it) and gP (the G1' B operand), MFMA operands
  // in AGPRs; the partial adjoint of L_{k-1} in LDS (als), of E_{k-1} (V4) in the workspace
  float AZ[NB][4], GP[MB][4];
  float pz[PV][2][4];  // Z_k rows of a G1' pair (set: pair parity when DEEP)
  float pg[PV][2][4];  // GZ: the cotangent of Z_k at those rows
  float pt[PV][2][4];  // ROWP: theta_z of those rows
  float pvs_all[PV][4][NS];  // the operands of row r of a G2' block (set: block parity, DEEP)
  auto set1 = [](int pair) { return DEEP ? (pair & 1) : 0; };
  auto set2 = [](int blk) { return DEEP ? (blk & 1) : 0; };
  float psz = 0.f, psb1 = 0.f, ps[5] = {0.f, 0.f, 0.f, 0.f, 0.f};  // parameter partials

  // ---------------------------------------------------------------- ring (LDS-DMA) stream
  // GEMM gi: 2 (K-1-k) = G1'(k) (A^T), 2 (K-1-k) + 1 = G2'(k) (M_k^T); past the end: A^T filler
  const int64_t wl = (int64_t)F::GF * kFrag;  // floats per packed M_k^T
  auto gsrc = [&](int gi) -> const float* {
    const int kk = K - 1 - (gi >> 1);
    return ((gi & 1) && kk >= 0) ? a.Mtp + (int64_t)kk * wl : a.Atp;
  };
  auto chunk_src = [&](int gi, int ch) -> const float* {
    uint64_t sb = (uint64_t)gsrc(gi + ch / NCH);
    asm volatile("" : "+s"(sb));
    return (const float*)sb + (ch % NCH) * CF * kFrag;
  };
  auto issue = [&](const float* base, int slot) {
    f32x4* dst = ring + slot * (CF * 64);
    if constexpr (DLADMM_DMA4 && CF % 16 == 0) {
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
  int cur = 0;
  auto frag = [&](int slot, int fc) -> f32x4 { return ring[(slot * CF + fc) * 64 + lane]; };
  // prime the ring first: its DMA overlaps the prologue
#pragma unroll
  for (int c = 0; c < F::SLOTS - 1; ++c) issue(chunk_src(0, c), c);

  // ---------------------------------------------------------------- initial state
  auto al_at = [&](int b, int r) -> int { return ((w * MB + b) * 64 + lane) * 4 + r; };
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      AZ[b][r] = 0.f;
      pin_agpr(AZ[b][r]);
    }
#pragma unroll
  for (int b = 0; b < MB; ++b)
    reinterpret_cast<f32x4*>(als)[(w * MB + b) * 64 + lane] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---------------------------------------------------------------- parameters
  cfloat_p sp = (cfloat_p)a.scal;
  // G2'(k): beta1 of BK3's layer k; BK1's layer j = k - 1 (the prologue: j = K - 1)
  struct LP2 { float b1k, b1, b2, b3, ss2, ss2b, the, cf; };
  auto lp2 = [&](int k, int jl) -> LP2 {
    LP2 p{};
    const int kk = k < K ? k : K - 1;
    const int jj = jl < 0 ? 0 : jl;
    p.cf = a.loss_kind ? ((cfloat_p)a.lcoef)[2 * jj + 1] : 0.f;
    if constexpr (ROWP) return p;  // per-row parameters: row-table operands (no scalar table)
    p.b1k = sp[kk * DLADMM_NSCALAR + DLADMM_P_BETA1];
    p.b1 = sp[jj * DLADMM_NSCALAR + DLADMM_P_BETA1];
    p.b2 = sp[jj * DLADMM_NSCALAR + DLADMM_P_BETA2];
    p.b3 = sp[jj * DLADMM_NSCALAR + DLADMM_P_BETA3];
    p.ss2 = sp[jj * DLADMM_NSCALAR + DLADMM_P_SS2];
    p.ss2b = sp[jj * DLADMM_NSCALAR + DLADMM_P_SS2B];
    p.the = sp[jj * DLADMM_NSCALAR + DLADMM_P_THETA_E];
    return p;
  };
  // G1'(k): the mask bound c from theta_z (0 for theta_z >= 0, else 2|theta_z|) and cz_k
  struct LP1 { float c, cz; };
  auto lp1 = [&](int k) -> LP1 {
    const float th = ROWP ? 0.f : sp[k * DLADMM_NSCALAR + DLADMM_P_THETA_Z];
    return LP1{th >= 0.f ? 0.f : -2.0f * th, a.loss_kind ? ((cfloat_p)a.lcoef)[2 * k] : 0.f};
  };

  // ---------------------------------------------------------------- operand views
  // BK1 of layer j reads P_j, E_{j-1}, L_{j-1} (E0 / L0 for j = 0, their own strides), T_j;
  // V1: beta1_{j+1} (BK3's), beta1_j, beta2_j and the BK1 part of beta1_{j+1}'s gradient; COT:
  // the cotangents of E_j, L_j and T_{j+1}.  The last G2' pass (BK3 of layer 0 alone) reads T_0
  // through the P slot (V1: and beta1_0's gradient so far)
  // ROWP: the row table [K][8][rstride] (lane: rows 4g.. of a block, the 16 lanes of a row on
  // one address; rows past m / n read finite table entries that meet zero adjoints) and the
  // per-row partials [K][8][RS][ncg], RS = max(MP, NP) rows so that the padded rows' partials
  // land in the buffer too -- a per-lane row test here would be hoisted out of the unrolled
  // passes as one live register per (block, row); the reduction reads rows < m / n only
  constexpr int RS = MP > NP ? MP : NP;
  const int64_t rst = ROWP ? a.rstride : 0;
  const rsrc_t rrow = ROWP ? mkrsrc(a.rowp, (uint32_t)(K * 8 * rst * 4)) : none;
  const uint32_t vr = (uint32_t)(16 * g);
  auto rbase = [&](int k, int slot) -> uint32_t {
    return __builtin_amdgcn_readfirstlane((uint32_t)(((int64_t)k * 8 + slot) * rst * 4));
  };
  const int64_t pslot = (int64_t)RS * a.ncg;   // floats per (layer, slot) of the partials
  auto rpart = [&](int k) {
    return urs(a.rpart + (int64_t)k * 8 * pslot, (uint32_t)(8 * pslot * 4));
  };
  const uint32_t vpr = (lane & 15) == 0 ? (uint32_t)(((int64_t)(4 * g) * a.ncg + cg) * 4) : kOOB;
  auto pso = [&](int slot) -> uint32_t {
    return __builtin_amdgcn_readfirstlane((uint32_t)(slot * pslot * 4));
  };
  const uint32_t ldp4 = (uint32_t)(a.ncg * 4);
  struct R2 {
    rsrc_t P, E, L, T, B1K, B1J, B2J, GB1K, GB1J, GB2J, GE, GL, GT;
    rsrc_t PK, PJ;                              // ROWP: per-row partials of layers k and j
    uint32_t rb1k, rb1j, rb2j, rthe, rb3j, rss2; // ROWP: row-table offsets
  };
  const uint32_t mbytes = (uint32_t)(ml * 4), ldo4 = (uint32_t)(ldo * 4);
  auto tview = [&](int t, int k) -> rsrc_t {
    const float* p = tptr(t, k);
    return urs(p, p ? mbytes : 0u);
  };
  auto res2 = [&](int j) -> R2 {
    R2 o;
    o.P = urs(a.P + j * ml, mbytes);
    o.T = urs(a.T + j * ml, mbytes);
    // E0 / L0 share the outputs' row stride (host: dladmm_capi.hip make_bwd_plan)
    o.E = kAE ? urs(j >= 1 ? a.E + (j - 1) * ml : a.E0, mbytes) : none;
    o.L = urs(j >= 1 ? a.L + (j - 1) * ml : a.L0, mbytes);
    if constexpr (kV1) {
      const bool bk3 = j + 1 < K;   // the prologue (j = K - 1) has no BK3
      o.B1K = bk3 ? tview(RT_B1, j + 1) : none;
      o.GB1K = bk3 ? tview(RT_GB1, j + 1) : none;
      o.B1J = tview(RT_B1, j);
      o.B2J = tview(RT_B2, j);
      o.GB1J = tview(RT_GB1, j);
      o.GB2J = tview(RT_GB2, j);
    }
    if constexpr (COT) {
      o.GE = tview(RT_GE, j);
      o.GL = tview(RT_GL, j);
      o.GT = tview(RT_GT, j + 1);
    }
    if constexpr (ROWP) {
      const bool bk3 = j + 1 < K;
      o.PK = bk3 ? rpart(j + 1) : none;
      o.PJ = rpart(j);
      o.rb1k = rbase(bk3 ? j + 1 : j, DLADMM_P_BETA1);
      o.rb1j = rbase(j, DLADMM_P_BETA1);
      o.rb2j = rbase(j, DLADMM_P_BETA2);
      o.rthe = rbase(j, DLADMM_P_THETA_E);
      o.rb3j = rbase(j, DLADMM_P_BETA3);
      o.rss2 = rbase(j, DLADMM_P_SS2);
    }
    return o;
  };
  auto res2_last = [&]() -> R2 {
    R2 o;
    o.P = mkrsrc(a.T, mbytes);
    o.L = urs(a.L0, mbytes);  // Var_0 = L0 + beta1_0 T_0 (E0 / L0: the outputs' row stride)
    o.E = o.T = none;
    o.B1J = o.B2J = o.GB1J = o.GB2J = o.GE = o.GL = o.GT = none;
    o.B1K = kV1 ? tview(RT_B1, 0) : none;
    o.GB1K = kV1 ? tview(RT_GB1, 0) : none;
    if constexpr (ROWP) {
      o.PK = rpart(0);
      o.PJ = none;
      o.rb1k = o.rb1j = o.rb2j = o.rthe = o.rb3j = o.rss2 = rbase(0, DLADMM_P_BETA1);
    }
    return o;
  };
  const rsrc_t rx = mkrsrc(a.X, (uint32_t)(m * a.ldx * 4));
  // Z_k and (GZ) its cotangent, same row stride (host: ld_g = ldo); ROWP: theta_z's row-table
  // offset and the layer's per-row partials
  struct R1 { rsrc_t z, gz, pk; uint32_t rthz; };
  auto rz = [&](int k) -> R1 {
    R1 o;
    o.z = urs(a.Z + k * zl, (uint32_t)(zl * 4));
    if constexpr (ROWP) {
      o.pk = rpart(k);
      o.rthz = rbase(k, DLADMM_P_THETA_Z);
    }
    if constexpr (GZ) {
      const float* gp = tptr(RT_GZ, k);
      o.gz = urs(gp, gp ? (uint32_t)(zl * 4) : 0u);
    } else {
      o.gz = o.z;
    }
    return o;
  };
  auto rgu = [&](int k) { return urs(a.GU + k * a.gus, (uint32_t)(NP * a.ldw * 4)); };
  // Var_j (rows 0..) and the adjoint of E_{j-1} (rows aeo / 4 / ldw ..) of layer j, plus the
  // next layer's block, which holds the adjoint of E_j that BK1(j) reads
  auto rvar = [&](int j) {
    return urs(a.VAR + j * a.vas, (uint32_t)((j + 1 < K ? 2 : 1) * a.vas * 4));
  };

  // uniform row offsets: loads of the pair being fetched, stores of the rows being finished
  SWalk wZ{0u, ldo4}, wPT{0u, ldo4}, wX{0u, (uint32_t)(a.ldx * 4)};
  const uint32_t ldw4 = (uint32_t)(a.ldw * 4);
  const uint32_t aeo = (uint32_t)(a.aer * a.ldw * 4);  // byte offset of the adjoint-of-E rows
  const uint32_t vas4 = (uint32_t)(a.vas * 4);
  SWalk wG{0u, ldw4}, wV{0u, ldw4}, wA{0u, ldw4}, wB{0u, ldo4};
  // ROWP: row-table loads (G1' / G2' operand rows) and per-row partial stores (G1' / G2' rows)
  SWalk wR1{0u, 4u}, wR2{0u, 4u}, wP1{0u, ldp4}, wP2{0u, ldp4};
  // per-row partial of one element row: the wave's 16 columns summed (the per-layer kernels'
  // col16_sum), stored by lanes l & 15 == 0
  auto pstore = [&](rsrc_t r, uint32_t soff, int row, int nrows, float v) {
    (void)row; (void)nrows;
    bstore_s(r, vpr, soff, row16_sum(v));
  };
  auto ld = [](rsrc_t r, uint32_t voff, uint32_t soff) -> float {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff,
                                                                         REV_LOAD_AUX));
  };
  auto pre1 = [&](const R1& r, int pair, int h, int rr) {
    const int st = set1(pair);
    if constexpr (REV_ABL & 8) { pz[st][h][rr] = 0.5f; return; }
    pz[st][h][rr] = ld(r.z, vo, wZ.at(rr));
    if constexpr (GZ) pg[st][h][rr] = ld(r.gz, vo, wZ.at(rr));
    if constexpr (ROWP) pt[st][h][rr] = ld(rrow, vr, r.rthz + wR1.at(rr));
    if (rr == 3) {
      wZ.next();
      if constexpr (ROWP) wR1.next();
    }
  };
  // G2' operands, one block ahead: slot rr <- row rr of block `blk` (rv: this pass's Var view,
  // whose next-layer block holds the incoming adjoint of E)
  auto pre2 = [&](const R2& o, rsrc_t rv, int blk, int rr) {
    auto& pw = pvs_all[set2(blk)];
    pw[rr][S_AL] = als[al_at(blk, rr)];
    if constexpr (REV_ABL & 32) {
      pw[rr][S_P] = 0.5f; pw[rr][S_L] = 0.125f; pw[rr][S_T] = 1.f; pw[rr][S_X] = 0.25f;
      return;
    }
    const uint32_t so = wPT.at(rr);
    // REV_ABL 4096 / 8192 / 16384 (timing only): X / P / the adjoint of E as ONE dwordx4 per
    // block (row 0's slot, fragment order) instead of a dword per row
    auto ld4 = [&](rsrc_t r, uint32_t soff, int S) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(lane * 16), (int)soff, REV_LOAD_AUX);
#pragma unroll
      for (int q = 0; q < 4; ++q) pw[q][S] = __builtin_bit_cast(float, v[q]);
    };
    if constexpr (REV_ABL & 8192) { if (rr == 0) ld4(o.P, so, S_P); }
    else pw[rr][S_P] = ld((REV_ABL & 512) ? none : o.P, vo, so);
    pw[rr][S_L] = ld((REV_ABL & 2048) ? none : o.L, vo, so);
    if constexpr (REV_ABL & 4096) { if (rr == 0) ld4(rx, wX.at(0), S_X); }
    else pw[rr][S_X] = ld((REV_ABL & 256) ? none : rx, vx, wX.at(rr));
    if constexpr (kAE) {
      pw[rr][S_E] = ld((REV_ABL & 1024) ? none : o.E, vo, so);
      if constexpr (REV_ABL & 16384) { if (rr == 0) ld4(rv, wA.at(0), S_AE); }
      else pw[rr][S_AE] = ld((REV_ABL & 128) ? none : rv, vw, wA.at(rr));
    }
    if constexpr (kV1) {
      pw[rr][S_B1K] = ld(o.B1K, vo, so);
      pw[rr][S_B1J] = ld(o.B1J, vo, so);
      pw[rr][S_B2J] = ld(o.B2J, vo, so);
      pw[rr][S_GB1] = ld(o.GB1K, vo, so);
    }
    if constexpr (ROWP) {
      const uint32_t rs = wR2.at(rr);
      pw[rr][S_RB1K] = ld(rrow, vr, o.rb1k + rs);
      pw[rr][S_RB1J] = ld(rrow, vr, o.rb1j + rs);
      pw[rr][S_RB2J] = ld(rrow, vr, o.rb2j + rs);
      pw[rr][S_RTHE] = ld(rrow, vr, o.rthe + rs);
      if constexpr (kAE) {
        pw[rr][S_RB3J] = ld(rrow, vr, o.rb3j + rs);
        pw[rr][S_RSS2J] = ld(rrow, vr, o.rss2 + rs);
      }
    }
    if constexpr (COT) {
      pw[rr][S_GE] = ld(o.GE, vo, so);
      pw[rr][S_GL] = ld(o.GL, vo, so);
      pw[rr][S_GT] = ld(o.GT, vo, so);
    }
    if (rr == 3) {
      wPT.next(); wX.next(); wA.next();
      if constexpr (ROWP) wR2.next();
    }
  };
  auto reset2 = [&]() {
    wPT.reset();
    wX.reset();
    wR2.reset();
    wA.cur = __builtin_amdgcn_readfirstlane(vas4 + aeo);
    asm volatile("" : "+s"(wA.cur));
  };

  // partial of (layer, slot): one fixed-order sum per wave, written by lane 0
  auto flush = [&](int layer, int slot, float v) {
    if constexpr (!kSC) return;  // V1: no scalar parameters; V2 / V3: per-row partials
    const float s = wave_sum(v);
    if (lane == 0) a.part[((int64_t)layer * DLADMM_NSCALAR + slot) * a.ncg + cg] = s;
  };
  auto flush_bk1 = [&](int j) {
    flush(j, DLADMM_P_BETA3, ps[0]);
    if constexpr (EMODE == EM_VVAR) {
      flush(j, DLADMM_P_BETA2, ps[1]);
      flush(j, DLADMM_P_THETA_E, ps[2]);
      flush(j, DLADMM_P_SS2, ps[3]);
    } else if constexpr (EMODE == EM_LASSO) {
      flush(j, DLADMM_P_SS2, ps[3]);
      flush(j, DLADMM_P_SS2B, ps[4]);
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) ps[i] = 0.f;
  };

  // ---------------------------------------------------------------- per-row epilogues
  // BK2 of layer k, block b row r (dladmm_backward.hip phase 5): q = R = A^T gP_k, pz = Z_k
  auto epi1_row = [&](const LP1& P1, const R1& rzk, rsrc_t rg, int b, int h, int r,
                      const f32x4& q) {
    if constexpr (REV_ABL & 4) { AZ[b][r] = q[r]; pin_agpr(AZ[b][r]); return; }
    const int st = set1(b / 2);
    const float zk = pz[st][h][r];
    float cth = P1.c;
    if constexpr (ROWP) {
      const float th = pt[st][h][r];
      cth = th >= 0.f ? 0.f : -2.0f * th;
    }
    float gZt = (GZ ? AZ[b][r] + pg[st][h][r] : AZ[b][r]) + q[r];
    // + d/dZ_k of cz_k sum|Z_k|: cz_k sgn(Z_k) is exact, so the fma is phase 5's mul + add
    const float sg = (zk > 0.f ? 1.f : 0.f) - (zk < 0.f ? 1.f : 0.f);
    gZt = __builtin_fmaf(P1.cz, sg, gZt);
    // S'(U) = [U - th > 0] + [-U - th > 0] in {0, 1, 2}, from Z_k = S(U, th); gZt * S' as a
    // sum of selected gZt (exact), d/dth = [-U - th > 0] - [U - th > 0]
    const float ga = zk > -cth ? gZt : 0.f, gb = zk < cth ? gZt : 0.f;
    const float gU = ga + gb;
    if constexpr (ROWP) {
      pstore(rzk.pk, pso(DLADMM_P_THETA_Z) + wP1.at(r), 16 * b + 4 * g + r, a.n, gb - ga);
    } else {
      psz += gb - ga;
      asm volatile("" : "+v"(psz));
    }
    AZ[b][r] = gU;  // adjoint of Z_{k-1}
    pin_agpr(AZ[b][r]);
    if constexpr (!(REV_ABL & 16)) bstore_s(rg, vw, wG.at(r), gU);
    if (r == 3) {
      wG.next();
      if constexpr (ROWP) wP1.next();
    }
  };
  // BK3 of layer k, then (MODE 0) BK1 of layer k - 1, block b row r (phase 6); q = gVar =
  // M_k^T gU_k.  MODE 1: BK3 of layer 0 alone (pv[r][S_P] = T_0).  MODE 2: the prologue, BK1 of
  // layer K-1 with zero incoming adjoints (q = 0).  Operands: pv[r] (block b's row r); o: the
  // pass's views (V1's beta gradients).  Every mode issues ST2 stores (dropped ones included) so
  // the ring barriers' counts hold.
  auto epi2_row = [&](auto MODE_, const LP2& P, const R2& o, rsrc_t rv, int b, int r,
                      const f32x4& q) {
    constexpr int MODE = decltype(MODE_)::value;
    const float gVar = q[r];
    if constexpr ((REV_ABL & 2) && MODE != 2) { GP[b][r] = gVar; pin_agpr(GP[b][r]); return; }
    auto& pv = pvs_all[set2(b)];
    const int row = 16 * b + 4 * g + r;  // this lane's row (ROWP partials)
    // pv slot S of row r, or `dflt` for a slot this instantiation does not have
    auto pvs = [&](auto S_, float dflt) -> float {
      constexpr int S = decltype(S_)::value;
      if constexpr (S < NS) return pv[r][S];
      else return dflt;
    };
    using S_B1K_t = std::integral_constant<int, kV1 ? S_B1K : ROWP ? S_RB1K : NS>;
    const float b1k = pvs(S_B1K_t{}, P.b1k);
    if constexpr (MODE == 1) {
      if constexpr (kV1) {
        // beta1_0's gradient: BK1(0)'s term (pv) + gVar T_0
        bstore_s(o.GB1K, vo, wB.at(r), pv[r][S_GB1] + gVar * pv[r][S_P]);
        bstore_s(none, vw, wV.at(r), 0.f);
        bstore_s(none, vw, wV.at(r), 0.f);
      } else if constexpr (ROWP) {
        // beta1_0's per-row partial: gVar T_0; the other slot stores keep the VM count
        pstore(o.PK, pso(DLADMM_P_BETA1) + wP2.at(r), row, m, gVar * pv[r][S_P]);
#pragma unroll
        for (int i = 1; i < NRS; ++i) bstore_s(none, vw, wV.at(r), 0.f);
      } else {
        psb1 += gVar * pv[r][S_P];
        asm volatile("" : "+v"(psb1));
      }
      // Var_0 = L0 + beta1_0 T_0, the forward's prologue expression (pv: T_0 in the P slot, L0)
      bstore_s(rv, vw, wV.at(r), pv[r][S_L] + b1k * pv[r][S_P]);
      if constexpr (kAE) bstore_s(none, vw, wV.at(r) + aeo, 0.f);  // keeps the row's VM count
      if (r == 3) {
        wV.next(); wB.next();
        if constexpr (ROWP) wP2.next();
      }
      return;
    } else {
      using S_B1J_t = std::integral_constant<int, kV1 ? S_B1J : ROWP ? S_RB1J : NS>;
      using S_B2J_t = std::integral_constant<int, kV1 ? S_B2J : ROWP ? S_RB2J : NS>;
      using S_B3J_t = std::integral_constant<int, (ROWP && kAE) ? S_RB3J : NS>;
      using S_SS2_t = std::integral_constant<int, (ROWP && kAE) ? S_RSS2J : NS>;
      using S_THE_t = std::integral_constant<int, ROWP ? S_RTHE : NS>;
      const float b2p = pvs(S_B2J_t{}, P.b2);
      const float b3p = pvs(S_B3J_t{}, P.b3);
      const float ss2p = pvs(S_SS2_t{}, P.ss2);
      const float thep = pvs(S_THE_t{}, P.the);
      using S_AE_t = std::integral_constant<int, kAE ? S_AE : NS>;
      using S_GE_t = std::integral_constant<int, COT ? S_GE : NS>;
      using S_GL_t = std::integral_constant<int, COT ? S_GL : NS>;
      using S_GT_t = std::integral_constant<int, COT ? S_GT : NS>;
      const float aLin = pv[r][S_AL] + gVar;  // complete adjoint of L_{k-1} (upstream aside)
      const float aTin = b1k * gVar;          // adjoint of T_k (main_syn_l1l1_scalar.py:117)
      const float aL = COT ? aLin + pvs(S_GL_t{}, 0.f) : aLin;
      const float aT = COT ? aTin + pvs(S_GT_t{}, 0.f) : aTin;
      // incoming adjoint of E_{k-1}: zero in the prologue (the buffer is not yet written)
      const float aE0 = MODE == 0 ? pvs(S_AE_t{}, 0.f) : 0.f;
      const float aE = COT ? aE0 + pvs(S_GE_t{}, 0.f) : aE0;
      const float Pv = pv[r][S_P], lp = pv[r][S_L], x = pv[r][S_X];
      const float b1 = pvs(S_B1J_t{}, P.b1);
      float gP, gEp = 0.f, gLp, t;
      (void)gEp;
      float p3 = 0.f, p2 = 0.f, pe = 0.f, ps2 = 0.f, ps2b = 0.f;
      if constexpr (EMODE == EM_V1) {
        const float b2 = b2p;
        const float u = (x - Pv) - b2 * lp;               // main_lena.py:87
        // E_{k-1} as the forward formed it (scalar theta: the clamp form; common.h)
        const float e = ROWP ? shrink(u, thep) : shrink_u(u, shrink_params(thep));
        t = (Pv + e) - x;                                 // T_k
        const float gTn = aT + b1 * aL;                   // L_{k-1} = L_{k-2} + b1 T_k (:89)
        p3 = aL * t;
        const float gEt = aE + gTn;
        const float ga = (u - thep) > 0.0f ? gEt : 0.f;
        const float gb = (-u - thep) > 0.0f ? gEt : 0.f;
        const float gEh = ga + gb;
        pe = gb - ga;                                     // V2's per-row theta_e
        gP = gTn - gEh;
        p2 = -gEh * lp;
        gLp = aL - b2 * gEh;
      } else if constexpr (EMODE == EM_VVAR) {
        const float ep = pv[r][S_E];
        const float r0 = (Pv + ep) - x;
        const float vv = lp + b2p * r0;                   // main_syn_l1l1_scalar.py:114
        const float eh = ep - ss2p * vv;                  // :115
        const float e = ROWP ? shrink(eh, thep) : shrink_u(eh, shrink_params(thep));
        t = (Pv + e) - x;                                 // T_k
        const float gTn = aT + b3p * aL;
        p3 = aL * t;
        const float gEt = aE + gTn;
        // shrink' = [eh - th > 0] + [-eh - th > 0]: gEt times it as a sum of selected gEt
        const float ga = (eh - thep) > 0.0f ? gEt : 0.f;
        const float gb = (-eh - thep) > 0.0f ? gEt : 0.f;
        const float gEh = ga + gb;
        pe = gb - ga;
        const float gVV = -ss2p * gEh;
        ps2 = -gEh * vv;
        gLp = aL + gVV;
        p2 = gVV * r0;
        gP = gTn + b2p * gVV;
        gEp = gEh + b2p * gVV;
      } else {
        const float e = P.ss2 * (x - Pv) - P.ss2b * lp;   // main_syn_lasso_scalar.py:102-103
        t = (Pv + e) - x;
        const float gTn = aT + P.b3 * aL;
        p3 = aL * t;
        const float gEt = aE + gTn;
        ps2 = gEt * (x - Pv);
        gP = gTn - P.ss2 * gEt;
        ps2b = -gEt * lp;
        gLp = aL - P.ss2b * gEt;
      }
      {  // d/dP of cf * fit (fit = sum|X - P|, torch sgn(0) = 0, or 0.5 sum (X - P)^2)
        const float res = x - Pv;
        const float sg = (res > 0.f ? 1.f : 0.f) - (res < 0.f ? 1.f : 0.f);
        // uniform select by bit mask (a per-row branch here splits the unrolled body)
        const float dfit = __builtin_bit_cast(
            float, (lqm & __builtin_bit_cast(uint32_t, res)) | (~lqm & __builtin_bit_cast(uint32_t, sg)));
        gP = gP - P.cf * dfit;
      }
      if constexpr (kV1) {
        // beta1_k's gradient = BK1(k)'s term + gVar T_k (the per-layer order); beta1_{k-1} gets
        // BK1(k-1)'s term aL T_k now and BK3(k-1)'s next pass; beta2_{k-1} complete
        bstore_s(MODE == 0 ? o.GB1K : none, vo, wB.at(r), pv[r][S_GB1] + gVar * t);
        bstore_s(o.GB1J, vo, wB.at(r), p3);
        bstore_s(o.GB2J, vo, wB.at(r), p2);
      } else if constexpr (ROWP) {
        // per-row partials: beta1 of layer k (BK3), then BK1(k-1)'s slots, as the per-layer
        // kernels group them (BK1's beta3 slot carries V2's beta1 L term)
        const uint32_t so2 = wP2.at(r);
        if constexpr (MODE == 0) pstore(o.PK, pso(DLADMM_P_BETA1) + so2, row, m, gVar * t);
        else bstore_s(none, vw, so2, 0.f);
        pstore(o.PJ, pso(DLADMM_P_BETA3) + so2, row, m, p3);
        pstore(o.PJ, pso(DLADMM_P_BETA2) + so2, row, m, p2);
        pstore(o.PJ, pso(DLADMM_P_THETA_E) + so2, row, m, pe);
        if constexpr (kAE) pstore(o.PJ, pso(DLADMM_P_SS2) + so2, row, m, ps2);
      } else {
        if constexpr (MODE == 0) {
          psb1 += gVar * t;  // beta1 of layer k: gVar * T_k
          asm volatile("" : "+v"(psb1));
        }
        ps[0] += p3; ps[1] += p2; ps[2] += pe; ps[3] += ps2; ps[4] += ps2b;
        asm volatile("" : "+v"(ps[0]), "+v"(ps[3]));
        if constexpr (EMODE == EM_VVAR) asm volatile("" : "+v"(ps[1]), "+v"(ps[2]));
        else asm volatile("" : "+v"(ps[4]));
      }
      GP[b][r] = gP;
      pin_agpr(GP[b][r]);
      als[al_at(b, r)] = gLp;
      // Var of layer k (BK3's): L_{k-1} + beta1_k T_k from the values just recomputed, the
      // forward's own expression (l = L_{k-2} + c T_k, then + beta1_k T_k; c = the L-update
      // coefficient), so T_{k-1} is never loaded.  The prologue's (layer K) is dropped: its
      // store runs past rv's last layer block.
      const float lcoef = EMODE == EM_V1 ? b1 : (EMODE == EM_VVAR ? b3p : P.b3);
      const float lk = lp + lcoef * t;
      const float vark = lk + b1k * t;
      if constexpr (!(REV_ABL & 64)) {
        bstore_s(rv, vw, vas4 + wV.at(r), vark);
        if constexpr (kAE) bstore_s((REV_ABL & 128) ? none : rv, vw, wV.at(r) + aeo, gEp);  // adjoint of E_{k-2}
      } else {
        asm volatile("" ::"v"(gEp), "v"(vark));
      }
      if (r == 3) {
        wV.next(); wB.next();
        if constexpr (ROWP) wP2.next();
      }
    }
  };

  // ---------------------------------------------------------------- one MFMA step
  f32x4 fr[4];
  auto step_head = [&](auto S_, int gi, auto WIN_) {
    constexpr int s = decltype(S_)::value;
    constexpr int WIN = decltype(WIN_)::value;
    constexpr int fi = 2 * s, fc = fi % CF, ch = fi / CF;
    if constexpr (fc + 2 < CF) {
      fr[(fi + 2) % 4] = frag(cur, fc + 2);
      fr[(fi + 3) % 4] = frag(cur, fc + 3);
    } else {
      if constexpr (WIN > 0) ring_barrier_cnt<WIN>();
      else ring_barrier();
      issue(chunk_src(gi, ch + F::SLOTS - 1), slot_add(cur, F::SLOTS - 1));
      const int nx = slot_add(cur, 1);
      fr[(fi + 2) % 4] = frag(nx, 0);
      fr[(fi + 3) % 4] = frag(nx, 1);
    }
  };
  auto step_tail = [&](auto S_) {
    constexpr int s = decltype(S_)::value;
    constexpr int fc = (2 * s) % CF;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (fc + 2 >= CF) cur = slot_add(cur, 1);
  };

  f32x4 qa = {0.f, 0.f, 0.f, 0.f}, qb = {0.f, 0.f, 0.f, 0.f};  // pending pair accumulators
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

  // ---------------------------------------------------------------- prologue: BK1(K-1)
  // On the saved P_{K-1} with zero incoming adjoints; no product, so the operand loads of
  // pair p + 1 are issued behind each row of pair p.
  {
    const LP2 P = lp2(K, K - 1);
    const R2 o = res2(K - 1);
    const rsrc_t rv = rvar(K - 1);
    reset2();
    wV.reset();
    wB.reset();
    wP2.reset();
    constexpr int AHEAD = DEEP ? 2 : 1;   // blocks the operand loads run ahead
    static_for<4 * AHEAD>([&](auto R_) {
      constexpr int q = decltype(R_)::value;
      pre2(o, rv, q / 4, q % 4);
    });
    static_for<MB / 2>([&](auto P_) {
      constexpr int p = decltype(P_)::value;
      static_for<8>([&](auto I_) {
        constexpr int i = decltype(I_)::value;
        constexpr int h = i / 4, r = i % 4;
        if constexpr (!(REV_ABL & 1))
        epi2_row(std::integral_constant<int, 2>{}, P, o, rv, 2 * p + h, r, zero4);
        if constexpr (2 * p + h + AHEAD < MB) pre2(o, rv, 2 * p + h + AHEAD, r);
      });
    });
    flush_bk1(K - 1);
  }
  ring_barrier();  // the primed chunks (and every prologue load / store) are complete
  fr[0] = frag(0, 0);
  fr[1] = frag(0, 1);

  // ---------------------------------------------------------------- the product passes
  // G1'(k): A^T gP_k over blocks (2p, 2p+1), contraction jb = 0..MB-1.  Pair 0 runs the rows of
  // G2'(k+1)'s last pair (Pp, op, rvp; none in the first pass), then flushes layer k+1's beta1
  // and layer k's BK1 partials.
  auto g1_pass = [&](auto FIRST_, int k, const LP1& P1, const R1& rzk, rsrc_t rg, const LP2& Pp,
                     const R2& op, rsrc_t rvp) {
    constexpr bool FIRST = decltype(FIRST_)::value;
    const int gi = 2 * (K - 1 - k);
    wZ.reset();
    wG.reset();
    wR1.reset();
    wP1.reset();
    static_for<NB / 2>([&](auto P_) {
      constexpr int p = decltype(P_)::value;
      f32x4 ca = zero4, cb = zero4;
      static_for<MB>([&](auto J_) {
        constexpr int jb = decltype(J_)::value;
        constexpr int s = p * MB + jb;
        step_head(std::integral_constant<int, s>{}, gi,
                  std::integral_constant<int, Win::template g1<s, FIRST>()>{});
        static_for<8>([&](auto I_) {
          constexpr int i = decltype(I_)::value;
          constexpr int h = i / 4, r = i % 4;
          if constexpr (rev_rows_at(jb, MB, i)) {
            if constexpr (p == 0) {
              if constexpr (!FIRST) {
                epi2_row(std::integral_constant<int, 0>{}, Pp, op, rvp, MB - 2 + h, r,
                         h ? qb : qa);
                // not DEEP: the last block's row r (DEEP: loaded in the G2' pass)
                if constexpr (h == 0 && !DEEP) pre2(op, rvp, MB - 1, r);
                if constexpr (i == 7) {
                  flush(k + 1, DLADMM_P_BETA1, psb1);
                  psb1 = 0.f;
                  flush_bk1(k);
                }
              }
            } else {
              epi1_row(P1, rzk, rg, 2 * p - 2 + h, h, r, h ? qb : qa);
              // this row's Z_k slot, for pair p (DEEP: p + 1)
              if constexpr (!DEEP) pre1(rzk, p, h, r);
              else if constexpr (p + 1 < NB / 2) pre1(rzk, p + 1, h, r);
            }
          }
        });
        if constexpr (p == 0) {
          static_for<Win::NP1>([&](auto PT_) {  // pair 0 (DEEP: and 1), one row per part
            constexpr int q = decltype(PT_)::value;
            if constexpr (rev_part_step(q, MB, Win::NP1) == jb) pre1(rzk, q / 8, (q / 4) % 2, q % 4);
          });
        }
        const f32x4 wa = fr[(2 * s) % 4], wb = fr[(2 * s + 1) % 4];
        ca = mfma4(wa.x, GP[jb][0], ca);
        cb = mfma4(wb.x, GP[jb][0], cb);
        ca = mfma4(wa.y, GP[jb][1], ca);
        cb = mfma4(wb.y, GP[jb][1], cb);
        ca = mfma4(wa.z, GP[jb][2], ca);
        cb = mfma4(wb.z, GP[jb][2], cb);
        ca = mfma4(wa.w, GP[jb][3], ca);
        cb = mfma4(wb.w, GP[jb][3], cb);
        step_tail(std::integral_constant<int, s>{});
      });
      qa = ca;
      qb = cb;
    });
  };
  // G2'(k): M_k^T gU_k over blocks (2p, 2p+1), contraction kb = 0..NB-1.  Pair 0 runs the rows
  // of G1'(k)'s last pair and then flushes layer k's theta_z partial; pair p > 0 those of pair
  // p - 1 (LAST: BK3 of layer 0 alone).
  auto g2_pass = [&](auto LAST_, int k, const LP2& P, const R2& o, rsrc_t rv, const LP1& P1,
                     const R1& rzk, rsrc_t rg) {
    constexpr bool LAST = decltype(LAST_)::value;
    const int gi = 2 * (K - 1 - k) + 1;
    wV.reset();
    wB.reset();
    wP2.reset();
    reset2();
    static_for<MB / 2>([&](auto P_) {
      constexpr int p = decltype(P_)::value;
      f32x4 ca = zero4, cb = zero4;
      static_for<NB>([&](auto K_) {
        constexpr int kb = decltype(K_)::value;
        constexpr int s = p * NB + kb;
        step_head(std::integral_constant<int, s>{}, gi,
                  std::integral_constant<int, Win::template g2<s>()>{});
        static_for<8>([&](auto I_) {
          constexpr int i = decltype(I_)::value;
          constexpr int h = i / 4, r = i % 4;
          if constexpr (rev_rows_at(kb, NB, i)) {
            if constexpr (p == 0) {
              epi1_row(P1, rzk, rg, NB - 2 + h, h, r, h ? qb : qa);
              if constexpr (i == 7) {
                if constexpr (!kV1) flush(k, DLADMM_P_THETA_Z, psz);
                psz = 0.f;
              }
            } else {
              epi2_row(std::integral_constant<int, LAST ? 1 : 0>{}, P, o, rv, 2 * p - 2 + h, r,
                       h ? qb : qa);
              // row r of block 2p - 1 + h (DEEP: 2p + h)
              pre2(o, rv, DEEP ? 2 * p + h : 2 * p - 1 + h, r);
            }
          }
        });
        if constexpr (p == 0) {
          static_for<Win::NP2>([&](auto PT_) {  // block 0's (DEEP: and 1's) rows, one per part
            constexpr int q = decltype(PT_)::value;
            if constexpr (rev_part_step(q, NB, Win::NP2) == kb) pre2(o, rv, q / 4, q % 4);
          });
        }
        const f32x4 wa = fr[(2 * s) % 4], wb = fr[(2 * s + 1) % 4];
        ca = mfma4(wa.x, AZ[kb][0], ca);
        cb = mfma4(wb.x, AZ[kb][0], cb);
        ca = mfma4(wa.y, AZ[kb][1], ca);
        cb = mfma4(wb.y, AZ[kb][1], cb);
        ca = mfma4(wa.z, AZ[kb][2], ca);
        cb = mfma4(wb.z, AZ[kb][2], cb);
        ca = mfma4(wa.w, AZ[kb][3], ca);
        cb = mfma4(wb.w, AZ[kb][3], cb);
        step_tail(std::integral_constant<int, s>{});
      });
      qa = ca;
      qb = cb;
    });
  };

  // ---------------------------------------------------------------- K layers, last to first
  LP1 P1 = lp1(K - 1);
  R1 Rk = rz(K - 1);
  g1_pass(std::true_type{}, K - 1, P1, Rk, rgu(K - 1), lp2(K, K - 1), res2_last(), none);
  for (int k = K - 1; k >= 1; --k) {
    const LP2 P = lp2(k, k - 1);
    const R2 o = res2(k - 1);
    const rsrc_t rv = rvar(k - 1);
    g2_pass(std::false_type{}, k, P, o, rv, P1, Rk, rgu(k));
    P1 = lp1(k - 1);
    Rk = rz(k - 1);
    g1_pass(std::false_type{}, k - 1, P1, Rk, rgu(k - 1), P, o, rv);
  }
  const LP2 P0 = lp2(0, -1);
  const R2 o0 = res2_last();
  const rsrc_t rv0 = rvar(0);  // the last pass stores Var_0
  g2_pass(std::true_type{}, 0, P0, o0, rv0, P1, Rk, rgu(0));
  // rows of layer 0's last G2' pair
  static_for<8>([&](auto I_) {
    constexpr int i = decltype(I_)::value;
    constexpr int h = i / 4, r = i % 4;
    epi2_row(std::integral_constant<int, 1>{}, P0, o0, rv0, MB - 2 + h, r, h ? qb : qa);
    if constexpr (h == 0 && !DEEP) pre2(o0, rv0, MB - 1, r);
  });
  flush(0, DLADMM_P_BETA1, psb1);
  // drain: the ring's last LDS-DMA must land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int MP, int NP, int EM, bool GZ, bool COT, bool ROWP>
void launch_rev1(const RevArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((reverse_kernel<MP, NP, EM, GZ, COT, ROWP>), dim3(grid), dim3(256), 0, s, a);
}

// ROWP: per-row parameters (V2 with EM_V1, V3 with EM_VVAR)
template <int MP, int NP, int EM, bool ROWP = false>
hipError_t launch_rev(const RevArgs& a, int grid, hipStream_t s) {
  if (a.has_gz && a.has_cot) launch_rev1<MP, NP, EM, true, true, ROWP>(a, grid, s);
  else if (a.has_gz) launch_rev1<MP, NP, EM, true, false, ROWP>(a, grid, s);
  else if (a.has_cot) launch_rev1<MP, NP, EM, false, true, ROWP>(a, grid, s);
  else launch_rev1<MP, NP, EM, false, false, ROWP>(a, grid, s);
  return hipGetLastError();
}

}  // namespace dladmm
