// dladmm_fused.hip -- MI355X (gfx950 / CDNA4) fused K-layer D-LADMM forward.
//
// Replaces the Python loop of DLADMMNet.forward (main_lena.py:57-98,
// main_syn_l1l1_scalar.py:80-127, main_syn_lasso_scalar.py:65-114 and the other variants
// listed in include/dladmm.h) with ONE persistent-state kernel per forward.
//
// Design (DESIGN.md has the full derivation):
//  * one workgroup = 4 waves = a tile of 64 batch columns; wave w owns columns 16w..16w+15;
//  * the whole per-column state -- Z (n), E, L, X and T/Var (m each) -- stays in registers for
//    all K layers, laid out exactly like the C/D fragment of v_mfma_f32_16x16x4_f32:
//    lane l holds column (l & 15) and feature rows 16*b + 4*(l >> 4) + r, r = 0..3;
//  * with that layout the accumulator of one GEMM IS the B operand of the next: U = W_k*Var
//    lands in Z's layout, P = A*Z lands in E/L/T's layout, and every shrink / AXPY of the
//    reference is lane-local -- no LDS transpose, no HBM round trip for the state;
//  * W_k and A are pre-packed (pack_frags_kernel) into "fragment order" (1 KiB per 16x16
//    fragment = exactly what one wave's lanes need for 4 MFMAs), streamed from L2/MALL by
//    global_load_lds_dwordx4 into a double-buffered LDS ring shared by the 4 waves;
//  * epilogues are deferred by one block so each block's HBM stores overlap the next block's
//    MFMAs instead of being drained by the next ring barrier.
// Elementwise arithmetic keeps the reference's evaluation order and is compiled with
// -ffp-contract=off so every mul/add rounds like the separate torch ops do.

#include "dladmm_common.h"
#include "dladmm_internal.h"

namespace dladmm {

template <int MP, int NP, int EMODE, int PKIND>
struct Fused {
  static constexpr int MB = MP / 16;
  static constexpr int NB = NP / 16;
  static constexpr int GF = MB * NB;                // fragments per GEMM
#ifndef DLADMM_CHUNK
#define DLADMM_CHUNK 16
#endif
  static constexpr int CF = GF < DLADMM_CHUNK ? GF : DLADMM_CHUNK;  // fragments per ring chunk
  static constexpr int NCH = GF / CF;               // chunks per GEMM
  static constexpr int TAB = 6 * MP + NP;           // per-row param table (floats)
  static constexpr int RING_F4 = 2 * CF * 64;
  static constexpr int TAB_F4 = (PKIND == PK_ROW) ? (3 * TAB) / 4 : 0;  // 3 layer buffers
  static constexpr int X_F4 = kWaves * MB * 64;  // the tile's X, resident in LDS (fragment order)
  static_assert(MP % 16 == 0 && NP % 16 == 0, "padded dims must be multiples of 16");
  static_assert(GF % CF == 0, "chunking");
  static_assert(TAB % 4 == 0, "table alignment");
};

template <int MP, int NP, int EMODE, int PKIND>
__global__ __launch_bounds__(256, 1) void fused_kernel(const FusedArgs a) {
  using F = Fused<MP, NP, EMODE, PKIND>;
  constexpr int MB = F::MB, NB = F::NB, CF = F::CF, NCH = F::NCH, TAB = F::TAB;
  constexpr int D = 2;         // fragments read ahead of the MFMAs that consume them
  constexpr int NBUF = D + 1;  // fragment registers in rotation
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

  float Zr[NB][4], Er[MB][4], Lr[MB][4], Vr[MB][4];
  float pb[2][3][4];  // per-element betas (PK_ELEM) of the G2 blocks in flight, by block parity
  float regsum = 0.f, fitsum = 0.f;

  // ---------------------------------------------------------------- ring (LDS-DMA) stream
  int cur = 0;  // slot of the chunk being consumed
  auto issue = [&](const float* src, int slot) {
    // opaque uniform base: stops the compiler from precomputing (and keeping live) the
    // 64-bit per-lane address of every chunk of the stream; the load becomes
    // global_load_lds_dwordx4 voff, s[base] with a loop-invariant 32-bit lane offset
    uint64_t sb = (uint64_t)src;
    asm volatile("" : "+s"(sb));
    const float* base = (const float*)sb;
    f32x4* dst = ring + slot * (CF * 64);
#pragma unroll
    for (int i = 0; i < (CF + 3) / 4; ++i) {
      if constexpr (CF % 4 == 0) {
        glds16(base + (i * 4 + w) * kFrag, lane * 16, dst + (i * 4 + w) * 64);
      } else {
        const int f = i * 4 + w;
        if (f < CF) glds16(base + f * kFrag, lane * 16, dst + f * 64);
      }
    }
  };
  // ring barrier for the chunk about to be consumed, then prefetch the next chunk into the
  // other slot (always a valid source: past the end of the stream it re-reads packed A)
  auto acquire = [&](const float* next_src) {
    ring_barrier();
    issue(next_src, cur ^ 1);
  };
  auto frag = [&](int fc) -> f32x4 { return ring[cur * (CF * 64) + fc * 64 + lane]; };

  // ---------------------------------------------------------------- parameters
  auto row_tab_load = [&](int k, int buf) {  // per-row params of layer k -> tab[buf]
    if constexpr (PKIND == PK_ROW) {
      float* t = tab + buf * TAB;
      const float* src = a.rowp + (int64_t)k * 8 * a.rstride;
      for (int i = tid; i < TAB; i += 256) {
        const int slot = i < 6 * MP ? i / MP : 6;
        const int row = i < 6 * MP ? i % MP : i - 6 * MP;
        const int lim = slot == 6 ? n : m;
        t[i] = row < lim ? src[(int64_t)slot * a.rstride + row] : 0.0f;
      }
    }
  };
  // uniform per-layer scalars (s_load).  k = -1 (prologue) reads layer 0; b1n = beta1 of the
  // layer whose Var the G2 epilogue of layer k produces (k+1, clamped).
  struct LayerP { float b1, b2, b3, ss2, ss2b, the, thz, s1, b1n; };
  auto layer_params = [&](int k) -> LayerP {
    LayerP p{};
    if constexpr (PKIND != PK_ROW) {
      const int kk = k < 0 ? 0 : k;
      const int kn = k < 0 ? 0 : (k + 1 < K ? k + 1 : k);
      cfloat_p sp = (cfloat_p)a.scal + kk * DLADMM_NSCALAR;
      p.b1 = sp[DLADMM_P_BETA1];
      p.b2 = sp[DLADMM_P_BETA2];
      p.b3 = sp[DLADMM_P_BETA3];
      p.ss2 = sp[DLADMM_P_SS2];
      p.ss2b = sp[DLADMM_P_SS2B];
      p.the = sp[DLADMM_P_THETA_E];
      p.thz = sp[DLADMM_P_THETA_Z];
      p.s1 = sp[DLADMM_P_S1];
      p.b1n = ((cfloat_p)a.scal)[kn * DLADMM_NSCALAR + DLADMM_P_BETA1];
    }
    return p;
  };
  // value of param `slot` for (layer k, block b, reg r)
  auto prm = [&](const LayerP& P, int k, int slot, int b, int r) -> float {
    if constexpr (PKIND == PK_ROW) {
      const int off = (slot == DLADMM_P_THETA_Z) ? 6 * MP : slot * MP;
      return tab[(k % 3) * TAB + off + 16 * b + 4 * g + r];
    } else {
      switch (slot) {
        case DLADMM_P_BETA1: return P.b1;
        case DLADMM_P_BETA2: return P.b2;
        case DLADMM_P_BETA3: return P.b3;
        case DLADMM_P_SS2: return P.ss2;
        case DLADMM_P_SS2B: return P.ss2b;
        case DLADMM_P_THETA_E: return P.the;
        case DLADMM_P_THETA_Z: return P.thz;
        default: return P.s1;
      }
    }
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
        Er[b][r] = bload(re, oe + (uint32_t)((16 * b + r) * a.lde0 * 4));
        Lr[b][r] = bload(rl, ol + (uint32_t)((16 * b + r) * a.ldl0 * 4));
        Vr[b][r] = 0.0f;
        pin_agpr(Vr[b][r]);
      }
      xs[(w * MB + b) * 64 + lane] = xv;  // read back only by this wave (no barrier needed)
    }
  }
  row_tab_load(0, 0);
  issue(a.Ap, 0);

  const uint32_t oo = lane_off(a.ldo);                    // output lane offset
  const uint32_t ob = lane_off(a.ldb);                    // per-element beta lane offset
  const uint32_t zbytes = (uint32_t)(n * a.ldo * 4), mbytes = (uint32_t)(m * a.ldo * 4);
  Walk zw{oo, (uint32_t)(a.ldo * 4)}, mw{oo, (uint32_t)(a.ldo * 4)};
  Walk bw{ob, (uint32_t)(a.ldb * 4)};

  // ---------------------------------------------------------------- per-row epilogues
  // Each block's epilogue is cut into its 4 accumulator rows; the rows of block b-1 are spread
  // over the MFMA steps of block b (row r before the MFMAs of step (r * steps) / 4), so the
  // VALU work and HBM stores issue in the MFMA shadow instead of stalling the matrix pipe.
  //
  // G1 block b, row r of layer k: Z = S(Z - s1*(W_k Var), theta_z)  main_lena.py:86 / tied :114
  auto epi1_row = [&](const LayerP& P, rsrc_t rzo, int k, int b, int r, f32x4 c0, f32x4 c1) {
    float u = c0[r] + c1[r];
    if constexpr (PKIND == PK_SCALAR) u = P.s1 * u;  // V5 ss1[k]; exactly 1.0 otherwise
    const float z = shrink(Zr[b][r] - u, prm(P, k, DLADMM_P_THETA_Z, b, r));
    Zr[b][r] = z;
    pin_agpr(Zr[b][r]);
    bstore(rzo, zw.at(r), z);
    // no column mask: padded columns hold exactly zero state (X = Z0 = E0 = L0 = 0)
    regsum += fabsf(z);
    if (r == 3) zw.next();
  };
  // G2 block b, row r of layer k.  Branch-free over k: for the prologue (k = -1) the E/L updates
  // are discarded and T0 = A Z0 + E0 - X (main_lena.py:70) falls out of the same expression;
  // its E/L stores go to 0-record buffers.
  struct OutR { rsrc_t e, l, t; };
  auto epi2_row = [&](const LayerP& P, const OutR& O, int k, int b, int r, f32x4 c0, f32x4 c1,
                      const f32x4& xv) {
    const bool pro = k < 0;
    const int kp = pro ? 0 : k;
    float(&pe)[3][4] = pb[b & 1];
    const float Pv = c0[r] + c1[r];
    const float x = xv[r];
    const uint32_t off = mw.at(r);
    const float l0 = Lr[b][r];
    float e;
    if constexpr (EMODE == EM_V1) {
      // E = S(X - A Z - b2*L, theta_e)                      main_lena.py:87
      const float b2 = (PKIND == PK_ELEM) ? pe[1][r] : prm(P, kp, DLADMM_P_BETA2, b, r);
      e = shrink((x - Pv) - b2 * l0, prm(P, kp, DLADMM_P_THETA_E, b, r));
    } else if constexpr (EMODE == EM_VVAR) {
      // VVar = L + b2*(A Z + E - X); E = S(E - ss2*VVar)    main_syn_l1l1_scalar.py:114-115
      const float vv = l0 + prm(P, kp, DLADMM_P_BETA2, b, r) * ((Pv + Er[b][r]) - x);
      e = shrink(Er[b][r] - prm(P, kp, DLADMM_P_SS2, b, r) * vv,
                 prm(P, kp, DLADMM_P_THETA_E, b, r));
    } else {
      // E = ss2_1*(X - A Z) - ss2_2*L                       main_syn_lasso_scalar.py:102-103
      e = prm(P, kp, DLADMM_P_SS2, b, r) * (x - Pv) - prm(P, kp, DLADMM_P_SS2B, b, r) * l0;
    }
    e = pro ? Er[b][r] : e;
    const float t = (Pv + e) - x;                            // main_lena.py:70 / :88
    const float b3 = (PKIND == PK_ELEM) ? pe[0][r] : prm(P, kp, DLADMM_P_BETA3, b, r);
    const float l = pro ? l0 : l0 + b3 * t;                  // main_lena.py:89 / scalar :118
    Er[b][r] = e;
    Lr[b][r] = l;
    bstore(O.e, off, e);
    bstore(O.l, off, l);
    bstore(O.t, off, t);
    const float res = x - Pv;
    fitsum += fabsf(res) * (lasso ? fabsf(res) : 1.0f);  // |r| or r^2; branch-free
    // Var of the next layer: L + b1*T  (main_lena.py:85); unused after the last layer
    float b1n;
    if constexpr (PKIND == PK_ELEM) b1n = pe[2][r];
    else if constexpr (PKIND == PK_ROW) b1n = prm(P, k + 1, DLADMM_P_BETA1, b, r);
    else b1n = P.b1n;
    Vr[b][r] = l + b1n * t;
    pin_agpr(Vr[b][r]);
    if (r == 3) mw.next();
  };
  // per-wave partial objective of layer k (k < 0: just reset the prologue's sums)
  auto flush_loss = [&](int k) {
    if (lossz && k >= 0) {
      const float rs = wave_sum(regsum), fs = wave_sum(fitsum);
      if (lane == 0) {
        const int gw = blockIdx.x * kWaves + w;
        a.lossp[(int64_t)(2 * k + 0) * a.nwaves + gw] = rs;
        a.lossp[(int64_t)(2 * k + 1) * a.nwaves + gw] = lasso ? 0.5f * fs : fs;
      }
    }
    regsum = 0.f;
    fitsum = 0.f;
  };
  auto prefetch_elem = [&](int k, int b) {  // betas the G2 epilogue of (k, b) will need
    if constexpr (PKIND == PK_ELEM) {
      float(&pe)[3][4] = pb[b & 1];
      const uint32_t eb = (uint32_t)(m * a.ldb * 4);
      const rsrc_t r1 = mkrsrc(k >= 0 ? a.b1e[k] : nullptr, k >= 0 ? eb : 0u);
      const rsrc_t r2 = mkrsrc(k >= 0 ? a.b2e[k] : nullptr, k >= 0 ? eb : 0u);
      const rsrc_t rn = mkrsrc(k + 1 < K ? a.b1e[k + 1] : nullptr, k + 1 < K ? eb : 0u);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t off = bw.at(r);
        pe[0][r] = bload(r1, off);
        pe[1][r] = bload(r2, off);
        pe[2][r] = bload(rn, off);
      }
      bw.next();
    }
  };

  // ---------------------------------------------------------------- the K-layer loop
  // Phase order: G2(-1) [P0 = A Z0], then per layer G1(k) [W_k Var], G2(k) [A Z_k].
  // Every MFMA step: prefetch the fragment D steps ahead from the LDS ring, run the epilogue
  // rows scheduled on this step, issue 4 MFMAs; a sched_barrier pins that order.
  const int64_t wl = (int64_t)F::GF * kFrag;  // floats per packed W_k
  f32x4 q0 = {0.f, 0.f, 0.f, 0.f}, q1 = {0.f, 0.f, 0.f, 0.f};  // pending block accumulators
  f32x4 xpend = {0.f, 0.f, 0.f, 0.f};                           // X rows of the pending G2 block
  f32x4 fr[NBUF];
  for (int k = -1; k < K; ++k) {
    const bool st = a.keep_all || k == K - 1;
    const int ko = a.keep_all ? k : 0;
    const LayerP P = layer_params(k);
    const LayerP Pp = layer_params(k - 1);
    // outputs of layer k (Z, E, L) and T[k+1]; num_records 0 = not stored
    const rsrc_t rzo = mkrsrc(a.Zo + (int64_t)ko * n * a.ldo, st && k >= 0 ? zbytes : 0u);
    const OutR O{mkrsrc(a.Eo + (int64_t)ko * m * a.ldo, st && k >= 0 ? mbytes : 0u),
                 mkrsrc(a.Lo + (int64_t)ko * m * a.ldo, st && k >= 0 ? mbytes : 0u),
                 mkrsrc(a.To ? a.To + (int64_t)(a.keep_all ? k + 1 : 0) * m * a.ldo : nullptr,
                        (a.To && st) ? mbytes : 0u)};
    // outputs of layer k-1 (its last G2 block's epilogue runs inside this layer's G1)
    const bool stp = a.keep_all || k - 1 == K - 1;
    const int kop = a.keep_all ? k - 1 : 0;
    const OutR Op{mkrsrc(a.Eo + (int64_t)kop * m * a.ldo, stp && k - 1 >= 0 ? mbytes : 0u),
                  mkrsrc(a.Lo + (int64_t)kop * m * a.ldo, stp && k - 1 >= 0 ? mbytes : 0u),
                  mkrsrc(a.To ? a.To + (int64_t)(a.keep_all ? k : 0) * m * a.ldo : nullptr,
                         (a.To && stp) ? mbytes : 0u)};
    const float* wk = a.Wp + (int64_t)(k < 0 ? 0 : k) * wl;

    // ---- G1(k): U[b] = sum_jb Wp_k[b][jb] * Var[jb]
    if (k >= 0) {
      zw.cur = oo;
      // layer k+1's row table -> buffer (k+1)%3.  Its previous content (layer k-2) was last
      // read in G1(k-1)'s deferred epilogue, several ring barriers ago; its readers (G2(k)
      // epilogues, layer k+1) all come after G1(k)'s first barrier.
      if (k + 1 < K) row_tab_load(k + 1, (k + 1) % 3);
      static_for<NB>([&](auto B_) {
        constexpr int b = decltype(B_)::value;
        f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
        static_for<MB>([&](auto J_) {
          constexpr int jb = decltype(J_)::value;
          constexpr int fi = b * MB + jb, fc = fi % CF;
          if constexpr (fc == 0) {
            constexpr int ch = fi / CF;
            acquire(ch + 1 < NCH ? wk + (int64_t)(ch + 1) * CF * kFrag : a.Ap);
            static_for<D>([&](auto Dd) {
              constexpr int d = decltype(Dd)::value;
              if constexpr (fc + d < CF) fr[(fi + d) % NBUF] = frag(fc + d);
            });
          }
          if constexpr (fc + D < CF) fr[(fi + D) % NBUF] = frag(fc + D);
          static_for<4>([&](auto R_) {
            constexpr int r = decltype(R_)::value;
            if constexpr ((r * MB) / 4 == jb) {
              if constexpr (b == 0) {  // last G2 block of the previous phase
                if constexpr (r == 0) xpend = xs[(w * MB + MB - 1) * 64 + lane];
                epi2_row(Pp, Op, k - 1, MB - 1, r, q0, q1, xpend);
                if constexpr (r == 3) flush_loss(k - 1);
              } else {
                epi1_row(P, rzo, k, b - 1, r, q0, q1);
              }
            }
          });
          const f32x4 wv = fr[fi % NBUF];
          c0 = mfma4(wv.x, Vr[jb][0], c0);
          c1 = mfma4(wv.y, Vr[jb][1], c1);
          c0 = mfma4(wv.z, Vr[jb][2], c0);
          c1 = mfma4(wv.w, Vr[jb][3], c1);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (fc == CF - 1) cur ^= 1;
        });
        q0 = c0;
        q1 = c1;
      });
    }
    // ---- G2(k): P[b] = sum_kb Ap[b][kb] * Z[kb]
    const float* next_base = (k + 1 < K) ? a.Wp + (int64_t)(k + 1) * wl : a.Ap;
    mw.cur = oo;
    bw.cur = ob;
    static_for<MB>([&](auto B_) {
      constexpr int b = decltype(B_)::value;
      f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
      static_for<NB>([&](auto K_) {
        constexpr int kb = decltype(K_)::value;
        constexpr int fi = b * NB + kb, fc = fi % CF;
        if constexpr (fc == 0) {
          constexpr int ch = fi / CF;
          acquire(ch + 1 < NCH ? a.Ap + (int64_t)(ch + 1) * CF * kFrag : next_base);
          static_for<D>([&](auto Dd) {
            constexpr int d = decltype(Dd)::value;
            if constexpr (fc + d < CF) fr[(fi + d) % NBUF] = frag(fc + d);
          });
        }
        if constexpr (fc + D < CF) fr[(fi + D) % NBUF] = frag(fc + D);
        if constexpr (kb == 0) prefetch_elem(k, b);
        static_for<4>([&](auto R_) {
          constexpr int r = decltype(R_)::value;
          if constexpr ((r * NB) / 4 == kb) {
            if constexpr (b == 0) {  // last G1 block of this layer
              if (k >= 0) epi1_row(P, rzo, k, NB - 1, r, q0, q1);
            } else {
              if constexpr (r == 0) xpend = xs[(w * MB + b - 1) * 64 + lane];
              epi2_row(P, O, k, b - 1, r, q0, q1, xpend);
            }
          }
        });
        const f32x4 wv = fr[fi % NBUF];
        c0 = mfma4(wv.x, Zr[kb][0], c0);
        c1 = mfma4(wv.y, Zr[kb][1], c1);
        c0 = mfma4(wv.z, Zr[kb][2], c0);
        c1 = mfma4(wv.w, Zr[kb][3], c1);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (fc == CF - 1) cur ^= 1;
      });
      q0 = c0;
      q1 = c1;
    });
  }
  {
    const LayerP P = layer_params(K - 1);
    const int ko = a.keep_all ? K - 1 : 0;
    const OutR O{mkrsrc(a.Eo + (int64_t)ko * m * a.ldo, mbytes),
                 mkrsrc(a.Lo + (int64_t)ko * m * a.ldo, mbytes),
                 mkrsrc(a.To ? a.To + (int64_t)(a.keep_all ? K : 0) * m * a.ldo : nullptr,
                        a.To ? mbytes : 0u)};
    xpend = xs[(w * MB + MB - 1) * 64 + lane];
#pragma unroll
    for (int r = 0; r < 4; ++r) epi2_row(P, O, K - 1, MB - 1, r, q0, q1, xpend);
    flush_loss(K - 1);
  }
}


template <int MP, int NP, int EM, int PK>
hipError_t launch_fused(const FusedArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((fused_kernel<MP, NP, EM, PK>), dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int MP, int NP>
hipError_t dispatch_variant(int variant, const FusedArgs& a, int grid, hipStream_t s) {
  switch (variant) {
    case DLADMM_V1_LENA: return launch_fused<MP, NP, EM_V1, PK_ELEM>(a, grid, s);
    case DLADMM_V2_LTHETA: return launch_fused<MP, NP, EM_V1, PK_ROW>(a, grid, s);
    case DLADMM_V3_FULL: return launch_fused<MP, NP, EM_VVAR, PK_ROW>(a, grid, s);
    case DLADMM_V4_SCALAR:
    case DLADMM_V5_TIED: return launch_fused<MP, NP, EM_VVAR, PK_SCALAR>(a, grid, s);
    case DLADMM_V6_LASSO: return launch_fused<MP, NP, EM_LASSO, PK_SCALAR>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_fused_shape(int shape, int variant, const FusedArgs& a, int grid,
                              hipStream_t s) {
  switch (shape) {
    case 0: return dispatch_variant<16, 32>(variant, a, grid, s);
    case 1: return dispatch_variant<64, 256>(variant, a, grid, s);
    case 2: return dispatch_variant<256, 512>(variant, a, grid, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace dladmm
