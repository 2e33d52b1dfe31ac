// dladmm_reverse_rs.hip -- the reverse-sweep backward for SMALL batches: one workgroup per 16
// batch columns, the ROWS of every product split over its 4 waves (the backward twin of
// dladmm_fused_rs.hip, path 5).
//
// The reverse sweep (dladmm_reverse_kernel.h) gives each wave 16 columns and all rows, so the
// reference training loops' batches of 20 / 25 (main_lena.py:155, main_syn_l1l1_scalar.py -bs
// 25) ran the whole backward on one CU.  Here, per layer k = K-1 .. 0, wave w owns
//   G1'(k)  R = A^T gP_k      rows n: blocks 8w .. 8w+7, epilogue BK2(k) (gU_k, the adjoint of Z)
//   G2'(k)  gVar = M_k^T gU_k rows m: blocks 4w .. 4w+3, epilogue BK3(k) + BK1(k-1)
// and the B operands (gP_k, then gU_k: whole column states) go through LDS, one barrier per
// product.  The products are the reverse sweep's -- same packed A^T / M_k^T fragments, one fma
// chain per output block in k order -- and so are the elementwise expressions, in the same
// order: gU_k and Var_k (and with them every weight gradient) are that kernel's bit for bit.
// The parameter partials are per (layer, slot, wave) as there, but each wave's partial covers a
// quarter of the rows of 16 columns, so the parameter gradients agree to rounding
// (tests/test_gpu_rowsplit.py); V1's per-sample beta gradients are per-element stores, equal
// bit for bit.  Scope: V1 (EM_V1), V4 / V5 (EM_VVAR) and V6 (EM_LASSO) at the 256 x 512 shape,
// with or without cotangents of Z and of E / L / T (the reference's torch-op losses over the
// returned states, main_lena.py:221-228).  The operands of a G2' output pair are loaded as the
// pair's products start, in flight across its 32 MFMA steps.
#include "dladmm_internal.h"

#ifndef RRS_PF
#define RRS_PF 4  // weight-fragment read-ahead (MFMA steps) per wave
#endif
#ifndef RRS_SPIN
#define RRS_SPIN (1 << 22)  // bound of every hand-off poll (bwd path 3)
#endif

namespace dladmm {

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

// MEM: workgroups per 16-column group.  1 = the one-workgroup form (bwd path 2); 4 = bwd path 3,
// after a path-6 forward: wave v = 4 member + w of the group's 16 owns G1' pair v and G2' block v
// (half of an M_k^T pair), and the B operands (gU_k, gP_k) go between the members through the
// group's exchange buffer once per product, by dladmm_fused_xs.hip's hand-off (sc1 stores, one
// agent-scope counter add per member, one bounded sc1 poll; NaN adjoints after a timeout)
template <int MP, int NP, int EMODE, bool GZ, bool COT, int MEM>
__global__ __launch_bounds__(256, 1) void reverse_rs_kernel(const RevArgs a) {
  constexpr int MB = MP / 16, NB = NP / 16;
  constexpr int WPG = kWaves * MEM;                     // waves per 16-column group
  constexpr int NB4 = NB / WPG, MB4 = MB / WPG;         // output blocks per wave
  static_assert(NB4 % 2 == 0 && (MB4 % 2 == 0 || MB4 == 1), "G1' whole pairs; G2' pairs or one block");
  constexpr int HP = MB4 >= 2 ? 2 : 1;                  // G2' blocks per output step group
  constexpr int S1 = (NB4 / 2) * MB, S2 = (MB4 / HP) * NB;  // MFMA steps of a wave's G1' / G2'
  constexpr bool kAE = EMODE == EM_VVAR;  // the adjoint of E is carried through the workspace
  constexpr bool kV1 = EMODE == EM_V1;     // V1: per-sample betas and their gradients
  // weight-fragment read-ahead: deeper in the four-workgroup form, whose waves wait on the
  // weight stream rather than on their MFMAs (dladmm_fused_xs.hip)
  constexpr int PF = MEM > 1 ? 8 : RRS_PF;
  __shared__ f32x4 gpx[MB * 64];  // gP_k of the 16 columns (G1''s B operand)
  __shared__ f32x4 gux[NB * 64];  // gU_k (G2''s B operand)

  const int xb = blockIdx.x;
  const int grp = MEM == 1 ? xb : (xb >> 5) * 8 + (xb & 7);  // members share xb % 8 (one XCD)
  const int mem = MEM == 1 ? 0 : (xb >> 3) & 3;
  if (MEM > 1 && grp * 16 >= a.B) return;   // a padding group: every member leaves
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int v = mem * kWaves + w;           // wave of the group
  const int g = lane >> 4;
  const int64_t col = (int64_t)grp * 16 + (lane & 15);
  const bool cv = col < a.B;
  const int m = a.m, K = a.K;
  const int cg = grp * WPG + v;  // partial slot of this wave
  const uint32_t lqm = __builtin_amdgcn_readfirstlane(a.loss_kind) == DLADMM_LOSS_LASSO ? ~0u : 0u;
  const int64_t ldo = a.ldo, ml = (int64_t)m * ldo, zl = (int64_t)a.n * ldo;
  auto lane_off = [&](int64_t ld, bool ok) -> uint32_t {
    return ok ? (uint32_t)((col + (int64_t)(4 * g) * ld) * 4) : kOOB;
  };
  const uint32_t vo = lane_off(ldo, cv), vx = lane_off(a.ldx, cv), vw = lane_off(a.ldw, col < a.Bw);
  const uint32_t ldo4 = (uint32_t)(ldo * 4), ldw4 = (uint32_t)(a.ldw * 4);
  const uint32_t aeo = (uint32_t)(a.aer * a.ldw * 4), vas4 = (uint32_t)(a.vas * 4);
  const uint32_t mbytes = (uint32_t)(ml * 4);
  const int b1o = v * NB4, b2o = v * MB4;
  const rsrc_t none = mkrsrc(nullptr, 0u);
  // MEM = 4: the group's exchange buffer (gU blocks [NB][64] f32x4, then gP blocks [MB][64]) and
  // its hand-off counter; MEM = 1: a workgroup barrier
  __shared__ int xerr;  // sticky: a hand-off timed out
  if (threadIdx.x == 0) xerr = 0;
  bool bad = false;
  auto fin = [&](float x) -> float { return bad ? __builtin_nanf("") : x; };
  const f32x4* xu = (const f32x4*)(MEM > 1 ? a.xch + (int64_t)grp * a.xstride : nullptr);
  const rsrc_t rxu = mkrsrc((const float*)xu, MEM > 1 ? (uint32_t)(NB * 64 * 16) : 0u);
  const rsrc_t rxp = mkrsrc((const float*)(xu + NB * 64), MEM > 1 ? (uint32_t)(MB * 64 * 16) : 0u);
  unsigned* cnt = MEM > 1 ? a.xcnt + grp * 64 : nullptr;
  unsigned hand = 0;
  auto xstore = [&](const rsrc_t& rb, int blk, const f32x4& val) {
    if constexpr (MEM > 1)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, val), rb,
                                             (blk * 64 + lane) * 16, 0, 16);
  };
  auto handoff = [&](const rsrc_t& rb, f32x4* dst, auto NBLK_) {
    if constexpr (MEM == 1) {
      __syncthreads();
    } else {
      constexpr int nblk = decltype(NBLK_)::value;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      hand += MEM;
      if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int it = 0;
        unsigned c = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (c < hand && ++it < RRS_SPIN) {
          __builtin_amdgcn_s_sleep(1);
          c = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (c < hand) xerr = 1;
      }
      __syncthreads();
      bad = __builtin_amdgcn_readfirstlane(xerr) != 0;
      constexpr int per = nblk * 64 / 256;
      f32x4 t[per];
#pragma unroll
      for (int q = 0; q < per; ++q)
        t[q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rb, (threadIdx.x + 256 * q) * 16, 0, 16));
#pragma unroll
      for (int q = 0; q < per; ++q) dst[threadIdx.x + 256 * q] = t[q];
      __syncthreads();
    }
  };
  // a wave-uniform (pointer, size) buffer view (readfirstlane: the selects stay in SGPRs)
  auto urs = [](const float* p, uint32_t bytes) -> rsrc_t {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return mkrsrc((const float*)(((uint64_t)hi << 32) | lo), __builtin_amdgcn_readfirstlane(bytes));
  };
  typedef const float* const __attribute__((address_space(4)))* ctab_p;
  const ctab_p tab = (ctab_p)a.ptab;
  auto ld = [](rsrc_t r, uint32_t voff, uint32_t soff) -> float {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 2));
  };
  auto row_off = [&](int b, int r, uint32_t ld4) -> uint32_t {  // opaque per-block base
    uint32_t o = (uint32_t)(16 * b) * ld4;
    asm volatile("" : "+s"(o));
    return o + (uint32_t)r * ld4;
  };

  // state of this wave's rows: the adjoint of Z (n rows: gU once BK2 formed it), the partial
  // adjoint of L_{k-1} (m rows), X
  float AZ[NB4][4], AL[MB4][4], Xr[MB4][4];
  {
    const rsrc_t rx = mkrsrc(a.X, (uint32_t)(m * a.ldx * 4));
#pragma unroll
    for (int b = 0; b < NB4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) AZ[b][r] = 0.f;
#pragma unroll
    for (int b = 0; b < MB4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        AL[b][r] = 0.f;
        Xr[b][r] = ld(rx, vx, row_off(b2o + b, r, (uint32_t)(a.ldx * 4)));
      }
  }
  float psz = 0.f, psb1 = 0.f, ps[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  auto flush = [&](int layer, int slot, float v) {
    if constexpr (kV1) return;  // V1: per-sample betas (element gradients), fixed thresholds
    const float s = wave_sum(v);
    if (lane == 0) a.part[((int64_t)layer * DLADMM_NSCALAR + slot) * a.ncg + cg] = fin(s);
  };
  auto flush_bk1 = [&](int j) {
    if constexpr (kV1) return;
    flush(j, DLADMM_P_BETA3, ps[0]);
    if constexpr (EMODE == EM_VVAR) {
      flush(j, DLADMM_P_BETA2, ps[1]);
      flush(j, DLADMM_P_THETA_E, ps[2]);
      flush(j, DLADMM_P_SS2, ps[3]);
    } else {
      flush(j, DLADMM_P_SS2, ps[3]);
      flush(j, DLADMM_P_SS2B, ps[4]);
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) ps[i] = 0.f;
  };

  // parameters (the reverse sweep's lp2 / lp1)
  cfloat_p sp = (cfloat_p)a.scal;
  struct LP2 { float b1k, b2, b3, ss2, ss2b, the, cf; };
  auto lp2 = [&](int k, int jl) -> LP2 {
    LP2 p{};
    const int kk = k < K ? k : K - 1;
    const int jj = jl < 0 ? 0 : jl;
    p.cf = a.loss_kind ? ((cfloat_p)a.lcoef)[2 * jj + 1] : 0.f;
    p.b1k = sp[kk * DLADMM_NSCALAR + DLADMM_P_BETA1];
    p.b2 = sp[jj * DLADMM_NSCALAR + DLADMM_P_BETA2];
    p.b3 = sp[jj * DLADMM_NSCALAR + DLADMM_P_BETA3];
    p.ss2 = sp[jj * DLADMM_NSCALAR + DLADMM_P_SS2];
    p.ss2b = sp[jj * DLADMM_NSCALAR + DLADMM_P_SS2B];
    p.the = sp[jj * DLADMM_NSCALAR + DLADMM_P_THETA_E];
    return p;
  };
  struct LP1 { float c, cz; };
  auto lp1 = [&](int k) -> LP1 {
    const float th = sp[k * DLADMM_NSCALAR + DLADMM_P_THETA_Z];
    return LP1{th >= 0.f ? 0.f : -2.0f * th, a.loss_kind ? ((cfloat_p)a.lcoef)[2 * k] : 0.f};
  };

  const uint32_t vf = (uint32_t)(lane * 16);
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  auto frag2 = [&](rsrc_t r, auto S_, f32x4& fa, f32x4& fb) {
    constexpr int s = decltype(S_)::value;
    fa = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)vf, 2 * s * 1024, 0));
    fb = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)vf, (2 * s + 1) * 1024, 0));
  };
  const int64_t wl = (int64_t)MB * NB * kFrag;  // floats per packed matrix
  // A^T [NB/2][MB][2] (G1': this wave's pairs from b1o / 2 on); M_k^T [K][MB/2][NB][2]
  const rsrc_t rat = mkrsrc(a.Atp + (int64_t)(b1o / 2) * MB * 2 * kFrag, (uint32_t)(S1 * 2 * kFrag * 4));

  // G1'(k): R = A^T gP_k for this wave's n blocks; BK2(k): gU_k = S'(U_k) (gZ + cz sgn Z_k + R)
  auto g1_pass = [&](int k) {
    const LP1 P1 = lp1(k);
    const rsrc_t rz = urs(a.Z + k * zl, (uint32_t)(zl * 4));
    const float* gzp = GZ ? tab[rev_tab_at(RT_GZ, K, k)] : nullptr;
    const rsrc_t rgz = GZ ? urs(gzp, gzp ? (uint32_t)(zl * 4) : 0u) : none;
    const rsrc_t rg = urs(a.GU + k * a.gus, (uint32_t)(NP * a.ldw * 4));
    float pz[NB4][4], pg[GZ ? NB4 : 1][4];
#pragma unroll
    for (int b = 0; b < NB4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t so = row_off(b1o + b, r, ldo4);
        pz[b][r] = ld(rz, vo, so);
        if constexpr (GZ) pg[b][r] = ld(rgz, vo, so);
      }
    f32x4 fa[PF], fb[PF];
    static_for<PF>([&](auto I_) {
      constexpr int i = decltype(I_)::value;
      if constexpr (i < S1) frag2(rat, I_, fa[i], fb[i]);
    });
    static_for<NB4 / 2>([&](auto P_) {
      constexpr int pp = decltype(P_)::value;
      f32x4 ca = zero4, cb = zero4;
      static_for<MB>([&](auto J_) {
        constexpr int jb = decltype(J_)::value;
        constexpr int s = pp * MB + jb;
        const f32x4 v = gpx[jb * 64 + lane];
        const f32x4 wa = fa[s % PF], wb = fb[s % PF];
        if constexpr (s + PF < S1)
          frag2(rat, std::integral_constant<int, s + PF>{}, fa[s % PF], fb[s % PF]);
        ca = mfma4(wa.x, v[0], ca);
        cb = mfma4(wb.x, v[0], cb);
        ca = mfma4(wa.y, v[1], ca);
        cb = mfma4(wb.y, v[1], cb);
        ca = mfma4(wa.z, v[2], ca);
        cb = mfma4(wb.z, v[2], cb);
        ca = mfma4(wa.w, v[3], ca);
        cb = mfma4(wb.w, v[3], cb);
      });
      static_for<2>([&](auto H_) {
        constexpr int h = decltype(H_)::value;
        constexpr int lb = 2 * pp + h;
        const f32x4 q = h ? cb : ca;
        f32x4 gu4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float zk = pz[lb][r];
          float gZt = (GZ ? AZ[lb][r] + pg[GZ ? lb : 0][r] : AZ[lb][r]) + q[r];
          const float sg = (zk > 0.f ? 1.f : 0.f) - (zk < 0.f ? 1.f : 0.f);
          gZt = __builtin_fmaf(P1.cz, sg, gZt);
          const float ga = zk > -P1.c ? gZt : 0.f, gb = zk < P1.c ? gZt : 0.f;
          const float gU = ga + gb;
          psz += gb - ga;
          AZ[lb][r] = gU;
          gu4[r] = fin(gU);
          bstore_s(rg, vw, row_off(b1o + lb, r, ldw4), gu4[r]);
        }
        gux[(b1o + lb) * 64 + lane] = gu4;
        xstore(rxu, b1o + lb, gu4);
      });
    });
    flush(k, DLADMM_P_THETA_Z, psz);
    psz = 0.f;
  };

  // G2'(k): gVar = M_k^T gU_k for this wave's m blocks.  MODE 0: BK3(k) + BK1(k-1) on layer
  // j = k - 1's saved state; 1: BK3 of layer 0 alone (T_0 in the P slot, L0); 2: the prologue,
  // BK1(K-1) with zero incoming adjoints (no product)
  auto g2_pass = [&](auto MODE_, int k) {
    constexpr int MODE = decltype(MODE_)::value;
    const int j = MODE == 2 ? K - 1 : k - 1;   // the BK1 layer
    const LP2 P = MODE == 2 ? lp2(K, K - 1) : (MODE == 1 ? lp2(0, -1) : lp2(k, k - 1));
    // operand views (the reverse sweep's res2 / res2_last)
    auto tview = [&](int t, int kk) -> rsrc_t {
      const float* p = tab[rev_tab_at(t, K, kk)];
      return urs(p, p ? mbytes : 0u);
    };
    rsrc_t oP, oL, oE = none;
    rsrc_t oB1K = none, oGB1K = none, oB1J = none, oB2J = none, oGB1J = none, oGB2J = none;
    rsrc_t oGE = none, oGL = none, oGT = none;
    if constexpr (MODE == 1) {
      oP = mkrsrc(a.T, mbytes);
      oL = urs(a.L0, mbytes);
      if constexpr (kV1) {
        oB1K = tview(RT_B1, 0);
        oGB1K = tview(RT_GB1, 0);
      }
    } else {
      oP = urs(a.P + j * ml, mbytes);
      oL = urs(j >= 1 ? a.L + (j - 1) * ml : a.L0, mbytes);
      if constexpr (kAE) oE = urs(j >= 1 ? a.E + (j - 1) * ml : a.E0, mbytes);
      if constexpr (kV1) {
        const bool bk3 = j + 1 < K;   // the prologue (j = K - 1) has no BK3
        oB1K = bk3 ? tview(RT_B1, j + 1) : none;
        oGB1K = bk3 ? tview(RT_GB1, j + 1) : none;
        oB1J = tview(RT_B1, j);
        oB2J = tview(RT_B2, j);
        oGB1J = tview(RT_GB1, j);
        oGB2J = tview(RT_GB2, j);
      }
      if constexpr (COT) {
        oGE = tview(RT_GE, j);
        oGL = tview(RT_GL, j);
        oGT = tview(RT_GT, j + 1);
      }
    }
    // Var_j's workspace block and the next layer's (which holds the adjoint of E_{j})
    const int jr = MODE == 1 ? 0 : j;
    const rsrc_t rv = urs(a.VAR + jr * a.vas, (uint32_t)((jr + 1 < K ? 2 : 1) * a.vas * 4));
    // operands of one pair of m blocks, loaded as the pair's products start (in flight during
    // its 32 MFMA steps)
    enum { O_P = 0, O_L = 1, O_E = 2, O_A = 3, O_B1K = 4, O_B1J = 5, O_B2J = 6, O_GB1 = 7,
           O_GE = 8, O_GL = 9, O_GT = 10 };
    float op[2][11][4];
    auto load_pair = [&](int pp) {
#pragma unroll
      for (int h = 0; h < HP; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int b = HP * pp + h;
          const uint32_t so = row_off(b2o + b, r, ldo4);
          op[h][O_P][r] = ld(oP, vo, so);
          op[h][O_L][r] = ld(oL, vo, so);
          if constexpr (kAE) {
            op[h][O_E][r] = MODE == 1 ? 0.f : ld(oE, vo, so);
            op[h][O_A][r] = MODE == 0 ? ld(rv, vw, vas4 + aeo + row_off(b2o + b, r, ldw4)) : 0.f;
          }
          if constexpr (kV1) {
            op[h][O_B1K][r] = ld(oB1K, vo, so);
            op[h][O_B1J][r] = ld(oB1J, vo, so);
            op[h][O_B2J][r] = ld(oB2J, vo, so);
            op[h][O_GB1][r] = ld(oGB1K, vo, so);
          }
          if constexpr (COT) {
            op[h][O_GE][r] = ld(oGE, vo, so);
            op[h][O_GL][r] = ld(oGL, vo, so);
            op[h][O_GT][r] = ld(oGT, vo, so);
          }
        }
    };
    // M_k^T: HP = 2, this wave's pairs from b2o / 2 on (steps read fragments 2s, 2s + 1);
    // HP = 1, half b2o & 1 of pair b2o / 2 (fragments 2 (P NB + kb) + h0: step s at 2s)
    const rsrc_t rmt =
        MODE == 2 ? none
        : HP == 2 ? mkrsrc(a.Mtp + (int64_t)k * wl + (int64_t)(b2o / 2) * NB * 2 * kFrag,
                           (uint32_t)(S2 * 2 * kFrag * 4))
                  : mkrsrc(a.Mtp + (int64_t)k * wl + ((int64_t)(b2o >> 1) * NB * 2 + (b2o & 1)) * kFrag,
                           (uint32_t)((2 * S2 - 1) * kFrag * 4));
    f32x4 fa[PF], fb[HP == 2 ? PF : 1];
    auto fetch = [&](auto S_, int slot) {
      constexpr int st = decltype(S_)::value;
      if constexpr (HP == 2) {
        frag2(rmt, S_, fa[slot], fb[slot]);
      } else {
        fa[slot] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 rmt, (int)vf, 2 * st * 1024, 0));
      }
    };
    if constexpr (MODE != 2) {
      static_for<PF>([&](auto I_) {
        constexpr int i = decltype(I_)::value;
        if constexpr (i < S2) fetch(I_, i);
      });
    }
    static_for<MB4 / HP>([&](auto P_) {
      constexpr int pp = decltype(P_)::value;
      load_pair(pp);
      f32x4 qa4[2] = {zero4, zero4};
      if constexpr (MODE != 2) {
        f32x4 ca = zero4, cb = zero4;
        static_for<NB>([&](auto K_) {
          constexpr int kb = decltype(K_)::value;
          constexpr int s = pp * NB + kb;
          const f32x4 u = gux[kb * 64 + lane];
          const f32x4 wa = fa[s % PF];
          const f32x4 wb = fb[HP == 2 ? s % PF : 0];
          if constexpr (s + PF < S2)
            fetch(std::integral_constant<int, s + PF>{}, s % PF);
          ca = mfma4(wa.x, u[0], ca);
          if constexpr (HP == 2) cb = mfma4(wb.x, u[0], cb);
          ca = mfma4(wa.y, u[1], ca);
          if constexpr (HP == 2) cb = mfma4(wb.y, u[1], cb);
          ca = mfma4(wa.z, u[2], ca);
          if constexpr (HP == 2) cb = mfma4(wb.z, u[2], cb);
          ca = mfma4(wa.w, u[3], ca);
          if constexpr (HP == 2) cb = mfma4(wb.w, u[3], cb);
        });
        qa4[0] = ca;
        qa4[1] = cb;
      }
      // epilogue rows (the reverse sweep's epi2_row)
#pragma unroll
    for (int h = 0; h < HP; ++h) {
      const int lb = HP * pp + h;
      f32x4 gp4;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float gVar = qa4[h][r];
        const uint32_t sw = row_off(b2o + lb, r, ldw4);
        const uint32_t sb = row_off(b2o + lb, r, ldo4);
        const float b1k = kV1 ? op[h][O_B1K][r] : P.b1k;
        if constexpr (MODE == 1) {
          if constexpr (kV1) {
            // beta1_0's gradient: BK1(0)'s term + gVar T_0
            bstore_s(oGB1K, vo, sb, op[h][O_GB1][r] + gVar * op[h][O_P][r]);
          } else {
            psb1 += gVar * op[h][O_P][r];   // beta1_0's gradient: gVar T_0
          }
          // Var_0 = L0 + beta1_0 T_0, the forward's prologue expression
          bstore_s(rv, vw, sw, op[h][O_L][r] + b1k * op[h][O_P][r]);
          continue;
        }
        const float aLin = AL[lb][r] + gVar;  // complete adjoint of L_{k-1} (upstream aside)
        const float aTin = b1k * gVar;        // adjoint of T_k
        const float aL = COT ? aLin + op[h][O_GL][r] : aLin;
        const float aT = COT ? aTin + op[h][O_GT][r] : aTin;
        const float aE0 = MODE == 0 ? (kAE ? op[h][O_A][r] : 0.f) : 0.f;
        const float aE = COT ? aE0 + op[h][O_GE][r] : aE0;
        const float Pv = op[h][O_P][r], lp = op[h][O_L][r], x = Xr[lb][r];
        const float b1 = kV1 ? op[h][O_B1J][r] : 0.f;
        float gP, gEp = 0.f, gLp, t;
        (void)gEp;
        float p3 = 0.f, p2 = 0.f, pe = 0.f, ps2 = 0.f, ps2b = 0.f;
        if constexpr (EMODE == EM_V1) {
          const float b2 = op[h][O_B2J][r];
          const float u = (x - Pv) - b2 * lp;               // main_lena.py:87
          const float e = shrink_u(u, shrink_params(P.the));
          t = (Pv + e) - x;                                 // T_k
          const float gTn = aT + b1 * aL;                   // L_{k-1} = L_{k-2} + b1 T_k (:89)
          p3 = aL * t;
          const float gEt = aE + gTn;
          const float ga = (u - P.the) > 0.0f ? gEt : 0.f;
          const float gb = (-u - P.the) > 0.0f ? gEt : 0.f;
          const float gEh = ga + gb;
          pe = gb - ga;
          gP = gTn - gEh;
          p2 = -gEh * lp;
          gLp = aL - b2 * gEh;
        } else if constexpr (EMODE == EM_VVAR) {
          const float ep = op[h][O_E][r];
          const float r0 = (Pv + ep) - x;
          const float vv = lp + P.b2 * r0;                  // main_syn_l1l1_scalar.py:114
          const float eh = ep - P.ss2 * vv;                 // :115
          const float e = shrink_u(eh, shrink_params(P.the));
          t = (Pv + e) - x;                                 // T_k
          const float gTn = aT + P.b3 * aL;
          p3 = aL * t;
          const float gEt = aE + gTn;
          const float ga = (eh - P.the) > 0.0f ? gEt : 0.f;
          const float gb = (-eh - P.the) > 0.0f ? gEt : 0.f;
          const float gEh = ga + gb;
          pe = gb - ga;
          const float gVV = -P.ss2 * gEh;
          ps2 = -gEh * vv;
          gLp = aL + gVV;
          p2 = gVV * r0;
          gP = gTn + P.b2 * gVV;
          gEp = gEh + P.b2 * gVV;
        } else {
          const float e = P.ss2 * (x - Pv) - P.ss2b * lp;  // main_syn_lasso_scalar.py:102-103
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
          const float dfit = __builtin_bit_cast(
              float, (lqm & __builtin_bit_cast(uint32_t, res)) | (~lqm & __builtin_bit_cast(uint32_t, sg)));
          gP = gP - P.cf * dfit;
        }
        if constexpr (kV1) {
          // beta1_k's gradient = BK1(k)'s term + gVar T_k; beta1_{k-1} gets BK1(k-1)'s term
          // aL T_k now and BK3(k-1)'s next pass; beta2_{k-1} complete
          bstore_s(MODE == 0 ? oGB1K : none, vo, sb, op[h][O_GB1][r] + gVar * t);
          bstore_s(oGB1J, vo, sb, p3);
          bstore_s(oGB2J, vo, sb, p2);
        } else {
          if constexpr (MODE == 0) psb1 += gVar * t;  // beta1 of layer k: gVar * T_k
          ps[0] += p3; ps[1] += p2; ps[2] += pe; ps[3] += ps2; ps[4] += ps2b;
        }
        gp4[r] = fin(gP);
        AL[lb][r] = gLp;
        // Var of layer k: L_{k-1} + beta1_k T_k from the recomputed values (the prologue's,
        // layer K, runs past the workspace: dropped)
        const float lcoef = kV1 ? b1 : P.b3;
        const float lk = lp + lcoef * t;
        const float vark = lk + b1k * t;
        bstore_s(rv, vw, vas4 + sw, vark);
        if constexpr (kAE) bstore_s(rv, vw, sw + aeo, gEp);  // adjoint of E_{k-2}
      }
      if constexpr (MODE != 1) {
        gpx[(b2o + lb) * 64 + lane] = gp4;
        xstore(rxp, b2o + lb, gp4);
      }
    }
    });
  };

  // prologue BK1(K-1), then per layer G1'(k), G2'(k)
  constexpr auto kNB = std::integral_constant<int, NB>{};
  constexpr auto kMB = std::integral_constant<int, MB>{};
  g2_pass(std::integral_constant<int, 2>{}, K);
  flush_bk1(K - 1);
  handoff(rxp, gpx, kMB);  // gP_{K-1} complete
  for (int k = K - 1; k >= 1; --k) {
    g1_pass(k);
    handoff(rxu, gux, kNB);  // gU_k complete; every wave is done reading gP_k
    g2_pass(std::integral_constant<int, 0>{}, k);
    flush(k, DLADMM_P_BETA1, psb1);
    psb1 = 0.f;
    flush_bk1(k - 1);
    handoff(rxp, gpx, kMB);  // gP_{k-1} complete; every wave is done reading gU_k
  }
  g1_pass(0);
  handoff(rxu, gux, kNB);
  g2_pass(std::integral_constant<int, 1>{}, 0);
  flush(0, DLADMM_P_BETA1, psb1);
}

template <int EM, bool GZ, bool COT, int MEM>
hipError_t launch_rrs(const RevArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((reverse_rs_kernel<kShapeMP[2], kShapeNP[2], EM, GZ, COT, MEM>), dim3(grid),
                     dim3(256), 0, s, a);
  return hipGetLastError();
}
template <int EM, int MEM = 1>
hipError_t launch_rrs_em(const RevArgs& a, int grid, hipStream_t s) {
  if (a.has_gz && a.has_cot) return launch_rrs<EM, true, true, MEM>(a, grid, s);
  if (a.has_gz) return launch_rrs<EM, true, false, MEM>(a, grid, s);
  if (a.has_cot) return launch_rrs<EM, false, true, MEM>(a, grid, s);
  return launch_rrs<EM, false, false, MEM>(a, grid, s);
}

size_t rev_xs_group_floats() {
  return (size_t)(kShapeNP[2] / 16 + kShapeMP[2] / 16) * 64 * 4;
}

hipError_t launch_reverse_xs(int shape, int variant, const RevArgs& a, hipStream_t s) {
  if (!reverse_rs_supports(shape, variant) || !a.xch || !a.xcnt) return hipErrorInvalidValue;
  const int grid = xs_grid(a.B);
  if (variant == DLADMM_V1_LENA) return launch_rrs_em<EM_V1, 4>(a, grid, s);
  if (variant == DLADMM_V6_LASSO) return launch_rrs_em<EM_LASSO, 4>(a, grid, s);
  return launch_rrs_em<EM_VVAR, 4>(a, grid, s);
}

bool reverse_rs_supports(int shape, int variant) {
  return shape == 2 && (variant == DLADMM_V1_LENA || variant == DLADMM_V4_SCALAR ||
                        variant == DLADMM_V5_TIED || variant == DLADMM_V6_LASSO);
}

hipError_t launch_reverse_rs(int shape, int variant, const RevArgs& a, int grid, hipStream_t s) {
  if (!reverse_rs_supports(shape, variant)) return hipErrorInvalidValue;
  if (variant == DLADMM_V1_LENA) return launch_rrs_em<EM_V1>(a, grid, s);
  if (variant == DLADMM_V6_LASSO) return launch_rrs_em<EM_LASSO>(a, grid, s);
  return launch_rrs_em<EM_VVAR>(a, grid, s);
}

}  // namespace dladmm
