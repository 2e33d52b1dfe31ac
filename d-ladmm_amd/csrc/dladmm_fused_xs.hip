// dladmm_fused_xs.hip -- the fused K-layer forward for the SMALLEST batches (path 6): four
// workgroups (on four CUs) per 16 batch columns, the rows of every product split over their 16
// waves.
//
// Path 5 (dladmm_fused_rs.hip) gives a 16-column group one workgroup: its 4 SIMDs run every
// MFMA of both products, so a layer costs ~15 us of f32 MFMA cycles per SIMD whatever the
// batch, and a batch of 20 columns (main_lena.py:155, the KM ground truth of
// test_syn_l1l1_scalar.py:478) uses 2 of 256 CUs.  Here a group is 4 workgroups: wave v = 4 *
// member + w of the group owns
//   G1 (Z = S(Z - s1 W_k Var)): output pair v (blocks 2v, 2v+1 of NP = 512), contraction over m;
//   G2 (A Z_k, the E / L / T / Var updates): output block v of MP = 256 (half of A pair v / 2),
//                                            contraction over n,
// a quarter of path 5's MFMAs per SIMD.  The B operand of each product is the group's whole column
// state, so after each product the members hand their blocks to each other through an exchange
// buffer in global memory (one hand-off per product): 16-byte `sc1` stores, every storing wave's
// `s_waitcnt vmcnt(0)`, a workgroup barrier, one agent-scope atomic add per member to the group's
// counter; the consumer's one lane polls the counter with `sc1` loads, a workgroup barrier, then
// `sc1` loads of the buffer into LDS (MI355X_MICROARCH.md, inter-workgroup visibility, the first
// hand-off row: valid at any placement).  Members are blocks b, b + 8, b + 16, b + 24, which the
// dispatcher deals to one XCD (observed, speed only: the hand-off stays in that XCD's L2).  Every
// spin is bounded (it ends after ~2^22 polls, never a hang; every output written after a timed-out
// hand-off is NaN, not silently wrong); a group is resident together because the plan launches at
// most one workgroup per CU.
//
// Arithmetic is path 5's, operation for operation (the same packed fragments, G1 one chain per
// block over k in order, G2 the two chains summed once, the same elementwise expressions): the
// outputs are the fused kernel's bit for bit (tests/test_gpu_xsplit.py).  The per-column
// objective sums its 16 wave partials in wave order: equal to fp32 rounding.
// Scope: V1, V4, V5, V6 at the 256 x 512 register shape, fp32.
#include "dladmm_internal.h"

#ifndef XS_PF
#define XS_PF 8  // weight-fragment read-ahead (MFMA steps) per wave; the first XS_PF steps of each
                 // pass are fetched during the hand-off before it
#endif
#ifndef XS_ABL
#define XS_ABL 0  // timing ablations only (wrong results): 1 no poll wait, 2 no exchange loads
                  // into LDS, 4 no exchange stores (tools/ablate_units.py)
#endif
#ifndef XS_PRE_LATE
#define XS_PRE_LATE 1  // 1: fetch the next pass's first fragments right behind the exchange
                       // loads (the LDS writes wait for those only); 0: before the poll.  V4
                       // K = 15 (ms, B = 20 / 1,000): 0.201 / 0.214 vs 0.207 / 0.221; read-ahead
                       // 12: 0.197 / 0.216; before both changes 0.27 (profiles/r06_xsplit_ab.json)
#endif
#ifndef XS_SPIN
#define XS_SPIN (1 << 22)  // bound of every hand-off poll
#endif

namespace dladmm {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kXsMembers = 4;   // workgroups per 16-column group
constexpr int kXsWaves = kXsMembers * kWaves;

template <int MP, int NP, int EMODE, int PKIND>
__global__ __launch_bounds__(256, 1) void fused_xs_kernel(const FusedArgs a) {
  constexpr int MB = MP / 16, NB = NP / 16;
  static_assert(NB == 2 * kXsWaves && MB == kXsWaves, "one G1 pair and one G2 block per wave");
  constexpr int S1 = MB, S2 = NB;  // MFMA steps of a wave's G1 / G2
  constexpr bool kElem = PKIND == PK_ELEM;
  __shared__ f32x4 zx[NB * 64];  // Z_k of the 16 columns, block b at zx[b * 64 + lane]
  __shared__ f32x4 vx[MB * 64];  // Var

  const int xb = blockIdx.x;
  const int grp = (xb >> 5) * 8 + (xb & 7);   // members share xb % 8
  const int mem = (xb >> 3) & 3;
  if (grp * 16 >= a.B) return;                // a padding group: every member leaves
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int v = mem * kWaves + w;             // wave of the group
  const int g = lane >> 4;
  const int64_t col = (int64_t)grp * 16 + (lane & 15);
  const bool cv = col < a.B;
  const int m = a.m, n = a.n, K = a.K;
  const bool lossz = a.loss_kind != 0;
  const bool lasso = __builtin_amdgcn_readfirstlane(a.loss_kind) == DLADMM_LOSS_LASSO;
  auto lane_off = [&](int64_t ld) -> uint32_t {
    return cv ? (uint32_t)((col + (int64_t)(4 * g) * ld) * 4) : kOOB;
  };
  const int b1o = 2 * v, b2o = v;  // this wave's G1 pair (blocks b1o, b1o + 1) and G2 block

  // the group's exchange buffer: Z blocks [NB][64] f32x4, Var blocks [MB][64], then the objective
  // partials [2][16 waves][16 columns]; its hand-off counter on a line of its own
  f32x4* xz = (f32x4*)(a.xch + (int64_t)grp * a.xstride);
  f32x4* xv = xz + NB * 64;
  float* xl = (float*)(xv + MB * 64);
  unsigned* cnt = a.xcnt + grp * 64;
  const rsrc_t rxz = mkrsrc((const float*)xz, (uint32_t)(NB * 64 * 16));
  const rsrc_t rxv = mkrsrc((const float*)xv, (uint32_t)(MB * 64 * 16));
  unsigned hand = 0;
  __shared__ int xerr;  // sticky: a hand-off timed out
  if (threadIdx.x == 0) xerr = 0;
  bool bad = false;
  // an output value, or NaN once a hand-off has timed out (the outputs of every later product
  // would be computed on incomplete operands: poisoned, not silently wrong)
  auto fin = [&](float x) -> float { return bad ? __builtin_nanf("") : x; };
  // hand-off: this member's stores are done; wait for every member's, then the buffer's blocks
  // (sc1: past this CU's L1) into LDS.  Called by every wave of the workgroup.
  auto handoff = [&](const rsrc_t& rb, f32x4* dst, auto NBLK_, auto&& pre) {
    constexpr int nblk = decltype(NBLK_)::value;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if constexpr (!XS_PRE_LATE) pre();  // the next pass's first weight fragments: in flight
                                        // while lane 0 polls
    hand += kXsMembers;
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int it = 0;
      unsigned c = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while (!(XS_ABL & 1) && c < hand && ++it < XS_SPIN) {
        __builtin_amdgcn_s_sleep(1);
        c = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (!(XS_ABL & 1) && c < hand) xerr = 1;  // a member never arrived: everything from here on is NaN
    }
    __syncthreads();
    bad = __builtin_amdgcn_readfirstlane(xerr) != 0;
    constexpr int per = (XS_ABL & 2) ? 0 : nblk * 64 / 256;  // f32x4 per thread
    f32x4 t[per > 0 ? per : 1];
#pragma unroll
    for (int j = 0; j < per; ++j)
      t[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           rb, (threadIdx.x + 256 * j) * 16, 0, 16));
    if constexpr (XS_PRE_LATE) pre();  // issued behind the exchange loads: the LDS writes below
                                       // wait for those only
#pragma unroll
    for (int j = 0; j < per; ++j) dst[threadIdx.x + 256 * j] = t[j];
    __syncthreads();
  };
  auto xstore = [&](const rsrc_t& rb, int blk, const f32x4& val) {
    if constexpr (XS_ABL & 4) return;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), rb, (blk * 64 + lane) * 16, 0, 16);
  };

  float Zr[2][4], Er[4], Lr[4], Xr[4];
  {
    const rsrc_t rz = mkrsrc(a.Z0, (uint32_t)(n * a.ldz0 * 4));
    const rsrc_t re = mkrsrc(a.E0, (uint32_t)(m * a.lde0 * 4));
    const rsrc_t rl = mkrsrc(a.L0, (uint32_t)(m * a.ldl0 * 4));
    const rsrc_t rx = mkrsrc(a.X, (uint32_t)(m * a.ldx * 4));
    const uint32_t oz = lane_off(a.ldz0), oe = lane_off(a.lde0), ol = lane_off(a.ldl0),
                   ox = lane_off(a.ldx);
    // Z0 of every block into LDS (an input: no hand-off), this wave's pair into registers
    for (int b = w; b < NB; b += kWaves) {
      f32x4 zv;
#pragma unroll
      for (int r = 0; r < 4; ++r) zv[r] = bload(rz, oz + (uint32_t)((16 * b + r) * a.ldz0 * 4));
      zx[b * 64 + lane] = zv;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) Zr[h][r] = bload(rz, oz + (uint32_t)((16 * (b1o + h) + r) * a.ldz0 * 4));
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t ro = (uint32_t)(16 * b2o + r);
      Xr[r] = bload(rx, ox + ro * (uint32_t)(a.ldx * 4));
      Er[r] = bload(re, oe + ro * (uint32_t)(a.lde0 * 4));
      Lr[r] = bload(rl, ol + ro * (uint32_t)(a.ldl0 * 4));
    }
  }

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

  float regsum = 0.f, fit1 = 0.f, fit2 = 0.f;
  float pb[kElem ? 3 : 1][4];
  const uint32_t vb = lane_off(a.ldb);
  auto load_betas = [&](int k) {
    if constexpr (kElem) {
      typedef const float* const __attribute__((address_space(4)))* ctab_p;
      const ctab_p t1 = (ctab_p)a.b1t, t2 = (ctab_p)a.b2t;
      const int kk = k < 0 ? 0 : k, kn = k + 1 < K ? k + 1 : kk;
      const uint32_t eb = (uint32_t)(m * a.ldb * 4);
      const rsrc_t r1 = mkrsrc(k < 0 ? nullptr : t1[kk], k < 0 ? 0u : eb);
      const rsrc_t r2 = mkrsrc(k < 0 ? nullptr : t2[kk], k < 0 ? 0u : eb);
      const rsrc_t rn = mkrsrc(k + 1 < K ? t1[kn] : nullptr, k + 1 < K ? eb : 0u);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t so = (uint32_t)(16 * b2o + r) * (uint32_t)(a.ldb * 4);
        pb[0][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r1, (int)vb, (int)so, 0));
        pb[1][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r2, (int)vb, (int)so, 0));
        pb[2][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rn, (int)vb, (int)so, 0));
      }
    }
  };
  // the layer's per-column objective: this wave's partial to the exchange buffer (handed off with
  // the Var blocks), summed over the 16 waves in order by member 0's wave 0 after that hand-off
  const rsrc_t rxl = mkrsrc(xl, (uint32_t)(2 * kXsWaves * 16 * 4));
  auto stage_loss = [&]() {
    const float rs_ = col_sum(regsum), fs = col_sum(lasso ? fit2 : fit1);
    if (g == 0) {
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, rs_), rxl, (v * 16 + lane) * 4, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, fs), rxl,
                                            ((kXsWaves + v) * 16 + lane) * 4, 0, 16);
    }
    regsum = fit1 = fit2 = 0.f;
  };
  auto flush_loss = [&](int k) {  // after the hand-off that follows stage_loss
    if (mem == 0 && w == 0 && g == 0) {
      auto ldl_ = [&](int i) -> float {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rxl, (i * 16 + lane) * 4, 0, 16));
      };
      float r0 = ldl_(0), f0 = ldl_(kXsWaves);
#pragma unroll
      for (int q = 1; q < kXsWaves; ++q) {
        r0 += ldl_(q);
        f0 += ldl_(kXsWaves + q);
      }
      // every slot of the group, padding columns too (their sums are zero): the reduction
      // reads ldl = 16 * groups columns
      a.lossp[(int64_t)(2 * k + 0) * a.ldl + col] = fin(r0);
      a.lossp[(int64_t)(2 * k + 1) * a.ldl + col] = fin(lasso ? 0.5f * f0 : f0);
    }
  };

  const uint32_t vo = lane_off(a.ldo);
  const uint32_t ld4 = (uint32_t)(a.ldo * 4);
  const uint32_t zbytes = (uint32_t)(n * a.ldo * 4), mbytes = (uint32_t)(m * a.ldo * 4);
  const int64_t wl = (int64_t)MB * NB * kFrag;
  const uint32_t vf = (uint32_t)(lane * 16);
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  auto frag = [&](rsrc_t r, int off) -> f32x4 {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)vf, off, 0));
  };
  auto row_off = [&](int b, int r) -> uint32_t {
    uint32_t o = (uint32_t)(16 * b) * ld4;
    asm volatile("" : "+s"(o));
    return o + (uint32_t)r * ld4;
  };

  // G1(k): this wave's Z pair; Var (all m rows) from vx.  Pack order 2: pair P's k-block kb at
  // fragments 2 (P MB + kb) + h
  f32x4 fa[XS_PF], fb[XS_PF];  // the weight-fragment window, shared by the passes
  auto rw_of = [&](int k) -> rsrc_t {
    const float* wk = a.Wp + (int64_t)(k * a.wstep) * wl + (int64_t)v * MB * 2 * kFrag;
    return mkrsrc(wk, (uint32_t)(S1 * 2 * kFrag * 4));
  };
  auto pre1 = [&](int k) {  // G1(k)'s first XS_PF steps
    const rsrc_t rw = rw_of(k);
    static_for<XS_PF>([&](auto I_) {
      constexpr int i = decltype(I_)::value;
      if constexpr (i < S1) { fa[i] = frag(rw, 2 * i * 1024); fb[i] = frag(rw, (2 * i + 1) * 1024); }
    });
  };
  auto g1_pass = [&](int k, const LayerP& P, rsrc_t rzo) {
    const rsrc_t rw = rw_of(k);
    f32x4 ca = zero4, cb = zero4;
    static_for<S1>([&](auto J_) {
      constexpr int s = decltype(J_)::value;
      const f32x4 vv = vx[s * 64 + lane];
      const f32x4 wa = fa[s % XS_PF], wb = fb[s % XS_PF];
      if constexpr (s + XS_PF < S1) {
        fa[s % XS_PF] = frag(rw, 2 * (s + XS_PF) * 1024);
        fb[s % XS_PF] = frag(rw, (2 * (s + XS_PF) + 1) * 1024);
      }
      ca = mfma4(wa.x, vv[0], ca);
      cb = mfma4(wb.x, vv[0], cb);
      ca = mfma4(wa.y, vv[1], ca);
      cb = mfma4(wb.y, vv[1], cb);
      ca = mfma4(wa.z, vv[2], ca);
      cb = mfma4(wb.z, vv[2], cb);
      ca = mfma4(wa.w, vv[3], ca);
      cb = mfma4(wb.w, vv[3], cb);
    });
    static_for<2>([&](auto H_) {
      constexpr int h = decltype(H_)::value;
      const f32x4 q = h ? cb : ca;
      f32x4 zv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float u = (PKIND == PK_S1) ? Zr[h][r] + P.s1 * q[r] : Zr[h][r] + q[r];
        const float z = shrink_u(u, P.thz);
        Zr[h][r] = z;
        zv[r] = z;
        bstore_s(rzo, vo, row_off(b1o + h, r), fin(z));
        regsum += fabsf(z);
      }
      xstore(rxz, b1o + h, zv);
    });
  };

  // G2(k): A Z_k for this wave's E / L / T block; Z_k (all n rows) from zx.  Its A fragments are
  // half h0 of pair v / 2: 2 (P NB + kb) + h0
  struct OutR { rsrc_t e, l, t, p; };
  const rsrc_t ra = mkrsrc(a.Ap + ((int64_t)(v >> 1) * NB * 2 + (v & 1)) * kFrag,
                           (uint32_t)((2 * S2 - 1) * kFrag * 4));
  auto pre2 = [&]() {  // G2's first XS_PF steps (A: the same every layer)
    static_for<XS_PF>([&](auto I_) {
      constexpr int i = decltype(I_)::value;
      if constexpr (i < S2) fa[i] = frag(ra, 2 * i * 1024);
    });
  };
  auto g2_pass = [&](auto PRO_, int k, const LayerP& P, const OutR& O) {
    constexpr bool PRO = decltype(PRO_)::value;
    load_betas(k);
    f32x4 ca = zero4, ca2 = zero4;
    static_for<S2>([&](auto K_) {
      constexpr int s = decltype(K_)::value;
      const f32x4 z = zx[s * 64 + lane];
      const f32x4 wa = fa[s % XS_PF];
      if constexpr (s + XS_PF < S2) fa[s % XS_PF] = frag(ra, 2 * (s + XS_PF) * 1024);
      ca = mfma4(wa.x, z[0], ca);
      ca2 = mfma4(wa.y, z[1], ca2);
      ca = mfma4(wa.z, z[2], ca);
      ca2 = mfma4(wa.w, z[3], ca2);
    });
    const f32x4 q = ca + ca2;
    f32x4 vv4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float Pv = q[r], x = Xr[r];
      const float l0 = Lr[r], e0 = Er[r];
      float b2 = P.b2, b3 = P.b3, b1n = P.b1n;
      if constexpr (kElem) {
        b3 = pb[0][r];
        b2 = pb[1][r];
        b1n = pb[2][r];
      }
      float e;
      if constexpr (EMODE == EM_V1) {
        const float u = (x - Pv) - b2 * l0;            // main_lena.py:87
        e = shrink_u(u, P.the);
      } else if constexpr (EMODE == EM_VVAR) {
        const float vv = l0 + b2 * ((Pv + e0) - x);    // main_syn_l1l1_scalar.py:114-115
        e = shrink_u(e0 - P.ss2 * vv, P.the);
      } else {
        e = P.ss2 * (x - Pv) - P.ss2b * l0;            // main_syn_lasso_scalar.py:102-103
      }
      e = PRO ? e0 : e;
      const float t = (Pv + e) - x;
      float l = l0 + b3 * t;
      l = PRO ? l0 : l;
      Er[r] = e;
      Lr[r] = l;
      const uint32_t so = row_off(b2o, r);
      bstore_s(O.e, vo, so, fin(e));
      bstore_s(O.l, vo, so, fin(l));
      bstore_s(O.t, vo, so, fin(t));
      bstore_s(O.p, vo, so, fin(Pv));
      const float res = x - Pv;
      fit1 += fabsf(res);
      fit2 = __builtin_fmaf(res, res, fit2);
      vv4[r] = l + b1n * t;
    }
    xstore(rxv, b2o, vv4);
  };

  const rsrc_t none = mkrsrc(nullptr, 0u);
  __syncthreads();  // every wave's Z0 blocks are in zx
  {
    const OutR Op{none, none,
                  mkrsrc(a.keep_all ? a.To : nullptr, (a.keep_all && a.To) ? mbytes : 0u), none};
    pre2();
    g2_pass(std::true_type{}, -1, layer_params(-1), Op);
  }
  regsum = fit1 = fit2 = 0.f;
  handoff(rxv, vx, std::integral_constant<int, MB>{}, [&] { if (K > 0) pre1(0); });  // Var_0 of the group
  for (int k = 0; k < K; ++k) {
    const bool st = a.keep_all || k == K - 1;
    const int ko = a.keep_all ? k : 0;
    const LayerP P = layer_params(k);
    g1_pass(k, P, mkrsrc(a.Zo + (int64_t)ko * n * a.ldo, st ? zbytes : 0u));
    handoff(rxz, zx, std::integral_constant<int, NB>{}, pre2);  // Z_k of the group
    const OutR O{mkrsrc(a.Eo + (int64_t)ko * m * a.ldo, st ? mbytes : 0u),
                 mkrsrc(a.Lo + (int64_t)ko * m * a.ldo, st ? mbytes : 0u),
                 mkrsrc(a.To ? a.To + (int64_t)(a.keep_all ? k + 1 : 0) * m * a.ldo : nullptr,
                        (a.To && st) ? mbytes : 0u),
                 mkrsrc(a.Po && a.keep_all ? a.Po + (int64_t)k * m * a.ldo : nullptr,
                        a.Po && a.keep_all ? mbytes : 0u)};
    g2_pass(std::false_type{}, k, P, O);
    if (lossz) stage_loss();
    handoff(rxv, vx, std::integral_constant<int, MB>{}, [&] { if (k + 1 < K) pre1(k + 1); });  // Var_{k+1} (and the layer's
                                                                  // objective partials)
    if (lossz) flush_loss(k);
  }
}

template <int MP, int NP, int EM, int PK>
hipError_t launch_xs(const FusedArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((fused_xs_kernel<MP, NP, EM, PK>), dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

int xs_grid(int64_t B) {
  const int64_t groups = (B + 15) / 16;
  return (int)(((groups + 7) / 8) * 8 * kXsMembers);
}

size_t xs_group_floats() {
  constexpr int MB = kShapeMP[2] / 16, NB = kShapeNP[2] / 16;
  return (size_t)(NB + MB) * 64 * 4 + 2 * kXsWaves * 16;
}

hipError_t launch_fused_xs(int shape, int variant, const FusedArgs& a, hipStream_t s) {
  if (shape != 2 || !a.xch || !a.xcnt) return hipErrorInvalidValue;
  constexpr int MP = kShapeMP[2], NP = kShapeNP[2];
  const int grid = xs_grid(a.B);
  switch (variant) {
    case DLADMM_V1_LENA: return launch_xs<MP, NP, EM_V1, PK_ELEM>(a, grid, s);
    case DLADMM_V4_SCALAR: return launch_xs<MP, NP, EM_VVAR, PK_SCALAR>(a, grid, s);
    case DLADMM_V5_TIED: return launch_xs<MP, NP, EM_VVAR, PK_S1>(a, grid, s);
    case DLADMM_V6_LASSO: return launch_xs<MP, NP, EM_LASSO, PK_SCALAR>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace dladmm
