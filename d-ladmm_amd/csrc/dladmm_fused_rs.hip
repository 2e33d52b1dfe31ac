// dladmm_fused_rs.hip -- the fused K-layer forward for SMALL batches (path 5): one workgroup per
// 16 batch columns, the ROWS of every product split over its 4 waves.
//
// The fused kernel (dladmm_fused_kernel.h) gives each wave 16 columns and ALL rows: a workgroup
// covers 64 columns, so a batch of B columns occupies ceil(B / 64) CUs and every layer costs one
// CU's time for both products over all rows (the KM ground truth of test_syn_l1l1_scalar.py:478,
// K = 2000 at B = 20 .. 1,000, ran at 67 us per step on 1-16 of the 256 CUs).
// Here a workgroup owns 16 columns and wave w owns a quarter of the output rows of each product:
//   G1 (Z = S(Z - s1 W_k Var)): output blocks 8w .. 8w+7 of n (NP = 512), contraction over all m;
//   G2 (A Z_k and the E / L / T / Var updates): blocks 4w .. 4w+3 of m (MP = 256), over all n.
// Each product's B operand (Var, then Z_k) is the whole column state, so the waves exchange it
// through LDS once per product (one barrier each); the weight fragments come straight from
// L2 by buffer loads, a few steps ahead, with compiler-counted waits (no LDS ring).
//
// Arithmetic is the fused kernel's, operation for operation: the same packed -W_k / A fragments
// (pack order 2), G1 one fma chain per output block over k in order, G2 two chains (k sub-steps
// x, z and y, w) summed once, the same elementwise expressions -- so the outputs are the fused
// kernel's bit for bit (tests/test_gpu_rowsplit.py), the saved products P_k = A Z_k of a
// training forward too.  The fused per-column objective is the same sum in another order (each
// wave sums its quarter of the rows, then the 4 quarters in wave order): equal to fp32 rounding.
// Scope: V1 (per-sample betas), V4, V5 (and the KM iteration built on it), V6 at the 256 x 512
// register shape; the plan (dladmm_capi.hip) picks it for batches that leave most CUs idle on
// the fused kernel.
#include "dladmm_internal.h"

#ifndef RS_PF
#define RS_PF 4  // weight-fragment read-ahead (MFMA steps) per wave: 2, 4 and 8 time the same
                 // (profiles/r06_rowsplit_ab.json) -- each CU fetches the whole weight pair per
                 // step for its 16 columns (1 MiB at 256 x 512), ~45 GB/s per CU at 22 us/step
#endif

namespace dladmm {

template <int MP, int NP, int EMODE, int PKIND>
__global__ __launch_bounds__(256, 1) void fused_rs_kernel(const FusedArgs a) {
  constexpr int MB = MP / 16, NB = NP / 16;
  constexpr int NB4 = NB / kWaves, MB4 = MB / kWaves;  // output blocks per wave
  static_assert(NB4 % 2 == 0 && MB4 % 2 == 0, "each wave computes whole pairs of blocks");
  constexpr int S1 = (NB4 / 2) * MB, S2 = (MB4 / 2) * NB;  // MFMA steps of a wave's G1 / G2
  constexpr bool kElem = PKIND == PK_ELEM;  // V1: per-sample betas (m, B) of every layer
  __shared__ f32x4 zx[NB * 64];  // Z_k of the 16 columns, block b at zx[b * 64 + lane]
  __shared__ f32x4 vx[MB * 64];  // Var
  __shared__ float red[kWaves][2][16];  // per-wave column partials of the fused objective

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int64_t col = (int64_t)blockIdx.x * 16 + (lane & 15);
  const bool cv = col < a.B;
  const int m = a.m, n = a.n, K = a.K;
  const bool lossz = a.loss_kind != 0;
  const bool lasso = __builtin_amdgcn_readfirstlane(a.loss_kind) == DLADMM_LOSS_LASSO;
  auto lane_off = [&](int64_t ld) -> uint32_t {
    return cv ? (uint32_t)((col + (int64_t)(4 * g) * ld) * 4) : kOOB;
  };
  const int b1o = w * NB4, b2o = w * MB4;  // first output block of this wave in G1 / G2

  float Zr[NB4][4], Er[MB4][4], Lr[MB4][4], Xr[MB4][4];
  {
    const rsrc_t rz = mkrsrc(a.Z0, (uint32_t)(n * a.ldz0 * 4));
    const rsrc_t re = mkrsrc(a.E0, (uint32_t)(m * a.lde0 * 4));
    const rsrc_t rl = mkrsrc(a.L0, (uint32_t)(m * a.ldl0 * 4));
    const rsrc_t rx = mkrsrc(a.X, (uint32_t)(m * a.ldx * 4));
    const uint32_t oz = lane_off(a.ldz0), oe = lane_off(a.lde0), ol = lane_off(a.ldl0),
                   ox = lane_off(a.ldx);
#pragma unroll
    for (int b = 0; b < NB4; ++b) {
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        Zr[b][r] = bload(rz, oz + (uint32_t)((16 * (b1o + b) + r) * a.ldz0 * 4));
        v[r] = Zr[b][r];
      }
      zx[(b1o + b) * 64 + lane] = v;
    }
#pragma unroll
    for (int b = 0; b < MB4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t ro = (uint32_t)(16 * (b2o + b) + r);
        Xr[b][r] = bload(rx, ox + ro * (uint32_t)(a.ldx * 4));
        Er[b][r] = bload(re, oe + ro * (uint32_t)(a.lde0 * 4));
        Lr[b][r] = bload(rl, ol + ro * (uint32_t)(a.ldl0 * 4));
      }
  }

  // uniform per-layer scalars, as the fused kernel's layer_params (k = -1: the prologue)
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

  float regsum = 0.f, fit1 = 0.f, fit2 = 0.f;  // this wave's rows of the layer's objective
  // V1: per-element betas of the G2 epilogue rows (b3 = beta1_k, b2 = beta2_k, b1n = beta1_k+1),
  // loaded at the start of the pass (scalar-loaded layer pointers, as the fused kernel)
  float pb[kElem ? MB4 : 1][3][4];
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
      for (int b = 0; b < MB4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t so = (uint32_t)(16 * (b2o + b) + r) * (uint32_t)(a.ldb * 4);
          pb[b][0][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r1, (int)vb, (int)so, 0));
          pb[b][1][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r2, (int)vb, (int)so, 0));
          pb[b][2][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rn, (int)vb, (int)so, 0));
        }
    }
  };
  // the layer's per-column objective (fused kernel: flush_loss): each wave's quarter of the rows
  // summed over its lane groups, then the 4 quarters in wave order by wave 0 after the barrier
  auto stage_loss = [&]() {
    const float rs_ = col_sum(regsum), fs = col_sum(lasso ? fit2 : fit1);
    if (g == 0) {
      red[w][0][lane] = rs_;
      red[w][1][lane] = fs;
    }
    regsum = fit1 = fit2 = 0.f;
  };
  auto flush_loss = [&](int k) {  // after the barrier that follows stage_loss
    if (w == 0 && g == 0) {
      float r0 = red[0][0][lane], f0 = red[0][1][lane];
#pragma unroll
      for (int q = 1; q < kWaves; ++q) {
        r0 += red[q][0][lane];
        f0 += red[q][1][lane];
      }
      a.lossp[(int64_t)(2 * k + 0) * a.ldl + col] = r0;
      a.lossp[(int64_t)(2 * k + 1) * a.ldl + col] = lasso ? 0.5f * f0 : f0;
    }
  };

  const uint32_t vo = lane_off(a.ldo);
  const uint32_t ld4 = (uint32_t)(a.ldo * 4);
  const uint32_t zbytes = (uint32_t)(n * a.ldo * 4), mbytes = (uint32_t)(m * a.ldo * 4);
  const int64_t wl = (int64_t)MB * NB * kFrag;  // floats per packed weight
  const uint32_t vf = (uint32_t)(lane * 16);    // lane offset inside a 1-KiB fragment
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

  // fragment pair of step s of this wave's pass.  Pack order 2 puts output pair P's k-block kb at
  // fragments 2 (P KB + kb) + h, so a wave's pairs are one contiguous run: its buffer view starts
  // at its first pair, and step s reads fragments 2s, 2s + 1 (compile-time offsets)
  auto frag2 = [&](rsrc_t r, auto S_, f32x4& fa, f32x4& fb) {
    constexpr int s = decltype(S_)::value;
    fa = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)vf, 2 * s * 1024, 0));
    fb = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)vf, (2 * s + 1) * 1024, 0));
  };
  // byte offset of row 16 b + r of a [rows][ldo] output (an opaque base, so the per-block values
  // are formed where they are used rather than all kept live across the layer loop)
  auto row_off = [&](int b, int r) -> uint32_t {
    uint32_t o = (uint32_t)(16 * b) * ld4;
    asm volatile("" : "+s"(o));
    return o + (uint32_t)r * ld4;
  };

  // G1(k): this wave's Z blocks; Var (all m rows) from vx
  auto g1_pass = [&](int k, const LayerP& P, rsrc_t rzo) {
    const float* wk = a.Wp + (int64_t)(k * a.wstep) * wl + (int64_t)(b1o / 2) * MB * 2 * kFrag;
    const rsrc_t rw = mkrsrc(wk, (uint32_t)(S1 * 2 * kFrag * 4));
    f32x4 fa[RS_PF], fb[RS_PF];
    static_for<RS_PF>([&](auto I_) {
      constexpr int i = decltype(I_)::value;
      if constexpr (i < S1) frag2(rw, I_, fa[i], fb[i]);
    });
    static_for<NB4 / 2>([&](auto P_) {
      constexpr int pp = decltype(P_)::value;
      f32x4 ca = zero4, cb = zero4;
      static_for<MB>([&](auto J_) {
        constexpr int jb = decltype(J_)::value;
        constexpr int s = pp * MB + jb;
        const f32x4 v = vx[jb * 64 + lane];
        const f32x4 wa = fa[s % RS_PF], wb = fb[s % RS_PF];
        if constexpr (s + RS_PF < S1)
          frag2(rw, std::integral_constant<int, s + RS_PF>{}, fa[s % RS_PF], fb[s % RS_PF]);
        ca = mfma4(wa.x, v[0], ca);
        cb = mfma4(wb.x, v[0], cb);
        ca = mfma4(wa.y, v[1], ca);
        cb = mfma4(wb.y, v[1], cb);
        ca = mfma4(wa.z, v[2], ca);
        cb = mfma4(wb.z, v[2], cb);
        ca = mfma4(wa.w, v[3], ca);
        cb = mfma4(wb.w, v[3], cb);
      });
      // Z = S(Z - s1*(W_k Var), theta_z): the fused kernel's epi1_row
      static_for<2>([&](auto H_) {
        constexpr int h = decltype(H_)::value;
        constexpr int lb = 2 * pp + h;
        const f32x4 q = h ? cb : ca;
        f32x4 zv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float u = (PKIND == PK_S1) ? Zr[lb][r] + P.s1 * q[r] : Zr[lb][r] + q[r];
          const float z = shrink_u(u, P.thz);
          Zr[lb][r] = z;
          zv[r] = z;
          bstore_s(rzo, vo, row_off(b1o + lb, r), z);
          regsum += fabsf(z);
        }
        zx[(b1o + lb) * 64 + lane] = zv;
      });
    });
  };

  // G2(k): A Z_k for this wave's E / L / T blocks; Z_k (all n rows) from zx.  PRO: the prologue
  // (T0 = A Z0 + E0 - X; E, L stay E0, L0)
  struct OutR { rsrc_t e, l, t, p; };
  const rsrc_t ra = mkrsrc(a.Ap + (int64_t)(b2o / 2) * NB * 2 * kFrag, (uint32_t)(S2 * 2 * kFrag * 4));
  auto g2_pass = [&](auto PRO_, int k, const LayerP& P, const OutR& O) {
    constexpr bool PRO = decltype(PRO_)::value;
    load_betas(k);
    f32x4 fa[RS_PF], fb[RS_PF];
    static_for<RS_PF>([&](auto I_) {
      constexpr int i = decltype(I_)::value;
      if constexpr (i < S2) frag2(ra, I_, fa[i], fb[i]);
    });
    static_for<MB4 / 2>([&](auto P_) {
      constexpr int pp = decltype(P_)::value;
      f32x4 ca = zero4, cb = zero4, ca2 = zero4, cb2 = zero4;
      static_for<NB>([&](auto K_) {
        constexpr int kb = decltype(K_)::value;
        constexpr int s = pp * NB + kb;
        const f32x4 z = zx[kb * 64 + lane];
        const f32x4 wa = fa[s % RS_PF], wb = fb[s % RS_PF];
        if constexpr (s + RS_PF < S2)
          frag2(ra, std::integral_constant<int, s + RS_PF>{}, fa[s % RS_PF], fb[s % RS_PF]);
        ca = mfma4(wa.x, z[0], ca);
        cb = mfma4(wb.x, z[0], cb);
        ca2 = mfma4(wa.y, z[1], ca2);
        cb2 = mfma4(wb.y, z[1], cb2);
        ca = mfma4(wa.z, z[2], ca);
        cb = mfma4(wb.z, z[2], cb);
        ca2 = mfma4(wa.w, z[3], ca2);
        cb2 = mfma4(wb.w, z[3], cb2);
      });
      const f32x4 qa = ca + ca2, qb = cb + cb2;
      // the fused kernel's epi2_row (scalar parameters)
      static_for<2>([&](auto H_) {
        constexpr int h = decltype(H_)::value;
        constexpr int lb = 2 * pp + h;
        const f32x4 q = h ? qb : qa;
        f32x4 vv4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float Pv = q[r], x = Xr[lb][r];
          const float l0 = Lr[lb][r], e0 = Er[lb][r];
          float b2 = P.b2, b3 = P.b3, b1n = P.b1n;
          if constexpr (kElem) {
            b3 = pb[lb][0][r];
            b2 = pb[lb][1][r];
            b1n = pb[lb][2][r];
          }
          float e;
          if constexpr (EMODE == EM_V1) {
            // E = S(X - A Z - b2*L, theta_e)                      main_lena.py:87
            const float u = (x - Pv) - b2 * l0;
            e = shrink_u(u, P.the);
          } else if constexpr (EMODE == EM_VVAR) {
            // VVar = L + b2*(A Z + E - X); E = S(E - ss2*VVar)    main_syn_l1l1_scalar.py:114-115
            const float vv = l0 + b2 * ((Pv + e0) - x);
            e = shrink_u(e0 - P.ss2 * vv, P.the);
          } else {
            // E = ss2_1*(X - A Z) - ss2_2*L                       main_syn_lasso_scalar.py:102-103
            e = P.ss2 * (x - Pv) - P.ss2b * l0;
          }
          e = PRO ? e0 : e;
          const float t = (Pv + e) - x;
          float l = l0 + b3 * t;
          l = PRO ? l0 : l;
          Er[lb][r] = e;
          Lr[lb][r] = l;
          const uint32_t so = row_off(b2o + lb, r);
          bstore_s(O.e, vo, so, e);
          bstore_s(O.l, vo, so, l);
          bstore_s(O.t, vo, so, t);
          bstore_s(O.p, vo, so, Pv);  // training forwards: A Z_k for the backward
          const float res = x - Pv;
          fit1 += fabsf(res);                       // |X - A Z|
          fit2 = __builtin_fmaf(res, res, fit2);    // (X - A Z)^2
          vv4[r] = l + b1n * t;  // Var of the next layer: L + b1*T
        }
        vx[(b2o + lb) * 64 + lane] = vv4;
      });
    });
  };

  const rsrc_t none = mkrsrc(nullptr, 0u);
  __syncthreads();  // every wave's Z0 blocks are in zx
  {
    const OutR Op{none, none,
                  mkrsrc(a.keep_all ? a.To : nullptr, (a.keep_all && a.To) ? mbytes : 0u), none};
    g2_pass(std::true_type{}, -1, layer_params(-1), Op);
  }
  regsum = fit1 = fit2 = 0.f;  // the prologue's sums are not an objective
  __syncthreads();  // Var_0 complete
  for (int k = 0; k < K; ++k) {
    const bool st = a.keep_all || k == K - 1;
    const int ko = a.keep_all ? k : 0;
    const LayerP P = layer_params(k);
    g1_pass(k, P, mkrsrc(a.Zo + (int64_t)ko * n * a.ldo, st ? zbytes : 0u));
    __syncthreads();  // Z_k complete; every wave is done reading Var_k
    const OutR O{mkrsrc(a.Eo + (int64_t)ko * m * a.ldo, st ? mbytes : 0u),
                 mkrsrc(a.Lo + (int64_t)ko * m * a.ldo, st ? mbytes : 0u),
                 mkrsrc(a.To ? a.To + (int64_t)(a.keep_all ? k + 1 : 0) * m * a.ldo : nullptr,
                        (a.To && st) ? mbytes : 0u),
                 mkrsrc(a.Po && a.keep_all ? a.Po + (int64_t)k * m * a.ldo : nullptr,
                        a.Po && a.keep_all ? mbytes : 0u)};
    g2_pass(std::false_type{}, k, P, O);
    if (lossz) stage_loss();
    __syncthreads();  // Var_{k+1} complete; every wave is done reading Z_k
    if (lossz) flush_loss(k);
  }
}

template <int MP, int NP, int EM, int PK>
hipError_t launch_rs(const FusedArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((fused_rs_kernel<MP, NP, EM, PK>), dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

bool rs_supports(int shape, int variant) {
  return shape == 2 && (variant == DLADMM_V1_LENA || variant == DLADMM_V4_SCALAR ||
                        variant == DLADMM_V5_TIED || variant == DLADMM_V6_LASSO);
}

hipError_t launch_fused_rs(int shape, int variant, const FusedArgs& a, int grid, hipStream_t s) {
  if (shape != 2) return hipErrorInvalidValue;
  constexpr int MP = kShapeMP[2], NP = kShapeNP[2];
  switch (variant) {
    case DLADMM_V1_LENA: return launch_rs<MP, NP, EM_V1, PK_ELEM>(a, grid, s);
    case DLADMM_V4_SCALAR: return launch_rs<MP, NP, EM_VVAR, PK_SCALAR>(a, grid, s);
    case DLADMM_V5_TIED: return launch_rs<MP, NP, EM_VVAR, PK_S1>(a, grid, s);
    case DLADMM_V6_LASSO: return launch_rs<MP, NP, EM_LASSO, PK_SCALAR>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace dladmm
