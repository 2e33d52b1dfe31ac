// dladmm_layer_epi.h -- the per-element epilogue of the per-layer forward kernels, shared by the
// one-dimensional slice kernels (dladmm_layered.hip) and the bf16 2-D tile kernel
// (dladmm_tile_bf16.hip).  One call finishes one output element (row, col) of the layer's
// product `accv` and returns the state value the NEXT product consumes as its B operand:
//   PH 0 (G1)  Z_k = S(Z_{k-1} - s1 * (W_k Var_k), theta_z)                  -> Z_k
//   PH 1 (G2)  E_k, L_k, T_{k+1} from P = A Z_k; Var_{k+1} = L_k + b1 T_{k+1} -> Var_{k+1}
//   PH 2       T_0 = A Z0 + E0 - X, Var_0 = L0 + b1 T_0 (main_lena.py:70, :85) -> Var_0
// (reference lines cited at each formula).  Invalid elements (row or column out of range) store
// nothing and return 0, which is exactly the zero padding the packed B operand needs.
#pragma once

#include "dladmm_common.h"
#include "dladmm_internal.h"

namespace dladmm {

#ifndef DLADMM_EPI_NT
#define DLADMM_EPI_NT 0  // non-temporal (nt) epilogue stores, by output: 1 Z, 2 E and L, 4 T
#endif
#ifndef DLADMM_EPI_ABL
#define DLADMM_EPI_ABL 0  // timing experiments only (WRONG results): 1 no fp32 output stores,
                          // 2 no operand loads (constants instead)
#endif
template <int WHICH>
__device__ __forceinline__ void epi_store(float* p, float v) {
  if constexpr (DLADMM_EPI_ABL & 1) asm volatile("" ::"v"(v));
  else if constexpr ((DLADMM_EPI_NT & WHICH) != 0) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int EMODE, int PKIND, int PH>
struct LayerEpi {
  const LayerArgs& a;
  bool lasso;
  cfloat_p sp, spn;
  const float* rp;
  const float* rpn;

  __device__ __forceinline__ explicit LayerEpi(const LayerArgs& a_) : a(a_) {
    const int k = a.k;
    lasso = a.loss_kind == DLADMM_LOSS_LASSO;
    sp = (cfloat_p)a.scal + (k < 0 ? 0 : k) * DLADMM_NSCALAR;
    spn = (cfloat_p)a.scal + (k + 1 < a.K ? k + 1 : (k < 0 ? 0 : k)) * DLADMM_NSCALAR;
    rp = a.rowp ? a.rowp + (int64_t)(k < 0 ? 0 : k) * 8 * a.rstride : nullptr;
    rpn = a.rowp ? a.rowp + (int64_t)(k + 1 < a.K ? k + 1 : 0) * 8 * a.rstride : nullptr;
  }
  __device__ __forceinline__ float prow(const float* base, int slot, int row) const {
    return base[(int64_t)slot * a.rstride + row];
  }

  // The epilogue runs in two passes over a batch of elements: load() gathers every input of an
  // element (its loads only), finish() computes and stores.  Issuing a whole batch's loads
  // before its first store matters: the compiler cannot move a load above a store it may alias,
  // so element-by-element code would pay one full memory round trip per element.
  struct In {
    float zp, thz;               // PH 0
    float x, e0, l0, b2, b3, b1n;  // PH 1 / 2
  };
  __device__ __forceinline__ In load(int row, bool cv, int64_t colc) const {
    In v{};
    if constexpr (DLADMM_EPI_ABL & 2) {
      v.zp = 0.25f; v.thz = 0.1f; v.x = 0.5f; v.e0 = 0.125f; v.l0 = 0.0625f;
      v.b2 = 1.f; v.b3 = 1.f; v.b1n = 1.f;
      asm volatile("" : "+v"(v.zp), "+v"(v.x), "+v"(v.e0), "+v"(v.l0));
      return v;
    }
    const int k = a.k;
    if constexpr (PH == 0) {
      const bool ok = cv && row < a.n;
      const int rowc = ok ? row : 0;
      v.zp = a.Zprev[(int64_t)rowc * a.ldzp + colc];
      v.thz = (PKIND == PK_ROW) ? prow(rp, DLADMM_P_THETA_Z, rowc) : sp[DLADMM_P_THETA_Z];
    } else {
      const bool ok = cv && row < a.m;
      const int rowc = ok ? row : 0;
      v.x = a.X[(int64_t)rowc * a.ldx + colc];
      v.e0 = a.Eprev[(int64_t)rowc * a.ldep + colc];
      v.l0 = a.Lprev[(int64_t)rowc * a.ldlp + colc];
      if constexpr (PH == 1) {
        auto pm = [&](int slot) -> float {
          return (PKIND == PK_ROW) ? prow(rp, slot, rowc) : sp[slot];
        };
        if constexpr (EMODE == EM_V1)
          v.b2 = (PKIND == PK_ELEM) ? a.b2e[(int64_t)rowc * a.ldb + colc] : pm(DLADMM_P_BETA2);
        v.b3 = (PKIND == PK_ELEM) ? a.b1e[(int64_t)rowc * a.ldb + colc] : pm(DLADMM_P_BETA3);
      }
      if constexpr (PKIND == PK_ELEM) v.b1n = a.b1n_e ? a.b1n_e[(int64_t)rowc * a.ldb + colc] : 0.f;
      else if constexpr (PKIND == PK_ROW) v.b1n = prow(rpn, DLADMM_P_BETA1, rowc);
      else v.b1n = (k < 0) ? sp[DLADMM_P_BETA1] : spn[DLADMM_P_BETA1];
    }
    return v;
  }

  // lsum accumulates this element's objective term (|Z_k| for PH 0, |X - P| or (X - P)^2 for
  // PH 1; nothing for PH 2)
  __device__ __forceinline__ float finish(int row, int64_t col, bool cv, const In& v, float accv,
                                          float& lsum) const {
    if constexpr (PH == 0) {
      const bool ok = cv && row < a.n;
      float u = accv;
      if constexpr (PKIND == PK_SCALAR) u = sp[DLADMM_P_S1] * u;
      const float z = shrink(v.zp - u, v.thz);                        // main_lena.py:79-80
      if (ok) epi_store<1>(a.Zo + (int64_t)row * a.ldo + col, z);
      lsum += ok ? fabsf(z) : 0.0f;
      return ok ? z : 0.0f;
    } else {
      const bool ok = cv && row < a.m;
      const int rowc = ok ? row : 0;
      const float P = accv;
      const float x = v.x, e0 = v.e0, l0 = v.l0;
      float t, l;
      if constexpr (PH == 2) {
        t = (P + e0) - x;  // T0 = A Z0 + E0 - X   main_lena.py:70
        l = l0;
      } else {
        float e;
        auto pm = [&](int slot) -> float {
          return (PKIND == PK_ROW) ? prow(rp, slot, rowc) : sp[slot];
        };
        if constexpr (EMODE == EM_V1) {
          e = shrink((x - P) - v.b2 * l0, pm(DLADMM_P_THETA_E));        // main_lena.py:87
        } else if constexpr (EMODE == EM_VVAR) {
          const float vv = l0 + pm(DLADMM_P_BETA2) * ((P + e0) - x);     // scalar :114
          e = shrink(e0 - pm(DLADMM_P_SS2) * vv, pm(DLADMM_P_THETA_E));  // scalar :115
        } else {
          e = pm(DLADMM_P_SS2) * (x - P) - pm(DLADMM_P_SS2B) * l0;        // lasso :102-103
        }
        t = (P + e) - x;                                                   // main_lena.py:88
        l = l0 + v.b3 * t;                                                 // main_lena.py:89
        if (ok) {
          epi_store<2>(a.Eo + (int64_t)row * a.ldo + col, e);
          epi_store<2>(a.Lo + (int64_t)row * a.ldo + col, l);
        }
        const float res = x - P;
        lsum += ok ? (lasso ? res * res : fabsf(res)) : 0.0f;
      }
      if (ok && a.To) epi_store<4>(a.To + (int64_t)row * a.ldo + col, t);
      const float var = l + v.b1n * t;                      // Var_{k+1} = L + b1 T  main_lena.py:85
      if (ok && a.Vo) epi_store<8>(a.Vo + (int64_t)row * a.ldv + col, var);
      return ok ? var : 0.0f;
    }
  }

  __device__ __forceinline__ float operator()(int row, int64_t col, bool cv, int64_t colc,
                                              float accv, float& lsum) const {
    return finish(row, col, cv, load(row, cv, colc), accv, lsum);
  }
};

}  // namespace dladmm
