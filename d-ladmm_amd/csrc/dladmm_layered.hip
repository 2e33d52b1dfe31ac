// dladmm_layered.hip -- per-layer D-LADMM kernels for shapes beyond the fused kernel's register
// budget (BASELINE config 4: LASSO m=512, n=2048, K=40; any m > 256 or n > 512).
//
// The per-column state no longer fits on chip (Z alone is n floats per column), so each layer is
// two GEMM kernels whose epilogues carry the whole elementwise part of the reference layer:
//   G1(k):  U = W_k * Var      -> Z_k = S(Z_{k-1} - s1*U, theta_z)          main_lena.py:85-86
//   G2(k):  P = A * Z_k        -> E_k, T_{k+1} = (P + E_k) - X, L_k, Var_{k+1} main_lena.py:87-89
//   G2(-1): P = A * Z0         -> T_0 = (P + E0) - X, Var_0                   main_lena.py:70-71
// so the reference's ~10 elementwise sweeps and its duplicated A*Z per layer disappear; HBM sees
// each state tensor read once and written once per layer (compute-bound: ~100 FLOP/B).
//
// Kernel geometry: a workgroup of NW waves owns 16*NW batch columns and a slice of SB output
// blocks (16*SB rows); wave w owns 16 columns and keeps the slice's SB 16x16 accumulators
// (4*SB registers).  The contraction runs as a RUNTIME loop over k-blocks of 16: the B operand
// (4 rows of the state, this lane's column) is loaded straight from HBM two k-blocks ahead, the
// A operands (packed weights, k-major fragment order) stream through a double-buffered LDS ring
// by LDS-DMA, shared by the NW waves.  Code size is one k-block of MFMAs, not a whole layer.
#include "dladmm_common.h"
#include "dladmm_internal.h"
#include "dladmm_slice.h"

namespace dladmm {

template <int EMODE, int PKIND, int PH, int NW, int SB, int BF16>
__global__ __launch_bounds__(NW * 64, 8 / NW) void layer_kernel(const LayerArgs a) {
  // fp32: 16-fragment chunks; bf16 (BASELINE config 5): one k-block of SB fragments per chunk
  __shared__ f32x4 ring[2 * (BF16 ? SB : kSliceCF) * 64];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int64_t col = (int64_t)blockIdx.x * (16 * NW) + w * 16 + (lane & 15);
  const bool cv = col < a.B;
  const int64_t colc = cv ? col : 0;
  const int ib0 = blockIdx.y * SB;  // first output block of this slice
  const int k = a.k;

  f32x4 acc[SB];
  if constexpr (BF16)
    slice_gemm_bf16<NW, SB>(ring, a.Wp, a.MBp, ib0, a.KB, a.S, a.ldS, a.Krows, colc, cv, acc);
  else
    slice_gemm<NW, SB>(ring, a.Wp, a.MBp, ib0, a.KB, a.S, a.ldS, a.Krows, colc, cv, acc);

  // ---------------------------------------------------------------- epilogue
  const bool lasso = a.loss_kind == DLADMM_LOSS_LASSO;
  float lsum = 0.f;
  cfloat_p sp = (cfloat_p)a.scal + (k < 0 ? 0 : k) * DLADMM_NSCALAR;
  cfloat_p spn = (cfloat_p)a.scal + (k + 1 < a.K ? k + 1 : (k < 0 ? 0 : k)) * DLADMM_NSCALAR;
  const float* rp = a.rowp ? a.rowp + (int64_t)(k < 0 ? 0 : k) * 8 * a.rstride : nullptr;
  const float* rpn = a.rowp ? a.rowp + (int64_t)(k + 1 < a.K ? k + 1 : 0) * 8 * a.rstride
                            : nullptr;
  auto prow = [&](const float* base, int slot, int row) -> float {  // per-row param
    return base[(int64_t)slot * a.rstride + row];
  };
  static_for<SB>([&](auto I_) {
    constexpr int i = decltype(I_)::value;
    static_for<4>([&](auto R_) {
      constexpr int r = decltype(R_)::value;
      const int row = 16 * (ib0 + i) + 4 * g + r;
      const float accv = acc[i][r];
      if constexpr (PH == 0) {
        // G1: Z_k = S(Z_{k-1} - s1*U, theta_z)
        const bool ok = cv && row < a.n;
        const int rowc = ok ? row : 0;
        float u = accv;
        if constexpr (PKIND == PK_SCALAR) u = sp[DLADMM_P_S1] * u;
        const float thz = (PKIND == PK_ROW) ? prow(rp, DLADMM_P_THETA_Z, rowc)
                                            : sp[DLADMM_P_THETA_Z];
        const float zp = a.Zprev[(int64_t)rowc * a.ldzp + colc];
        const float z = shrink(zp - u, thz);
        if (ok) a.Zo[(int64_t)row * a.ldo + col] = z;
        lsum += ok ? fabsf(z) : 0.0f;
      } else {
        const bool ok = cv && row < a.m;
        const int rowc = ok ? row : 0;
        const float P = accv;
        const float x = a.X[(int64_t)rowc * a.ldx + colc];
        const float e0 = a.Eprev[(int64_t)rowc * a.ldep + colc];
        const float l0 = a.Lprev[(int64_t)rowc * a.ldlp + colc];
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
            const float b2 = (PKIND == PK_ELEM) ? a.b2e[(int64_t)rowc * a.ldb + colc]
                                                : pm(DLADMM_P_BETA2);
            e = shrink((x - P) - b2 * l0, pm(DLADMM_P_THETA_E));          // main_lena.py:87
          } else if constexpr (EMODE == EM_VVAR) {
            const float vv = l0 + pm(DLADMM_P_BETA2) * ((P + e0) - x);     // scalar :114
            e = shrink(e0 - pm(DLADMM_P_SS2) * vv, pm(DLADMM_P_THETA_E));  // scalar :115
          } else {
            e = pm(DLADMM_P_SS2) * (x - P) - pm(DLADMM_P_SS2B) * l0;        // lasso :102-103
          }
          t = (P + e) - x;                                                   // main_lena.py:88
          const float b3 = (PKIND == PK_ELEM) ? a.b1e[(int64_t)rowc * a.ldb + colc]
                                              : pm(DLADMM_P_BETA3);
          l = l0 + b3 * t;                                                   // main_lena.py:89
          if (ok) {
            a.Eo[(int64_t)row * a.ldo + col] = e;
            a.Lo[(int64_t)row * a.ldo + col] = l;
          }
          const float res = x - P;
          lsum += ok ? (lasso ? res * res : fabsf(res)) : 0.0f;
        }
        if (ok && a.To) a.To[(int64_t)row * a.ldo + col] = t;
        // Var of layer k+1 = L + b1*T (main_lena.py:85)
        float b1n;
        if constexpr (PKIND == PK_ELEM) b1n = a.b1n_e ? a.b1n_e[(int64_t)rowc * a.ldb + colc] : 0.f;
        else if constexpr (PKIND == PK_ROW) b1n = prow(rpn, DLADMM_P_BETA1, rowc);
        else b1n = (k < 0) ? sp[DLADMM_P_BETA1] : spn[DLADMM_P_BETA1];
        if (ok) a.Vo[(int64_t)row * a.ldv + col] = l + b1n * t;
      }
    });
  });
  if (a.lossp && k >= 0 && !(PH == 2)) {
    // per-column partial over this slice's rows
    const float s = col_sum(lsum);
    if (g == 0) {
      const float v = (PH == 1 && lasso) ? 0.5f * s : s;
      a.lossp[(int64_t)(2 * k + (PH == 0 ? 0 : 1)) * a.nslots + (int64_t)blockIdx.y * a.ldl +
              (int64_t)blockIdx.x * (16 * NW) + w * 16 + (lane & 15)] = v;
    }
  }
}

template <int EM, int PK, int PH>
hipError_t launch_layer_v(const LayerArgs& a, dim3 grid, int sb, hipStream_t s) {
  constexpr int NW = kLayerWaves;
  if (sb == -32)  // bf16 operands (config 5)
    hipLaunchKernelGGL((layer_kernel<EM, PK, PH, NW, 32, 1>), grid, dim3(NW * 64), 0, s, a);
  else if (sb == 32)
    hipLaunchKernelGGL((layer_kernel<EM, PK, PH, NW, 32, 0>), grid, dim3(NW * 64), 0, s, a);
  else
    hipLaunchKernelGGL((layer_kernel<EM, PK, PH, NW, 16, 0>), grid, dim3(NW * 64), 0, s, a);
  return hipGetLastError();
}

template <int PH>
hipError_t launch_layer_ph(int variant, const LayerArgs& a, dim3 grid, int sb, hipStream_t s) {
  switch (variant) {
    case DLADMM_V1_LENA: return launch_layer_v<EM_V1, PK_ELEM, PH>(a, grid, sb, s);
    case DLADMM_V2_LTHETA: return launch_layer_v<EM_V1, PK_ROW, PH>(a, grid, sb, s);
    case DLADMM_V3_FULL: return launch_layer_v<EM_VVAR, PK_ROW, PH>(a, grid, sb, s);
    case DLADMM_V4_SCALAR:
    case DLADMM_V5_TIED: return launch_layer_v<EM_VVAR, PK_SCALAR, PH>(a, grid, sb, s);
    case DLADMM_V6_LASSO: return launch_layer_v<EM_LASSO, PK_SCALAR, PH>(a, grid, sb, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_layer(int phase, int variant, const LayerArgs& a, dim3 grid, int sb,
                        hipStream_t s) {
  switch (phase) {
    case 0: return launch_layer_ph<0>(variant, a, grid, sb, s);
    case 1: return launch_layer_ph<1>(variant, a, grid, sb, s);
    case 2: return launch_layer_ph<2>(variant, a, grid, sb, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace dladmm
