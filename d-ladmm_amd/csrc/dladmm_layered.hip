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
// (4 rows of the state, this lane's column) is LDS-DMA'd two k-blocks ahead, the A operands
// (packed weights, k-major fragment order) stream through a double-buffered LDS ring by LDS-DMA,
// shared by the NW waves (dladmm_slice.h).  Code size is one k-block of MFMAs, not a whole layer.
#include "dladmm_common.h"
#include "dladmm_internal.h"
#include "dladmm_slice.h"
#include "dladmm_layer_epi.h"

namespace dladmm {

template <int EMODE, int PKIND, int PH, int NW, int SB>
__global__ __launch_bounds__(NW * 64, 8 / NW) void layer_kernel(const LayerArgs a) {
  __shared__ f32x4 ring[slice_lds_f4<NW, 3>()];

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
  slice_gemm<NW, SB, 3>(ring, a.Wp, a.MBp, ib0, a.KB, a.S, a.ldS, a.Krows, a.B, acc);

  // ---------------------------------------------------------------- epilogue
  // units of IB output blocks, software-pipelined: the loads of unit u + 1 are issued before
  // unit u computes and stores (see LayerEpi::load)
  const LayerEpi<EMODE, PKIND, PH> epi(a);
  using In = typename LayerEpi<EMODE, PKIND, PH>::In;
  constexpr int IB = (PH == 0 && PKIND != PK_ROW) ? 4 : 2;
  constexpr int NU = SB / IB;
  float lsum = 0.f;
  In buf[2][IB][4];
  auto load_unit = [&](auto U_) {
    constexpr int u = decltype(U_)::value;
#pragma unroll
    for (int ii = 0; ii < IB; ++ii)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        buf[u & 1][ii][r] = epi.load(16 * (ib0 + u * IB + ii) + 4 * g + r, cv, colc);
  };
  load_unit(std::integral_constant<int, 0>{});
  static_for<NU>([&](auto U_) {
    constexpr int u = decltype(U_)::value;
    if constexpr (u + 1 < NU) load_unit(std::integral_constant<int, u + 1>{});
#pragma unroll
    for (int ii = 0; ii < IB; ++ii)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        epi.finish(16 * (ib0 + u * IB + ii) + 4 * g + r, col, cv, buf[u & 1][ii][r],
                   acc[u * IB + ii][r], lsum);
  });
  if (a.lossp && k >= 0 && !(PH == 2)) {
    // per-column partial over this slice's rows
    const float s = col_sum(lsum);
    if (g == 0) {
      const float v = (PH == 1 && epi.lasso) ? 0.5f * s : s;
      a.lossp[(int64_t)(2 * k + (PH == 0 ? 0 : 1)) * a.nslots + (int64_t)blockIdx.y * a.ldl +
              (int64_t)blockIdx.x * (16 * NW) + w * 16 + (lane & 15)] = v;
    }
  }
}

template <int EM, int PK, int PH>
hipError_t launch_layer_v(const LayerArgs& a, dim3 grid, int sb, hipStream_t s) {
  constexpr int NW = kLayerWaves;
  if (sb == 32)
    hipLaunchKernelGGL((layer_kernel<EM, PK, PH, NW, 32>), grid, dim3(NW * 64), 0, s, a);
  else
    hipLaunchKernelGGL((layer_kernel<EM, PK, PH, NW, 16>), grid, dim3(NW * 64), 0, s, a);
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
