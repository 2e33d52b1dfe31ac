// dladmm_tile_bf16_pair.hip -- the bf16 mode's per-layer products (BASELINE config 5), two phases
// per launch: the batch is split into two column halves that run ONE PHASE APART, and every
// launch carries one layer product of each half -- the G1 (W_k Var_k -> Z_k) tiles of one half
// beside the G2 (A Z_k -> E_k, L_k, T_{k+1}) tiles of the other:
//
//   launch t:   half 0 at phase t,   half 1 at phase t - 1
//   phases:     0 = prologue (A Z0 -> T_0, Var_0), 2k + 1 = G1(k), 2k + 2 = G2(k)
//
// Columns are independent samples, so the two halves of one launch share no data; each phase's
// inputs were completed by an earlier launch (kernel boundaries order them, no in-launch
// hand-off).  Why: a one-phase launch runs all its workgroups through the same main loop and then
// the same HBM-bound epilogue at about the same time, so the matrix cores idle during the
// epilogues and the HBM during the main loops (main loops ~4.1 ms and
// epilogues ~4.0 ms of the 7.1-ms forward overlap by ~1 ms).  Here the blocks of the two halves
// are interleaved in dispatch order, so the two workgroups a CU holds are, most of the time, one
// G2 tile (K = n: a long main loop, a light epilogue) and one G1 tile (K = m: a short main loop,
// the heavy Z epilogue) at unrelated points of their lives.  Every tile is computed by exactly
// the code of the one-phase kernel (tile_body), so the outputs are bit-identical to it.
//
// Dispatch order: the G2-shaped (long) tiles are spread evenly over the first `F` blocks of the
// launch and the rest are G1 tiles, so the long tiles start early and the launch ends on short
// ones (F = total: an even interleave).
#include "dladmm_tile_bf16_body.h"

namespace dladmm {

template <int EMODE, int PKIND, int PH0, int PH1>
__global__ __launch_bounds__(256, 2) void tile_bf16_pair_kernel(const TilePairArgs pa) {
  using G = TileG<4>;
  __shared__ f32x4 ring[G::NST * G::SF * 64];
  constexpr int LH = PH0 != 0 ? 0 : 1;  // the half whose tiles are G2-shaped (long main loop)
  const int b = blockIdx.x;
  const int nL = LH ? pa.n[1] : pa.n[0], F = pa.F;
  int h, i;
  if (b < F) {
    const int q0 = (int)((int64_t)b * nL / F), q1 = (int)((int64_t)(b + 1) * nL / F);
    if (q1 > q0) { h = LH; i = q0; } else { h = 1 - LH; i = b - q0; }
  } else {
    h = 1 - LH;
    i = b - nL;
  }
  h = __builtin_amdgcn_readfirstlane(h);
  i = __builtin_amdgcn_readfirstlane(i);
  // no dynamic index into the kernel argument (it would be copied to scratch and read per lane)
  const int gx = h ? pa.gx[1] : pa.gx[0];
  const int x0 = h ? pa.x0[1] : pa.x0[0];
  // wave-uniform (the DMA source addresses live in SGPRs)
  const int tx = __builtin_amdgcn_readfirstlane(x0 + i % gx);
  const int ty = __builtin_amdgcn_readfirstlane(i / gx);
  if (h == 0) tile_body<EMODE, PKIND, PH0, 4>(pa.a[0], ring, tx, ty);
  else tile_body<EMODE, PKIND, PH1, 4>(pa.a[1], ring, tx, ty);
}

template <int PH0, int PH1>
hipError_t launch_pair_ph(int variant, const TilePairArgs& pa, hipStream_t s) {
  const dim3 grid(pa.n[0] + pa.n[1]), blk(256);
  switch (variant) {
    case DLADMM_V1_LENA:
      hipLaunchKernelGGL((tile_bf16_pair_kernel<EM_V1, PK_ELEM, PH0, PH1>), grid, blk, 0, s, pa); break;
    case DLADMM_V2_LTHETA:
      hipLaunchKernelGGL((tile_bf16_pair_kernel<EM_V1, PK_ROW, PH0, PH1>), grid, blk, 0, s, pa); break;
    case DLADMM_V3_FULL:
      hipLaunchKernelGGL((tile_bf16_pair_kernel<EM_VVAR, PK_ROW, PH0, PH1>), grid, blk, 0, s, pa); break;
    case DLADMM_V4_SCALAR:
    case DLADMM_V5_TIED:
      hipLaunchKernelGGL((tile_bf16_pair_kernel<EM_VVAR, PK_SCALAR, PH0, PH1>), grid, blk, 0, s, pa); break;
    case DLADMM_V6_LASSO:
      hipLaunchKernelGGL((tile_bf16_pair_kernel<EM_LASSO, PK_SCALAR, PH0, PH1>), grid, blk, 0, s, pa); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_tile_bf16_pair(int ph0, int ph1, int variant, const TilePairArgs& pa,
                                 hipStream_t s) {
  if (pa.n[0] + pa.n[1] == 0) return hipSuccess;
  if (ph0 == 0 && ph1 == 2) return launch_pair_ph<0, 2>(variant, pa, s);
  if (ph0 == 1 && ph1 == 0) return launch_pair_ph<1, 0>(variant, pa, s);
  if (ph0 == 0 && ph1 == 1) return launch_pair_ph<0, 1>(variant, pa, s);
  if (ph0 == 2 && ph1 == 0) return launch_pair_ph<2, 0>(variant, pa, s);
  return hipErrorInvalidValue;
}

}  // namespace dladmm
