// dladmm_fused.hip -- instantiations of the fused K-layer forward (inference form).
// The kernel template and its design notes: dladmm_fused_kernel.h.
#include "dladmm_fused_kernel.h"

namespace dladmm {

template <int MP, int NP>
hipError_t dispatch_variant(int variant, const FusedArgs& a, int grid, hipStream_t s) {
  switch (variant) {
    case DLADMM_V1_LENA: return launch_fused<MP, NP, EM_V1, PK_ELEM, false>(a, grid, s);
    case DLADMM_V2_LTHETA: return launch_fused<MP, NP, EM_V1, PK_ROW, false>(a, grid, s);
    case DLADMM_V3_FULL: return launch_fused<MP, NP, EM_VVAR, PK_ROW, false>(a, grid, s);
    case DLADMM_V4_SCALAR: return launch_fused<MP, NP, EM_VVAR, PK_SCALAR, false>(a, grid, s);
    case DLADMM_V5_TIED: return launch_fused<MP, NP, EM_VVAR, PK_S1, false>(a, grid, s);
    case DLADMM_V6_LASSO: return launch_fused<MP, NP, EM_LASSO, PK_SCALAR, false>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_fused_shape(int shape, int variant, const FusedArgs& a, int grid,
                              hipStream_t s) {
  switch (shape) {
    case 0: return dispatch_variant<kShapeMP[0], kShapeNP[0]>(variant, a, grid, s);
    case 1: return dispatch_variant<kShapeMP[1], kShapeNP[1]>(variant, a, grid, s);
    case 2: return dispatch_variant<kShapeMP[2], kShapeNP[2]>(variant, a, grid, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace dladmm
