// dladmm_fused_x3.hip -- instantiations of the split-f16 fused forward (dladmm_fused_x3_kernel.h),
// inference form, and the variant support query of the C ABI plan.
#include "dladmm_fused_x3_kernel.h"

namespace dladmm {

bool x3_supports(int variant) {
  return variant == DLADMM_V4_SCALAR || variant == DLADMM_V5_TIED ||
         variant == DLADMM_V6_LASSO || variant == DLADMM_V1_LENA;
}

hipError_t launch_fused_x3_shape(int shape, int variant, const FusedArgs& a, int grid,
                                 hipStream_t s) {
  return launch_x3_shape<false>(shape, variant, a, grid, s);
}

}  // namespace dladmm
