// dladmm_fused_x3_savep.hip -- instantiations of the split-f16 fused forward that also store
// P_k = A Z_k for the backward (training forwards, include/dladmm.h fwd_desc.P).
#include "dladmm_fused_x3_kernel.h"

namespace dladmm {

hipError_t launch_fused_x3_shape_savep(int shape, int variant, const FusedArgs& a, int grid,
                                       hipStream_t s) {
  return launch_x3_shape<true>(shape, variant, a, grid, s);
}

}  // namespace dladmm
