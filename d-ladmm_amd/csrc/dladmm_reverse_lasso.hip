// dladmm_reverse_lasso.hip -- reverse-sweep instantiations: E-step form EM_LASSO, the 256 x 512
// shape (dladmm_reverse_kernel.h; dispatch: dladmm_reverse.hip).
#include "dladmm_reverse_kernel.h"

namespace dladmm {

hipError_t launch_rev_lasso_s2(const RevArgs& a, int grid, hipStream_t s) {
  return launch_rev<kShapeMP[2], kShapeNP[2], EM_LASSO>(a, grid, s);
}

}  // namespace dladmm
