// dladmm_reverse_v2_small.hip -- reverse-sweep instantiations: V2 (main_syn_l1l1_ltheta.py), per-row
// parameters, E-step form EM_V1, the two small shapes (dladmm_reverse_kernel.h; dispatch:
// dladmm_reverse.hip).
#include "dladmm_reverse_kernel.h"

namespace dladmm {

hipError_t launch_rev_v2_s01(int shape, const RevArgs& a, int grid, hipStream_t s) {
  if (shape == 0) return launch_rev<kShapeMP[0], kShapeNP[0], EM_V1, true>(a, grid, s);
  return launch_rev<kShapeMP[1], kShapeNP[1], EM_V1, true>(a, grid, s);
}

}  // namespace dladmm
