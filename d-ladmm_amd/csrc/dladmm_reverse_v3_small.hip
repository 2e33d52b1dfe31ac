// dladmm_reverse_v3_small.hip -- reverse-sweep instantiations: V3 (main_syn_l1l1_full.py), per-row
// parameters, E-step form EM_VVAR, the two small shapes (dladmm_reverse_kernel.h; dispatch:
// dladmm_reverse.hip).
#include "dladmm_reverse_kernel.h"

namespace dladmm {

hipError_t launch_rev_v3_s01(int shape, const RevArgs& a, int grid, hipStream_t s) {
  if (shape == 0) return launch_rev<kShapeMP[0], kShapeNP[0], EM_VVAR, true>(a, grid, s);
  return launch_rev<kShapeMP[1], kShapeNP[1], EM_VVAR, true>(a, grid, s);
}

}  // namespace dladmm
