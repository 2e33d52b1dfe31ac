// dladmm_reverse_v2.hip -- reverse-sweep instantiations: V2 (main_syn_l1l1_ltheta.py), per-row parameters,
// E-step form EM_V1, the 256 x 512 shape (dladmm_reverse_kernel.h; dispatch: dladmm_reverse.hip).
#include "dladmm_reverse_kernel.h"

namespace dladmm {

hipError_t launch_rev_v2_s2(const RevArgs& a, int grid, hipStream_t s) {
  return launch_rev<kShapeMP[2], kShapeNP[2], EM_V1, true>(a, grid, s);
}

}  // namespace dladmm
