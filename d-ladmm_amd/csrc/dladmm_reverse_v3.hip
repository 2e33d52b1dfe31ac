// dladmm_reverse_v3.hip -- reverse-sweep instantiations: V3 (main_syn_l1l1_full.py), per-row parameters,
// E-step form EM_VVAR, the 256 x 512 shape (dladmm_reverse_kernel.h; dispatch: dladmm_reverse.hip).
#include "dladmm_reverse_kernel.h"

namespace dladmm {

hipError_t launch_rev_v3_s2(const RevArgs& a, int grid, hipStream_t s) {
  return launch_rev<kShapeMP[2], kShapeNP[2], EM_VVAR, true>(a, grid, s);
}

}  // namespace dladmm
