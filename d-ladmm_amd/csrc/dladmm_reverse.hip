// dladmm_reverse.hip -- dispatch of the reverse-sweep backward (dladmm_reverse_kernel.h) to its
// instantiations: one translation unit per E-step form for the 256 x 512 shape and one for the
// two small shapes (dladmm_reverse_{v1,vvar,lasso}[_small].hip).
#include "dladmm_common.h"
#include "dladmm_internal.h"

namespace dladmm {

// defined by the instantiation units: shape 2 (`_s2`) and shapes 0 / 1 (`_s01`)
#define DLADMM_REV_DECL(NAME)                                                                \
  hipError_t launch_rev_##NAME##_s2(const RevArgs& a, int grid, hipStream_t s);             \
  hipError_t launch_rev_##NAME##_s01(int shape, const RevArgs& a, int grid, hipStream_t s);
DLADMM_REV_DECL(v1)
DLADMM_REV_DECL(vvar)
DLADMM_REV_DECL(lasso)
DLADMM_REV_DECL(v2)
DLADMM_REV_DECL(v3)
#undef DLADMM_REV_DECL

// V5 (tied, a trainable step ss1_k on W Var): M_k^T packs -ss1_k W^T, the masks come from Z_k as
// for V4, and ss1_k's gradient -<W, gU_k Var_k^T> is taken from the weight gradient's sums
// (wgrad_reduce_kernel), so the sweep needs no q = W Var_k.  V1: per-sample betas, fixed
// thresholds (scalar table: theta_z, theta_e, s1 = 1).  V2 / V3: per-row parameters from the row
// table, per-row gradient partials
bool reverse_supports(int variant) {
  return variant == DLADMM_V1_LENA || variant == DLADMM_V2_LTHETA || variant == DLADMM_V3_FULL ||
         variant == DLADMM_V4_SCALAR || variant == DLADMM_V5_TIED || variant == DLADMM_V6_LASSO;
}

hipError_t launch_reverse_shape(int shape, int variant, const RevArgs& a, int grid,
                                hipStream_t s) {
  static_assert(kNumShapes == 3, "one case per register-resident shape");
  if (shape < 0 || shape > 2) return hipErrorInvalidValue;
  switch (variant) {
    case DLADMM_V1_LENA:
      return shape == 2 ? launch_rev_v1_s2(a, grid, s) : launch_rev_v1_s01(shape, a, grid, s);
    case DLADMM_V2_LTHETA:
      return shape == 2 ? launch_rev_v2_s2(a, grid, s) : launch_rev_v2_s01(shape, a, grid, s);
    case DLADMM_V3_FULL:
      return shape == 2 ? launch_rev_v3_s2(a, grid, s) : launch_rev_v3_s01(shape, a, grid, s);
    case DLADMM_V4_SCALAR:
    case DLADMM_V5_TIED:
      return shape == 2 ? launch_rev_vvar_s2(a, grid, s)
                        : launch_rev_vvar_s01(shape, a, grid, s);
    case DLADMM_V6_LASSO:
      return shape == 2 ? launch_rev_lasso_s2(a, grid, s)
                        : launch_rev_lasso_s01(shape, a, grid, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace dladmm
