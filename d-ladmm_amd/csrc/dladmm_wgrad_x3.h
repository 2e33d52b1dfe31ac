// dladmm_wgrad_x3.h -- the weight-gradient GEMM of the backward (part[c] = G V^T over batch chunk
// c) on the f16 matrix cores with exactly split operands, for precision DLADMM_PREC_F32_SPLIT
// (dladmm_wgrad_x3.hip).  Same arguments, grid and partial layout as wgrad_kernel.
#pragma once

#include "dladmm_internal.h"

namespace dladmm {

// the split-f16 form applies when every chunk (and the padded batch) is whole 32-column
// sub-chunks
inline bool wgrad_x3_fits(const WgradArgs& a) { return a.chunk % 32 == 0 && a.Bpad % 32 == 0; }

hipError_t launch_wgrad_x3(const WgradArgs& a, int tiles, hipStream_t s, int layers = 1);

}  // namespace dladmm
