// dladmm_tile_bf16.hip -- the per-layer products of the bf16 mode (BASELINE config 5: m = 1024,
// n = 4096) as 2-D tiled GEMMs on v_mfma_f32_16x16x32_bf16 with the layer's elementwise update
// fused into the epilogue (dladmm_layer_epi.h, the same per-element code as the fp32 kernels).
//
// Why a second kernel shape: the fp32 slice kernels keep the B operand (state columns) in the
// wave's registers and stream only the weights through LDS, so every 1 KiB weight fragment read
// from LDS feeds a single MFMA.  A bf16 MFMA is 4x the work of an fp32 one in the same time, so
// that shape needs 256 B/clk of LDS reads per CU (the LDS delivers 128) and its 1-k-block prefetch
// leaves the HBM latency exposed at every barrier.  Here:
//   * both operands are packed bf16 fragments (1 KiB: 16 rows/columns x 32 k, lane l holds row
//     or column l & 15 and k 8(l >> 4) .. +7 -- the operand layout of the MFMA, so every
//     ds_read_b128 is one contiguous, conflict-free KiB).  The weights are packed once per call;
//     the state is packed by the PREVIOUS product's epilogue, which writes its output both as
//     the fp32 tensor the API returns (Z_k) and as the next product's bf16 B operand (Z_k or
//     Var_{k+1}) -- Var itself is never stored in fp32.
//   * a workgroup owns a 256-row output tile; every wave owns 128 rows x 64 columns = 8 x 4
//     accumulator blocks, so per k-block of 32 it reads 12 fragments and issues 32 MFMAs (96 KiB
//     of LDS reads per CU per 1024 MFMA cycles).  Two widths (TileG):
//       - wide: 8 waves, 256 columns; a stage (one k-block: 16 A + 16 B fragments = 32 KiB) is
//         LDS-DMA'd 4 fragments per wave, 4 stages in the ring (128 KiB, one workgroup per CU);
//       - narrow: 4 waves, 128 columns; 16 A + 8 B fragments = 24 KiB per stage, 6 per wave, 3
//         stages (72 KiB), two workgroups per CU: while one streams its epilogue to HBM the
//         other's main loop keeps the matrix cores busy;
//     the ring barrier waits with a COUNTED vmcnt so the younger stages stay in flight.
// Every output block is one accumulation chain over k-blocks in order, on the same packed
// operands (weights RNE-rounded, state RNE-rounded) as the restated bf16 oracle.
#include "dladmm_tile_bf16_body.h"
#ifndef DLADMM_TILE_LDSPAD
#define DLADMM_TILE_LDSPAD 0  // experiment: extra dynamic LDS bytes per workgroup (occupancy)
#endif

namespace dladmm {

template <int EMODE, int PKIND, int PH, int NW>
__global__ __launch_bounds__(NW * 64, 8 / NW) void tile_bf16_kernel(const LayerArgs a) {
  using G = TileG<NW>;
  __shared__ f32x4 ring[G::NST * G::SF * 64];
  tile_body<EMODE, PKIND, PH, NW>(a, ring, blockIdx.x, blockIdx.y);
}

template <int PH, int NW>
hipError_t launch_tile_ph(int variant, const LayerArgs& a, dim3 grid, hipStream_t s) {
  const dim3 blk(NW * 64);
  switch (variant) {
    case DLADMM_V1_LENA:
      hipLaunchKernelGGL((tile_bf16_kernel<EM_V1, PK_ELEM, PH, NW>), grid, blk, DLADMM_TILE_LDSPAD, s, a); break;
    case DLADMM_V2_LTHETA:
      hipLaunchKernelGGL((tile_bf16_kernel<EM_V1, PK_ROW, PH, NW>), grid, blk, DLADMM_TILE_LDSPAD, s, a); break;
    case DLADMM_V3_FULL:
      hipLaunchKernelGGL((tile_bf16_kernel<EM_VVAR, PK_ROW, PH, NW>), grid, blk, DLADMM_TILE_LDSPAD, s, a); break;
    case DLADMM_V4_SCALAR:
    case DLADMM_V5_TIED:
      hipLaunchKernelGGL((tile_bf16_kernel<EM_VVAR, PK_SCALAR, PH, NW>), grid, blk, DLADMM_TILE_LDSPAD, s, a); break;
    case DLADMM_V6_LASSO:
      hipLaunchKernelGGL((tile_bf16_kernel<EM_LASSO, PK_SCALAR, PH, NW>), grid, blk, DLADMM_TILE_LDSPAD, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_tile_bf16(int phase, int variant, bool narrow, const LayerArgs& a, dim3 grid,
                            hipStream_t s) {
  switch (phase * 2 + (narrow ? 1 : 0)) {
    case 0: return launch_tile_ph<0, 8>(variant, a, grid, s);
    case 1: return launch_tile_ph<0, 4>(variant, a, grid, s);
    case 2: return launch_tile_ph<1, 8>(variant, a, grid, s);
    case 3: return launch_tile_ph<1, 4>(variant, a, grid, s);
    case 4: return launch_tile_ph<2, 8>(variant, a, grid, s);
    case 5: return launch_tile_ph<2, 4>(variant, a, grid, s);
  }
  return hipErrorInvalidValue;
}

// ---- Z0 -> packed bf16 B operand: one thread per 16-byte lane slot of a fragment
__global__ __launch_bounds__(256) void pack_state_bf16_kernel(const float* S, int64_t ld, int rows,
                                                              int64_t cols, int64_t nslot, int nbp,
                                                              uint4* out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= nslot) return;
  const int L = (int)(t & 63);
  const int64_t frag = t >> 6;
  const int64_t cb = frag % nbp, kb = frag / nbp;
  const int64_t col = cb * 16 + (L & 15);
  const int r0 = (int)(32 * kb) + 8 * (L >> 4);
  uint32_t h[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int row = r0 + q;
    const float x = (row < rows && col < cols) ? S[(int64_t)row * ld + col] : 0.0f;
    h[q] = __builtin_bit_cast(uint16_t, (__bf16)x);
  }
  out[t] = make_uint4(h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16),
                      h[6] | (h[7] << 16));
}

hipError_t pack_state_bf16(const float* S, int64_t ld, int rows, int64_t cols, int KB, int nbp,
                           void* out, hipStream_t s) {
  const int64_t nslot = (int64_t)KB * nbp * 64;
  hipLaunchKernelGGL(pack_state_bf16_kernel, dim3((unsigned)((nslot + 255) / 256)), dim3(256), 0,
                     s, S, ld, rows, cols, nslot, nbp, (uint4*)out);
  return hipGetLastError();
}

}  // namespace dladmm
