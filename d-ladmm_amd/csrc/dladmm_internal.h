// dladmm_internal.h -- host-side contracts between the C ABI (dladmm_capi.hip) and the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dladmm_common.h"

namespace dladmm {

struct FusedArgs {
  int m, n, B, K;
  int keep_all, loss_kind, ldl;   // ldl: columns per row of lossp (tiles * 64)
  int pad0;
  const float* X;  int64_t ldx;
  const float* Z0; int64_t ldz0;
  const float* E0; int64_t lde0;
  const float* L0; int64_t ldl0;
  const float* Ap;   // packed A          [MB/2][NB][2] fragments (pair order)
  const float* Wp;   // packed -W_k  [K][NB/2][MB][2] fragments (V5: s1 applied in the epilogue)
  int wstep;         // 1: layer k reads packed weight k; 0: every layer reads the one shared weight
  int pad1;
  const float* scal; // [K][8]
  const float* rowp; int64_t rstride;  // [K][8][rstride]
  int64_t ldb;
  // V1 per-sample betas: device tables of the K layer pointers (workspace), any depth
  const float* const* b1t;
  const float* const* b2t;
  float* Zo; float* Eo; float* Lo; float* To; int64_t ldo;
  float* Po;         // training: A Z_k of every layer [K][m][ldo] (the SAVEP instantiations)
  float* lossp;      // [K][2][ldl] per-column objective terms
  // split-f16 path (dladmm_fused_x3.hip): per-tensor weight scale exponents (wexp[0] = A,
  // wexp[1 + k] = -W_k) and the lean-mode Z_k workspace [2][n][ldzw]
  const int* wexp;
  float* Zw; int64_t ldzw;
  // diagnostic builds only (X3_STAMP): per-wave cycle sums; DLADMM_DBG_PTR (device address)
  unsigned long long* dbg;
  // path 6 (dladmm_fused_xs.hip): per-group exchange buffers (xstride floats each) and hand-off
  // counters (64 per group, zeroed before the launch)
  float* xch; int64_t xstride;
  unsigned* xcnt;
};


// Register-resident instantiations of the fused kernel, by index: (MP, NP).
constexpr int kNumShapes = 3;
constexpr int kShapeMP[kNumShapes] = {32, 64, 256};
constexpr int kShapeNP[kNumShapes] = {32, 256, 512};

hipError_t launch_fused_shape(int shape, int variant, const FusedArgs& a, int grid,
                              hipStream_t s);
// the same kernels that also store P_k = A Z_k (a.Po) for the backward (dladmm_fused_savep.hip)
hipError_t launch_fused_shape_savep(int shape, int variant, const FusedArgs& a, int grid,
                                    hipStream_t s);
// small-batch row-split form of the fused kernel (path 5, dladmm_fused_rs.hip): 16 columns per
// workgroup, grid = ceil(B / 16)
bool rs_supports(int shape, int variant);
hipError_t launch_fused_rs(int shape, int variant, const FusedArgs& a, int grid, hipStream_t s);
// the smallest batches (path 6, dladmm_fused_xs.hip): four workgroups per 16 columns, exchange
// through a.xch / a.xcnt; xs_grid(B) workgroups, xs_group_floats() floats per group's buffer
int xs_grid(int64_t B);
size_t xs_group_floats();
hipError_t launch_fused_xs(int shape, int variant, const FusedArgs& a, hipStream_t s);
// split-f16 fused kernel (DLADMM_PREC_F32_SPLIT); Ap / Wp hold [step][hi|lo] f16 fragments
bool x3_supports(int variant);
hipError_t launch_fused_x3_shape(int shape, int variant, const FusedArgs& a, int grid,
                                 hipStream_t s);
// the same kernels that also store P_k = A Z_k (a.Po) for the backward (dladmm_fused_x3_savep.hip)
hipError_t launch_fused_x3_shape_savep(int shape, int variant, const FusedArgs& a, int grid,
                                       hipStream_t s);

}  // namespace dladmm

namespace dladmm {

// ---- per-layer path (dladmm_layered.hip)
#ifndef DLADMM_LAYER_WAVES
#define DLADMM_LAYER_WAVES 4
#endif
// waves per layer-kernel workgroup: 4 (one per SIMD) with two workgroups per CU, so one
// workgroup's epilogue (HBM-bound) overlaps the other's MFMA main loop
constexpr int kLayerWaves = DLADMM_LAYER_WAVES;
constexpr int kLayerCols = 16 * kLayerWaves;        // batch columns per workgroup

struct LayerArgs {
  int m, n, B, K, k;          // k = layer index; -1 = prologue (T0, Var0)
  int loss_kind, nslots;      // lossp row length: slices * ldl (per slice, per column)
  int ldl;                    // columns per slice row of lossp (gx * 16 * NW)
  int KB;                     // 16-row blocks of the contraction
  int MBp;                    // packed output row-blocks (padded to the slice size)
  int Krows;                  // valid rows of the B operand
  const float* Wp;            // packed weights, k-major fragment order [KB][MBp]
  const float* S; int64_t ldS;          // B operand: Var (G1) or Z_k / Z0 (G2)
  const float* Zprev; int64_t ldzp;     // G1: Z_{k-1}
  const float* X; int64_t ldx;          // G2
  const float* Eprev; int64_t ldep;     // G2: E_{k-1}
  const float* Lprev; int64_t ldlp;     // G2: L_{k-1}
  float* Zo; float* Eo; float* Lo; float* To; int64_t ldo;
  float* Vo; int64_t ldv;               // Var of layer k+1 (workspace)
  const float* scal;
  const float* rowp; int64_t rstride;
  const float* b1e; const float* b2e; const float* b1n_e; int64_t ldb;  // V1 betas
  float* lossp;
  // bf16 tile path (path 3): S is the PACKED bf16 B operand ([KB][nbp] fragments of 32 rows x
  // 16 columns); Pb receives this product's output state packed the same way for the next
  // product (pb_kb k-blocks); Vo is unused there
  void* Pb; int nbp, pb_kb;
};

// phase 0 = G1 (W_k Var -> Z_k), 1 = G2 (A Z_k -> E_k, L_k, T_{k+1}, Var_{k+1}),
// 2 = prologue G2 (A Z0 -> T_0, Var_0).  sb = output blocks per slice (16 or 32).
hipError_t launch_layer(int phase, int variant, const LayerArgs& a, dim3 grid, int sb,
                        hipStream_t s);

// ---- bf16 2-D tile kernels (dladmm_tile_bf16.hip), BASELINE config 5
// A workgroup owns a 256-row output tile (16 row blocks); both operands are packed bf16
// fragments streamed by LDS-DMA through a ring.  Two widths (wave tile 128 x 64 either way):
//   wide   8 waves, 256 columns, 4-stage ring (128 KiB): one workgroup per CU;
//   narrow 4 waves, 128 columns, 3-stage ring (72 KiB): two workgroups per CU, so one
//          workgroup's HBM-bound epilogue runs beside the other's MFMA main loop.
constexpr int kTileBlocks = 16;                 // row blocks per tile
constexpr int bf16_tile_cols(bool narrow) { return narrow ? 128 : 256; }
hipError_t launch_tile_bf16(int phase, int variant, bool narrow, const LayerArgs& a, dim3 grid,
                            hipStream_t s);
// Z0 [rows][ld] fp32 -> packed bf16 B operand [KB][nbp] (RNE, zero padding)
hipError_t pack_state_bf16(const float* S, int64_t ld, int rows, int64_t cols, int KB, int nbp,
                           void* out, hipStream_t s);

}  // namespace dladmm

namespace dladmm {

// ---- backward (dladmm_backward.hip)
// 4 waves per workgroup = 1 wave per SIMD: the epilogues' adjoint algebra needs the full
// 512-register budget next to 64-128 accumulator registers.
constexpr int kBwdWaves = 4;
constexpr int kBwdCols = 16 * kBwdWaves;
struct BwdArgs {
  int m, n, B, K, k;
  int KB, MBp, Krows;         // slice GEMM geometry (BK2: both GEMMs share it)
  int nslots, ncg;            // scalar partial slots per param slot; column groups (row kind)
  const float* Wp; const float* S; int64_t ldS;     // GEMM 1: packed operand, B operand
  const float* Wp2; const float* S2; int64_t ldS2;  // GEMM 2 (BK2 only)
  const float* X; int64_t ldx;
  const float* Ep; int64_t ldep;   // E_{k-1}
  const float* Lp; int64_t ldlp;   // L_{k-1}
  const float* Zp; int64_t ldzp;   // Z_{k-1}
  const float* Tk; int64_t ldt;    // T_k
  const float* Pk;                 // BK1 with the forward's saved A Z_k (row stride ldt)
  const float* Zk; int64_t ldzk;   // BK2: the forward's Z_k (its shrink mask, zk_mask)
  int zk_mask;                     // BK2, scalar kinds: 2 = the layer runs a PH 5 launch
                                   // (theta_z >= 0: the mask comes from Z_k, q = W_k Var_k is
                                   // not formed; V5's ss1 gradient comes from the weight
                                   // gradient) beside a PH 2 launch (theta_z < 0), each exiting
                                   // unless theta_z's sign is its case; 0 = PH 2 only.  Per-row
                                   // kinds run PH 5 alone (each row's sign in the epilogue)
  const float* gZ; const float* gE; const float* gL; const float* gT; int64_t ldg;  // upstream
  int loss_kind; const float* lcoef;  // fused training objective: device [K][2] (cz_k, cf_k)
  float* AZ; float* AE; float* AL; float* AT; float* GP; float* VAR; int64_t ldw;   // workspace
  const float* scal;
  const float* rowp; int64_t rstride;
  const float* b1e; const float* b2e; int64_t ldb;  // V1 betas of layer k
  float* gb1e; float* gb2e;                          // V1 beta grads of layer k
  float* part;
  // PH 6 (BK3 of layer k3 fused with BK1 of layer k = k3 - 1): the BK3 layer's T_k3, V1 beta1 and
  // its gradient, and the partial buffer of its parameter slot (beta1)
  int k3;
  const float* Tk3; const float* b1e3; float* gb1e3;
  float* part3;
};

struct WgradArgs {
  const float* G; const float* V; int64_t ld;  // gU (NR x ld), Var (MR x ld), zero-padded
  int n, m;                                    // valid rows of G / V
  int NBp16, MBp16;                            // padded rows / 16 (multiples of 8)
  int64_t Bpad, chunk;                         // padded batch; columns per split-K chunk
  int nchunks;
  float* part;                                 // [nchunks][n][m]
  int64_t gls, vls, pls;                       // layer strides (grid.z = layer of a batch)
};

hipError_t launch_bwd(int phase, int variant, const BwdArgs& a, dim3 grid, int sb,
                      hipStream_t s);

// every argument struct travels by value as a kernel argument: keep them small
static_assert(sizeof(FusedArgs) <= 2048, "kernel argument size");
static_assert(sizeof(LayerArgs) <= 2048, "kernel argument size");
static_assert(sizeof(BwdArgs) <= 2048, "kernel argument size");
static_assert(sizeof(WgradArgs) <= 2048, "kernel argument size");
hipError_t launch_wgrad(const WgradArgs& a, int tiles, hipStream_t s, int layers = 1);
// fixed-order chunk sums of `nl` consecutive layers' split-K partials (part + y*pls, layers
// klo + y): gW_k = -s1_k * sum (each its own output, layer stride gls), or (tied) all of them
// added into one gW in the order k = klo + nl - 1 .. klo -- the per-layer reduce's order
struct WredArgs {
  const float* part; int64_t pls; int nchunks; int64_t nm;
  const float* scal; int klo, nl, tied;
  float* gW; int64_t gls, ldgw; int m;
  const float* Wd; int64_t ldwd;  // V5: <W, G_k> per layer -> dotp + k*nbd
  double* dotp; int nbd;
};
hipError_t launch_wgrad_reduce_layers(const WredArgs& a, hipStream_t s);

// ---- backward as one reverse sweep (dladmm_reverse.hip): V1 / V4 / V5 / V6 after a saved-
// product fused forward, register-resident shapes (kShapeMP / kShapeNP), optional upstream
// cotangents of Z, E, L, T
// Device pointer table of the sweep (written per call by write_ptr_table, graph-capturable):
// entry blocks of K (gT: K + 1) pointers, NULL = absent / zero
enum RevTab { RT_GZ = 0, RT_GE = 1, RT_GL = 2, RT_GT = 3, RT_B1 = 4, RT_B2 = 5, RT_GB1 = 6,
              RT_GB2 = 7, RT_NTAB = 8 };
__host__ __device__ constexpr int rev_tab_at(int tab, int K, int k) {
  return tab * K + (tab > RT_GT ? 1 : 0) + k;   // gT holds K + 1 entries
}
struct RevArgs {
  int m, n, B, K;
  int loss_kind, ncg;              // ncg: waves (column groups) = partial entries per slot
  int64_t Bw;                      // padded batch of the gU / Var workspaces (stored as zeros)
  const float* X; int64_t ldx;
  const float* E0; int64_t lde0;
  const float* L0; int64_t ldl0;
  const float* Z; const float* E; const float* L; const float* T; const float* P;
  int64_t ldo;                     // the forward's outputs: Z, E, L, P [K][.][ldo], T [K+1];
                                   // also the row stride of the betas, their gradients and the
                                   // cotangents (host: make_bwd_plan)
  const float* Atp;                // packed A^T            [NB/2][MB][2] fragments (pair order)
  const float* Mtp;                // packed (-s1 W_k)^T [K][MB/2][NB][2]
  const float* scal;               // [K][8]
  const float* lcoef;              // fused objective [K][2] (cz_k, cf_k), or null
  float* GU; float* VAR; int64_t ldw, gus, vas;   // gU_k [K][gus], Var_k [K][vas], row stride ldw
  int64_t aer;                     // V4: rows aer.. of layer k's Var block hold the adjoint of
                                   // E_{k-1} (carried from BK1(k) to BK1(k-1))
  float* part;                     // parameter partials [K][8][ncg]
  const float* const* ptab;        // RevTab pointer table (device)
  int has_gz, has_cot;             // cotangents of Z; of E / L / T
  const float* rowp; int64_t rstride;  // V2 / V3: per-row parameter table [K][8][rstride]
  float* rpart;                    // V2 / V3: per-row partials [K][8][rstride][ncg]
  // the four-workgroup row split (bwd path 3): per-group exchange buffers (xstride floats each)
  // and hand-off counters (64 per group, zeroed before the launch)
  float* xch; int64_t xstride; unsigned* xcnt;
};
static_assert(sizeof(RevArgs) <= 2048, "kernel argument size");
bool reverse_supports(int variant);
hipError_t launch_reverse_shape(int shape, int variant, const RevArgs& a, int grid, hipStream_t s);
// the small-batch row-split reverse sweep (dladmm_reverse_rs.hip): 16 columns per workgroup,
// grid = ceil(B / 16), after a path-5 forward; V4 / V5 / V6 at the 256 x 512 shape, no E / L / T
// cotangents
bool reverse_rs_supports(int shape, int variant);
hipError_t launch_reverse_rs(int shape, int variant, const RevArgs& a, int grid, hipStream_t s);
// its four-workgroup form (bwd path 3, after path 6): grid xs_grid(B), exchange a.xch / a.xcnt
// (rev_xs_group_floats() floats per group)
size_t rev_xs_group_floats();
hipError_t launch_reverse_xs(int shape, int variant, const RevArgs& a, hipStream_t s);
// fused main_lena.py objective (dladmm_lena.hip, dladmm_lena_f32): one workgroup per 64 columns,
// every layer; mode 0 = per-column partial sums part[K][4][ldl], mode 1 = the cotangents gE / gL
struct LenaArgs {
  int m, n, B, K, mode, ldl;
  float alpha, inv_mb, inv_nb;
  float xsign;  // +1 / -1: the sign of X in gL (main_lena.py:226 / main_syn_l1l1-dgap_ltheta.py:205)
  float gc[8];  // dual_gap constants (a, 1 + e^-2a, e^-a, e^a + e^-a) for a = alpha, then a = 1
  const float* X; int64_t ldx;
  const float* E; const float* L; int64_t ls, ld;  // layer k at + k*ls, row stride ld
  const float* Ap;   // packed A   [MB/2][NB][2] fragments (the forward's G2 order)
  const float* Atp;  // packed A^T [NB/2][MB][2] fragments
  float* part;
  float* gE; float* gL; int64_t gls, ldg;
  const float* coef;  // mode 1: [K]
};
hipError_t launch_lena(int shape, const LenaArgs& a, int grid, hipStream_t s);
// its small-batch row-split form (16 columns per workgroup, grid = ceil(B / 16), shape 2)
hipError_t launch_lena_rs(const LenaArgs& a, int grid, hipStream_t s);

hipError_t launch_wgrad_reduce(const float* part, int nchunks, int n, int m, const float* scal,
                               int k, int accumulate, float* gW, int64_t ldgw, hipStream_t s,
                               const float* Wd = nullptr, int64_t ldwd = 0,
                               double* dotp = nullptr);
// V5: ss1_k's gradient from the weight gradient's sums (-<W, gU_k Var_k^T>): dotp holds
// s1_dot_blocks(n, m) fp64 block partials of one layer
int s1_dot_blocks(int n, int m);
hipError_t launch_s1_dot_finish(const double* dotp, int n, int m, double* out, hipStream_t s);

}  // namespace dladmm
