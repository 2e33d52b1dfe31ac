/*
 * dladmm.h -- C ABI of the MI355X-native fused D-LADMM forward (libdladmm_hip.so).
 *
 * The reference (xhchrn/D-LADMM) has no FFI: its interface for this path is the Python
 * nn.Module `DLADMMNet` whose forward() runs the K-layer Z/E/lambda update loop
 * (main_lena.py:57-98, main_syn_l1l1_scalar.py:80-127, main_syn_lasso_scalar.py:65-114, ...).
 * This header is the boundary underneath the drop-in Python module (d-ladmm_amd/model.py):
 * the whole K-layer loop of one forward() is ONE call of dladmm_fwd_f32().
 *
 * Conventions
 *  - Every matrix is fp32, row-major "features x batch" exactly like the reference tensors
 *    (X, E, L, T: m x B; Z: n x B; A: m x n; fc[k].weight = W_k: n x m), batch contiguous.
 *    Row strides (leading dims, in elements) are explicit so batch shards can be views.
 *  - All pointers are DEVICE pointers except the pointer tables inside the descriptor
 *    (W, beta1_elem, beta2_elem), which are host arrays of `layers` device pointers.
 *  - The library never allocates: the caller provides outputs and a workspace of
 *    dladmm_fwd_workspace_bytes() bytes (device memory, 256-byte aligned).
 *  - The call is asynchronous on `stream` (a hipStream_t passed as void*); nothing syncs.
 *  - Return value: 0 on success, a negative DLADMM_E_* code for an invalid descriptor, or a
 *    positive hipError_t from the HIP runtime.  dladmm_error_string() maps either to text.
 */
#ifndef DLADMM_H_
#define DLADMM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DLADMM_ABI_VERSION 6
#define DLADMM_MAX_LAYERS 65536   /* K limit, every variant (e.g. the K=2000 KM ground-truth run) */

/* Reference variants (class DLADMMNet of the named reference script). */
enum dladmm_variant {
  DLADMM_V1_LENA = 1,   /* main_lena.py:16-102          beta (m,B) per sample, fixed thetas   */
  DLADMM_V2_LTHETA = 2, /* main_syn_l1l1_ltheta.py:16-95 beta (m,1), learned (d,1)/(m,1) thetas */
  DLADMM_V3_FULL = 3,   /* main_syn_l1l1_full.py:16-96   per-row beta1/2/3, ss2, thetas         */
  DLADMM_V4_SCALAR = 4, /* main_syn_l1l1_scalar.py:34-131 all params (1,1)                     */
  DLADMM_V5_TIED = 5,   /* main_syn_l1l1_scalar_tied.py:34-104 shared fc, per-layer ss1       */
  DLADMM_V6_LASSO = 6   /* main_syn_lasso_scalar.py:17-118 linear E-step                      */
};

/* Per-layer objective reduced inside the kernel (the reference training loop's loss[k]). */
enum dladmm_loss_kind {
  DLADMM_LOSS_NONE = 0,
  DLADMM_LOSS_L1L1 = 1, /* sum|Z_k| and sum|X - A Z_k|        main_syn_l1l1_scalar.py:290-294   */
  DLADMM_LOSS_LASSO = 2 /* sum|Z_k| and 0.5*sum (X - A Z_k)^2  main_syn_lasso_scalar.py:276-281 */
};

/* Error codes (negative). */
#define DLADMM_E_ABI_VERSION (-1)
#define DLADMM_E_VARIANT (-2)
#define DLADMM_E_SHAPE (-3)
#define DLADMM_E_LAYERS (-4)
#define DLADMM_E_NULL (-5)
#define DLADMM_E_WORKSPACE (-6)
#define DLADMM_E_UNSUPPORTED (-7)
#define DLADMM_E_ALIGN (-8)

/*
 * Scalar parameter slots, per layer: scalar_params[k * DLADMM_NSCALAR + slot].
 * For the per-row variants (V2, V3) the same slots live in row_params (see below); for V1 the
 * betas are per-element tensors and only the two fixed thresholds are read from here.
 *   beta1  main_lena.py:35            b1 in  Var = L + b1*T                      (all)
 *   beta2  main_lena.py:36            b2 in  E-step                                (V1-V5)
 *   beta3  main_syn_l1l1_scalar.py:61 b3 in  L = L + b3*T   (V1/V2 pass beta1)    (all)
 *   ss2    main_syn_l1l1_scalar.py:62 E = S(E - ss2*VVar)   / LASSO ss2_1          (V3-V6)
 *   ss2b   main_syn_lasso_scalar.py:47 LASSO ss2_2                                 (V6)
 *   theta_z / theta_e  active_para / active_para1 (V1: 0.025 / 0.06 fixed)         (all)
 *   s1     main_syn_l1l1_scalar_tied.py:34 ss1 (1.0 for untied variants)            (V5)
 */
enum dladmm_param_slot {
  DLADMM_P_BETA1 = 0,
  DLADMM_P_BETA2 = 1,
  DLADMM_P_BETA3 = 2,
  DLADMM_P_SS2 = 3,
  DLADMM_P_SS2B = 4,
  DLADMM_P_THETA_E = 5,
  DLADMM_P_THETA_Z = 6,
  DLADMM_P_S1 = 7,
  DLADMM_NSCALAR = 8
};

typedef struct dladmm_fwd_desc {
  int32_t abi_version; /* = DLADMM_ABI_VERSION */
  int32_t variant;     /* enum dladmm_variant */
  int32_t m;           /* rows of A (reference ctor arg m)        */
  int32_t n;           /* columns of A (reference ctor arg d)     */
  int32_t batch;       /* columns of X processed by this call     */
  int32_t layers;      /* K (reference ctor arg layers), <= DLADMM_MAX_LAYERS */
  int32_t keep_all;    /* 1: write Z/E/L for every layer and T[0..K] (reference return lists);
                          0: write only layer K-1 (Z,E,L) and T[K]                              */
  int32_t loss_kind;   /* enum dladmm_loss_kind */

  /* inputs (device) */
  const float* X;  int64_t ld_x;   /* m x batch */
  const float* A;  int64_t ld_a;   /* m x n     */
  const float* Z0; int64_t ld_z0;  /* n x batch */
  const float* E0; int64_t ld_e0;  /* m x batch */
  const float* L0; int64_t ld_l0;  /* m x batch */

  /* weights: host array of `layers` device pointers to fc[k].weight (n x m, row stride ld_w).
     V5 (tied) passes the same pointer `layers` times; when every entry is the same pointer the
     weight is packed once (any K). */
  const float* const* W; int64_t ld_w;

  /* parameters (device), see dladmm_param_slot:
       V4/V5/V6: scalar_params  [layers][DLADMM_NSCALAR]
       V2/V3:    row_params     [layers][DLADMM_NSCALAR][rows] with rows = max(m, n); the
                 theta_z slot holds n values, every other slot m values; s1 unused
       V1:       scalar_params (theta_z/theta_e only) + beta1_elem/beta2_elem: host arrays of
                 `layers` device pointers to the (m x batch) per-sample betas, row stride ld_beta */
  const float* scalar_params;
  const float* row_params; int64_t row_stride; /* elements between slots of one layer */
  const float* const* beta1_elem;
  const float* const* beta2_elem;
  int64_t ld_beta;

  /* outputs (device).  keep_all: Z [K][n][ld_out], E/L [K][m][ld_out], T [K+1][m][ld_out];
     else one layer each.  T may be NULL (V1-V3 do not return it). */
  float* Z; float* E; float* L; float* T;
  int64_t ld_out;

  /* per-layer loss sums (device, fp64): loss_sums[k*2+0] = sum|Z_k|,
     loss_sums[k*2+1] = sum|X-AZ_k| (L1L1) or 0.5*sum(X-AZ_k)^2 (LASSO).  NULL if loss_kind=0. */
  double* loss_sums;

  void* workspace; size_t workspace_bytes;

  /* optional profiling: hipEvent_t handles recorded on `stream` immediately before / after the
     fused K-layer kernel (NULL = not recorded) */
  void* ev_kernel_start;
  void* ev_kernel_stop;

  /* optional per-column objective terms (device, needs loss_kind): col_loss[(k*2+t)*batch + b]
     = sum_i |Z_k[i,b]| (t = 0) and the column's fit term (t = 1) -- the per-sample values the
     reference's evaluation objectives reduce (test_syn_l1l1_scalar.py:460-478). NULL = off. */
  float* col_loss;

  /* GEMM operand precision:
       DLADMM_PREC_F32 (default; the reference's fp32): fp32 MFMA (v_mfma_f32_16x16x4_f32), an
         exact fp32 fma chain per output;
       DLADMM_PREC_F32_SPLIT: the same fp32 GEMMs on the f16 matrix cores -- both operands scaled
         by powers of two (weights per tensor, state per batch column) and split exactly into
         hi + lo f16 halves (22 significant bits), the product formed as hi*hi + hi*lo + lo*hi with
         fp32 accumulation (every f16 x f16 product is exact in fp32).  Error of an fp32 GEMM
         (same tolerance tests as PREC_F32); every elementwise update stays fp32.  Fused path
         (m <= 256, n <= 512) for V1 (per-sample betas) and V4/V5/V6; other shapes / variants
         run PREC_F32;
       DLADMM_PREC_BF16 (BASELINE config 5: A, W_k and the state operands Var / Z_k rounded to bf16
         for the MFMAs, fp32 accumulation, every elementwise update -- shrinks, E, dual L, T -- in
         fp32).  bf16 runs on the per-layer kernels (path 3). */
  int32_t precision;
  /* plan options, a bitwise OR of enum dladmm_flags (0 = the default plan).  They change which
     kernels run -- never the arithmetic a kernel performs -- and the descriptor is the whole
     input of the plan: the library reads no environment variable. */
  int32_t flags;

  /* optional (training): P [K][m][ld_out] receives A Z_k of every layer, exactly the product the
     E/L/T updates consumed (main_syn_l1l1_scalar.py:114-117).  Written only on paths 1, 4 and 5
     (fused kernels, keep_all = 1; dladmm_fwd_path() tells); ignored on every other path.  A backward
     whose fwd.P is set reads it instead of recomputing the product (one GEMM per layer less). */
  float* P;
} dladmm_fwd_desc;

enum dladmm_precision { DLADMM_PREC_F32 = 0, DLADMM_PREC_BF16 = 1, DLADMM_PREC_F32_SPLIT = 2 };

/* dladmm_fwd_desc.flags (also read from dladmm_bwd_desc.fwd.flags by the backward). */
enum dladmm_flags {
  DLADMM_F_PER_LAYER = 1,      /* forward: the per-layer kernel pair (path 2) even where the fused
                                  kernel fits (equivalence tests, A/B timing)                      */
  DLADMM_F_BF16_WIDE = 2,      /* bf16 tiles: 256-column tiles, one workgroup per CU (default: 128
                                  columns, two per CU -- 2 % faster at BASELINE config 5)          */
  DLADMM_F_BWD_PER_LAYER = 4,  /* backward: the per-layer kernels even where the reverse sweep
                                  applies (dladmm_bwd_path 0)                                      */
  DLADMM_F_BWD_UNFUSED = 8,    /* per-layer backward after a saved-product forward: BK1 as its own
                                  launch instead of inside BK3's (bit-identical)                   */
  DLADMM_F_BWD_NO_ZMASK = 16,  /* per-layer backward, V2 / V3: form q = W_k Var_k in BK2 instead of
                                  reading the shrink masks off the saved Z_k                       */
  DLADMM_F_WGRAD_F32 = 32,     /* split-f16 backward: the weight gradient on the fp32-MFMA kernel  */
  DLADMM_F_NO_ROWSPLIT = 64,   /* forward: the fused kernel (path 1) where the small-batch
                                  row-split kernels (paths 5 / 6) would run (equivalence tests,
                                  A/B)                                                             */
  DLADMM_F_NO_XSPLIT = 128     /* forward: the one-workgroup row split (path 5) where the
                                  four-workgroup one (path 6) would run                            */
};

/* ABI version the library was built with. */
int dladmm_abi_version(void);

/* Workspace the call needs for this descriptor (0 on an invalid descriptor). */
size_t dladmm_fwd_workspace_bytes(const dladmm_fwd_desc* d);

/* Which kernel path this descriptor takes: 1 = fused persistent K-layer kernel,
   2 = per-layer kernel pair (large shapes, or one layer's matrix >= 2^31 bytes), 3 = per-layer
   tile kernels on bf16 operands, 4 = fused kernel on split-f16 operands (DLADMM_PREC_F32_SPLIT),
   5 = fused kernel with each workgroup's rows split over its waves (16 columns per workgroup):
   small fp32 batches (at most three workgroups per CU) of V1 / V4 / V5 / V6 at m <= 256,
   n <= 512 (and m > 64 or n > 256) -- the same arithmetic as path 1, bit for bit (the fused
   objective's per-column sums: to fp32 rounding), 6 = the same split over four workgroups per
   16 columns (16 waves; the column state handed between them through the workspace once per
   product) where that grid fits one workgroup per CU (B <= 1,024 on 256 CUs), also bit for bit;
   <0 = DLADMM_E_* error.  Host-only: no device work. */
int dladmm_fwd_path(const dladmm_fwd_desc* d);

/* Enqueue the whole K-layer forward on `stream` (hipStream_t). */
int dladmm_fwd_f32(const dladmm_fwd_desc* d, void* stream);

/*
 * Backward: the vector-Jacobian product of one forward call.
 *
 * The reference trains by `total_loss.backward()` through DLADMMNet.forward
 * (main_lena.py:229, main_syn_l1l1_scalar.py:298, main_syn_lasso_scalar.py:285); torch autograd
 * then produces .grad for every parameter.  dladmm_bwd_f32() produces the same gradients from
 * the saved forward outputs and the upstream cotangents of those outputs:
 *   grad of  sum_k <gZ_k, Z_k> + <gE_k, E_k> + <gL_k, L_k> + sum_j <gT_j, T_j>
 * with respect to W_k (fc[k].weight), every per-layer parameter slot and, for V1, the
 * per-sample betas.  There are no gradients for X, A, Z0, E0, L0 (plain tensors in the
 * reference, never parameters).
 *
 * `fwd` must describe the forward call whose outputs are differentiated, run with keep_all = 1
 * and T != NULL (all K layers of Z/E/L and T[0..K] saved; V1-V3 keep T internally).  Its
 * workspace fields are ignored.
 */
typedef struct dladmm_bwd_desc {
  /* the forward's descriptor (keep_all, T, and P where it was saved).  fwd.precision:
     DLADMM_PREC_F32, or DLADMM_PREC_F32_SPLIT after a split-f16 training forward -- then the
     weight-gradient GEMM (gU_k Var_k^T over the batch) also runs on the f16 matrix cores with
     exactly split operands (any batch on the reverse sweep, whose operand columns are padded to
     32; whole 32-column chunks on the per-layer backward, else the fp32 kernel), unless
     fwd.flags holds DLADMM_F_WGRAD_F32; every other backward kernel is fp32 either way.
     Accuracy: fp32-GEMM error relative to the largest product in each 64 x 64 block of gW --
     the split scales are per wave, so a row of gU_k or Var_k more than ~2^17 below the largest
     row of its 64-row block keeps fewer bits (measured within 1e-5 of the fp32 kernel per row
     at a 2^20 spread; rows ~2^29 below contribute nothing) */
  dladmm_fwd_desc fwd;

  /* upstream cotangents: HOST arrays of device pointers, one per layer (gT: K+1), each a
     (rows x ld_g) matrix; a NULL array or a NULL entry is a zero cotangent */
  const float* const* gZ;  /* K entries, n x ld_g */
  const float* const* gE;  /* K entries, m x ld_g */
  const float* const* gL;  /* K entries, m x ld_g */
  const float* const* gT;  /* K+1 entries, m x ld_g (entry 0 reaches no parameter) */
  int64_t ld_g;

  /* fused training objective (optional): adds the gradient of
       sum_k  cz_k * sum|Z_k|  +  cf_k * fit_k,   fit = sum|X - A Z_k| (L1L1) or
                                                     0.5 * sum (X - A Z_k)^2 (LASSO)
     -- the reference training loss (main_syn_l1l1_scalar.py:283-296, lasso :270-283) with
     cz_k = decay_k * alpha / B and cf_k = decay_k / B -- without materialising A Z_k.
     loss_kind = DLADMM_LOSS_NONE disables it; loss_coef: DEVICE array [K][2] = (cz_k, cf_k). */
  int32_t loss_kind;
  int32_t gw_sum;             /* 1: every layer shares ONE weight (V5 tied, tied newS): gW is one
                                 n x m block holding the sum over layers; 0: gW[k] per layer */
  const float* loss_coef;

  /* outputs (device) */
  float* gW; int64_t ld_gw;   /* [K][n][ld_gw], or [1][n][ld_gw] when gw_sum */
  double* g_scalar;           /* V4-V6: [K][DLADMM_NSCALAR] per-slot grads (slots the variant
                                 does not use are 0; V1: unused).  Slot DLADMM_P_S1 (the step
                                 scaling W_k Var_k) holds ss1_k's gradient for the tied variant
                                 (V5); for the others s1 is the constant 1 and the slot is 0 */
  double* g_row;              /* V2/V3: [K][DLADMM_NSCALAR][fwd.row_stride] per-row grads */
  float* const* g_beta1_elem; /* V1: host arrays of K device pointers, (m x fwd.ld_beta) each: */
  float* const* g_beta2_elem; /*     grads of the per-sample beta1[k] / beta2[k]              */

  void* workspace; size_t workspace_bytes;
} dladmm_bwd_desc;

/* Workspace the backward needs for this descriptor (0 on an invalid descriptor). */
size_t dladmm_bwd_workspace_bytes(const dladmm_bwd_desc* d);

/* Which kernels the backward runs: 1 = one reverse-sweep kernel for every layer's adjoints,
   2 = the same sweep in its small-batch row-split form (16 columns per workgroup, each
   product's rows over its waves; after an fp32 path-5 / 6 forward of V1 / V4 / V5 / V6, any
   cotangents, at most one 16-column workgroup per CU: gU_k, Var_k, the weight gradients and
   V1's beta gradients bit-equal to path 1's, the scalar-parameter gradients to rounding),
   3 = that form over four workgroups per 16 columns after a path-6 forward (the same
   guarantees), 0 = per-layer kernels,
   <0 = DLADMM_E_* error.  The reverse sweep
   runs when ALL of these hold:
     - any variant V1-V6 (and the newS models built on V4 / V5);
     - the forward saved P (fwd.P != NULL, keep_all): the fused fp32 path or the split-f16
       path (precision DLADMM_PREC_F32_SPLIT), both of which store the product A Z_k their
       E / L / T updates consumed;
     - cotangents (gZ, gE, gL, gT; any subset, any depth) only with ld_g == fwd.ld_out;
     - fwd.ld_e0 == fwd.ld_l0 == fwd.ld_out; V1: fwd.ld_beta == fwd.ld_out;
     - its 32-bit workspace offsets hold and its workspace, about
       (layers + 1) * MP * NP * 4 + layers * (Rn + 2 * MP) * Bpad * 4 bytes (MP, NP: the
       instantiation's padded m, n; Rn = NP rounded up to 128; Bpad = batch rounded up to 16;
       V2 / V3 add 8 * layers * max(MP, NP) * (batch / 16, rounded up to 4) * 4 bytes of per-row
       partials), stays under a quarter of the device memory;
     - fwd.flags does not hold DLADMM_F_BWD_PER_LAYER.
   dladmm_bwd_workspace_bytes() reports the size of whichever path this returns. */
int dladmm_bwd_path(const dladmm_bwd_desc* d);

/* Enqueue the whole reverse sweep on `stream` (hipStream_t).  Deterministic: every reduction
   (parameter slots, per-row params, weight gradients) is summed in a fixed order. */
int dladmm_bwd_f32(const dladmm_bwd_desc* d, void* stream);

/*
 * Safeguard step of learned + safeguarded KM (LSKM):
 * test_syn_l1l1_scalar.py:227-266 with the mu updaters of mu_updater.py:18-116.
 * Given, for every batch column, the L2O candidate (Zl, El, Ll, Tl), the classic KM candidate
 * (Zk, Ek, Lk, Tk) -- both one step from the same state whose E is Ep -- and the KM step taken
 * from the L2O candidate (Es, Ts), it computes
 *   |S| = sqrt(sum_i (beta Ts_i)^2 + (c ((Es_i - 2 El_i) + Ep_i))^2),   keep = |S| < (1-delta) mu,
 * updates mu, writes the selected candidate to (Zo, Eo, Lo, To) and adds the number of
 * safeguarded (not kept) columns to *count.  All matrices share the row stride ld.
 * With Zo == NULL it only initialises mu = |S| (mu_0 = |S(Z0, E0, L0, T0, X, E0)|, :190-197;
 * pass the KM step from the initial state as Es/Ts and E0 as El and Ep).
 */
enum dladmm_mu_updater {
  DLADMM_MU_NONE = 0, /* BlankUpdater: mu = 1e10 after the first step (mu_updater.py:98-110)  */
  DLADMM_MU_EMA = 1,  /* mu = keep ? p|S| + (1-p) mu : mu                  (:18-32)            */
  DLADMM_MU_GS = 2,   /* mu = keep ? (1-p) mu : mu                         (:34-52)            */
  DLADMM_MU_RT = 3    /* mu = keep ? |S| : mu                              (:55-73)            */
};

typedef struct dladmm_safeguard_desc {
  int32_t abi_version;
  int32_t m, n, batch;
  int64_t ld;
  const float *Zl, *El, *Ll, *Tl;  /* L2O candidate (Z: n rows, others m rows) */
  const float *Zk, *Ek, *Lk, *Tk;  /* KM candidate */
  const float *Es, *Ts;            /* KM step from the L2O candidate */
  const float* Ep;                 /* E of the state both candidates started from */
  float *Zo, *Eo, *Lo, *To;        /* selected outputs (may alias neither input) */
  float* mu;                       /* [batch] in/out */
  float* norm_out;                 /* [batch] |S| or NULL */
  int32_t* count;                  /* += safeguarded columns */
  float beta, c;
  double delta;
  int32_t updater;                 /* enum dladmm_mu_updater */
  float mu_param;
} dladmm_safeguard_desc;

int dladmm_safeguard_f32(const dladmm_safeguard_desc* d, void* stream);

/*
 * Per-column evaluation objectives over saved layers: for every
 * layer k and batch column b (fp64 sums over the rows)
 *   reg[k*batch+b] = sum_i |Z_k|,  fit = sum_i |E_k - T_{k+1}| (L1L1) or 0.5 sum (E_k - T_{k+1})^2
 *   (LASSO) -- i.e. |X - A Z_k| without re-forming A Z_k --, dz = sum_i (Zref - Z_k)^2,
 *   de = sum_i (Eref - E_k)^2.
 * The reference test scripts reduce these per-sample values into NMSE, L1L1, Normalized-L1L1,
 * GT and Normalized-GT (test_syn_l1l1_scalar.py:436-489).  Any output may be NULL.
 */
typedef struct dladmm_colobj_desc {
  int32_t abi_version;
  int32_t m, n, batch, layers;
  int32_t fit_kind;                            /* DLADMM_LOSS_L1L1 / DLADMM_LOSS_LASSO */
  const float* Z; int64_t z_layer_stride; int64_t ld_z;   /* layer k at Z + k*z_layer_stride */
  const float* E; int64_t e_layer_stride; int64_t ld_e;
  const float* T; int64_t t_layer_stride; int64_t ld_t;   /* layer k reads T_{k+1} */
  const float* Zref; int64_t ld_zref;                      /* n x batch or NULL */
  const float* Eref; int64_t ld_eref;                      /* m x batch or NULL */
  double* reg; double* fit; double* dz; double* de;        /* [layers][batch] each, or NULL */
} dladmm_colobj_desc;

int dladmm_colobj_f32(const dladmm_colobj_desc* d, void* stream);

/*
 * Fused main_lena.py training objective over a forward's saved layers (SURVEY.md section 8 rows
 * a11 / f1; main_lena.py:221-228, dual_gap :145-147), for any variant:
 *   l_k = alpha/(n N) sum|Z_k| + 1/(m N) sum|E_k| + 1/(n N) sum dual_gap(A^T L_k, alpha)
 *         + 1/(m N) sum dual_gap(L_k, 1) +/- 1/(m N) sum L_k * X,
 *   dual_gap(x, c) = softplus(x - c) + softplus(-x - c)   (torch softplus: beta 1, threshold 20),
 * N = the batch of the mean (a data-parallel shard passes the global batch).  The sum|Z_k| term is
 * the forward's own loss_sums[k*2+0] (loss_kind DLADMM_LOSS_L1L1); this call forms the other four
 * without storing A^T L_k:
 *   mode 0: sums[k*4 + t] (fp64, fixed order): t = 0 sum|E_k|, 1 sum dual_gap(A^T L_k, alpha)
 *           (rows < n), 2 sum dual_gap(L_k, 1), 3 sum L_k * X;
 *   mode 1: the cotangents of coef[k] * those terms with their means, i.e. for inv_mb = 1/(m N),
 *           inv_nb = 1/(n N):  gE_k = coef[k] inv_mb sgn(E_k),
 *           gL_k = coef[k] inv_nb A S_k + coef[k] inv_mb (softplus'(L_k - 1) - softplus'(-L_k - 1)
 *           + X),  S_k = softplus'(A^T L_k - alpha) - softplus'(-A^T L_k - alpha)
 *           -- what a dladmm_bwd_f32 call then takes as its gE / gL cotangents;
 *   mode 2: both (a training forward: one pass over the layers; the backward scales the
 *           cotangents by its upstream gradient with dladmm_scale_f32).
 * E_k and L_k (m x batch) sit at E + k*layer_stride (row stride ld), likewise the outputs (gE, gL
 * at + k*g_layer_stride, row stride ld_g).  coef: device [layers] (mode 1).  Shapes: m <= 256 and
 * n <= 512 (the fused forward's register-resident shapes); otherwise DLADMM_E_UNSUPPORTED.
 * lx_negate: 0 = + mean(L_k X) (main_lena.py:226), 1 = - mean(L_k X)
 * (main_syn_l1l1-dgap_ltheta.py:205-206): the sign of X in gL (modes 1, 2); sums[k*4+3] is the
 * unsigned sum L_k X either way.
 */
typedef struct dladmm_lena_desc {
  int32_t abi_version;
  int32_t m, n, batch, layers;
  int32_t mode;
  float alpha, inv_mb, inv_nb;
  int32_t lx_negate;                              /* 0: + mean(L_k X); 1: - mean(L_k X) */
  const float* X; int64_t ld_x;
  const float* A; int64_t ld_a;
  const float* E; const float* L; int64_t layer_stride; int64_t ld;
  double* sums;                                   /* modes 0, 2: [layers][4] */
  float* gE; float* gL; int64_t g_layer_stride; int64_t ld_g;   /* modes 1, 2 */
  const float* coef;                              /* modes 1, 2: device [layers] */
  void* workspace; size_t workspace_bytes;
} dladmm_lena_desc;

size_t dladmm_lena_workspace_bytes(const dladmm_lena_desc* d);
int dladmm_lena_f32(const dladmm_lena_desc* d, void* stream);

/* x[0 .. n) *= *s on `stream`, unless *s == 1 (s: a device scalar, read on the device). */
int dladmm_scale_f32(float* x, int64_t n, const float* s, void* stream);

/* Text for a return code of this library (DLADMM_E_* or hipError_t). */
const char* dladmm_error_string(int code);

#ifdef __cplusplus
}
#endif
#endif /* DLADMM_H_ */
