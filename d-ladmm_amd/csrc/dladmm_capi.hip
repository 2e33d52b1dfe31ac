// dladmm_capi.hip -- the C ABI of include/dladmm.h: descriptor validation, planning, weight
// packing, the loss reduction, and dispatch to the fused (dladmm_fused.hip) or per-layer
// (dladmm_layered.hip) kernels.
#include <stdlib.h>

#include "dladmm_common.h"
#include "dladmm_internal.h"

namespace dladmm {

// ------------------------------------------------------------------------ weight packing
struct PackArgs {
  const float* src[DLADMM_MAX_LAYERS + 1];
  int R, C, RB, CB;  // valid rows/cols of each source; row-blocks (padded) / col-blocks packed
  int order;         // fragment (ib, jb) at: 0 ib*CB + jb; 1 jb*RB + ib (per-layer path);
                     // 2 ((ib/2)*CB + jb)*2 + ib%2 (fused path: output blocks in pairs)
  int64_t ld;
  float* dst;
  float sign;          // every element is multiplied by sign * (scal ? scal[t][S1] : 1)
  const float* scal;   // device [T][DLADMM_NSCALAR] (V4-V6 s1) or null
};

// fragment (ib, jb) of source t: dst[..][lane][q] = src_t[16 ib + (lane & 15)][16 jb + 4 (lane >> 4) + q]
// (0 outside R x C) -- exactly the A operand of one v_mfma_f32_16x16x4_f32 k-step group
__global__ __launch_bounds__(256) void pack_frags_kernel(const PackArgs p) {
  const int t = blockIdx.y;
  const int64_t fr = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (fr >= (int64_t)p.RB * p.CB) return;
  const int lane = threadIdx.x & 63;
  int ib, jb;
  if (p.order == 0) { ib = (int)(fr / p.CB); jb = (int)(fr % p.CB); }
  else if (p.order == 1) { ib = (int)(fr % p.RB); jb = (int)(fr / p.RB); }
  else { const int64_t q = fr >> 1; jb = (int)(q % p.CB); ib = 2 * (int)(q / p.CB) + (int)(fr & 1); }
  const float f = p.sign * (p.scal ? p.scal[t * DLADMM_NSCALAR + DLADMM_P_S1] : 1.0f);
  const int row = 16 * ib + (lane & 15);
  const int c0 = 16 * jb + 4 * (lane >> 4);
  const float* s = p.src[t];
  f32x4 v;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    v[q] = (row < p.R && c0 + q < p.C) ? f * s[(int64_t)row * p.ld + c0 + q] : 0.0f;
  reinterpret_cast<f32x4*>(p.dst)[((int64_t)t * p.RB * p.CB + fr) * 64 + lane] = v;
}

// ------------------------------------------------------------------------ loss reduction
// sums[i] = sum_w part[i][w] in fp64, fixed order (bitwise reproducible)
__global__ __launch_bounds__(256) void loss_reduce_kernel(const float* part, int nw, double* sums) {
  __shared__ double red[256];
  const int i = blockIdx.x;
  double s = 0.0;
  for (int wv = threadIdx.x; wv < nw; wv += 256) s += (double)part[(int64_t)i * nw + wv];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) sums[i] = red[0];
}

}  // namespace dladmm

// ======================================================================== host side / C ABI
namespace dladmm {

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

inline int pick_shape(int m, int n) {
  for (int i = 0; i < kNumShapes; ++i)
    if (m <= kShapeMP[i] && n <= kShapeNP[i]) return i;
  return -1;
}

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

struct Plan {
  int path;  // 1 fused, 2 per-layer
  // fused
  int shape, MP, NP, tiles;
  // per-layer
  int KB1, KB2, SB1, SB2, MBp1, MBp2, slices1, slices2, gx;
  int nslots;  // loss partial slots per (layer, term)
  size_t off_ap, off_wp, off_v, off_zw, off_ew, off_lw, off_loss, total;
};

inline int validate(const dladmm_fwd_desc* d) {
  if (!d) return DLADMM_E_NULL;
  if (d->abi_version != DLADMM_ABI_VERSION) return DLADMM_E_ABI_VERSION;
  if (d->variant < DLADMM_V1_LENA || d->variant > DLADMM_V6_LASSO) return DLADMM_E_VARIANT;
  if (d->m < 1 || d->n < 1 || d->batch < 1) return DLADMM_E_SHAPE;
  if (d->layers < 1 || d->layers > DLADMM_MAX_LAYERS) return DLADMM_E_LAYERS;
  if (d->loss_kind < 0 || d->loss_kind > 2) return DLADMM_E_UNSUPPORTED;
  if (!d->X || !d->A || !d->Z0 || !d->E0 || !d->L0 || !d->W || !d->Z || !d->E || !d->L)
    return DLADMM_E_NULL;
  for (int k = 0; k < d->layers; ++k)
    if (!d->W[k]) return DLADMM_E_NULL;
  if (d->loss_kind && !d->loss_sums) return DLADMM_E_NULL;
  const int v = d->variant;
  if (v == DLADMM_V2_LTHETA || v == DLADMM_V3_FULL) {
    if (!d->row_params) return DLADMM_E_NULL;
    if (d->row_stride < d->m || d->row_stride < d->n) return DLADMM_E_SHAPE;
  } else if (!d->scalar_params) {
    return DLADMM_E_NULL;
  }
  if (v == DLADMM_V1_LENA) {
    if (!d->beta1_elem || !d->beta2_elem) return DLADMM_E_NULL;
    for (int k = 0; k < d->layers; ++k)
      if (!d->beta1_elem[k] || !d->beta2_elem[k]) return DLADMM_E_NULL;
    if (d->ld_beta < d->batch) return DLADMM_E_SHAPE;
  }
  const int64_t B = d->batch;
  if (d->ld_x < B || d->ld_z0 < B || d->ld_e0 < B || d->ld_l0 < B || d->ld_out < B)
    return DLADMM_E_SHAPE;
  if (d->ld_a < d->n || d->ld_w < d->m) return DLADMM_E_SHAPE;
  return 0;
}

// The fused kernel addresses every per-column matrix with 32-bit buffer offsets.
inline bool fits_32bit(const dladmm_fwd_desc* d) {
  const int64_t lim = (int64_t)1 << 31;
  const int64_t mx = d->m > d->n ? d->m : d->n;
  return !(mx * d->ld_x * 4 >= lim || mx * d->ld_z0 * 4 >= lim || mx * d->ld_e0 * 4 >= lim ||
           mx * d->ld_l0 * 4 >= lim || mx * d->ld_out * 4 >= lim ||
           (d->variant == DLADMM_V1_LENA && mx * d->ld_beta * 4 >= lim));
}

inline int make_plan(const dladmm_fwd_desc* d, Plan* p) {
  *p = Plan{};
  const int s = pick_shape(d->m, d->n);
  const int K = d->layers;
  const int64_t B = d->batch;
  // DLADMM_PATH=layered forces the per-layer kernels (tests / A-B measurements)
  const char* force = getenv("DLADMM_PATH");
  const bool force_layered = force && force[0] == 'l';
  if (s >= 0 && fits_32bit(d) && !force_layered) {
    p->path = 1;
    p->shape = s;
    p->MP = kShapeMP[s];
    p->NP = kShapeNP[s];
    p->tiles = ceil_div(d->batch, kTileCols);
    p->nslots = p->tiles * kWaves;
    const size_t frag_bytes = (size_t)p->MP * p->NP * sizeof(float);
    p->off_ap = 0;
    p->off_wp = align256(frag_bytes);
    p->off_loss = p->off_wp + align256(frag_bytes * K);
    p->total = p->off_loss + align256((size_t)2 * K * p->nslots * sizeof(float));
    return 0;
  }
  // per-layer path
  p->path = 2;
  const int MB = ceil_div(d->m, 16), NB = ceil_div(d->n, 16);
  p->KB1 = MB;                       // G1 contracts over m
  p->KB2 = NB;                       // G2 contracts over n
  p->SB1 = NB >= 32 ? 32 : 16;       // G1 output rows: n
  p->SB2 = MB >= 32 ? 32 : 16;       // G2 output rows: m
  p->MBp1 = ceil_div(NB, p->SB1) * p->SB1;
  p->MBp2 = ceil_div(MB, p->SB2) * p->SB2;
  p->slices1 = p->MBp1 / p->SB1;
  p->slices2 = p->MBp2 / p->SB2;
  p->gx = ceil_div(d->batch, kLayerCols);
  p->nslots = p->gx * (p->slices1 > p->slices2 ? p->slices1 : p->slices2) * kLayerWaves;
  const size_t fb = (size_t)kFrag * sizeof(float);
  p->off_ap = 0;
  p->off_wp = align256(fb * p->KB2 * p->MBp2);
  p->off_v = p->off_wp + align256(fb * p->KB1 * p->MBp1 * K);
  p->off_zw = p->off_v + align256((size_t)d->m * B * sizeof(float));
  const bool lean = !d->keep_all && K > 1;
  p->off_ew = p->off_zw + (lean ? align256((size_t)d->n * B * sizeof(float)) : 0);
  p->off_lw = p->off_ew + (lean ? align256((size_t)d->m * B * sizeof(float)) : 0);
  p->off_loss = p->off_lw + (lean ? align256((size_t)d->m * B * sizeof(float)) : 0);
  p->total = p->off_loss + align256((size_t)2 * K * p->nslots * sizeof(float));
  return 0;
}

// ---- pack helpers
inline hipError_t pack(const float* const* srcs, int T, int R, int C, int64_t ld, int RB, int CB,
                       int order, float* dst, hipStream_t s, float sign = 1.0f,
                       const float* scal = nullptr) {
  PackArgs pa{};
  for (int t = 0; t < T; ++t) pa.src[t] = srcs[t];
  pa.R = R; pa.C = C; pa.RB = RB; pa.CB = CB; pa.order = order; pa.ld = ld; pa.dst = dst;
  pa.sign = sign; pa.scal = scal;
  hipLaunchKernelGGL(pack_frags_kernel, dim3((RB * CB + 3) / 4, T), dim3(256), 0, s, pa);
  return hipGetLastError();
}

inline int run_fused(const dladmm_fwd_desc* d, const Plan& p, char* ws, hipStream_t s) {
  float* Ap = (float*)(ws + p.off_ap);
  float* Wp = (float*)(ws + p.off_wp);
  float* lossp = (float*)(ws + p.off_loss);
  const int MB = p.MP / 16, NB = p.NP / 16;
  // 1. pack A and every -s1_k W_k into paired MFMA fragment order (zero-padded to MP x NP);
  //    s1 is ss1[k] for V5 and 1.0 in the V4/V6 tables; V1-V3 have no step size
  const float* asrc[1] = {d->A};
  const bool has_s1 = d->variant >= DLADMM_V4_SCALAR;
  if (hipError_t e = pack(asrc, 1, d->m, d->n, d->ld_a, MB, NB, 2, Ap, s)) return (int)e;
  if (hipError_t e = pack(d->W, d->layers, d->n, d->m, d->ld_w, NB, MB, 2, Wp, s, -1.0f,
                          has_s1 ? d->scalar_params : nullptr))
    return (int)e;
  // 2. the fused K-layer forward
  FusedArgs a{};
  a.m = d->m; a.n = d->n; a.B = d->batch; a.K = d->layers;
  a.keep_all = d->keep_all ? 1 : 0; a.loss_kind = d->loss_kind; a.nwaves = p.nslots;
  a.X = d->X; a.ldx = d->ld_x;
  a.Z0 = d->Z0; a.ldz0 = d->ld_z0;
  a.E0 = d->E0; a.lde0 = d->ld_e0;
  a.L0 = d->L0; a.ldl0 = d->ld_l0;
  a.Ap = Ap; a.Wp = Wp;
  a.scal = d->scalar_params;
  a.rowp = d->row_params; a.rstride = d->row_stride;
  a.ldb = d->ld_beta;
  if (d->variant == DLADMM_V1_LENA)
    for (int k = 0; k < d->layers; ++k) { a.b1e[k] = d->beta1_elem[k]; a.b2e[k] = d->beta2_elem[k]; }
  a.Zo = d->Z; a.Eo = d->E; a.Lo = d->L; a.To = d->T; a.ldo = d->ld_out;
  a.lossp = lossp;
  if (d->ev_kernel_start) {
    if (hipError_t e = hipEventRecord((hipEvent_t)d->ev_kernel_start, s)) return (int)e;
  }
  if (hipError_t e = launch_fused_shape(p.shape, d->variant, a, p.tiles, s)) return (int)e;
  if (d->ev_kernel_stop) {
    if (hipError_t e = hipEventRecord((hipEvent_t)d->ev_kernel_stop, s)) return (int)e;
  }
  return 0;
}

inline int run_layered(const dladmm_fwd_desc* d, const Plan& p, char* ws, hipStream_t s) {
  const int K = d->layers, m = d->m, n = d->n;
  const int64_t B = d->batch;
  float* Ap = (float*)(ws + p.off_ap);
  float* Wp = (float*)(ws + p.off_wp);
  float* V = (float*)(ws + p.off_v);
  float* Zw = (float*)(ws + p.off_zw);
  float* Ew = (float*)(ws + p.off_ew);
  float* Lw = (float*)(ws + p.off_lw);
  float* lossp = (float*)(ws + p.off_loss);
  const size_t wl = (size_t)kFrag * p.KB1 * p.MBp1;  // floats per packed W_k
  // 1. pack A (rows m, contraction n) and every W_k (rows n, contraction m), k-major
  const float* asrc[1] = {d->A};
  if (hipError_t e = pack(asrc, 1, m, n, d->ld_a, p.MBp2, p.KB2, 1, Ap, s)) return (int)e;
  if (hipError_t e = pack(d->W, K, n, m, d->ld_w, p.MBp1, p.KB1, 1, Wp, s)) return (int)e;
  if (d->loss_kind) {
    if (hipError_t e = hipMemsetAsync(lossp, 0, (size_t)2 * K * p.nslots * sizeof(float), s))
      return (int)e;
  }
  const bool lean = !d->keep_all;
  const int64_t ldo = d->ld_out;
  const int64_t zl = (int64_t)n * ldo, ml = (int64_t)m * ldo;
  LayerArgs a{};
  a.m = m; a.n = n; a.B = d->batch; a.K = K;
  a.loss_kind = d->loss_kind; a.nslots = p.nslots;
  a.X = d->X; a.ldx = d->ld_x;
  a.Vo = V; a.ldv = B;
  a.scal = d->scalar_params;
  a.rowp = d->row_params; a.rstride = d->row_stride;
  a.ldb = d->ld_beta;
  a.lossp = d->loss_kind ? lossp : nullptr;
  const dim3 g1(p.gx, p.slices1), g2(p.gx, p.slices2);
  const bool v1 = d->variant == DLADMM_V1_LENA;
  if (d->ev_kernel_start) {
    if (hipError_t e = hipEventRecord((hipEvent_t)d->ev_kernel_start, s)) return (int)e;
  }
  // prologue: P0 = A Z0 -> T0, Var0
  {
    LayerArgs b = a;
    b.k = -1; b.KB = p.KB2; b.MBp = p.MBp2; b.Krows = n; b.Wp = Ap;
    b.S = d->Z0; b.ldS = d->ld_z0;
    b.Eprev = d->E0; b.ldep = d->ld_e0; b.Lprev = d->L0; b.ldlp = d->ld_l0;
    b.ldo = ldo;
    b.To = (d->T && !lean) ? d->T : nullptr;
    b.b1n_e = v1 ? d->beta1_elem[0] : nullptr;
    if (hipError_t e = launch_layer(2, d->variant, b, g2, p.SB2, s)) return (int)e;
  }
  for (int k = 0; k < K; ++k) {
    const bool last = k == K - 1;
    // where layer k-1's Z/E/L live, and where layer k's go
    const float* Zp = k == 0 ? d->Z0 : (lean ? Zw : d->Z + (k - 1) * zl);
    const int64_t ldzp = k == 0 ? d->ld_z0 : (lean ? B : ldo);
    const float* Ep = k == 0 ? d->E0 : (lean ? Ew : d->E + (k - 1) * ml);
    const int64_t ldep = k == 0 ? d->ld_e0 : (lean ? B : ldo);
    const float* Lp = k == 0 ? d->L0 : (lean ? Lw : d->L + (k - 1) * ml);
    const int64_t ldlp = k == 0 ? d->ld_l0 : (lean ? B : ldo);
    float* Zo = lean ? (last ? d->Z : Zw) : d->Z + k * zl;
    float* Eo = lean ? (last ? d->E : Ew) : d->E + k * ml;
    float* Lo = lean ? (last ? d->L : Lw) : d->L + k * ml;
    const int64_t ldout = (lean && !last) ? B : ldo;
    // G1(k): Z_k = S(Z_{k-1} - s1 * W_k Var_k)
    LayerArgs b = a;
    b.k = k; b.KB = p.KB1; b.MBp = p.MBp1; b.Krows = m; b.Wp = Wp + k * wl;
    b.S = V; b.ldS = B;
    b.Zprev = Zp; b.ldzp = ldzp;
    b.Zo = Zo; b.ldo = ldout;
    if (hipError_t e = launch_layer(0, d->variant, b, g1, p.SB1, s)) return (int)e;
    // G2(k): P = A Z_k -> E_k, L_k, T_{k+1}, Var_{k+1}
    LayerArgs c = a;
    c.k = k; c.KB = p.KB2; c.MBp = p.MBp2; c.Krows = n; c.Wp = Ap;
    c.S = Zo; c.ldS = ldout;
    c.Eprev = Ep; c.ldep = ldep; c.Lprev = Lp; c.ldlp = ldlp;
    c.Eo = Eo; c.Lo = Lo; c.ldo = ldout;
    c.To = d->T ? (lean ? (last ? d->T : nullptr) : d->T + (k + 1) * ml) : nullptr;
    if (v1) {
      c.b1e = d->beta1_elem[k];
      c.b2e = d->beta2_elem[k];
      c.b1n_e = k + 1 < K ? d->beta1_elem[k + 1] : nullptr;
    }
    if (hipError_t e = launch_layer(1, d->variant, c, g2, p.SB2, s)) return (int)e;
  }
  if (d->ev_kernel_stop) {
    if (hipError_t e = hipEventRecord((hipEvent_t)d->ev_kernel_stop, s)) return (int)e;
  }
  return 0;
}

}  // namespace dladmm

extern "C" {

int dladmm_abi_version(void) { return DLADMM_ABI_VERSION; }

size_t dladmm_fwd_workspace_bytes(const dladmm_fwd_desc* d) {
  using namespace dladmm;
  if (validate(d)) return 0;
  Plan p;
  if (make_plan(d, &p)) return 0;
  return p.total;
}

int dladmm_fwd_path(const dladmm_fwd_desc* d) {
  using namespace dladmm;
  if (int e = validate(d)) return e;
  Plan p;
  if (int e = make_plan(d, &p)) return e;
  return p.path;
}

int dladmm_fwd_f32(const dladmm_fwd_desc* d, void* stream) {
  using namespace dladmm;
  if (int e = validate(d)) return e;
  Plan p;
  if (int e = make_plan(d, &p)) return e;
  if (!d->workspace || d->workspace_bytes < p.total) return DLADMM_E_WORKSPACE;
  if (((uintptr_t)d->workspace) & 255) return DLADMM_E_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)d->workspace;
  const int rc = p.path == 1 ? run_fused(d, p, ws, s) : run_layered(d, p, ws, s);
  if (rc) return rc;
  // per-layer loss sums, fixed-order fp64 reduction of the per-wave partials
  if (d->loss_kind) {
    hipLaunchKernelGGL(loss_reduce_kernel, dim3(2 * d->layers), dim3(256), 0, s,
                       (const float*)(ws + p.off_loss), p.nslots, d->loss_sums);
    if (hipError_t e = hipGetLastError()) return (int)e;
  }
  return 0;
}

const char* dladmm_error_string(int code) {
  switch (code) {
    case 0: return "success";
    case DLADMM_E_ABI_VERSION: return "dladmm: descriptor abi_version mismatch";
    case DLADMM_E_VARIANT: return "dladmm: unknown variant";
    case DLADMM_E_SHAPE: return "dladmm: invalid shape or leading dimension";
    case DLADMM_E_LAYERS: return "dladmm: layers must be in [1, DLADMM_MAX_LAYERS]";
    case DLADMM_E_NULL: return "dladmm: required pointer is NULL";
    case DLADMM_E_WORKSPACE: return "dladmm: workspace missing or too small";
    case DLADMM_E_UNSUPPORTED: return "dladmm: unsupported configuration";
    case DLADMM_E_ALIGN: return "dladmm: workspace must be 256-byte aligned";
  }
  if (code > 0) return hipGetErrorString((hipError_t)code);
  return "dladmm: unknown error";
}

}  // extern "C"
