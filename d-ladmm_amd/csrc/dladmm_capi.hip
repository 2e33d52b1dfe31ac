// dladmm_capi.hip -- the C ABI of include/dladmm.h: descriptor validation, planning, weight
// packing, the loss reduction, and dispatch to the fused (dladmm_fused.hip) or per-layer
// (dladmm_layered.hip) kernels.
#include <math.h>
#include <stdlib.h>

#include <vector>

#include "dladmm_common.h"
#include "dladmm_wgrad_x3.h"
#include "dladmm_internal.h"

namespace dladmm {

// ------------------------------------------------------------------------ weight packing
constexpr int kPackBatch = 64;  // sources per pack launch (the struct is a kernel argument)

struct PackArgs {
  const float* src[kPackBatch];
  int R, C, RB, CB;  // valid rows/cols of each source; row-blocks (padded) / col-blocks packed
  int order;         // fragment (ib, jb) at: 0 ib*CB + jb; 1 jb*RB + ib (per-layer path);
                     // 2 ((ib/2)*CB + jb)*2 + ib%2 (fused path: output blocks in pairs)
  int64_t ld;
  float* dst;
  float sign;          // every element is multiplied by sign * (scal ? scal[t][S1] : 1)
  const float* scal;   // device [T][DLADMM_NSCALAR] (V4-V6 s1) or null
  int trans;           // 1: pack the transpose (element (row, c) = src[c][row])
  int t0;              // scal row of source t is t0 + t
  int bf16;            // 1: v_mfma_f32_16x16x32_bf16 A fragments (16 x 32, 8 bf16 per lane)
  int vec;             // 1: every source 16-B aligned and ld % 4 == 0: a lane's in-range
                       // piece is read with 16-B loads (the same values, fewer instructions)
};
static_assert(sizeof(PackArgs) <= 2048, "kernel argument size");

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
  const float f = p.sign * (p.scal ? p.scal[(p.t0 + t) * DLADMM_NSCALAR + DLADMM_P_S1] : 1.0f);
  const int row = 16 * ib + (lane & 15);
  if (p.bf16) {
    // lane l: M[16 ib + (l & 15)][32 jb + 8 (l >> 4) + j], j = 0..7, rounded to bf16 (RNE)
    const int c8 = 32 * jb + 8 * (lane >> 4);
    const float* s8 = p.src[t];
    bf16x8 v;
    if (p.vec && !p.trans && row < p.R && c8 + 8 <= p.C) {
      const f32x4* q4 = reinterpret_cast<const f32x4*>(s8 + (int64_t)row * p.ld + c8);
      const f32x4 lo = q4[0], hi = q4[1];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[q] = (__bf16)(f * lo[q]);
        v[4 + q] = (__bf16)(f * hi[q]);
      }
      reinterpret_cast<bf16x8*>(p.dst)[((int64_t)t * p.RB * p.CB + fr) * 64 + lane] = v;
      return;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float x = (row < p.R && c8 + q < p.C)
                          ? f * (p.trans ? s8[(int64_t)(c8 + q) * p.ld + row]
                                         : s8[(int64_t)row * p.ld + c8 + q])
                          : 0.0f;
      v[q] = (__bf16)x;
    }
    reinterpret_cast<bf16x8*>(p.dst)[((int64_t)t * p.RB * p.CB + fr) * 64 + lane] = v;
    return;
  }
  const int c0 = 16 * jb + 4 * (lane >> 4);
  const float* s = p.src[t];
  f32x4 v;
  if (p.vec && !p.trans && row < p.R && c0 + 4 <= p.C) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(s + (int64_t)row * p.ld + c0);
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = f * x[q];
    reinterpret_cast<f32x4*>(p.dst)[((int64_t)t * p.RB * p.CB + fr) * 64 + lane] = v;
    return;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
    v[q] = (row < p.R && c0 + q < p.C)
               ? f * (p.trans ? s[(int64_t)(c0 + q) * p.ld + row] : s[(int64_t)row * p.ld + c0 + q])
               : 0.0f;
  reinterpret_cast<f32x4*>(p.dst)[((int64_t)t * p.RB * p.CB + fr) * 64 + lane] = v;
}

// ------------------------------------------------------------------------ zero fill
// Stream-ordered zeroing of workspace regions as a kernel launch rather than hipMemsetAsync: a
// forward captured into a HIP graph (torch.cuda.graph) and replayed measured stale partial sums
// with hipMemsetAsync nodes (tests/test_gpu_graph.py); kernel nodes replay in stream order.
__global__ __launch_bounds__(256) void zero_fill_kernel(uint32_t* p, int64_t words,
                                                        uint8_t* tail, int ntail) {
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (int64_t i = i0; i < words; i += (int64_t)gridDim.x * 256) p[i] = 0u;
  if (i0 < ntail) tail[i0] = 0;
}
inline hipError_t zero_async(void* p, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  const uintptr_t a = (uintptr_t)p;
  const size_t head = (4 - (a & 3)) & 3;  // workspace regions are 256-B aligned: head = 0
  if (head) {
    hipLaunchKernelGGL(zero_fill_kernel, dim3(1), dim3(256), 0, s, (uint32_t*)nullptr,
                       (int64_t)0, (uint8_t*)p, (int)(head < bytes ? head : bytes));
    if (hipError_t e = hipGetLastError()) return e;
    if (head >= bytes) return hipSuccess;
    p = (uint8_t*)p + head;
    bytes -= head;
  }
  const int64_t words = (int64_t)(bytes / 4);
  const int ntail = (int)(bytes & 3);
  int64_t blocks = (words + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks);
  hipLaunchKernelGGL(zero_fill_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (uint32_t*)p,
                     words, (uint8_t*)p + 4 * words, ntail);
  return hipGetLastError();
}

// rows x cols fp32 at leading dimension ld (the tied weight gradient; no hipMemset2DAsync, for
// the same capture reason as zero_async)
__global__ __launch_bounds__(256) void zero_2d_kernel(float* p, int64_t ld, int cols, int rows) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < (int64_t)rows * cols) p[(t / cols) * ld + t % cols] = 0.0f;
}
inline hipError_t zero_2d_async(float* p, int64_t ld, int cols, int rows, hipStream_t s) {
  const int64_t total = (int64_t)rows * cols;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(zero_2d_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p, ld,
                     cols, rows);
  return hipGetLastError();
}

// ------------------------------------------------------------------------ device pointer tables
// dst[0 .. n) = src[0 .. n) for host arrays of device pointers, kPtrChunk entries per launch,
// the values travelling as kernel arguments (graph-capturable; no host buffer outlives the call)
constexpr int kPtrChunk = 64;
struct PtrChunk {
  const void* p[kPtrChunk];
  const void** dst;
  int n;
};
__global__ __launch_bounds__(64) void ptr_table_kernel(const PtrChunk c) {
  if ((int)threadIdx.x < c.n) c.dst[threadIdx.x] = c.p[threadIdx.x];
}
inline hipError_t write_ptr_table(const void* const* src, int n, const void** dst, hipStream_t s) {
  for (int b = 0; b < n; b += kPtrChunk) {
    PtrChunk c{};
    c.n = n - b < kPtrChunk ? n - b : kPtrChunk;
    for (int i = 0; i < c.n; ++i) c.p[i] = src[b + i];
    c.dst = dst + b;
    hipLaunchKernelGGL(ptr_table_kernel, dim3(1), dim3(64), 0, s, c);
    if (hipError_t e = hipGetLastError()) return e;
  }
  return hipSuccess;
}

// ------------------------------------------------------------------------ split-f16 packing
// (DLADMM_PREC_F32_SPLIT, dladmm_fused_x3.hip).  Matrix M (R x C valid, zero padded to RB
// blocks of 16 rows x KS steps of 32) -> per-tensor scale 2^sw (max|M| * 2^sw in [2^14, 2^15)),
// then x = sign * M * 2^sw split into hi = f16(x), lo = f16(x - hi).  Fragment (ib, s) = step
// ib*KS + s: [hi | lo][lane] f16x8, lane l = row 16 ib + (l & 15), element q = column
// 32 s + 16 (q >> 2) + 4 (l >> 4) + (q & 3) -- the k order in which the state registers of two
// consecutive 16-row blocks form one v_mfma_f32_16x16x32_f16 B operand.
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
struct X3PackArgs {
  const float* src[kPackBatch];
  int R, C, RB, KS, t0;
  int64_t ld;
  float sign;
  f16x8_t* dst;          // [T][RB*KS][2][64]
  unsigned* umax;        // [t0 + T] max |M| bits
  int* wexp;             // [t0 + T] scale exponents
};
static_assert(sizeof(X3PackArgs) <= 2048, "kernel argument size");

__global__ __launch_bounds__(256) void absmax_kernel(const X3PackArgs p) {
  const int t = blockIdx.y;
  const float* src = p.src[t];
  const int64_t total = (int64_t)p.R * p.C;
  float mx = 0.0f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256)
    mx = fmaxf(mx, fabsf(src[(i / p.C) * p.ld + i % p.C]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(p.umax + p.t0 + t, __float_as_uint(mx));  // non-negative floats order as uints
  }
}

__global__ __launch_bounds__(256) void pack_x3_kernel(const X3PackArgs p) {
  const int t = blockIdx.y;
  const int st = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (st >= p.RB * p.KS) return;
  const int lane = threadIdx.x & 63;
  const int ib = st / p.KS, ks = st % p.KS;
  int sw = 15 - __builtin_amdgcn_frexp_expf(__uint_as_float(p.umax[p.t0 + t]));
  sw = sw < -126 ? -126 : (sw > 126 ? 126 : sw);
  if (st == 0 && lane == 0) p.wexp[p.t0 + t] = sw;
  const float f = p.sign * __builtin_amdgcn_ldexpf(1.0f, sw);
  const float* src = p.src[t];
  const int row = 16 * ib + (lane & 15);
  f16x8_t hi, lo;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int c = 32 * ks + 16 * (q >> 2) + 4 * (lane >> 4) + (q & 3);
    const float x = (row < p.R && c < p.C) ? src[(int64_t)row * p.ld + c] * f : 0.0f;
    const _Float16 h = (_Float16)x;
    hi[q] = h;
    lo[q] = (_Float16)(x - (float)h);
  }
  f16x8_t* d = p.dst + ((int64_t)t * p.RB * p.KS + st) * 128;
  d[lane] = hi;
  d[64 + lane] = lo;
}

// ------------------------------------------------------------------------ loss reduction
// per-column objective terms: out[r][b] = sum_s part[r][s][b] over the slices, in order
__global__ __launch_bounds__(256) void col_loss_kernel(const float* part, int nslice, int ldl,
                                                       int B, float* out) {
  const int r = blockIdx.y;
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  float s = 0.0f;
  for (int sl = 0; sl < nslice; ++sl) s += part[((int64_t)r * nslice + sl) * ldl + b];
  out[(int64_t)r * B + b] = s;
}

// Backward scalar-parameter slots: sums[sl] = sum_{w < cnt} part[sl][w], fp64, fixed order.
// cnt: entries the owning kernel wrote (BK2's slots theta_z / s1 cover the n-row slices, the
// others the m-row slices).  1024 threads: one launch per layer, no memset of the partials.
__global__ __launch_bounds__(1024) void param_reduce_kernel(const float* part, int stride,
                                                            int cnt_m, int cnt_n, double* sums) {
  __shared__ double red[1024];
  const int sl = blockIdx.x;
  if (sl == DLADMM_P_S1) {  // V5 writes ss1's gradient afterwards; for the others s1 is 1: 0
    if (threadIdx.x == 0) sums[sl] = 0.0;
    return;
  }
  const int cnt = (sl == DLADMM_P_THETA_Z || sl == DLADMM_P_S1) ? cnt_n : cnt_m;
  double s = 0.0;
  for (int w = threadIdx.x; w < cnt; w += 1024) s += (double)part[(int64_t)sl * stride + w];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) sums[sl] = red[0];
}

// fp64 sum of row[0 .. nw) by a 1024-thread block in a fixed order (bitwise reproducible);
// the result is valid in thread 0
__device__ __forceinline__ double fixed_sum_1024(const float* row, int nw, double* red) {
  // 8 independent running sums per thread (loads in flight), combined in a fixed order
  double acc8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int wv = threadIdx.x;
  for (; wv + 7 * 1024 < nw; wv += 8 * 1024) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc8[u] += (double)row[wv + u * 1024];
  }
  for (int u = 0; wv < nw; wv += 1024, ++u) acc8[u & 7] += (double)row[wv];
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += acc8[u];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  return red[0];
}

// sums[i] = sum_w part[i][w] in fp64, fixed order (bitwise reproducible)
__global__ __launch_bounds__(1024) void loss_reduce_kernel(const float* part, int nw, double* sums) {
  __shared__ double red[1024];
  const int i = blockIdx.x;
  const double s = fixed_sum_1024(part + (int64_t)i * nw, nw, red);
  if (threadIdx.x == 0) sums[i] = s;
}

// Reverse sweep, per-row parameters (V2 / V3): out[k][slot][row] (row stride ors) = the
// fixed-order sum of the per-wave partials part[k][slot][row][0 .. nw) (row stride prs >= ors,
// the kernel's padded rows) for the slots in `mask` and the rows the slot has (theta_z: n, the
// others: m); every other entry 0
__global__ __launch_bounds__(1024) void row_reduce_kernel(const float* part, int nw, int prs,
                                                          int ors, int m, int n, unsigned mask,
                                                          double* out) {
  __shared__ double red[1024];
  const int i = blockIdx.x;                 // over [K][8][ors]
  const int row = i % ors, ks = i / ors;    // ks = k * 8 + slot
  const int slot = ks % 8;
  const bool ok = ((mask >> slot) & 1u) && row < (slot == DLADMM_P_THETA_Z ? n : m);
  if (!ok) {
    if (threadIdx.x == 0) out[i] = 0.0;
    return;
  }
  const double s = fixed_sum_1024(part + ((int64_t)ks * prs + row) * nw, nw, red);
  if (threadIdx.x == 0) out[i] = s;
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
  int path;  // 1 fused, 2 per-layer, 3 bf16 tiles, 4 fused split-f16, 5 fused row-split
  // fused
  int shape, MP, NP, tiles;
  // per-layer
  int KB1, KB2, SB1, SB2, MBp1, MBp2, slices1, slices2, gx;
  int nslots;  // loss partials per (layer, term): slices x ldl per-column entries
  int ldl;     // columns per slice
  int nbp;     // bf16 path: 16-column blocks of the packed state
  bool narrow;  // bf16 path: 128-column tiles (two workgroups per CU; DLADMM_F_BF16_WIDE: 256)
  size_t off_ap, off_wp, off_v, off_zb, off_zw, off_ew, off_lw, off_loss, total;
  size_t off_btab;            // path 1, V1: device tables of the per-layer beta pointers
  size_t off_xch, off_xcnt;   // path 6: exchange buffers, hand-off counters
  size_t off_wexp, off_umax;  // path 4
  int64_t ldzw;               // path 4: lean-mode Z_k workspace row stride
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
  if (d->col_loss && !d->loss_kind) return DLADMM_E_UNSUPPORTED;
  if (d->precision != DLADMM_PREC_F32 && d->precision != DLADMM_PREC_BF16 &&
      d->precision != DLADMM_PREC_F32_SPLIT)
    return DLADMM_E_UNSUPPORTED;
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

// The split-f16 kernel moves every batch row in 16-B pieces (4 columns per lane): the batch must
// be a multiple of 4 and the state / output rows 16-B aligned.  Otherwise: the fp32 kernel.
inline bool x3_layout_ok(const dladmm_fwd_desc* d) {
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  return d->batch % 4 == 0 && d->ld_out % 4 == 0 && d->ld_z0 % 4 == 0 && al(d->Z0) &&
         al(d->Z) && al(d->E) && al(d->L) && (!d->T || al(d->T));
}

// every layer uses the same weight tensor (V5 tied, the KM iteration): packed once
inline bool shared_weight(const dladmm_fwd_desc* d) {
  for (int k = 1; k < d->layers; ++k)
    if (d->W[k] != d->W[0]) return false;
  return true;
}

// the split-f16 weight-gradient kernel: precision "f32_split" (make_bwd_plan rounds its chunks
// to whole 32-column sub-chunks), unless fwd.flags holds DLADMM_F_WGRAD_F32
inline bool use_wgrad_x3(bool x3w, const WgradArgs& wa) { return x3w && wgrad_x3_fits(wa); }

// CUs of the current device (cached; the plan is host-only)
inline int device_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return n;
}

// Path 5: the fused kernel's arithmetic with each workgroup's 16 columns' rows split over its 4
// waves, where the fused kernel's 64-column workgroups would leave most CUs idle -- a batch of at
// most three 16-column workgroups per CU (KM ground truth, m = 250, n = 500: 22 / 39 us per step
// at one / two per CU against path 1's 67), e.g. the reference training loops' batches of
// 20 / 25 and BASELINE config 2.  DLADMM_F_NO_ROWSPLIT keeps path 1.
#ifndef DLADMM_RS_PER_CU
#define DLADMM_RS_PER_CU 3  // path 5 up to this many 16-column workgroups per CU: V4 K = 15
                            // with the fused objective, path 5 vs path 1 (ms): B = 4,096 0.52 /
                            // 1.08, 8,192 0.72 / 1.10, 10,000 0.94 / 1.12 (3 per CU), 16,384
                            // 1.28 / 1.17 (profiles/r06_rowsplit_ab.json)
#endif
inline bool use_rowsplit(const dladmm_fwd_desc* d, int shape) {
  return rs_supports(shape, d->variant) && d->precision == DLADMM_PREC_F32 &&
         !(d->flags & DLADMM_F_NO_ROWSPLIT) &&
         ceil_div(d->batch, 16) <= DLADMM_RS_PER_CU * device_cus();
}

// Path 6: the row split spread over four workgroups per 16 columns (exchange through global
// memory once per product), where the whole grid fits one workgroup per CU (B <= 1,024 on 256
// CUs): a quarter of path 5's MFMA cycles per SIMD.  DLADMM_F_NO_XSPLIT keeps path 5.
inline bool use_xsplit(const dladmm_fwd_desc* d, int shape) {
  return use_rowsplit(d, shape) && !(d->flags & DLADMM_F_NO_XSPLIT) &&
         xs_grid(d->batch) <= device_cus();
}

inline int make_plan(const dladmm_fwd_desc* d, Plan* p) {
  *p = Plan{};
  const int s = pick_shape(d->m, d->n);
  const int K = d->layers;
  const int64_t B = d->batch;
  // DLADMM_F_PER_LAYER forces the per-layer kernels (tests / A-B measurements)
  const bool force_layered = (d->flags & DLADMM_F_PER_LAYER) != 0;
  const bool bf16 = d->precision == DLADMM_PREC_BF16;
  // split-f16 fused kernel: register-resident shapes, scalar-parameter variants (V4-V6); other
  // cases run the fp32 kernels (same results up to fp32 GEMM rounding)
  if (s >= 0 && fits_32bit(d) && !force_layered && d->precision == DLADMM_PREC_F32_SPLIT &&
      x3_supports(d->variant) && x3_layout_ok(d)) {
    p->path = 4;
    p->shape = s < 1 ? 1 : s;  // the x3 kernel's smallest instantiation is shape 1
    p->MP = kShapeMP[p->shape];
    p->NP = kShapeNP[p->shape];
    p->tiles = ceil_div(d->batch, kTileCols);
    p->ldl = p->tiles * kTileCols;
    p->nslots = p->ldl;
    p->ldzw = p->ldl;
    const size_t tb = (size_t)p->MP * p->NP * 2 * sizeof(_Float16);  // hi + lo per tensor
    const int nw = shared_weight(d) ? 1 : K;
    p->off_ap = 0;
    p->off_wp = align256(tb);
    p->off_wexp = p->off_wp + align256(tb * nw);
    p->off_umax = p->off_wexp + align256((size_t)(nw + 1) * sizeof(int));
    p->off_zw = p->off_umax + align256((size_t)(nw + 1) * sizeof(unsigned));
    const bool lean = !d->keep_all && K > 1;
    p->off_loss = p->off_zw + (lean ? align256((size_t)2 * d->n * p->ldzw * sizeof(float)) : 0);
    p->off_btab = p->off_loss + align256((size_t)2 * K * p->nslots * sizeof(float));
    p->total = p->off_btab +
               (d->variant == DLADMM_V1_LENA ? align256((size_t)2 * K * sizeof(void*)) : 0);
    return 0;
  }
  if (s >= 0 && fits_32bit(d) && !force_layered && !bf16) {
    p->path = use_xsplit(d, s) ? 6 : use_rowsplit(d, s) ? 5 : 1;
    p->shape = s;
    p->MP = kShapeMP[s];
    p->NP = kShapeNP[s];
    p->tiles = ceil_div(d->batch, kTileCols);
    // per-column objective slots: every column the grid covers (64 / 16 per workgroup)
    p->ldl = p->path >= 5 ? ceil_div(d->batch, 16) * 16 : p->tiles * kTileCols;
    p->nslots = p->ldl;  // one slice
    const size_t frag_bytes = (size_t)p->MP * p->NP * sizeof(float);
    p->off_ap = 0;
    p->off_wp = align256(frag_bytes);
    p->off_loss = p->off_wp + align256(frag_bytes * (shared_weight(d) ? 1 : K));
    p->off_btab = p->off_loss + align256((size_t)2 * K * p->nslots * sizeof(float));
    p->total = p->off_btab +
               (d->variant == DLADMM_V1_LENA ? align256((size_t)2 * K * sizeof(void*)) : 0);
    if (p->path == 6) {  // exchange buffers and hand-off counters of every (padded) group
      const size_t groups = (size_t)xs_grid(d->batch) / 4;
      p->off_xch = p->total;
      p->off_xcnt = p->off_xch + align256(groups * xs_group_floats() * sizeof(float));
      p->total = p->off_xcnt + align256(groups * 64 * sizeof(unsigned));
    }
    return 0;
  }
  // per-layer path; path 3 = bf16 operands: 2-D tiles of 256 x 256, k-blocks of 32
  p->path = bf16 ? 3 : 2;
  const int MB = ceil_div(d->m, 16), NB = ceil_div(d->n, 16);
  p->KB1 = bf16 ? ceil_div(d->m, 32) : MB;  // G1 contracts over m
  p->KB2 = bf16 ? ceil_div(d->n, 32) : NB;  // G2 contracts over n
  p->SB1 = bf16 ? kTileBlocks : (NB >= 32 ? 32 : 16);  // G1 output rows: n
  p->SB2 = bf16 ? kTileBlocks : (MB >= 32 ? 32 : 16);  // G2 output rows: m
  p->MBp1 = ceil_div(NB, p->SB1) * p->SB1;
  p->MBp2 = ceil_div(MB, p->SB2) * p->SB2;
  p->slices1 = p->MBp1 / p->SB1;
  p->slices2 = p->MBp2 / p->SB2;
  // bf16 tile width: 128 columns (2 % faster at config 5) unless DLADMM_F_BF16_WIDE
  p->narrow = bf16 && !(d->flags & DLADMM_F_BF16_WIDE);
  const int cols = bf16 ? bf16_tile_cols(p->narrow) : kLayerCols;
  p->gx = ceil_div(d->batch, cols);
  p->ldl = p->gx * cols;
  p->nbp = p->ldl / 16;
  // loss partial slots per column: one per slice (bf16 tiles: one per slice and wave row)
  p->nslots = p->ldl * (p->slices1 > p->slices2 ? p->slices1 : p->slices2) * (bf16 ? 2 : 1);
  const size_t fb = (size_t)kFrag * sizeof(float);
  p->off_ap = 0;
  p->off_wp = align256(fb * p->KB2 * p->MBp2);
  p->off_v = p->off_wp + align256(fb * p->KB1 * p->MBp1 * (shared_weight(d) ? 1 : K));
  // fp32 Var [m][B], or (bf16) packed Var [KB1][nbp] and packed Z [KB2][nbp] fragments
  p->off_zb = p->off_v + align256(bf16 ? fb * p->KB1 * p->nbp : (size_t)d->m * B * sizeof(float));
  p->off_zw = p->off_zb + (bf16 ? align256(fb * p->KB2 * p->nbp) : 0);
  const bool lean = !d->keep_all && K > 1;
  p->off_ew = p->off_zw + (lean ? align256((size_t)d->n * B * sizeof(float)) : 0);
  p->off_lw = p->off_ew + (lean ? align256((size_t)d->m * B * sizeof(float)) : 0);
  p->off_loss = p->off_lw + (lean ? align256((size_t)d->m * B * sizeof(float)) : 0);
  p->total = p->off_loss + align256((size_t)2 * K * p->nslots * sizeof(float));
  return 0;
}

// ---- pack helpers
// Pack T sources (layer t uses scal row t0 + t) into consecutive [RB*CB] fragment blocks, at
// most kPackBatch sources per launch.
inline hipError_t pack(const float* const* srcs, int T, int R, int C, int64_t ld, int RB, int CB,
                       int order, float* dst, hipStream_t s, float sign = 1.0f,
                       const float* scal = nullptr, int trans = 0, int t0 = 0, int bf16 = 0) {
  for (int b = 0; b < T; b += kPackBatch) {
    const int nb = T - b < kPackBatch ? T - b : kPackBatch;
    PackArgs pa{};
    pa.trans = trans; pa.t0 = t0 + b;
    for (int t = 0; t < nb; ++t) pa.src[t] = srcs[b + t];
    pa.R = R; pa.C = C; pa.RB = RB; pa.CB = CB; pa.order = order; pa.ld = ld;
    pa.dst = dst + (size_t)b * RB * CB * kFrag;
    pa.sign = sign; pa.scal = scal; pa.bf16 = bf16;
    pa.vec = ld % 4 == 0 ? 1 : 0;
    for (int t = 0; t < nb; ++t)
      if ((uintptr_t)pa.src[t] & 15) pa.vec = 0;
    hipLaunchKernelGGL(pack_frags_kernel, dim3((RB * CB + 3) / 4, nb), dim3(256), 0, s, pa);
    if (hipError_t e = hipGetLastError()) return e;
  }
  return hipSuccess;
}

// Device address of the per-wave cycle-sum buffer of the diagnostic stamp builds (built with
// -DX3_STAMP by tools/x3_stamp.py, which passes the address in DLADMM_DBG_PTR); product builds
// compile no stamp code and read nothing
inline unsigned long long* dbg_ptr() {
#if defined(X3_STAMP) && X3_STAMP
  static unsigned long long* const p = [] {
    const char* e = getenv("DLADMM_DBG_PTR");
    return e ? (unsigned long long*)strtoull(e, nullptr, 0) : nullptr;
  }();
  return p;
#else
  return nullptr;
#endif
}

inline int run_fused(const dladmm_fwd_desc* d, const Plan& p, char* ws, hipStream_t s) {
  float* Ap = (float*)(ws + p.off_ap);
  float* Wp = (float*)(ws + p.off_wp);
  float* lossp = (float*)(ws + p.off_loss);
  const int MB = p.MP / 16, NB = p.NP / 16;
  // 1. pack A and every -W_k into paired MFMA fragment order (zero-padded to MP x NP); a weight
  //    shared by every layer is packed once
  const float* asrc[1] = {d->A};
  const bool shared = shared_weight(d);
  if (hipError_t e = pack(asrc, 1, d->m, d->n, d->ld_a, MB, NB, 2, Ap, s)) return (int)e;
  if (hipError_t e = pack(d->W, shared ? 1 : d->layers, d->n, d->m, d->ld_w, NB, MB, 2, Wp, s,
                          -1.0f))
    return (int)e;
  // 2. the fused K-layer forward
  FusedArgs a{};
  a.m = d->m; a.n = d->n; a.B = d->batch; a.K = d->layers;
  a.keep_all = d->keep_all ? 1 : 0; a.loss_kind = d->loss_kind; a.ldl = p.ldl;
  a.X = d->X; a.ldx = d->ld_x;
  a.Z0 = d->Z0; a.ldz0 = d->ld_z0;
  a.E0 = d->E0; a.lde0 = d->ld_e0;
  a.L0 = d->L0; a.ldl0 = d->ld_l0;
  a.Ap = Ap; a.Wp = Wp;
  a.wstep = shared ? 0 : 1;
  a.scal = d->scalar_params;
  a.rowp = d->row_params; a.rstride = d->row_stride;
  a.ldb = d->ld_beta;
  if (d->variant == DLADMM_V1_LENA) {
    // the K per-layer beta pointers of each table go to the workspace (no depth limit), written
    // by a kernel whose arguments carry them: a graph capture records the pointer values with
    // the launch, where a memcpy from the caller's (short-lived) host array would replay from
    // freed memory
    const void** tab = (const void**)(ws + p.off_btab);
    if (hipError_t e = write_ptr_table((const void* const*)d->beta1_elem, d->layers, tab, s))
      return (int)e;
    if (hipError_t e = write_ptr_table((const void* const*)d->beta2_elem, d->layers,
                                       tab + d->layers, s))
      return (int)e;
    a.b1t = (const float* const*)tab;
    a.b2t = (const float* const*)(tab + d->layers);
  }
  a.Zo = d->Z; a.Eo = d->E; a.Lo = d->L; a.To = d->T; a.ldo = d->ld_out;
  a.lossp = lossp;
  a.dbg = dbg_ptr();  // diagnostic builds (DLADMM_STAMP) write per-wave cycle sums here
  // training forwards also store P_k = A Z_k for the backward (fwd_desc.P, keep_all only)
  const bool savep = d->P != nullptr && d->keep_all;
  a.Po = savep ? d->P : nullptr;
  if (d->ev_kernel_start) {
    if (hipError_t e = hipEventRecord((hipEvent_t)d->ev_kernel_start, s)) return (int)e;
  }
  if (p.path == 6) {
    a.xch = (float*)(ws + p.off_xch);
    a.xstride = (int64_t)xs_group_floats();
    a.xcnt = (unsigned*)(ws + p.off_xcnt);
    if (hipError_t e = zero_async(a.xcnt, p.total - p.off_xcnt, s)) return (int)e;
  }
  hipError_t e = p.path == 6 ? launch_fused_xs(p.shape, d->variant, a, s)
                 : p.path == 5
                    ? launch_fused_rs(p.shape, d->variant, a, ceil_div(d->batch, 16), s)
                    : (savep ? launch_fused_shape_savep : launch_fused_shape)(p.shape, d->variant,
                                                                             a, p.tiles, s);
  if (e) return (int)e;
  if (d->ev_kernel_stop) {
    if (hipError_t e = hipEventRecord((hipEvent_t)d->ev_kernel_stop, s)) return (int)e;
  }
  return 0;
}

// absmax + split pack of T sources (scale exponents at wexp[t0 ..]), kPackBatch per launch
inline hipError_t pack_x3(const float* const* srcs, int T, int R, int C, int64_t ld, int RB,
                          int KS, float sign, _Float16* dst, unsigned* umax, int* wexp, int t0,
                          hipStream_t s) {
  for (int b = 0; b < T; b += kPackBatch) {
    const int nb = T - b < kPackBatch ? T - b : kPackBatch;
    X3PackArgs pa{};
    for (int t = 0; t < nb; ++t) pa.src[t] = srcs[b + t];
    pa.R = R; pa.C = C; pa.RB = RB; pa.KS = KS; pa.t0 = t0 + b; pa.ld = ld; pa.sign = sign;
    pa.dst = reinterpret_cast<f16x8_t*>(dst) + (size_t)b * RB * KS * 128;
    pa.umax = umax; pa.wexp = wexp;
    const int blocks = ceil_div((int)(((int64_t)R * C + 255) / 256), 8);
    hipLaunchKernelGGL(absmax_kernel, dim3(blocks < 64 ? blocks : 64, nb), dim3(256), 0, s, pa);
    if (hipError_t e = hipGetLastError()) return e;
    hipLaunchKernelGGL(pack_x3_kernel, dim3(ceil_div(RB * KS, 4), nb), dim3(256), 0, s, pa);
    if (hipError_t e = hipGetLastError()) return e;
  }
  return hipSuccess;
}

inline int run_fused_x3(const dladmm_fwd_desc* d, const Plan& p, char* ws, hipStream_t s) {
  _Float16* Ap = (_Float16*)(ws + p.off_ap);
  _Float16* Wp = (_Float16*)(ws + p.off_wp);
  int* wexp = (int*)(ws + p.off_wexp);
  unsigned* umax = (unsigned*)(ws + p.off_umax);
  const int MB = p.MP / 16, NB = p.NP / 16, KS1 = p.MP / 32, KS2 = p.NP / 32;
  const bool shared = shared_weight(d);
  const int nw = shared ? 1 : d->layers;
  if (hipError_t e = zero_async(umax, (size_t)(nw + 1) * sizeof(unsigned), s)) return (int)e;
  // A (rows m, contraction n) and every -W_k (rows n, contraction m)
  const float* asrc[1] = {d->A};
  if (hipError_t e = pack_x3(asrc, 1, d->m, d->n, d->ld_a, MB, KS2, 1.0f, Ap, umax, wexp, 0, s))
    return (int)e;
  if (hipError_t e = pack_x3(d->W, nw, d->n, d->m, d->ld_w, NB, KS1, -1.0f, Wp, umax, wexp, 1, s))
    return (int)e;
  FusedArgs a{};
  a.m = d->m; a.n = d->n; a.B = d->batch; a.K = d->layers;
  a.keep_all = d->keep_all ? 1 : 0; a.loss_kind = d->loss_kind; a.ldl = p.ldl;
  a.X = d->X; a.ldx = d->ld_x;
  a.Z0 = d->Z0; a.ldz0 = d->ld_z0;
  a.E0 = d->E0; a.lde0 = d->ld_e0;
  a.L0 = d->L0; a.ldl0 = d->ld_l0;
  a.Ap = (const float*)Ap; a.Wp = (const float*)Wp;
  a.wstep = shared ? 0 : 1;
  a.scal = d->scalar_params;
  a.Zo = d->Z; a.Eo = d->E; a.Lo = d->L; a.To = d->T; a.ldo = d->ld_out;
  a.lossp = (float*)(ws + p.off_loss);
  a.wexp = wexp;
  a.Zw = (float*)(ws + p.off_zw); a.ldzw = p.ldzw;
  a.dbg = dbg_ptr();  // diagnostic builds (X3_STAMP) write per-wave cycle sums here
  if (d->variant == DLADMM_V1_LENA) {
    // V1: the per-layer beta pointers as device tables (scalar-loaded per G2 pass, any depth)
    a.ldb = d->ld_beta;
    const void** tab = (const void**)(ws + p.off_btab);
    if (hipError_t e = write_ptr_table((const void* const*)d->beta1_elem, d->layers, tab, s))
      return (int)e;
    if (hipError_t e = write_ptr_table((const void* const*)d->beta2_elem, d->layers,
                                       tab + d->layers, s))
      return (int)e;
    a.b1t = (const float* const*)tab;
    a.b2t = (const float* const*)(tab + d->layers);
  }
  if (d->ev_kernel_start) {
    if (hipError_t e = hipEventRecord((hipEvent_t)d->ev_kernel_start, s)) return (int)e;
  }
  // training forwards also store P_k = A Z_k for the backward (fwd_desc.P, keep_all only)
  const bool savep = d->P != nullptr && d->keep_all;
  a.Po = savep ? d->P : nullptr;
  if (hipError_t e = (savep ? launch_fused_x3_shape_savep : launch_fused_x3_shape)(
          p.shape, d->variant, a, p.tiles, s))
    return (int)e;
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
  const int bf = p.path == 3 ? 1 : 0;
  const int sb1 = p.SB1, sb2 = p.SB2;
  char* Vb = ws + p.off_v;   // bf16: packed Var_k (B operand of G1)
  char* Zb = ws + p.off_zb;  // bf16: packed Z_k / Z0 (B operand of G2)
  auto launch = [&](int phase, const LayerArgs& la, dim3 grid, int sb) -> hipError_t {
    return bf ? launch_tile_bf16(phase, d->variant, p.narrow, la, grid, s)
              : launch_layer(phase, d->variant, la, grid, sb, s);
  };
  // 1. pack A (rows m, contraction n) and every W_k (rows n, contraction m), k-major
  const float* asrc[1] = {d->A};
  if (hipError_t e = pack(asrc, 1, m, n, d->ld_a, p.MBp2, p.KB2, 1, Ap, s, 1.0f, nullptr, 0, 0, bf))
    return (int)e;
  const bool shared = shared_weight(d);
  if (hipError_t e = pack(d->W, shared ? 1 : K, n, m, d->ld_w, p.MBp1, p.KB1, 1, Wp, s, 1.0f,
                          nullptr, 0, 0, bf))
    return (int)e;
  if (d->loss_kind) {
    if (hipError_t e = zero_async(lossp, (size_t)2 * K * p.nslots * sizeof(float), s))
      return (int)e;
  }
  const bool lean = !d->keep_all;
  const int64_t ldo = d->ld_out;
  const int64_t zl = (int64_t)n * ldo, ml = (int64_t)m * ldo;
  LayerArgs a{};
  a.m = m; a.n = n; a.B = d->batch; a.K = K;
  a.loss_kind = d->loss_kind; a.nslots = p.nslots; a.ldl = p.ldl;
  a.X = d->X; a.ldx = d->ld_x;
  a.Vo = bf ? nullptr : V; a.ldv = B;
  a.nbp = p.nbp;
  a.scal = d->scalar_params;
  a.rowp = d->row_params; a.rstride = d->row_stride;
  a.ldb = d->ld_beta;
  a.lossp = d->loss_kind ? lossp : nullptr;
  const dim3 g1(p.gx, p.slices1), g2(p.gx, p.slices2);
  const bool v1 = d->variant == DLADMM_V1_LENA;
  auto run = [&](int phase, const LayerArgs& la, dim3 grid, int sb) -> hipError_t {
    return launch(phase, la, grid, sb);
  };
  if (d->ev_kernel_start) {
    if (hipError_t e = hipEventRecord((hipEvent_t)d->ev_kernel_start, s)) return (int)e;
  }
  // prologue: P0 = A Z0 -> T0, Var0
  {
    LayerArgs b = a;
    b.k = -1; b.KB = p.KB2; b.MBp = p.MBp2; b.Krows = n; b.Wp = Ap;
    b.S = d->Z0; b.ldS = d->ld_z0;
    if (bf) {
      if (hipError_t e = pack_state_bf16(d->Z0, d->ld_z0, n, B, p.KB2, p.nbp, Zb, s))
        return (int)e;
      b.S = (const float*)Zb;
      b.Pb = Vb; b.pb_kb = p.KB1;
    }
    b.Eprev = d->E0; b.ldep = d->ld_e0; b.Lprev = d->L0; b.ldlp = d->ld_l0;
    b.ldo = ldo;
    b.To = (d->T && !lean) ? d->T : nullptr;
    b.b1n_e = v1 ? d->beta1_elem[0] : nullptr;
    if (hipError_t e = run(2, b, g2, sb2)) return (int)e;
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
    b.k = k; b.KB = p.KB1; b.MBp = p.MBp1; b.Krows = m; b.Wp = Wp + (shared ? 0 : k * wl);
    b.S = bf ? (const float*)Vb : V; b.ldS = B;
    b.Zprev = Zp; b.ldzp = ldzp;
    b.Zo = Zo; b.ldo = ldout;
    if (bf) { b.Pb = Zb; b.pb_kb = p.KB2; }
    if (hipError_t e = run(0, b, g1, sb1)) return (int)e;
    // G2(k): P = A Z_k -> E_k, L_k, T_{k+1}, Var_{k+1}
    LayerArgs c = a;
    c.k = k; c.KB = p.KB2; c.MBp = p.MBp2; c.Krows = n; c.Wp = Ap;
    c.S = bf ? (const float*)Zb : Zo; c.ldS = ldout;
    if (bf && !last) { c.Pb = Vb; c.pb_kb = p.KB1; }  // the last Var feeds nothing
    c.Eprev = Ep; c.ldep = ldep; c.Lprev = Lp; c.ldlp = ldlp;
    c.Eo = Eo; c.Lo = Lo; c.ldo = ldout;
    c.To = d->T ? (lean ? (last ? d->T : nullptr) : d->T + (k + 1) * ml) : nullptr;
    if (v1) {
      c.b1e = d->beta1_elem[k];
      c.b2e = d->beta2_elem[k];
      c.b1n_e = k + 1 < K ? d->beta1_elem[k + 1] : nullptr;
    }
    if (hipError_t e = run(1, c, g2, sb2)) return (int)e;
  }
  if (d->ev_kernel_stop) {
    if (hipError_t e = hipEventRecord((hipEvent_t)d->ev_kernel_stop, s)) return (int)e;
  }
  return 0;
}

// ======================================================================== backward driver
struct BwdPlan {
  Plan fwd;                       // the forward's plan (which kernel formed U)
  int MB, NB, SBm, MBpm, NBpn, slices_m, slices_n, gx;
  int64_t Bpad, Rn, Rm;           // padded batch; padded rows of the gU / Var buffers
  int nslots, ncg;
  int wtiles, nchunks; int64_t chunk;
  int wgl;  // reverse path: layers per batched weight-gradient launch
  bool saved_p;                   // BK1 reads the forward's A Z_k (fwd_desc.P)
  bool x3w;                       // weight gradient on the f16 cores (precision "f32_split")
  size_t off_a1, off_at, off_m, off_mt, off_az, off_ae, off_al, off_at_, off_gp, off_var,
      off_part, off_part2, off_wpart, off_s1dot, total;
  // reverse-sweep kernel (dladmm_reverse.hip): packed A^T and M_k^T, gU_k / Var_k of every
  // layer (rows padded to Rn2 / Rm2 for the weight gradient), per-wave parameter partials
  bool rev;
  int rtiles, rncg;
  bool rrs;  // reverse sweep on the row-split kernel (16 columns per workgroup)
  bool rxs;  // ... over four workgroups per 16 columns (bwd path 3, after path 6)
  size_t off_rxcnt, off_rxch;  // rxs: hand-off counters (zeroed with the partials), exchange
  int64_t Rn2, Rm2;
  size_t off_ratp, off_rmtp, off_gu, off_rvar, off_rpart, off_rptab, off_rrow;
};

// plan options of the backward, from the forward descriptor it carries (enum dladmm_flags)
inline bool bwd_flag(const dladmm_fwd_desc& f, int flag) { return (f.flags & flag) != 0; }

inline int validate_bwd(const dladmm_bwd_desc* d) {
  if (!d) return DLADMM_E_NULL;
  if (int e = validate(&d->fwd)) return e;
  const dladmm_fwd_desc& f = d->fwd;
  if (!f.keep_all || !f.T) return DLADMM_E_UNSUPPORTED;
  // backward kernels are fp32; F32_SPLIT moves only the weight-gradient GEMM (make_bwd_plan)
  if (f.precision != DLADMM_PREC_F32 && f.precision != DLADMM_PREC_F32_SPLIT)
    return DLADMM_E_UNSUPPORTED;
  // the backward epilogues address every per-layer matrix with 32-bit buffer offsets
  if (!fits_32bit(&f)) return DLADMM_E_UNSUPPORTED;
  {
    const int64_t mx = f.m > f.n ? f.m : f.n, lim = (int64_t)1 << 31;
    const int64_t bpad = (f.batch + 15) / 16 * 16;
    if (mx * bpad * 4 >= lim || mx * d->ld_g * 4 >= lim) return DLADMM_E_UNSUPPORTED;
  }
  if (!d->gW) return DLADMM_E_NULL;
  if (d->ld_gw < f.m) return DLADMM_E_SHAPE;
  if ((d->gZ || d->gE || d->gL || d->gT) && d->ld_g < f.batch) return DLADMM_E_SHAPE;
  if (d->loss_kind < 0 || d->loss_kind > 2) return DLADMM_E_UNSUPPORTED;
  if (d->loss_kind && !d->loss_coef) return DLADMM_E_NULL;
  const int v = f.variant;
  if (v >= DLADMM_V4_SCALAR && !d->g_scalar) return DLADMM_E_NULL;
  if ((v == DLADMM_V2_LTHETA || v == DLADMM_V3_FULL) && !d->g_row) return DLADMM_E_NULL;
  if (v == DLADMM_V1_LENA) {
    if (!d->g_beta1_elem || !d->g_beta2_elem) return DLADMM_E_NULL;
    for (int k = 0; k < f.layers; ++k)
      if (!d->g_beta1_elem[k] || !d->g_beta2_elem[k]) return DLADMM_E_NULL;
  }
  return 0;
}

inline int64_t round_up(int64_t x, int64_t q) { return (x + q - 1) / q * q; }
inline int64_t K_of(const dladmm_fwd_desc& f) { return f.layers; }

// Largest workspace the reverse sweep may ask for: a quarter of the device's memory (72 GB on an
// MI355X)
inline size_t rev_ws_cap() {
  static size_t cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return (size_t)64 << 30;
  if (!cache[dev]) {
    size_t total = 0;
    cache[dev] = hipDeviceTotalMem(&total, dev) == hipSuccess && total ? total / 4
                                                                        : (size_t)64 << 30;
  }
  return cache[dev];
}

inline int make_bwd_plan(const dladmm_bwd_desc* d, BwdPlan* p) {
  *p = BwdPlan{};
  const dladmm_fwd_desc& f = d->fwd;
  // the backward's kernels are planned on the fp32 forward's geometry whatever GEMM form produced
  // the saved state; fwd_desc.precision "f32_split" (a split-f16 training forward) also moves
  // the weight-gradient GEMM to the f16 matrix cores (x3w)
  dladmm_fwd_desc f32 = f;
  f32.precision = DLADMM_PREC_F32;
  if (int e = make_plan(&f32, &p->fwd)) return e;
  p->x3w = f.precision == DLADMM_PREC_F32_SPLIT && !bwd_flag(f, DLADMM_F_WGRAD_F32);
  // the forward stored A Z_k only on the fused paths, fp32 and split-f16 (fwd_desc.P)
  p->saved_p = f.P != nullptr && f.keep_all &&
               (p->fwd.path == 1 || p->fwd.path == 4 || p->fwd.path >= 5);
  const int m = f.m, n = f.n;
  const int64_t B = f.batch;
  p->MB = ceil_div(m, 16);
  p->NB = ceil_div(n, 16);
  p->SBm = 16;                          // BK1 / BK3 output rows: m (SB = 32 spills registers)
  p->MBpm = ceil_div(p->MB, p->SBm) * p->SBm;
  p->NBpn = ceil_div(p->NB, 32) * 32;   // BK2 output rows: n (16-block slices with two
                                        // accumulator sets, 32-block ones with one: PH 5)
  p->slices_m = p->MBpm / p->SBm;
  p->slices_n = p->NBpn / 16;
  p->gx = ceil_div(f.batch, kBwdCols);
  p->Bpad = round_up(B, 16);
  p->Rn = round_up(n, 128);
  p->Rm = round_up(m, 128);
  p->ncg = p->gx * kBwdWaves;
  p->nslots = p->ncg * (p->slices_m > p->slices_n ? p->slices_m : p->slices_n);
  const int64_t rs = f.row_stride > 0 ? f.row_stride : 1;
  const int64_t part_floats = 8 * (p->nslots > rs * p->ncg ? (int64_t)p->nslots : rs * p->ncg);
  // one reverse-sweep kernel: any variant after a saved-product fused forward, cotangents with
  // the outputs' row stride, 32-bit workspace offsets, workspace under rev_ws_cap()
  // (the conditions include/dladmm.h documents at dladmm_bwd_path)
  p->rev = false;
  // (E0 / L0 addressed with the outputs' row stride)
  // upstream cotangents (a torch-op loss over the returned Z_k / E_k / L_k / T_k, as the
  // reference's training loops build it) ride along when they share the outputs' row stride;
  // V1's per-sample betas and their gradients too
  const bool cot_ok = !(d->gZ || d->gE || d->gL || d->gT) || d->ld_g == f.ld_out;
  const bool v1_ok = f.variant != DLADMM_V1_LENA || f.ld_beta == f.ld_out;
  if (p->saved_p && reverse_supports(f.variant) && cot_ok && v1_ok &&
      f.ld_e0 == f.ld_out && f.ld_l0 == f.ld_out && !bwd_flag(f, DLADMM_F_BWD_PER_LAYER)) {
    const int MP = kShapeMP[p->fwd.shape], NP = kShapeNP[p->fwd.shape];
    // the split-f16 weight gradient runs whole 32-column sub-chunks: pad its operand columns to
    // 32 (the sweep writes zeros up to bpad; its tiles cover 64 columns) so every batch takes it
    const int64_t bpad = p->x3w ? round_up(B, 32) : p->Bpad;
    p->Rn2 = round_up(NP, 128);
    p->Rm2 = round_up(MP, 128);
    const int64_t lim = (int64_t)1 << 31;
    // the sweep keeps gU_k and Var_k of every layer: (Rn2 + Rm2 + MP) x Bpad floats per layer
    // (≈256 MiB per layer at 256 x 512, B = 65,536) where the per-layer phases need O(1) in K;
    // above rev_ws_cap() the per-layer phases run instead of a workspace that may not fit
    const bool rowv = f.variant == DLADMM_V2_LTHETA || f.variant == DLADMM_V3_FULL;
    const size_t rev_bytes = (size_t)(K_of(f) + 1) * MP * NP * 4 +
                             (size_t)K_of(f) * (p->Rn2 + p->Rm2 + MP) * bpad * 4 +
                             (rowv ? (size_t)8 * K_of(f) * (MP > NP ? MP : NP) *
                                         ((B + 63) / 64 * 4) * 4 : 0);
    if ((int64_t)NP * bpad * 4 < lim && 2 * (p->Rm2 + MP) * bpad * 4 < lim &&
        rev_bytes <= rev_ws_cap()) {
      p->rev = true;
      p->Bpad = bpad;
      p->Rn = p->Rn2;  // the weight gradient reads the reverse kernel's row padding
      p->Rm = p->Rm2;
      // after a path-5 forward (a small batch), the row-split sweep: 16 columns per workgroup,
      // each product's rows over its waves (bit-equal gU_k / Var_k)
      // (the forward itself ran path 5: an fp32 forward -- the plan above is recomputed in fp32
      // for every forward precision)
      // At most one workgroup per CU: backward (V4, K = 15, fused objective) 0.68 vs 1.32 ms at
      // B = 25, 1.03 vs 1.66 at 4,096, but 2.42 vs 1.90 at 10,000 (profiles/r06_rowsplit_ab.json)
      p->rrs = p->fwd.path >= 5 && f.precision == DLADMM_PREC_F32 &&
               reverse_rs_supports(p->fwd.shape, f.variant) &&
               ceil_div((int)f.batch, 16) <= device_cus();
      // after a path-6 forward, the same sweep over four workgroups per 16 columns (its grid one
      // workgroup per CU at most, as the forward's)
      p->rxs = p->rrs && p->fwd.path == 6;
      p->rtiles = p->rxs ? xs_grid(f.batch)
                  : p->rrs ? ceil_div(f.batch, 16) : ceil_div(f.batch, kTileCols);
      p->rncg = p->rtiles * kWaves;
    }
  }
  p->wtiles = (int)((p->Rn / 128) * (p->Rm / 128));
  // split-K chunks: whole 16-column k-steps, or 32-column sub-chunks for the split-f16 kernel
  // (the reverse sweep's Bpad is then a multiple of 32; the per-layer backward keeps 16 and its
  // odd-16 chunks take the fp32 kernel)
  const int q = p->x3w && p->rev ? 32 : 16;
  const int64_t steps = p->Bpad / q;
  int64_t nch = (512 + p->wtiles - 1) / p->wtiles;
  if (nch > steps) nch = steps;
  if (nch < 1) nch = 1;
  p->chunk = ceil_div((int)steps, (int)nch) * q;
  p->nchunks = (int)((p->Bpad + p->chunk - 1) / p->chunk);
  const size_t fb = (size_t)kFrag * sizeof(float);
  const size_t colb = (size_t)p->Bpad * sizeof(float);
  size_t o = 0;
  if (p->rev) {
    const size_t wb = (size_t)kShapeMP[p->fwd.shape] * kShapeNP[p->fwd.shape] * sizeof(float);
    const size_t K = (size_t)f.layers;
    p->off_ratp = o; o += align256(wb);
    p->off_rmtp = o; o += align256(wb * K);
    p->off_gu = o; o += align256(colb * p->Rn2 * K);
    // per layer: Var_k rows (Rm2, zero padded for the weight gradient), then MP rows of the
    // adjoint of E_{k-1} (V4) that the next-lower layer's BK1 reads
    p->off_rvar = o; o += align256(colb * (p->Rm2 + kShapeMP[p->fwd.shape]) * K);
    p->off_rpart = o; o += align256(sizeof(float) * DLADMM_NSCALAR * K * p->rncg);
    p->off_rxcnt = o;
    if (p->rxs) o += align256(sizeof(unsigned) * 64 * (size_t)(p->rtiles / 4));
    // the weight gradients of up to wgl layers per launch (one grid over their tiles and
    // chunks; partials <= 256 MiB): no per-layer launch gaps and tails
    const size_t lpart = sizeof(float) * (size_t)p->nchunks * n * m;
    p->wgl = (int)((size_t)256 * 1024 * 1024 / lpart);
    if (p->wgl < 1) p->wgl = 1;
    if (p->wgl > (int)K) p->wgl = (int)K;
    p->off_wpart = o; o += align256(lpart * p->wgl);
    p->off_s1dot = o; o += align256(sizeof(double) * (size_t)s1_dot_blocks(n, m) * K);
    p->off_rptab = o; o += align256(sizeof(void*) * (size_t)(RT_NTAB * K + 1));
    // V2 / V3: per-row partials [K][8][max(MP, NP)][waves] (the kernel's padded rows)
    const bool rowk = f.variant == DLADMM_V2_LTHETA || f.variant == DLADMM_V3_FULL;
    p->off_rrow = o;
    const int RS = kShapeMP[p->fwd.shape] > kShapeNP[p->fwd.shape] ? kShapeMP[p->fwd.shape]
                                                                    : kShapeNP[p->fwd.shape];
    if (rowk) o += align256(sizeof(float) * 8 * K * (size_t)RS * p->rncg);
    p->off_rxch = o;
    if (p->rxs) o += align256(sizeof(float) * rev_xs_group_floats() * (size_t)(p->rtiles / 4));
    p->total = o;
    return 0;
  }
  p->off_a1 = o; o += align256(fb * p->NB * p->MBpm);     // A      [NB][MBpm]   (BK1)
  p->off_at = o; o += align256(fb * p->MB * p->NBpn);     // A^T    [MB][NBpn]   (BK2)
  p->off_m = o; o += align256(fb * p->MB * p->NBpn);      // M_k    [MB][NBpn]   (BK2)
  p->off_mt = o; o += align256(fb * p->NB * p->MBpm);     // M_k^T  [NB][MBpm]   (BK3)
  p->off_az = o; o += align256(colb * p->Rn);
  p->off_ae = o; o += align256(colb * m);
  p->off_al = o; o += align256(colb * m);
  p->off_at_ = o; o += align256(colb * m);
  p->off_gp = o; o += align256(colb * m);
  p->off_var = o; o += align256(colb * p->Rm);
  p->off_part = o; o += align256(sizeof(float) * part_floats);
  p->off_part2 = o; o += align256(sizeof(float) * part_floats);  // phase 6: layers of odd k
  p->off_wpart = o; o += align256(sizeof(float) * (size_t)p->nchunks * n * m);
  p->off_s1dot = o; o += align256(sizeof(double) * (size_t)s1_dot_blocks(n, m));
  p->total = o;
  return 0;
}

// The reverse-sweep kernel: every layer's adjoints in one launch, then the weight gradients of
// the K layers from the gU_k / Var_k it wrote, then the parameter slots.
inline int run_reverse(const dladmm_bwd_desc* d, const BwdPlan& p, char* ws, hipStream_t s) {
  const dladmm_fwd_desc& f = d->fwd;
  const int K = f.layers, m = f.m, n = f.n;
  const int shape = p.fwd.shape, MP = kShapeMP[shape], NP = kShapeNP[shape];
  const int MB = MP / 16, NB = NP / 16;
  float* Atp = (float*)(ws + p.off_ratp);
  float* Mtp = (float*)(ws + p.off_rmtp);
  float* GU = (float*)(ws + p.off_gu);
  float* VAR = (float*)(ws + p.off_rvar);
  float* rpart = (float*)(ws + p.off_rpart);
  float* wpart = (float*)(ws + p.off_wpart);
  const int64_t ldw = p.Bpad, gus = p.Rn2 * ldw, vas = (p.Rm2 + MP) * ldw;
  // A^T (rows n, contraction m) and every M_k^T = (-s1 W_k)^T (rows m, contraction n), in the
  // fused forward's paired fragment order
  const float* asrc[1] = {f.A};
  if (hipError_t e = pack(asrc, 1, n, m, f.ld_a, NB, MB, 2, Atp, s, 1.0f, nullptr, 1))
    return (int)e;
  if (hipError_t e = pack(f.W, K, m, n, f.ld_w, MB, NB, 2, Mtp, s, -1.0f, f.scalar_params, 1, 0))
    return (int)e;
  // slots a variant never writes stay 0; rows past NP / MP (to the weight gradient's 128-row
  // tiles) are never written by the kernel
  if (hipError_t e = zero_async(rpart, p.off_wpart - p.off_rpart, s)) return (int)e;
  for (int k = 0; k < K && (p.Rn2 > NP || p.Rm2 > MP); ++k) {
    if (p.Rn2 > NP)
      if (hipError_t e = zero_async(GU + k * gus + NP * ldw,
                                        (size_t)(p.Rn2 - NP) * ldw * sizeof(float), s))
        return (int)e;
    if (p.Rm2 > MP)
      if (hipError_t e = zero_async(VAR + k * vas + MP * ldw,
                                        (size_t)(p.Rm2 - MP) * ldw * sizeof(float), s))
        return (int)e;
  }
  RevArgs r{};
  r.m = m; r.n = n; r.B = (int)f.batch; r.K = K;
  r.loss_kind = d->loss_kind; r.ncg = p.rncg;
  r.Bw = p.Bpad;
  r.X = f.X; r.ldx = f.ld_x;
  r.E0 = f.E0; r.lde0 = f.ld_e0;
  r.L0 = f.L0; r.ldl0 = f.ld_l0;
  r.Z = f.Z; r.E = f.E; r.L = f.L; r.T = f.T; r.P = f.P; r.ldo = f.ld_out;
  r.Atp = Atp; r.Mtp = Mtp;
  r.scal = f.scalar_params;
  r.lcoef = d->loss_kind ? d->loss_coef : nullptr;
  r.GU = GU; r.VAR = VAR; r.ldw = ldw; r.gus = gus; r.vas = vas;
  r.aer = p.Rm2;
  r.part = rpart;
  // the sweep's pointer table (cotangents, V1's betas and their gradients), written by a kernel
  // whose arguments carry the pointers (graph-capturable; the host array dies with this call)
  {
    std::vector<const void*> tab((size_t)RT_NTAB * K + 1, nullptr);
    auto put = [&](int t, const void* const* src, int cnt) {
      for (int k = 0; src && k < cnt; ++k) tab[rev_tab_at(t, K, k)] = src[k];
    };
    put(RT_GZ, (const void* const*)d->gZ, K);
    put(RT_GE, (const void* const*)d->gE, K);
    put(RT_GL, (const void* const*)d->gL, K);
    put(RT_GT, (const void* const*)d->gT, K + 1);
    if (f.variant == DLADMM_V1_LENA) {
      put(RT_B1, (const void* const*)f.beta1_elem, K);
      put(RT_B2, (const void* const*)f.beta2_elem, K);
      put(RT_GB1, (const void* const*)d->g_beta1_elem, K);
      put(RT_GB2, (const void* const*)d->g_beta2_elem, K);
    }
    const void** ptab = (const void**)(ws + p.off_rptab);
    if (hipError_t e = write_ptr_table(tab.data(), (int)tab.size(), ptab, s)) return (int)e;
    r.ptab = (const float* const*)ptab;
  }
  r.has_gz = d->gZ ? 1 : 0;
  r.has_cot = (d->gE || d->gL || d->gT) ? 1 : 0;
  const bool rowk = f.variant == DLADMM_V2_LTHETA || f.variant == DLADMM_V3_FULL;
  if (rowk) {
    r.rowp = f.row_params; r.rstride = f.row_stride;
    r.rpart = (float*)(ws + p.off_rrow);
  }
  if (p.rxs) {
    r.xch = (float*)(ws + p.off_rxch);
    r.xstride = (int64_t)rev_xs_group_floats();
    r.xcnt = (unsigned*)(ws + p.off_rxcnt);   // zeroed with the partials above
  }
  if (hipError_t e = p.rxs ? launch_reverse_xs(shape, f.variant, r, s)
                     : p.rrs ? launch_reverse_rs(shape, f.variant, r, p.rtiles, s)
                             : launch_reverse_shape(shape, f.variant, r, p.rtiles, s))
    return (int)e;
  // weight gradients gW_k = -s1 gU_k Var_k^T (split-K over the batch, fixed-order reduction),
  // layers K-1 .. 0 as the per-layer sweep visits them (a tied weight sums them in that order);
  // V5: each layer's <W, gU_k Var_k^T> for ss1_k's gradient
  const bool tied = d->gw_sum != 0, v5 = f.variant == DLADMM_V5_TIED;
  double* s1dot = (double*)(ws + p.off_s1dot);
  const int nbd = s1_dot_blocks(n, m);
  if (tied)
    if (hipError_t e = zero_2d_async(d->gW, d->ld_gw, m, n, s)) return (int)e;
  // batches of wgl layers, highest first (the tied sum keeps the per-layer order K-1 .. 0)
  // V5 with distinct per-layer weights (not what the module passes): one layer per batch, so
  // each layer's <W_k, G_k> reads its own W_k
  bool wsame = true;
  for (int k = 1; k < K; ++k) wsame = wsame && f.W[k] == f.W[0];
  const int wgl = v5 && !wsame ? 1 : p.wgl;
  for (int khi = K - 1; khi >= 0; khi -= wgl) {
    const int nl = khi + 1 < wgl ? khi + 1 : wgl, klo = khi - nl + 1;
    WgradArgs wa{};
    wa.G = GU + klo * gus; wa.V = VAR + klo * vas; wa.ld = ldw; wa.n = n; wa.m = m;
    wa.NBp16 = (int)(p.Rn2 / 16); wa.MBp16 = (int)(p.Rm2 / 16);
    wa.Bpad = p.Bpad; wa.chunk = p.chunk; wa.nchunks = p.nchunks; wa.part = wpart;
    wa.gls = gus; wa.vls = vas; wa.pls = (int64_t)p.nchunks * n * m;
    // precision "f32_split": the weight-gradient GEMM on the f16 matrix cores with exactly split
    // operands too (dladmm_wgrad_x3.hip; DLADMM_WGRAD_X3=0 keeps the fp32-MFMA kernel)
    if (hipError_t e = (use_wgrad_x3(p.x3w, wa) ? launch_wgrad_x3 : launch_wgrad)(wa, p.wtiles, s, nl))
      return (int)e;
    WredArgs ra{};
    ra.part = wpart; ra.pls = wa.pls; ra.nchunks = p.nchunks; ra.nm = (int64_t)n * m;
    ra.scal = f.scalar_params; ra.klo = klo; ra.nl = nl; ra.tied = tied ? 1 : 0;
    ra.gW = d->gW; ra.gls = (int64_t)n * d->ld_gw; ra.ldgw = d->ld_gw; ra.m = m;
    ra.Wd = v5 ? f.W[klo] : nullptr; ra.ldwd = f.ld_w;  // V5: the batch's (shared) weight
    ra.dotp = v5 ? s1dot : nullptr; ra.nbd = nbd;
    if (hipError_t e = launch_wgrad_reduce_layers(ra, s)) return (int)e;
  }
  // parameter slots of every layer: fixed-order fp64 sums of the per-wave partials (V1: its
  // per-sample beta gradients were written elementwise by the sweep)
  if (rowk) {
    // V2: theta_z, beta1 (BK3), beta3 (its L term), beta2, theta_e; V3 also ss2
    unsigned mask = (1u << DLADMM_P_THETA_Z) | (1u << DLADMM_P_BETA1) | (1u << DLADMM_P_BETA3) |
                    (1u << DLADMM_P_BETA2) | (1u << DLADMM_P_THETA_E);
    if (f.variant == DLADMM_V3_FULL) mask |= 1u << DLADMM_P_SS2;
    hipLaunchKernelGGL(row_reduce_kernel, dim3((unsigned)(8 * K * f.row_stride)), dim3(1024), 0,
                       s, (const float*)r.rpart, p.rncg, MP > NP ? MP : NP, (int)f.row_stride, m,
                       n, mask, d->g_row);
    if (hipError_t e = hipGetLastError()) return (int)e;
  } else if (f.variant != DLADMM_V1_LENA) {
    hipLaunchKernelGGL(loss_reduce_kernel, dim3((unsigned)(DLADMM_NSCALAR * K)), dim3(1024), 0,
                       s, (const float*)rpart, p.rncg, d->g_scalar);
    if (hipError_t e = hipGetLastError()) return (int)e;
  }
  for (int k = 0; k < K && v5; ++k)
    if (hipError_t e = launch_s1_dot_finish(s1dot + (int64_t)k * nbd, n, m,
                                            d->g_scalar + (int64_t)k * DLADMM_NSCALAR +
                                                DLADMM_P_S1, s))
      return (int)e;
  return 0;
}

inline int run_bwd(const dladmm_bwd_desc* d, const BwdPlan& p, char* ws, hipStream_t s) {
  if (p.rev) return run_reverse(d, p, ws, s);
  const dladmm_fwd_desc& f = d->fwd;
  const int K = f.layers, m = f.m, n = f.n;
  const int64_t B = f.batch, ldo = f.ld_out, ldw = p.Bpad;
  const int v = f.variant;
  const bool has_s1 = v >= DLADMM_V4_SCALAR;
  const bool tied = d->gw_sum != 0;
  const bool rowk = v == DLADMM_V2_LTHETA || v == DLADMM_V3_FULL;
  float* A1 = (float*)(ws + p.off_a1);
  float* At = (float*)(ws + p.off_at);
  float* Mp = (float*)(ws + p.off_m);
  float* Mt = (float*)(ws + p.off_mt);
  float* AZ = (float*)(ws + p.off_az);
  float* AE = (float*)(ws + p.off_ae);
  float* AL = (float*)(ws + p.off_al);
  float* AT = (float*)(ws + p.off_at_);
  float* GP = (float*)(ws + p.off_gp);
  float* VAR = (float*)(ws + p.off_var);
  float* const part = (float*)(ws + p.off_part);
  float* wpart = (float*)(ws + p.off_wpart);
  // adjoints start at zero; the padded rows / columns of gU and Var stay zero (wgrad reads them)
  if (hipError_t e = zero_async(ws + p.off_az, p.off_part - p.off_az, s)) return (int)e;
  if (tied) {
    if (hipError_t e = zero_2d_async(d->gW, d->ld_gw, m, n, s)) return (int)e;
  }
  const bool v5 = v == DLADMM_V5_TIED;
  double* s1dot = (double*)(ws + p.off_s1dot);
  const float* asrc[1] = {f.A};
  // BK1 operand: A (rows m, contraction n); BK2 operand: A^T (rows n, contraction m)
  if (hipError_t e = pack(asrc, 1, m, n, f.ld_a, p.MBpm, p.NB, 1, A1, s)) return (int)e;
  if (hipError_t e = pack(asrc, 1, n, m, f.ld_a, p.NBpn, p.MB, 1, At, s, 1.0f, nullptr, 1))
    return (int)e;
  const int64_t zl = (int64_t)n * ldo, ml = (int64_t)m * ldo;
  BwdArgs a{};
  a.m = m; a.n = n; a.B = (int)B; a.K = K;
  a.nslots = p.nslots; a.ncg = p.ncg;
  a.X = f.X; a.ldx = f.ld_x;
  a.ldg = d->ld_g;
  a.loss_kind = d->loss_kind;
  a.lcoef = d->loss_coef;
  a.AZ = AZ; a.AE = AE; a.AL = AL; a.AT = AT; a.GP = GP; a.VAR = VAR; a.ldw = ldw;
  a.scal = f.scalar_params;
  a.rowp = f.row_params; a.rstride = f.row_stride;
  a.ldb = f.ld_beta;
  a.part = part;
  const dim3 gm(p.gx, p.slices_m), gn(p.gx, p.slices_n);
  const size_t part_bytes = p.off_part2 - p.off_part;
  // with the forward's saved products (p.saved_p) BK1 of layer k-1 runs inside BK3(k)'s launch
  // (phase 6); the parameter-slot partials of layer k then live in part buffer k & 1 (layer k's
  // BK1 slots are written one iteration before its BK2 / BK3 ones)
  const bool fuse = p.saved_p && !bwd_flag(f, DLADMM_F_BWD_UNFUSED);
  float* part2 = (float*)(ws + p.off_part2);
  auto partk = [&](int k) { return (fuse && (k & 1)) ? part2 : part; };
  // phase 4: a wave covers 64 columns (one per lane), so its grid has a quarter of the tiles
  const dim3 gm4(ceil_div((int)B, 64 * kBwdWaves), p.slices_m);
  auto layer_args = [&](BwdArgs& x, int k) {
    x.k = k;
    x.Ep = k ? f.E + (k - 1) * ml : f.E0; x.ldep = k ? ldo : f.ld_e0;
    x.Lp = k ? f.L + (k - 1) * ml : f.L0; x.ldlp = k ? ldo : f.ld_l0;
    x.Zp = k ? f.Z + (k - 1) * zl : f.Z0; x.ldzp = k ? ldo : f.ld_z0;
    x.Tk = f.T + k * ml; x.ldt = ldo;
    x.gZ = d->gZ ? d->gZ[k] : nullptr;
    x.gE = d->gE ? d->gE[k] : nullptr;
    x.gL = d->gL ? d->gL[k] : nullptr;
    x.gT = d->gT ? d->gT[k + 1] : nullptr;
    if (v == DLADMM_V1_LENA) {
      x.b1e = f.beta1_elem[k]; x.b2e = f.beta2_elem[k];
      x.gb1e = d->g_beta1_elem[k]; x.gb2e = d->g_beta2_elem[k];
    }
    x.part = partk(k);
  };
  if (fuse) {
    // scalar kinds: every slot of both buffers is rewritten per layer, zeroed once; per-row
    // kinds re-zero a buffer before its layer's first write
    if (hipError_t e = zero_async(rowk ? partk(K - 1) : part,
                                      rowk ? part_bytes : 2 * part_bytes, s))
      return (int)e;
    BwdArgs b1 = a;
    layer_args(b1, K - 1);
    b1.Pk = f.P + (int64_t)(K - 1) * ml;
    if (hipError_t e = launch_bwd(4, v, b1, gm4, p.SBm, s)) return (int)e;
  }
  for (int k = K - 1; k >= 0; --k) {
    // W_k (q = W_k Var_k; both forward paths formed U = Z_{k-1} - s1 q bit for bit) and
    // (-s1 W_k)^T
    const float* wsrc[1] = {f.W[k]};
    if (hipError_t e = pack(wsrc, 1, n, m, f.ld_w, p.NBpn, p.MB, 1, Mp, s)) return (int)e;
    if (hipError_t e = pack(wsrc, 1, m, n, f.ld_w, p.MBpm, p.NB, 1, Mt, s, -1.0f,
                            has_s1 ? f.scalar_params : nullptr, 1, k))
      return (int)e;
    // scalar kinds: every slot's entries are rewritten per layer (counts fixed), so the
    // partials are zeroed once; per-row kinds re-zero (rows past m/n are never written)
    if (!fuse && (rowk || k == K - 1))
      if (hipError_t e = zero_async(part, part_bytes, s)) return (int)e;
    layer_args(a, k);
    if (!fuse) {
      // BK1: P = A Z_k, recomputed -- or (phase 4) read from the forward's saved P_k, the same
      // values bit for bit (the forward's own product), which leaves BK1 without a GEMM
      BwdArgs b1 = a;
      b1.KB = p.NB; b1.MBp = p.MBpm; b1.Krows = n; b1.Wp = A1;
      b1.S = f.Z + k * zl; b1.ldS = ldo;
      b1.Pk = p.saved_p ? f.P + k * ml : nullptr;
      if (hipError_t e = launch_bwd(p.saved_p ? 4 : 1, v, b1, p.saved_p ? gm4 : gm, p.SBm, s))
        return (int)e;
    }
    // BK2: R = A^T gP, q = M_k Var_k
    BwdArgs b2 = a;
    b2.KB = p.MB; b2.MBp = p.NBpn; b2.Krows = m;
    b2.Wp = At; b2.S = GP; b2.ldS = ldw;
    b2.Wp2 = Mp; b2.S2 = VAR; b2.ldS2 = ldw;
    // S'(U_k) from the saved Z_k unless a parameter scales W_k Var_k (V5's ss1) or theta_z is
    // per row (V2, V3); the kernel also checks theta_z >= 0
    b2.Zk = f.Z + k * zl; b2.ldzk = ldo;
    // (V5: ss1's gradient comes from the weight gradient's sums, so q is not needed either)
    const bool zm = v == DLADMM_V1_LENA || v == DLADMM_V4_SCALAR || v == DLADMM_V5_TIED ||
                    v == DLADMM_V6_LASSO;
    // per-row theta_z (V2, V3): PH 5 when no row of the layer has theta_z < 0 (checked on the
    // device), PH 2 otherwise (DLADMM_BWD_ZMASK=0: the recomputing PH 2 for these too -- A/B
    // and equivalence tests)
    const bool zrow = (v == DLADMM_V2_LTHETA || v == DLADMM_V3_FULL) && !bwd_flag(f, DLADMM_F_BWD_NO_ZMASK);
    // mask variants: a PH 5 launch (32-block slices, one GEMM) does the layer when theta_z >= 0,
    // the PH 2 launch when theta_z < 0; the other exits at once (the sign is read on the device)
    // (per-row kinds: the PH 5 launch when every row's theta_z >= 0, else the PH 2 launch)
    b2.zk_mask = (zm || zrow) ? 2 : 0;
    if (zm || zrow) {
      if (hipError_t e = launch_bwd(5, v, b2, dim3(p.gx, p.slices_n / 2), 32, s)) return (int)e;
    }
    if (hipError_t e = launch_bwd(2, v, b2, gn, 16, s)) return (int)e;
    // weight gradient gW_k = -s1 * gU Var_k^T (split-K over the batch, fixed-order reduction);
    // before BK3: with phase 6 that launch overwrites Var with Var_{k-1}
    WgradArgs wa{};
    wa.G = AZ; wa.V = VAR; wa.ld = ldw; wa.n = n; wa.m = m;
    wa.NBp16 = (int)(p.Rn / 16); wa.MBp16 = (int)(p.Rm / 16);
    wa.Bpad = p.Bpad; wa.chunk = p.chunk; wa.nchunks = p.nchunks; wa.part = wpart;
    // split-f16 GEMM after a split-f16 forward, as on the reverse sweep
    if (hipError_t e = (use_wgrad_x3(p.x3w, wa) ? launch_wgrad_x3 : launch_wgrad)(wa, p.wtiles, s, 1))
      return (int)e;
    float* gWk = tied ? d->gW : d->gW + (int64_t)k * n * d->ld_gw;
    if (hipError_t e = launch_wgrad_reduce(wpart, p.nchunks, n, m,
                                           has_s1 ? f.scalar_params : nullptr, k, tied ? 1 : 0,
                                           gWk, d->ld_gw, s, v5 ? f.W[k] : nullptr, f.ld_w,
                                           v5 ? s1dot : nullptr))
      return (int)e;
    // BK3: gVar = M_k^T gU -- with phase 6 fused with BK1 of layer k-1
    BwdArgs b3 = a;
    b3.KB = p.NB; b3.MBp = p.MBpm; b3.Krows = n; b3.Wp = Mt;
    b3.S = AZ; b3.ldS = ldw;
    if (fuse && k > 0) {
      layer_args(b3, k - 1);           // the BK1 layer
      b3.Pk = f.P + (int64_t)(k - 1) * ml;
      b3.k3 = k;
      b3.Tk3 = f.T + k * ml;
      if (v == DLADMM_V1_LENA) { b3.b1e3 = f.beta1_elem[k]; b3.gb1e3 = d->g_beta1_elem[k]; }
      b3.part3 = partk(k);
      if (rowk)
        if (hipError_t e = zero_async(partk(k - 1), part_bytes, s)) return (int)e;
      if (hipError_t e = launch_bwd(6, v, b3, gm, p.SBm, s)) return (int)e;
    } else {
      if (hipError_t e = launch_bwd(3, v, b3, gm, p.SBm, s)) return (int)e;
    }
    float* const pk = partk(k);   // this layer's slots, for the reductions below
    // parameter slots: fixed-order fp64 sums of the per-wave partials
    if (v >= DLADMM_V4_SCALAR) {
      hipLaunchKernelGGL(param_reduce_kernel, dim3(DLADMM_NSCALAR), dim3(1024), 0, s,
                         (const float*)pk, p.nslots, p.gx * kBwdWaves * p.slices_m,
                         p.gx * kBwdWaves * p.slices_n,
                         d->g_scalar + (int64_t)k * DLADMM_NSCALAR);
      if (hipError_t e = hipGetLastError()) return (int)e;
      if (v5)  // ss1_k: the weight gradient's <W, gU_k Var_k^T> replaces BK2's partials
        if (hipError_t e = launch_s1_dot_finish(s1dot, n, m, d->g_scalar +
                                                (int64_t)k * DLADMM_NSCALAR + DLADMM_P_S1, s))
          return (int)e;
    } else if (rowk) {
      hipLaunchKernelGGL(loss_reduce_kernel, dim3((unsigned)(DLADMM_NSCALAR * f.row_stride)),
                         dim3(1024), 0, s, (const float*)pk, p.ncg,
                         d->g_row + (int64_t)k * DLADMM_NSCALAR * f.row_stride);
      if (hipError_t e = hipGetLastError()) return (int)e;
    }
  }
  return 0;
}

// x *= *s, unless *s == 1 (read on the device: no host synchronisation; the common
// total.backward() scale 1 costs one launch)
__global__ __launch_bounds__(256) void scale_if_kernel(float* x, int64_t n, const float* s) {
  const float v = *s;
  if (v == 1.0f) return;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    x[i] *= v;
}

// ---- fused main_lena.py objective (dladmm_lena.hip)
struct LenaPlan {
  int shape, MP, NP, tiles, ldl;
  bool rs;  // the row-split form (16 columns per workgroup) at small batches
  size_t off_ap, off_atp, off_part, total;
};

inline int lena_plan(const dladmm_lena_desc* d, LenaPlan* p) {
  *p = LenaPlan{};
  if (!d) return DLADMM_E_NULL;
  if (d->abi_version != DLADMM_ABI_VERSION) return DLADMM_E_ABI_VERSION;
  if (d->m < 1 || d->n < 1 || d->batch < 1) return DLADMM_E_SHAPE;
  if (d->layers < 1 || d->layers > 65535) return DLADMM_E_LAYERS;  // grid.y
  if (d->mode < 0 || d->mode > 2) return DLADMM_E_UNSUPPORTED;
  if (d->lx_negate != 0 && d->lx_negate != 1) return DLADMM_E_UNSUPPORTED;
  if (!d->X || !d->A || !d->E || !d->L) return DLADMM_E_NULL;
  if (d->mode != 1 && !d->sums) return DLADMM_E_NULL;
  if (d->mode != 0 && (!d->gE || !d->gL || !d->coef)) return DLADMM_E_NULL;
  const int64_t B = d->batch;
  if (d->ld < B || d->ld_x < B || d->ld_a < d->n) return DLADMM_E_SHAPE;
  if (d->layers > 1 && d->layer_stride < (int64_t)d->m * d->ld) return DLADMM_E_SHAPE;
  if (d->mode != 0) {
    if (d->ld_g < B) return DLADMM_E_SHAPE;
    if (d->layers > 1 && d->g_layer_stride < (int64_t)d->m * d->ld_g) return DLADMM_E_SHAPE;
  }
  const int s = pick_shape(d->m, d->n);
  if (s < 0) return DLADMM_E_UNSUPPORTED;
  // 32-bit buffer offsets per layer.  The kernel walks the instantiation's padded rows
  // (kShapeMP[s] >= m), and a lane outside the batch starts at kOOB = 2^31 plus the row offset:
  // that sum must stay below 2^32 to land out of range, so the padded extent is what is bounded
  // (ADVICE r04).  The same holds for the loss-partial rows (4K rows of ldl floats).
  const int64_t lim = (int64_t)1 << 31;
  const int64_t MPs = kShapeMP[s];
  if (MPs * d->ld * 4 >= lim || MPs * d->ld_x * 4 >= lim ||
      (d->mode != 0 && MPs * d->ld_g * 4 >= lim))
    return DLADMM_E_UNSUPPORTED;
  p->shape = s;
  p->MP = kShapeMP[s];
  p->NP = kShapeNP[s];
  // at most one 16-column workgroup per CU at the 256 x 512 shape: the row-split kernel
  p->rs = s == 2 && ceil_div(d->batch, 16) <= device_cus();
  p->tiles = p->rs ? ceil_div(d->batch, 16) : ceil_div(d->batch, kTileCols);
  p->ldl = p->tiles * (p->rs ? 16 : kTileCols);
  if (d->mode != 1 && (int64_t)16 * d->layers * p->ldl >= lim) return DLADMM_E_UNSUPPORTED;
  const size_t fb = (size_t)p->MP * p->NP * sizeof(float);
  p->off_ap = 0;
  p->off_atp = align256(fb);
  p->off_part = p->off_atp + align256(fb);
  p->total = p->off_part +
             (d->mode != 1 ? align256((size_t)4 * d->layers * p->ldl * sizeof(float)) : 0);
  return 0;
}

}  // namespace dladmm

extern "C" {

size_t dladmm_lena_workspace_bytes(const dladmm_lena_desc* d) {
  using namespace dladmm;
  LenaPlan p;
  return lena_plan(d, &p) ? 0 : p.total;
}

int dladmm_lena_f32(const dladmm_lena_desc* d, void* stream) {
  using namespace dladmm;
  LenaPlan p;
  if (int e = lena_plan(d, &p)) return e;
  if (!d->workspace || d->workspace_bytes < p.total) return DLADMM_E_WORKSPACE;
  if (((uintptr_t)d->workspace) & 255) return DLADMM_E_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  char* ws = (char*)d->workspace;
  float* Ap = (float*)(ws + p.off_ap);
  float* Atp = (float*)(ws + p.off_atp);
  const int MB = p.MP / 16, NB = p.NP / 16;
  const float* asrc[1] = {d->A};
  if (hipError_t e = pack(asrc, 1, d->m, d->n, d->ld_a, MB, NB, 2, Ap, s)) return (int)e;
  if (hipError_t e = pack(asrc, 1, d->n, d->m, d->ld_a, NB, MB, 2, Atp, s, 1.0f, nullptr, 1))
    return (int)e;
  LenaArgs a{};
  a.m = d->m; a.n = d->n; a.B = d->batch; a.K = d->layers; a.mode = d->mode; a.ldl = p.ldl;
  a.alpha = d->alpha; a.inv_mb = d->inv_mb; a.inv_nb = d->inv_nb;
  a.xsign = d->lx_negate ? -1.0f : 1.0f;
  for (int i = 0; i < 2; ++i) {  // dual_gap constants (dladmm_lena.hip)
    const double c = i == 0 ? (double)d->alpha : 1.0;
    a.gc[4 * i + 0] = (float)c;
    a.gc[4 * i + 1] = (float)(1.0 + exp(-2.0 * c));
    a.gc[4 * i + 2] = (float)exp(-c);
    a.gc[4 * i + 3] = (float)(exp(c) + exp(-c));
  }
  a.X = d->X; a.ldx = d->ld_x;
  a.E = d->E; a.L = d->L; a.ls = d->layer_stride; a.ld = d->ld;
  a.Ap = Ap; a.Atp = Atp;
  a.part = (float*)(ws + p.off_part);
  a.gE = d->gE; a.gL = d->gL; a.gls = d->g_layer_stride; a.ldg = d->ld_g;
  a.coef = d->coef;
  if (hipError_t e = p.rs ? launch_lena_rs(a, p.tiles, s) : launch_lena(p.shape, a, p.tiles, s))
    return (int)e;
  if (d->mode != 1) {
    hipLaunchKernelGGL(loss_reduce_kernel, dim3((unsigned)(4 * d->layers)), dim3(1024), 0, s,
                       (const float*)a.part, p.ldl, d->sums);
    if (hipError_t e = hipGetLastError()) return (int)e;
  }
  return 0;
}

int dladmm_scale_f32(float* x, int64_t n, const float* s, void* stream) {
  using namespace dladmm;
  if (n < 0) return DLADMM_E_SHAPE;
  if (n == 0) return 0;
  if (!x || !s) return DLADMM_E_NULL;
  int64_t blocks = (n + 255) / 256;
  blocks = blocks > 4096 ? 4096 : blocks;
  hipLaunchKernelGGL(scale_if_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     x, n, s);
  return (int)hipGetLastError();
}

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
  const int rc = p.path == 1 || p.path >= 5 ? run_fused(d, p, ws, s)
                 : p.path == 4 ? run_fused_x3(d, p, ws, s)
                               : run_layered(d, p, ws, s);
  if (rc) return rc;
  // per-layer loss sums, fixed-order fp64 reduction of the per-column partials
  if (d->loss_kind) {
    hipLaunchKernelGGL(loss_reduce_kernel, dim3(2 * d->layers), dim3(1024), 0, s,
                       (const float*)(ws + p.off_loss), p.nslots, d->loss_sums);
    if (hipError_t e = hipGetLastError()) return (int)e;
    if (d->col_loss) {
      hipLaunchKernelGGL(col_loss_kernel, dim3(ceil_div(d->batch, 256), 2 * d->layers),
                         dim3(256), 0, s, (const float*)(ws + p.off_loss), p.nslots / p.ldl,
                         p.ldl, d->batch, d->col_loss);
      if (hipError_t e = hipGetLastError()) return (int)e;
    }
  }
  return 0;
}

size_t dladmm_bwd_workspace_bytes(const dladmm_bwd_desc* d) {
  using namespace dladmm;
  if (validate_bwd(d)) return 0;
  BwdPlan p;
  if (make_bwd_plan(d, &p)) return 0;
  return p.total;
}

int dladmm_bwd_path(const dladmm_bwd_desc* d) {
  using namespace dladmm;
  if (int e = validate_bwd(d)) return e;
  BwdPlan p;
  if (int e = make_bwd_plan(d, &p)) return e;
  return p.rev ? (p.rxs ? 3 : p.rrs ? 2 : 1) : 0;
}

int dladmm_bwd_f32(const dladmm_bwd_desc* d, void* stream) {
  using namespace dladmm;
  if (int e = validate_bwd(d)) return e;
  BwdPlan p;
  if (int e = make_bwd_plan(d, &p)) return e;
  if (!d->workspace || d->workspace_bytes < p.total) return DLADMM_E_WORKSPACE;
  if (((uintptr_t)d->workspace) & 255) return DLADMM_E_ALIGN;
  return run_bwd(d, p, (char*)d->workspace, (hipStream_t)stream);
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
