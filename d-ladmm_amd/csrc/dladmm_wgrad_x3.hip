// dladmm_wgrad_x3.hip -- MI355X (gfx950) weight gradient of the backward, part[c][i][j] =
// sum_{b in chunk c} G[i][b] V[j][b] (G = gU_k, V = Var_k: the product BK2 / BK3 hand to the
// weight update of main_syn_l1l1_scalar.py:298's backward), with its fp32 products formed on the
// f16 matrix cores: the split-f16 scheme of the forward applied to the
// backward's third GEMM under precision "f32_split".
//
// Why: wgrad_kernel runs v_mfma_f32_16x16x4_f32 at 0.81 of the fp32 MFMA peak (2.0 ms of a 7.1-ms
// backward at the headline shape).  Here each 16 x 16 x 32 block is three
// v_mfma_f32_16x16x32_f16 (hi hi + hi lo + lo hi) at 16x the f32 MFMA's rate per instruction.
//
// Numerics.  Per 32-column sub-chunk every wave scales its own operand values (its 64 G rows and
// its 64 V rows) by powers of two that put their largest magnitude in [2^14, 2^15), splits each
// x into hi = f16(x s), lo = f16(x s - hi) (22 significant bits; both roundings exact-input RNE),
// accumulates the three products in fp32 by MFMA over the sub-chunk, and adds the sub-chunk's sum
// to the running fp32 accumulator after one exact power-of-two unscale.  The dropped lo lo term is
// 2^-22 of a product; elements more than 2^-29 below their sub-tile's largest go subnormal in
// f16, i.e. contribute below 2^-29 of that largest product.  Fixed order throughout: the result is
// deterministic.  Not bit-equal to wgrad_kernel (a different rounding sequence of the same sum).
//
// Geometry.  Grid and partial layout of wgrad_kernel: a workgroup = 4 waves over a 128 x 128
// output tile (wave (wr, wc): G rows 64 wr .., V rows 64 wc ..), one chunk of batch columns.
// Operands reach LDS by LDS-DMA in MFMA fragment order (a 1-KiB piece = 16 rows x 4 columns per
// lane-quarter, so every fragment read is one conflict-free ds_read_b128): per 32-column
// sub-chunk 16 G and 16 V pieces (32 KiB), two buffers (64 KiB), two workgroups per CU: the
// operands stream from HBM and the second workgroup's waves cover their latency (measured: 677
// us per 8-layer launch against 820 for four buffers at one workgroup per CU and 990 for
// wgrad_kernel, profiles/r05_wgrad_x3.json).
#include "dladmm_common.h"
#include "dladmm_internal.h"
#include "dladmm_wgrad_x3.h"

namespace dladmm {

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma_h(const h8& a, const h8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// exponent e with max * 2^e in [2^14, 2^15) (0 for an all-zero operand)
__device__ __forceinline__ int split_exp(float mx) {
  if (!(mx > 0.0f)) return 0;
  int ex;
  (void)frexpf(mx, &ex);  // mx = f 2^ex, f in [0.5, 1)
  return 15 - ex;
}

// max over the wave of non-negative values: on their bit patterns (order-preserving for x >= 0)
// by DPP row shifts and row broadcasts (a few cycles each; a ds_bpermute chain costs its LDS
// latency per step), the result read from lane 63
__device__ __forceinline__ float wave_max(float v) {
  int x = __builtin_bit_cast(int, v);
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false));  // row_shr:1
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false));  // row_shr:2
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false));  // row_shr:4
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false));  // row_shr:8
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false));  // row_bcast:15
  x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(x, 63));
}

// 8 consecutive k-values (two 16-B pieces) -> hi / lo halves at scale sc: hi = f16(x sc),
// lo = f16(x sc - hi), each one RNE rounding of an exact value (the forms lower to
// v_fma_mix{lo,hi}_f16, as in the split-f16 forward)
__device__ __forceinline__ void split8(const f32x4& p0, const f32x4& p1, float sc, h8& hi,
                                       h8& lo) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const _Float16 h0 = (_Float16)__builtin_fmaf(p0[q], sc, 0.0f);
    const _Float16 h1 = (_Float16)__builtin_fmaf(p1[q], sc, 0.0f);
    hi[q] = h0;
    hi[4 + q] = h1;
    lo[q] = (_Float16)__builtin_fmaf(p0[q], sc, -(float)h0);
    lo[4 + q] = (_Float16)__builtin_fmaf(p1[q], sc, -(float)h1);
  }
}

constexpr int kSub = 32;   // batch columns per sub-chunk (one k-step of 32)
constexpr int kBufs = 2;   // sub-chunk buffers: the next one streams in while this one is read

// Tile geometry by V-tile width TJ: 128 G rows x TJ V rows, waves of 64 x 64 (2 wave rows x
// TJ / 64 wave columns); a sub-chunk is 16 G pieces + TJ / 8 V pieces of 1 KiB.  TJ = 128: 4
// waves, 64 KiB of LDS, two workgroups per CU; TJ = 256: 8 waves, 96 KiB, one workgroup per CU
// -- the same two waves per SIMD, and every G row is read once per V tile instead of twice.
template <int TJ>
struct WgX3 {
  static constexpr int WC = TJ / 64, NW = 2 * WC;
  static constexpr int GP = 16, VP = TJ / 8, PIECES = GP + VP, PPW = PIECES / NW;
  static constexpr int OCC = TJ == 128 ? 2 : 1;
  static_assert(PIECES % NW == 0, "even DMA share per wave");
};

template <int TJ>
__global__ __launch_bounds__(WgX3<TJ>::NW * 64, WgX3<TJ>::OCC) void wgrad_x3_kernel(
    const WgradArgs a) {
  using T = WgX3<TJ>;
  __shared__ f32x4 img[kBufs * T::PIECES * 64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w / T::WC, wc = w % T::WC;
  const int tiles_j = a.MBp16 / (TJ / 16);
  const int tile = blockIdx.x;
  const int64_t zl = blockIdx.z;
  const int ti = tile / tiles_j, tj = tile % tiles_j;
  const int64_t b0 = (int64_t)blockIdx.y * a.chunk;
  int64_t b1 = b0 + a.chunk;
  if (b1 > a.Bpad) b1 = a.Bpad;
  const int nsub = b1 > b0 ? (int)((b1 - b0) / kSub) : 0;
  const int r = lane & 15, g = lane >> 4;

  // DMA: piece p < GP is G's (row block p / 2), else V's (row block (p - GP) / 2); hf = p & 1
  // is the 4-column half of the lane's 8: lane l copies row 16 blk + (l & 15), columns
  // 8 (l >> 4) + 4 hf .. +3 of the sub-chunk.  Wave w issues pieces PPW w .. PPW w + PPW - 1.
  const float* gb = a.G + zl * a.gls + (int64_t)(ti * 128) * a.ld;
  const float* vb = a.V + zl * a.vls + (int64_t)(tj * TJ) * a.ld;
  const uint32_t vl = (uint32_t)(((int64_t)r * a.ld + 8 * g) * 4);
  auto issue = [&](int sub, int buf) {
#pragma unroll
    for (int q = 0; q < T::PPW; ++q) {
      const int p = T::PPW * w + q;
      const bool isg = p < T::GP;
      const int pp = isg ? p : p - T::GP;
      const float* base = isg ? gb : vb;
      uint64_t sb = (uint64_t)(base + (int64_t)(16 * (pp >> 1)) * a.ld + b0 +
                               (int64_t)kSub * sub + 4 * (pp & 1));
      // both halves through uint32_t: readfirstlane returns int, and a sign-extended low half
      // (address bit 31 set) would overwrite the high half
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)sb);
      const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(sb >> 32));
      sb = ((uint64_t)hi << 32) | lo;
      asm volatile("" : "+s"(sb));
      glds16((const float*)sb, vl, img + (buf * T::PIECES + p) * 64);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nsub > 0) issue(0, 0);
  // Software-pipelined: iteration s reads and splits sub-chunk s, then runs the MFMAs of s - 1
  // (split in the previous iteration) while the LDS reads of s land.
  h8 ah[4], al[4], bh[4], bl[4];
  float uns = 0.f;
  auto mfmas = [&]() {
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
        c = mfma_h(ah[x], bh[y], c);
        c = mfma_h(ah[x], bl[y], c);
        c = mfma_h(al[x], bh[y], c);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[x][y][q] = __builtin_fmaf(c[q], uns, acc[x][y][q]);
      }
  };
  for (int s = 0; s < nsub; ++s) {
    // sub-chunk s landed for every wave; every wave is past its reads of sub-chunk s - 1
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    const f32x4* im = img + (s % kBufs) * T::PIECES * 64;
    f32x4 fa[4][2], fb[4][2];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        fa[x][hf] = im[((4 * wr + x) * 2 + hf) * 64 + lane];
        fb[x][hf] = im[(T::GP + (4 * wc + x) * 2 + hf) * 64 + lane];
      }
    // the other buffer (sub-chunk s - 1's) is free: it receives sub-chunk s + 1
    if (s + 1 < nsub) issue(s + 1, (s + 1) % kBufs);
    if (s > 0) mfmas();  // sub-chunk s - 1, while the reads above land
    float ma = 0.f, mb = 0.f;
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ma = fmaxf(ma, fabsf(fa[x][hf][q]));
          mb = fmaxf(mb, fabsf(fb[x][hf][q]));
        }
    const int ea = split_exp(wave_max(ma)), eb = split_exp(wave_max(mb));
    const float sa = ldexpf(1.0f, ea), sbs = ldexpf(1.0f, eb);
    uns = ldexpf(1.0f, -(ea + eb));
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      split8(fa[x][0], fa[x][1], sa, ah[x], al[x]);
      split8(fb[x][0], fb[x][1], sbs, bh[x], bl[x]);
    }
  }
  if (nsub > 0) mfmas();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA in flight when the LDS is released
  // C/D layout: lane holds column (l & 15) = V row j, rows 4 g + q = G rows
  const int i0 = ti * 128 + wr * 64, j0 = tj * TJ + wc * 64;
  float* out = a.part + zl * a.pls + (int64_t)blockIdx.y * a.n * a.m;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = i0 + 16 * x + 4 * g + q;
        const int j = j0 + 16 * y + r;
        if (i < a.n && j < a.m) out[(int64_t)i * a.m + j] = acc[x][y][q];
      }
}

}  // namespace

hipError_t launch_wgrad_x3(const WgradArgs& a, int tiles, hipStream_t s, int layers) {
  (void)tiles;  // the tile count follows the V-tile width chosen here
  if (!wgrad_x3_fits(a)) return hipErrorInvalidValue;
  // 256-row V tiles where the padded V rows allow (DLADMM_WGRAD_X3_TJ=128 forces the narrow
  // form: A/B)
  const char* e = getenv("DLADMM_WGRAD_X3_TJ");
  const bool wide = a.MBp16 % 16 == 0 && !(e && atoi(e) == 128);
  const int ti = a.NBp16 / 8;
  if (wide) {
    hipLaunchKernelGGL((wgrad_x3_kernel<256>), dim3(ti * (a.MBp16 / 16), a.nchunks, layers),
                       dim3(WgX3<256>::NW * 64), 0, s, a);
  } else {
    hipLaunchKernelGGL((wgrad_x3_kernel<128>), dim3(ti * (a.MBp16 / 8), a.nchunks, layers),
                       dim3(WgX3<128>::NW * 64), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace dladmm
