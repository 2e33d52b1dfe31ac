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
// Numerics.  Every wave scales its own operand values (its 64 G rows and its 64 V rows) by powers
// of two that put their largest magnitude SO FAR in the chunk in [2^14, 2^15), splits each x into
// hi = f16(x s), lo = f16(x s - hi) (22 significant bits; both roundings exact-input RNE) and
// accumulates the three products by MFMA straight into fp32 accumulators held at scale
// 2^(ea + eb).  A 32-column sub-chunk with a larger magnitude (one ballot per sub-chunk detects
// it) lowers the exponent and rescales the accumulators by the exact power of two; one exact
// unscale at the end.  The dropped lo lo term is 2^-22 of a product; elements more than 2^-29
// below the running largest go subnormal in f16, i.e. contribute below 2^-29 of that largest
// product.  Fixed order throughout: the result is deterministic.  Not bit-equal to wgrad_kernel
// (a different rounding sequence of the same sum).
//
// Dynamic range.  The scales are per wave, not per row: a G (or V) row more than ~2^17 below
// the largest magnitude its wave has seen in the chunk keeps fewer than 22 significant bits in
// hi + lo, and one ~2^29 below it contributes nothing.  The error of every output element is
// therefore bounded relative to the largest product in its wave's 64 x 64 block (the bound of
// an fp32 GEMM relative to |G| |V|^T), not to that element's own rows
// (tests/test_gpu_split.py::test_split_weight_gradient_row_range measures it).
//
// Geometry.  Partial layout of wgrad_kernel, a 1-D grid over (tile, chunk, layer).  A workgroup
// covers 128 G rows x TJ V rows (TJ = 256 where the padded V rows allow: 8 waves of 64 x 64, one
// workgroup per CU; else 128: 4 waves, two per CU), one chunk of batch columns; the tiles of one
// (chunk, layer) run on one XCD so its L2 serves their shared V rows.  Operands reach LDS by
// LDS-DMA in MFMA fragment order (a 1-KiB piece = 16 rows x 4 columns per lane-quarter, so every
// fragment read is one conflict-free ds_read_b128); per 32-column sub-chunk 16 G and TJ / 8 V
// pieces, three buffers at TJ = 256 (144 KiB: two sub-chunks in flight), two at 128.  Measured
// (profiles/r05_wgrad_x3.json, r05_wgrad_tj.json, r05_wgrad_x3_steps.json): 561 us per 8-layer
// launch at the headline shape against 662 for the round's first form and 990 for wgrad_kernel;
// the LDS-DMA issued after the MFMAs rather than beside the fragment reads: ~545 us.
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
// lo = f16(x sc - hi), each one RNE rounding of an exact value.  Per pair of values: one packed
// multiply and one v_cvt_pk_f16_f32 form the hi pair; v_fma_mixlo / mixhi form each lo straight
// from x, sc and the f16 hi (2 VALU per value; the compiler's own lowering of the same
// expressions converted hi back to f32 first, ~2.9 per value)
__device__ __forceinline__ void split8(const f32x4& p0, const f32x4& p1, float sc, h8& hi,
                                       h8& lo) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  uint32_t H[4], L[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float x0 = k < 2 ? p0[2 * k] : p1[2 * k - 4];
    const float x1 = k < 2 ? p0[2 * k + 1] : p1[2 * k - 3];
    const f32x2 y = f32x2{x0, x1} * f32x2{sc, sc};  // exact: sc is a power of two
    const h2 hp = __builtin_convertvector(y, h2);
    H[k] = __builtin_bit_cast(uint32_t, hp);
    asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]"
        : "=v"(L[k]) : "v"(x0), "v"(sc), "v"(H[k]));
    asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "+v"(L[k]) : "v"(x1), "v"(sc), "v"(H[k]));
  }
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  hi = __builtin_bit_cast(h8, u32x4{H[0], H[1], H[2], H[3]});
  lo = __builtin_bit_cast(h8, u32x4{L[0], L[1], L[2], L[3]});
}

constexpr int kSub = 32;   // batch columns per sub-chunk (one k-step of 32)

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

// One running scale per operand over the chunk (below).  NBUF sub-chunk buffers: NBUF - 1
// sub-chunks stream in while one is read.  DPOS: where the LDS-DMA of sub-chunk s + NBUF - 1 is
// issued in iteration s: 0 right after the fragment reads, 1 after the MFMAs of s - 1 (an
// LDS-DMA instruction costs its wave ~60 cycles among MFMAs / VALU but 100-185 beside ds_reads,
// MI355X_MICROARCH.md).  Round 5 also measured a per-sub-chunk scale, a speculative split beside
// the MFMAs and the DMA spread over the split: all slower (profiles/r05_wgrad_x3_steps.json).
template <int TJ, int NBUF, int DPOS>
__global__ __launch_bounds__(WgX3<TJ>::NW * 64, WgX3<TJ>::OCC) void wgrad_x3_kernel(
    const WgradArgs a, int xcd) {
  using T = WgX3<TJ>;
  constexpr int kBufs = NBUF;
  static_assert(NBUF == 2 || NBUF == 3, "two or three sub-chunk buffers");
  __shared__ f32x4 img[kBufs * T::PIECES * 64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w / T::WC, wc = w % T::WC;
  const int tiles_j = a.MBp16 / (TJ / 16);
  const int ntiles = (a.NBp16 / 8) * tiles_j;
  // 1-D grid over (tile, chunk, layer).  Workgroups are dispatched to the 8 XCDs round-robin by
  // linear id; xcd: the ntiles tiles of one (chunk, layer) go to ONE XCD, back to back, so its
  // L2 serves their shared operand rows (each V row block is read by every G tile) once from
  // HBM.  Otherwise consecutive ids: the tiles of a chunk spread over XCDs.
  const int L = blockIdx.x;
  int tile, grp;
  if (xcd) {
    const int slot = L >> 3;
    tile = slot % ntiles;
    grp = (slot / ntiles) * 8 + (L & 7);
  } else {
    tile = L % ntiles;
    grp = L / ntiles;
  }
  const int64_t zl = grp / a.nchunks;
  const int cy = grp % a.nchunks;
  const int ti = tile / tiles_j, tj = tile % tiles_j;
  const int64_t b0 = (int64_t)cy * a.chunk;
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
  auto issue_piece = [&](int sub, int buf, int q) {
    {
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
  auto issue = [&](int sub, int buf) {
#pragma unroll
    for (int q = 0; q < T::PPW; ++q) issue_piece(sub, buf, q);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nsub > 0) issue(0, 0);
  if (kBufs == 3 && nsub > 1) issue(1, 1);
  // Software-pipelined: iteration s reads and splits sub-chunk s, then runs the MFMAs of s - 1
  // (split in the previous iteration) while the LDS reads of s land.
  h8 ah[4], al[4], bh[4], bl[4];
  // The accumulators hold the sum at scale 2^(ea + eb), where 2^ea / 2^eb put the largest
  // G / V magnitude of this wave's rows SO FAR in the chunk in [2^14, 2^15); a sub-chunk that
  // exceeds it (any lane at or above lim) lowers the exponent and rescales the accumulators by
  // the exact power of two, so the MFMAs accumulate straight into them and the per-sub-chunk
  // unscale and both wave maxima drop out of the steady state.  127: no magnitude >= 2^-112 seen.
  int ea = 127, eb = 127;
  float sa = ldexpf(1.0f, 127), sbs = sa, lima = ldexpf(1.0f, -112), limb = lima;
  auto mfmas = [&]() {
    // three passes over the 16 independent accumulators (no back-to-back dependent MFMAs)
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[x][y] = mfma_h(ah[x], bh[y], acc[x][y]);
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[x][y] = mfma_h(ah[x], bl[y], acc[x][y]);
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[x][y] = mfma_h(al[x], bh[y], acc[x][y]);
  };
  auto wait_bar = [&](int s) {
    // sub-chunk s landed for every wave (three buffers: this wave's PPW DMAs of s + 1 may stay
    // in flight); every wave is past its reads of sub-chunk s - 1
    if (kBufs == 3 && s + 1 < nsub)
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(T::PPW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  };
  {
    for (int s = 0; s < nsub; ++s) {
      wait_bar(s);
      const f32x4* im = img + (s % kBufs) * T::PIECES * 64;
      f32x4 fa[4][2], fb[4][2];
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          fa[x][hf] = im[((4 * wr + x) * 2 + hf) * 64 + lane];
          fb[x][hf] = im[(T::GP + (4 * wc + x) * 2 + hf) * 64 + lane];
        }
      // sub-chunk s - 1's buffer is free: it receives sub-chunk s + kBufs - 1
      const bool more = s + kBufs - 1 < nsub;
      const int nx = s + kBufs - 1, nbuf = (s + kBufs - 1) % kBufs;
      if (DPOS == 0 && more) issue(nx, nbuf);
      if (s > 0) mfmas();  // sub-chunk s - 1, while the reads above land
      if (DPOS == 1 && more) issue(nx, nbuf);
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
      {
        // (after the MFMAs of s - 1, which used the old scales)
        const bool ga = __builtin_amdgcn_ballot_w64(ma >= lima) != 0;
        const bool gb = __builtin_amdgcn_ballot_w64(mb >= limb) != 0;
        if (ga || gb) {
          const int na = ga ? split_exp(wave_max(ma)) : ea;
          const int nb = gb ? split_exp(wave_max(mb)) : eb;
          const float fa2 = ldexpf(1.0f, na - ea), fb2 = ldexpf(1.0f, nb - eb);
#pragma unroll
          for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y)
#pragma unroll
              for (int q = 0; q < 4; ++q) acc[x][y][q] = acc[x][y][q] * fa2 * fb2;
          ea = na;
          eb = nb;
          sa = ldexpf(1.0f, ea);
          sbs = ldexpf(1.0f, eb);
          lima = ldexpf(1.0f, 15 - ea);
          limb = ldexpf(1.0f, 15 - eb);
        }
      }
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        split8(fa[x][0], fa[x][1], sa, ah[x], al[x]);
        split8(fb[x][0], fb[x][1], sbs, bh[x], bl[x]);
      }
    }
    if (nsub > 0) mfmas();
  }
  {
    // one exact unscale (two factors: 2^-(ea + eb) alone could leave the float range)
    const float ua = ldexpf(1.0f, -ea), ub = ldexpf(1.0f, -eb);
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[x][y][q] = acc[x][y][q] * ua * ub;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA in flight when the LDS is released
  // C/D layout: lane holds column (l & 15) = V row j, rows 4 g + q = G rows
  const int i0 = ti * 128 + wr * 64, j0 = tj * TJ + wc * 64;
  float* out = a.part + zl * a.pls + (int64_t)cy * a.n * a.m;
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
  // tiles: the caller's 128 x 128 count (the launch re-tiles at the V-tile width chosen here)
  if (!wgrad_x3_fits(a) || tiles != (a.NBp16 / 8) * (a.MBp16 / 8)) return hipErrorInvalidValue;
  // 256-row V tiles where the padded V rows allow: three sub-chunk buffers (144 KiB: two
  // sub-chunks in flight), the LDS-DMA issued after the MFMAs (539-556 vs 558-582 us right after
  // the fragment reads).  Else 128-row tiles, two workgroups per CU, two buffers, the early issue
  // (409 vs 418-421 us at m = 64).  XCD-grouped tiles where the (chunk, layer) count is a
  // multiple of 8.
  const bool wide = a.MBp16 % 16 == 0;
  const int ti = a.NBp16 / 8;
  const int groups = a.nchunks * layers;
  const int xcd = groups % 8 == 0 ? 1 : 0;
  const int nt = ti * (wide ? a.MBp16 / 16 : a.MBp16 / 8);
  const dim3 grid(nt * groups);
  if (wide)
    hipLaunchKernelGGL((wgrad_x3_kernel<256, 3, 1>), grid, dim3(WgX3<256>::NW * 64), 0, s, a, xcd);
  else
    hipLaunchKernelGGL((wgrad_x3_kernel<128, 2, 0>), grid, dim3(WgX3<128>::NW * 64), 0, s, a, xcd);
  return hipGetLastError();
}

}  // namespace dladmm
