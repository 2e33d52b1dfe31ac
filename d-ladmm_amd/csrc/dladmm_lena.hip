// dladmm_lena.hip -- MI355X (gfx950 / CDNA4) fused main_lena.py training objective over a
// forward's saved layers (include/dladmm.h, dladmm_lena_f32): main_lena.py:221-228 with
// dual_gap of :145-147,
//   l_k = a/(nN) sum|Z_k| + 1/(mN) sum|E_k| + 1/(nN) sum dual_gap(A^T L_k, a)
//         + 1/(mN) sum dual_gap(L_k, 1) + 1/(mN) sum L_k * X,
//   dual_gap(x, c) = softplus(x - c) + softplus(-x - c).
// The reference builds it from the returned E_k, L_k with torch ops: K products A^T L_k (n x B
// each, 128 MB per layer at B = 65,536) and a dozen elementwise passes over them forward, as many
// backward plus the products A (d/dY).  Here one launch covers every layer (grid = tiles x K) and
// A^T L_k never leaves the registers:
//  * one workgroup = 4 waves = 64 batch columns of one layer; wave w owns 16.  L_k's tile sits in
//    registers in the C/D layout of v_mfma_f32_16x16x4_f32 (lane l: column l & 15, rows
//    16 b + 4 (l >> 4) + r), i.e. as the B operand of
//      G1: Y = A^T L_k     (rows n, contraction m)  -- A^T packed in paired fragment order
//    whose epilogue either sums dual_gap(Y, a) (mode 0) or keeps S = softplus'(Y - a) -
//    softplus'(-Y - a) in registers (mode 1), S then being the B operand of
//      G2: G = A S         (rows m, contraction n)  -- A packed as for the forward's G2
//    with the epilogue gL_k = c_k/(nN) G + c_k/(mN) (sigma'(L_k) + X), gE_k = c_k/(mN) sgn(E_k);
//  * A^T and A stream through a 4-slot LDS-DMA ring shared by the four waves (the forward's
//    scheme, dladmm_fused_kernel.h), two output blocks per MFMA pass;
//  * mode 0's per-column partial sums go to part[k][t][col], reduced in fp64 in a fixed order by
//    loss_reduce_kernel (dladmm_capi.hip).
// softplus / its derivative follow torch's (beta 1, threshold 20): x > 20 ? x : log1p(exp(x)),
// x > 20 ? 1 : e / (e + 1), e = exp(x).
#include "dladmm_common.h"
#include "dladmm_internal.h"

namespace dladmm {

// Hardware exp2 / log2 (v_exp_f32, v_log_f32: ~1 ulp): softplus(x) = log(1 + e^x) for x <= 20
// is within ~1e-7 absolute of torch's log1p form (below e^x < 2^-24 the 1 + e^x rounds to 1 and
// the value to 0 instead of e^x); its derivative e / (e + 1) keeps full relative accuracy.  The
// OCML expf / log1pf sequences cost the unrolled G1 epilogue its registers (scratch spills).
__device__ __forceinline__ float exp_h(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896341f); }
__device__ __forceinline__ float softplus_t(float x) {
  return x > 20.0f ? x : 0.693147180559945309f * __builtin_amdgcn_logf(1.0f + exp_h(x));
}
__device__ __forceinline__ float softplus_d(float x) {
  const float e = exp_h(x);
  return x > 20.0f ? 1.0f : e / (e + 1.0f);
}

template <int MP, int NP, int MODE>
__global__ __launch_bounds__(256, 1) void lena_kernel(const LenaArgs a) {
  constexpr int MB = MP / 16, NB = NP / 16;
  constexpr int GF = MB * NB;                  // fragments per product
  constexpr int CF = GF < 16 ? GF : 16;        // fragments per ring chunk
  constexpr int NCH = GF / CF;                 // chunks per product
  constexpr int SLOTS = 4;
  static_assert(MB % 2 == 0 && NB % 2 == 0 && GF % CF == 0 && CF % 2 == 0, "shape");
  __shared__ f32x4 ring[SLOTS * CF * 64];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int k = blockIdx.y;
  const int64_t col = (int64_t)blockIdx.x * kTileCols + w * 16 + (lane & 15);
  const bool cv = col < a.B;
  const int m = a.m, n = a.n;

  // ---- ring: product gi = 0 (A^T, G1), 1 (A, G2); past the end: A again (harmless filler)
  auto chunk_src = [&](int ch) -> const float* {
    uint64_t sb = (uint64_t)(ch < NCH ? a.Atp : a.Ap);
    asm volatile("" : "+s"(sb));
    return (const float*)sb + (ch % NCH) * CF * kFrag;
  };
  auto issue = [&](const float* base, int slot) {
    f32x4* dst = ring + slot * (CF * 64);
    if constexpr (CF % 16 == 0) {
#pragma unroll
      for (int i = 0; i < CF / 16; ++i)
        glds16x4(base + (16 * i + 4 * w) * kFrag, lane * 16, dst + (16 * i + 4 * w) * 64);
    } else {
#pragma unroll
      for (int i = 0; i < (CF + 3) / 4; ++i) {
        const int f = i * 4 + w;
        if (CF % 4 == 0 || f < CF) glds16(base + f * kFrag, lane * 16, dst + f * 64);
      }
    }
  };
  int cur = 0;
  auto frag = [&](int slot, int fc) -> f32x4 { return ring[(slot * CF + fc) * 64 + lane]; };
#pragma unroll
  for (int c = 0; c < SLOTS - 1; ++c) issue(chunk_src(c), c);

  // ---- L_k's tile (rows past m and columns past B read 0)
  const int64_t ld = a.ld;
  const uint32_t vo = cv ? (uint32_t)((col + (int64_t)(4 * g) * ld) * 4) : kOOB;
  const uint32_t vx = cv ? (uint32_t)((col + (int64_t)(4 * g) * a.ldx) * 4) : kOOB;
  const uint32_t mbytes = (uint32_t)((int64_t)m * ld * 4);
  const rsrc_t rl = mkrsrc(a.L + (int64_t)k * a.ls, mbytes);
  const rsrc_t re = mkrsrc(a.E + (int64_t)k * a.ls, mbytes);
  const rsrc_t rx = mkrsrc(a.X, (uint32_t)((int64_t)m * a.ldx * 4));
  float Lr[MB][4];
#pragma unroll
  for (int b = 0; b < MB; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      Lr[b][r] = bload(rl, vo + (uint32_t)((int64_t)(16 * b + r) * ld * 4));
      pin_agpr(Lr[b][r]);
    }

  // mode 0: the elementwise terms over L_k's rows -- |E_k|, dual_gap(L_k, 1), L_k * X -- one
  // block at a time (the scheduling barrier keeps the unrolled blocks' loads from piling up)
  float se = 0.f, sdl = 0.f, slx = 0.f;
  if constexpr (MODE == 0) {
#pragma unroll
    for (int b = 0; b < MB; ++b) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = cv && (16 * b + 4 * g + r) < m;
        const float l = Lr[b][r];
        const float e = bload(re, vo + (uint32_t)((int64_t)(16 * b + r) * ld * 4));
        const float x = bload(rx, vx + (uint32_t)((int64_t)(16 * b + r) * a.ldx * 4));
        se += fabsf(e);
        sdl += ok ? softplus_t(l - 1.0f) + softplus_t(-l - 1.0f) : 0.f;
        slx += l * x;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  ring_barrier();  // the primed chunks landed; every load above is complete
  f32x4 fr[4];
  fr[0] = frag(0, 0);
  fr[1] = frag(0, 1);
  // step s of the stream (compile time): fragments 2s, 2s+1; the next step's two are read ahead
  // (at a chunk's last step: ring barrier, the next chunk's first fragments, and the DMA of the
  // chunk SLOTS - 1 ahead into the slot every wave has finished)
  auto step_head = [&](auto S_) {
    constexpr int s = decltype(S_)::value;
    constexpr int fi = 2 * s, fc = fi % CF, ch = fi / CF;
    if constexpr (fc + 2 < CF) {
      fr[(fi + 2) % 4] = frag(cur, fc + 2);
      fr[(fi + 3) % 4] = frag(cur, fc + 3);
    } else {
      ring_barrier();
      issue(chunk_src(ch + SLOTS - 1), (cur + SLOTS - 1) % SLOTS);
      const int nx = (cur + 1) % SLOTS;
      fr[(fi + 2) % 4] = frag(nx, 0);
      fr[(fi + 3) % 4] = frag(nx, 1);
    }
  };
  auto step_tail = [&](auto S_) {
    constexpr int s = decltype(S_)::value;
    constexpr int fc = (2 * s) % CF;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (fc + 2 >= CF) cur = (cur + 1) % SLOTS;
  };
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  const float al = a.alpha;

  // ---- G1: Y = A^T L_k, blocks (2p, 2p+1) of the n rows over jb = 0..MB-1
  float S[MODE == 1 ? NB : 1][4];
  float sdy = 0.f;  // mode 0: this lane's sum of dual_gap(Y, alpha) over valid rows
  static_for<NB / 2>([&](auto P_) {
    constexpr int p = decltype(P_)::value;
    f32x4 ca = zero4, cb = zero4;
    static_for<MB>([&](auto J_) {
      constexpr int jb = decltype(J_)::value;
      constexpr int s = p * MB + jb;
      step_head(std::integral_constant<int, s>{});
      const f32x4 wa = fr[(2 * s) % 4], wb = fr[(2 * s + 1) % 4];
      ca = mfma4(wa.x, Lr[jb][0], ca);
      cb = mfma4(wb.x, Lr[jb][0], cb);
      ca = mfma4(wa.y, Lr[jb][1], ca);
      cb = mfma4(wb.y, Lr[jb][1], cb);
      ca = mfma4(wa.z, Lr[jb][2], ca);
      cb = mfma4(wb.z, Lr[jb][2], cb);
      ca = mfma4(wa.w, Lr[jb][3], ca);
      cb = mfma4(wb.w, Lr[jb][3], cb);
      step_tail(std::integral_constant<int, s>{});
    });
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float y = h ? cb[r] : ca[r];
        if constexpr (MODE == 0) {
          const bool ok = cv && (16 * (2 * p + h) + 4 * g + r) < n;
          const float dg = softplus_t(y - al) + softplus_t(-y - al);
          sdy += ok ? dg : 0.f;
        } else {
          // rows past n: y = 0 exactly (zero-padded A^T), so S = 0 there
          S[2 * p + h][r] = softplus_d(y - al) - softplus_d(-y - al);
          pin_agpr(S[2 * p + h][r]);
        }
      }
  });

  if constexpr (MODE == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's filler DMA has landed
    const float v[4] = {col_sum(se), col_sum(sdy), col_sum(sdl), col_sum(slx)};
    if (g == 0) {  // padded columns write their zero sums (the reduction reads every column)
#pragma unroll
      for (int t = 0; t < 4; ++t) a.part[((int64_t)k * 4 + t) * a.ldl + col] = v[t];
    }
    return;
  } else {
    // ---- G2: G = A S, blocks (2p, 2p+1) of the m rows over kb = 0..NB-1; epilogue gL, gE
    const float c = a.coef[k];
    const float cn = c * a.inv_nb, cm = c * a.inv_mb;
    const uint32_t vg = cv ? (uint32_t)((col + (int64_t)(4 * g) * a.ldg) * 4) : kOOB;
    const uint32_t gbytes = (uint32_t)((int64_t)m * a.ldg * 4);
    const rsrc_t rgl = mkrsrc(a.gL + (int64_t)k * a.gls, gbytes);
    const rsrc_t rge = mkrsrc(a.gE + (int64_t)k * a.gls, gbytes);
    static_for<MB / 2>([&](auto P_) {
      constexpr int p = decltype(P_)::value;
      // this pair's X and E rows, in flight during its MFMAs
      float xv[2][4], ev[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * (2 * p + h) + r;
          xv[h][r] = bload(rx, vx + (uint32_t)((int64_t)row * a.ldx * 4));
          ev[h][r] = bload(re, vo + (uint32_t)((int64_t)row * ld * 4));
        }
      f32x4 ca = zero4, cb = zero4;
      static_for<NB>([&](auto K_) {
        constexpr int kb = decltype(K_)::value;
        constexpr int s = (NB / 2) * MB + p * NB + kb;  // G2 follows G1 in the stream
        step_head(std::integral_constant<int, s>{});
        const f32x4 wa = fr[(2 * s) % 4], wb = fr[(2 * s + 1) % 4];
        ca = mfma4(wa.x, S[kb][0], ca);
        cb = mfma4(wb.x, S[kb][0], cb);
        ca = mfma4(wa.y, S[kb][1], ca);
        cb = mfma4(wb.y, S[kb][1], cb);
        ca = mfma4(wa.z, S[kb][2], ca);
        cb = mfma4(wb.z, S[kb][2], cb);
        ca = mfma4(wa.w, S[kb][3], ca);
        cb = mfma4(wb.w, S[kb][3], cb);
        step_tail(std::integral_constant<int, s>{});
      });
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int b = 2 * p + h;
          const uint32_t so = (uint32_t)((int64_t)(16 * b + r) * a.ldg * 4);
          const float l = Lr[b][r];
          const float dl = softplus_d(l - 1.0f) - softplus_d(-l - 1.0f);
          const float gl = cn * (h ? cb[r] : ca[r]) + cm * (dl + xv[h][r]);
          const float e = ev[h][r];
          const float sg = (e > 0.f ? 1.f : 0.f) - (e < 0.f ? 1.f : 0.f);
          bstore_s(rgl, vg, so, gl);
          bstore_s(rge, vg, so, cm * sg);
        }
    });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's last DMA has landed
  }
}

template <int MP, int NP>
hipError_t launch_lena_s(const LenaArgs& a, int grid, hipStream_t s) {
  if (a.mode == 0)
    hipLaunchKernelGGL((lena_kernel<MP, NP, 0>), dim3(grid, a.K), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((lena_kernel<MP, NP, 1>), dim3(grid, a.K), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_lena(int shape, const LenaArgs& a, int grid, hipStream_t s) {
  switch (shape) {
    case 0: return launch_lena_s<kShapeMP[0], kShapeNP[0]>(a, grid, s);
    case 1: return launch_lena_s<kShapeMP[1], kShapeNP[1]>(a, grid, s);
    case 2: return launch_lena_s<kShapeMP[2], kShapeNP[2]>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace dladmm
