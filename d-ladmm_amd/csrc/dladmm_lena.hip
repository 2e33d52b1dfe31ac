// dladmm_lena.hip -- MI355X (gfx950 / CDNA4) fused main_lena.py training objective over a
// forward's saved layers (include/dladmm.h, dladmm_lena_f32): main_lena.py:221-228 with
// dual_gap of :145-147,
//   l_k = a/(nN) sum|Z_k| + 1/(mN) sum|E_k| + 1/(nN) sum dual_gap(A^T L_k, a)
//         + 1/(mN) sum dual_gap(L_k, 1) +/- 1/(mN) sum L_k * X   (- : main_syn_l1l1-dgap_ltheta.py:205),
//   dual_gap(x, c) = softplus(x - c) + softplus(-x - c).
// The reference builds it from the returned E_k, L_k with torch ops: K products A^T L_k (n x B
// each, 128 MB per layer at B = 65,536) and a dozen elementwise passes over them forward, as many
// backward plus the products A (d/dY).  Here one launch covers every layer and A^T L_k never
// leaves the registers:
//  * one workgroup = 4 waves = 64 batch columns for all K layers; wave w owns 16.  L_k's tile
//    sits in registers (L_{k+1}'s blocks load as L_k's last reads of them pass) in the C/D layout of v_mfma_f32_16x16x4_f32 (lane l: column l & 15, rows
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
// dual_gap and its derivative in closed form (below), to torch's softplus (beta 1, threshold 20)
// within fp32 precision.
#include "dladmm_common.h"
#include "dladmm_internal.h"

#ifndef LENA_ABL
#define LENA_ABL 0  // timing experiments only (WRONG results): 1 no G1 epilogue transcendentals,
                    // 2 no mode-0 elementwise sums (E / X loads), 8 no G1 MFMAs, 16 mode-0
                    // E loads without the sums' math, 32 the math without the E loads
#endif

namespace dladmm {

// dual_gap(y, a) = softplus(y - a) + softplus(-y - a) = ln((1 + e^(y-a)) (1 + e^(-y-a)))
//                 = ln(c1 + c2 (e^y + e^-y)),  c1 = 1 + e^-2a, c2 = e^-a,
// and its derivative softplus'(y - a) - softplus'(-y - a) = (e^y - e^-y) / (e^y + e^-y + c3),
// c3 = e^a + e^-a.  With t = e^|y| (>= 1) both need ONE exponential:
//   dual_gap = ln(c2 t^2 + c1 t + c2) - |y|,   derivative = sgn(y) (t^2 - 1) / (t^2 + c3 t + 1)
// -- exp + log for the value, exp + rcp for the derivative, exp + log + rcp for both (the
// e^y, e^-y form needed one transcendental more each); no cancellation in the log (its
// argument is >= c2 (1 + t)^2 > 0) and t^2 - 1 as one fma, so the derivative near y = 0 is as
// exact as t.  Past |y| = 30 they are |y| - a and sgn(y) (what torch's softplus threshold of 20
// gives to fp32 precision; t^2 may overflow there and is discarded).  Hardware v_exp_f32 /
// v_log_f32 / v_rcp_f32 (~1 ulp each): within ~1e-7 of the torch values, relative to the
// terms' scale; branch-free (selects), so no lane diverges around the transcendental work.
// dual_gap and dual_gap_vd (dual_gap_d and dual_gap_vd) form the value (the derivative) by the
// same operations, so modes 0, 1 and 2 agree bit for bit.
struct Gap { float a, c1, c2, c3; };
__device__ __forceinline__ float exp_h(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896341f); }
__device__ __forceinline__ float gap_v(float t, float ay, const Gap& G) {
  return 0.693147180559945309f * __builtin_amdgcn_logf(fmaf(fmaf(G.c2, t, G.c1), t, G.c2)) - ay;
}
__device__ __forceinline__ float gap_d(float t, const Gap& G) {
  return fmaf(t, t, -1.0f) * __builtin_amdgcn_rcpf(fmaf(t + G.c3, t, 1.0f));
}
__device__ __forceinline__ float dual_gap(float y, const Gap& G) {
  const float ay = fabsf(y);
  float v = gap_v(exp_h(ay), ay, G);
  asm("" : "+v"(v));  // computed on every lane: the select below must not become a branch
  return ay > 30.0f ? ay - G.a : v;
}
// both at once (mode 2): they share t
__device__ __forceinline__ void dual_gap_vd(float y, const Gap& G, float& val, float& der) {
  const float ay = fabsf(y);
  const float t = exp_h(ay);
  float v = gap_v(t, ay, G);
  float d = gap_d(t, G);
  asm("" : "+v"(v), "+v"(d));
  val = ay > 30.0f ? ay - G.a : v;
  der = copysignf(ay > 30.0f ? 1.0f : d, y);
}
__device__ __forceinline__ float dual_gap_d(float y, const Gap& G) {
  const float ay = fabsf(y);
  float d = gap_d(exp_h(ay), G);
  asm("" : "+v"(d));
  return copysignf(ay > 30.0f ? 1.0f : d, y);
}

// Static VM-operation counts of one layer body, for the counted ring barriers (the scheme of the
// forward's WinCount).  Steps: mode 0 = G1 only (T1 steps per layer), mode 1 = G1 then G2.  Ops
// issued in the body of local step t (after its head, i.e. after any barrier / DMA of t):
//   mode 0: at the start of G1 pair p the E loads of the L blocks assigned to p (blocks go to
//           pairs 0 .. NB/2 - 2, their sums formed one step before the pair's last; NB/2 = 1:
//           at the layer start); in the last pair, after each step's MFMAs, L_{k+1}'s block jb
//           (4 loads); after the layer's last step the 4 sum stores;
//   mode 1: at the start of G2 pair p the E loads of its two blocks (8); after its last step
//           the gL / gE stores (16) and L_{k+1}'s two blocks (8).
// A barrier at step s (last step of a chunk of SPC steps) awaits the chunk DMA issued SLOTS - 2
// barriers back: newer are the DMAs of the barriers in between and every op of the steps since
// (VM operations complete in issue order for vmcnt, so a load must have landed by the barrier
// that awaits the first chunk DMA issued after it: a deeper ring gives the E loads, which miss
// to HBM, more steps);
// ops of the previous layer are not counted (fewer counted only waits longer).  X sits in LDS.
template <int MB, int NB, int CF, int MODE, int SLOTS>
struct LenaWin {
  static constexpr int SPC = CF / 2;
  static constexpr int DMAOPS = CF % 16 == 0 ? 4 * (CF / 16) : 1;  // VM ops of one chunk DMA
  static constexpr int NP1 = NB / 2;                                // G1 pairs
  static constexpr int T1 = NP1 * MB;
  static constexpr int pair_of_block(int b) { return NP1 > 1 ? (b * (NP1 - 1)) / MB : 0; }
  static constexpr int blocks_at(int p) {
    int c = 0;
    for (int b = 0; b < MB; ++b) c += pair_of_block(b) == p ? 1 : 0;
    return c;
  }
  static constexpr int ops(int t) {
    int c = 0;
    if constexpr (MODE == 0) {
      const int p = t / MB, j = t % MB;
      if (j == 0 && NP1 > 1 && !(LENA_ABL & 2)) c += 4 * blocks_at(p);
      if (p == NP1 - 1) c += 4;
      if (t == T1 - 1) c += 4;
    } else {
      if (t >= T1) {
        const int u = t - T1, j = u % NB;
        if (j == 0) c += 8;
        if (j == NB - 1) c += 24;
      }
    }
    return c;
  }
  template <int S>
  static constexpr int at() {
    int n = DMAOPS * (SLOTS - 3);
    for (int t = S - (SLOTS - 2) * SPC; t < S; ++t)
      if (t >= 0) n += ops(t);
    return n < 63 ? n : 63;
  }
};

template <int MP, int NP, int MODE>
__global__ __launch_bounds__(256, 1) void lena_kernel(const LenaArgs a) {
  constexpr int MB = MP / 16, NB = NP / 16;
  constexpr int GF = MB * NB;                  // fragments per product
  constexpr int CF = GF < 16 ? GF : 16;        // fragments per ring chunk
  constexpr int NCH = GF / CF;                 // chunks per product
  // MODE 0: the sums; 1: the cotangents; 2: both (a training forward: the backward then only
  // scales the cotangents by its upstream gradient)
  constexpr bool GRAD = MODE >= 1, SUMS = MODE != 1;
  constexpr int CPL = GRAD ? 2 * NCH : NCH;  // chunks per layer
  // ring slots: 6 where they fit beside the X tile (160 KiB at 256 x 512), else 4
  constexpr int SLOTS = (6 * CF + kWaves * MB) * 64 * 16 <= 160 * 1024 ? 6 : 4;
  using Win = LenaWin<MB, NB, CF, MODE, SLOTS>;
  constexpr int NP1 = NB / 2, T1 = Win::T1;
  static_assert(MB % 2 == 0 && NB % 2 == 0 && GF % CF == 0 && CF % 2 == 0, "shape");
  __shared__ f32x4 ring[SLOTS * CF * 64];
  __shared__ f32x4 xs[kWaves * MB * 64];  // xs[w][b][lane] = X rows 16 b + 4 g .. +3 (read by w)

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int K = a.K;
  const int64_t col = (int64_t)blockIdx.x * kTileCols + w * 16 + (lane & 15);
  const bool cv = col < a.B;
  const int m = a.m, n = a.n;

  // ---- ring: per layer A^T (G1) [, A (G2)], layer after layer; past the end: harmless filler
  auto chunk_src = [&](int ch) -> const float* {
    const int q = ch % CPL;
    uint64_t sb = (uint64_t)(q < NCH ? a.Atp : a.Ap);
    asm volatile("" : "+s"(sb));
    return (const float*)sb + (q % NCH) * CF * kFrag;
  };
  auto issue = [&](const float* base, int slot) {
    f32x4* dst = ring + slot * (CF * 64);
    if constexpr (CF % 16 == 0) {
#pragma unroll
      for (int i = 0; i < CF / 16; ++i)
        glds16x4(base + (16 * i + 4 * w) * kFrag, lane * 16, dst + (16 * i + 4 * w) * 64);
    } else {
      // CF < 16 (the 32 x 32 shape): fragment w per wave; waves past CF issue a harmless
      // duplicate so every wave's VM count is the same
      const int f = w < CF ? w : 0;
      glds16(base + f * kFrag, lane * 16, dst + f * 64);
    }
  };
  int cur = 0;
  auto frag = [&](int slot, int fc) -> f32x4 { return ring[(slot * CF + fc) * 64 + lane]; };
#pragma unroll
  for (int c = 0; c < SLOTS - 1; ++c) issue(chunk_src(c), c);

  // ---- views (rows past m and columns past B read 0 / are dropped)
  const int64_t ld = a.ld;
  const uint32_t vo = cv ? (uint32_t)((col + (int64_t)(4 * g) * ld) * 4) : kOOB;
  const uint32_t vx = cv ? (uint32_t)((col + (int64_t)(4 * g) * a.ldx) * 4) : kOOB;
  const uint32_t mbytes = (uint32_t)((int64_t)m * ld * 4);
  const rsrc_t rx = mkrsrc(a.X, (uint32_t)((int64_t)m * a.ldx * 4));
  auto lview = [&](int k) { return mkrsrc(k < K ? a.L + (int64_t)k * a.ls : nullptr, k < K ? mbytes : 0u); };
  auto row_off = [&](int b, int r, int64_t stride) { return (uint32_t)((int64_t)(16 * b + r) * stride * 4); };
  float Lr[MB][4];
  {
    const rsrc_t rl = lview(0);
#pragma unroll
    for (int b = 0; b < MB; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        Lr[b][r] = bload(rl, vo + row_off(b, r, ld));
        pin_agpr(Lr[b][r]);
      }
  }
#pragma unroll
  for (int b = 0; b < MB; ++b) {
    f32x4 xv;
#pragma unroll
    for (int r = 0; r < 4; ++r) xv[r] = bload(rx, vx + row_off(b, r, a.ldx));
    xs[(w * MB + b) * 64 + lane] = xv;  // this wave's own columns: no barrier needed
  }
  ring_barrier();  // the primed chunks landed; L_0 and X are in
  f32x4 fr[4];
  fr[0] = frag(0, 0);
  fr[1] = frag(0, 1);
  int chb = 0;  // stream chunk of the current layer's first chunk
  auto step_head = [&](auto S_) {
    constexpr int s = decltype(S_)::value;
    constexpr int fi = 2 * s, fc = fi % CF, ch = fi / CF;
    if constexpr (fc + 2 < CF) {
      fr[(fi + 2) % 4] = frag(cur, fc + 2);
      fr[(fi + 3) % 4] = frag(cur, fc + 3);
    } else {
      ring_barrier_cnt<Win::template at<s>()>();
      issue(chunk_src(chb + ch + SLOTS - 1), (cur + SLOTS - 1) % SLOTS);
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
  // constants of dual_gap(., alpha) and dual_gap(., 1), formed on the host (lena_gap_consts)
  const Gap Gac{a.gc[0], a.gc[1], a.gc[2], a.gc[3]}, G1c{a.gc[4], a.gc[5], a.gc[6], a.gc[7]};
  // mode 0: per-column sums of the layer; part[k][t] through a buffer view (lanes g > 0 and
  // padded columns write nothing / their zero sums: every lane issues the store)
  const rsrc_t rpart = mkrsrc(a.part, (uint32_t)((int64_t)4 * K * a.ldl * 4));
  const uint32_t vp = g == 0 ? (uint32_t)(col * 4) : kOOB;

  // valid rows of this lane: 16 b + r < lim (no rows for a padded column)
  const int limm = cv ? m - 4 * g : -1, limn = cv ? n - 4 * g : -1;
  float S[GRAD ? NB : 1][4];
  for (int k = 0; k < K; ++k) {
    // opaque ring slot at the layer start, so the compiler cannot precompute the unrolled
    // body's LDS addresses and keep them all live across the layer loop
    cur = __builtin_amdgcn_readfirstlane(cur);
    asm volatile("" : "+s"(cur));
    const rsrc_t rln = lview(k + 1);
    const rsrc_t re = mkrsrc(a.E + (int64_t)k * a.ls, mbytes);
    float se = 0.f, sdl = 0.f, slx = 0.f, sdy = 0.f;
    // mode 0: |E_k|, dual_gap(L_k, 1), L_k X over block b's rows (E / X rows in ev / xv)
    // Row masks: row 16 b + 4 g + r is valid iff 16 b + r < lim (lim folds in the lane's 4 g
    // and its column); lim goes through an opaque copy where it is used, so the compiler can
    // neither precompute every (b, r) mask at the top (hundreds of live lane masks: spills) nor
    // branch around the transcendental work of masked-off lanes.
    auto masked_add = [](float& acc, float v, int rr, int lim0) {
      int lim = lim0;
      asm volatile("" : "+v"(lim), "+v"(v));
      acc += rr < lim ? v : 0.f;
    };
    auto elem_sums = [&](int b, const float (&ev)[4]) {
      const f32x4 xv = xs[(w * MB + b) * 64 + lane];
      if constexpr (LENA_ABL & 16) {  // loads kept, no math
        se += ev[0] + ev[1] + ev[2] + ev[3] + xv[0];
        return;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float l = Lr[b][r];
        se += fabsf(ev[r]);
        masked_add(sdl, dual_gap(l, G1c), 16 * b + r, limm);
        slx += l * xv[r];
      }
    };
    if constexpr (MODE == 0 && NP1 == 1) {
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        float ev[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) ev[r] = bload(re, vo + row_off(b, r, ld));
        elem_sums(b, ev);
      }
    }
    // ---- G1: Y = A^T L_k, blocks (2p, 2p+1) of the n rows over jb = 0..MB-1
    static_for<NP1>([&](auto P_) {
      constexpr int p = decltype(P_)::value;
      constexpr int NBP = MODE == 0 && NP1 > 1 && !(LENA_ABL & 2) ? Win::blocks_at(p) : 0;
      float ev[NBP > 0 ? NBP : 1][4];
      f32x4 ca = zero4, cb = zero4;
      static_for<MB>([&](auto J_) {
        constexpr int jb = decltype(J_)::value;
        constexpr int s = p * MB + jb;
        step_head(std::integral_constant<int, s>{});
        if constexpr (jb == 0 && NBP > 0) {  // E rows of this pair's blocks
          int q = 0;
#pragma unroll
          for (int b = 0; b < MB; ++b) {
            if (Win::pair_of_block(b) != p) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r)
              ev[q][r] = (LENA_ABL & 32) ? 0.5f : bload(re, vo + row_off(b, r, ld));
            ++q;
          }
        }
        // the sums of this pair's blocks one step before the pair's last step: their E rows are
        // then waited for before that step's ring barrier issues the next DMA (the compiler's
        // own wait for a loaded value counts every VM operation after it, the LDS-DMA included)
        if constexpr (jb == MB - 2 && NBP > 0) {
          int q = 0;
#pragma unroll
          for (int b = 0; b < MB; ++b) {
            if (Win::pair_of_block(b) != p) continue;
            elem_sums(b, ev[q]);
            ++q;
          }
        }
        const f32x4 wa = fr[(2 * s) % 4], wb = fr[(2 * s + 1) % 4];
        if constexpr (LENA_ABL & 8) {  // no MFMAs: the ring, barriers and epilogues alone
          ca += wa * Lr[jb][0];
          cb += wb * Lr[jb][1];
          step_tail(std::integral_constant<int, s>{});
          return;
        }
        ca = mfma4(wa.x, Lr[jb][0], ca);
        cb = mfma4(wb.x, Lr[jb][0], cb);
        ca = mfma4(wa.y, Lr[jb][1], ca);
        cb = mfma4(wb.y, Lr[jb][1], cb);
        ca = mfma4(wa.z, Lr[jb][2], ca);
        cb = mfma4(wb.z, Lr[jb][2], cb);
        ca = mfma4(wa.w, Lr[jb][3], ca);
        cb = mfma4(wb.w, Lr[jb][3], cb);
        if constexpr (MODE == 0 && p == NP1 - 1) {
          // L_{k+1}'s block jb: this was the last read of L_k's block jb
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            Lr[jb][r] = bload(rln, vo + row_off(jb, r, ld));
            pin_agpr(Lr[jb][r]);
          }
        }
        step_tail(std::integral_constant<int, s>{});
      });
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float y = h ? cb[r] : ca[r];
          if constexpr (MODE == 0) {
            if constexpr (LENA_ABL & 1) sdy += y;
            else masked_add(sdy, dual_gap(y, Gac), 16 * (2 * p + h) + r, limn);
          } else if constexpr (MODE == 2) {
            float dv, dd;
            dual_gap_vd(y, Gac, dv, dd);
            masked_add(sdy, dv, 16 * (2 * p + h) + r, limn);
            S[2 * p + h][r] = dd;  // rows past n: y = 0 exactly, so S = 0 there
            pin_agpr(S[2 * p + h][r]);
          } else {
            // rows past n: y = 0 exactly (zero-padded A^T), so S = 0 there
            if constexpr (LENA_ABL & 1) S[2 * p + h][r] = y;
            else S[2 * p + h][r] = dual_gap_d(y, Gac);
            pin_agpr(S[2 * p + h][r]);
          }
        }
    });

    if constexpr (MODE == 0) {
      const float v[4] = {col_sum(se), col_sum(sdy), col_sum(sdl), col_sum(slx)};
#pragma unroll
      for (int t = 0; t < 4; ++t)
        bstore_s(rpart, vp, (uint32_t)(((int64_t)k * 4 + t) * a.ldl * 4), v[t]);
    } else {
      // ---- G2: G = A S, blocks (2p, 2p+1) of the m rows over kb = 0..NB-1; epilogue gL, gE
      const float c = a.coef[k];
      const float cn = c * a.inv_nb, cm = c * a.inv_mb, xsg = a.xsign;
      const uint32_t vg = cv ? (uint32_t)((col + (int64_t)(4 * g) * a.ldg) * 4) : kOOB;
      const uint32_t gbytes = (uint32_t)((int64_t)m * a.ldg * 4);
      const rsrc_t rgl = mkrsrc(a.gL + (int64_t)k * a.gls, gbytes);
      const rsrc_t rge = mkrsrc(a.gE + (int64_t)k * a.gls, gbytes);
      static_for<MB / 2>([&](auto P_) {
        constexpr int p = decltype(P_)::value;
        float ev[2][4], base[2][4], gsg[2][4];
        f32x4 ca = zero4, cb = zero4;
        static_for<NB>([&](auto K_) {
          constexpr int kb = decltype(K_)::value;
          constexpr int s = T1 + p * NB + kb;  // G2 follows G1 in the stream
          step_head(std::integral_constant<int, s>{});
          if constexpr (kb == 0) {  // this pair's E rows, in flight during its MFMAs
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int r = 0; r < 4; ++r) ev[h][r] = bload(re, vo + row_off(2 * p + h, r, ld));
          }
          if constexpr (kb == NB - 2) {
            // the parts of the epilogue that need no product, one step before the pair's last
            // (E waited for before the last step's barrier issues the next DMA; see G1)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const f32x4 xv = xs[(w * MB + 2 * p + h) * 64 + lane];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float l = Lr[2 * p + h][r];
                const float e = ev[h][r];
                float dl;
                if constexpr (MODE == 2) {  // the elementwise sums of the objective too
                  float gv;
                  dual_gap_vd(l, G1c, gv, dl);
                  se += fabsf(e);
                  masked_add(sdl, gv, 16 * (2 * p + h) + r, limm);
                  slx += l * xv[r];
                } else {
                  dl = dual_gap_d(l, G1c);
                }
                base[h][r] = cm * (dl + xsg * xv[r]);  // xsg = +-1: exact
                gsg[h][r] = cm * ((e > 0.f ? 1.f : 0.f) - (e < 0.f ? 1.f : 0.f));
              }
            }
          }
          const f32x4 wa = fr[(2 * s) % 4], wb = fr[(2 * s + 1) % 4];
          ca = mfma4(wa.x, S[kb][0], ca);
          cb = mfma4(wb.x, S[kb][0], cb);
          ca = mfma4(wa.y, S[kb][1], ca);
          cb = mfma4(wb.y, S[kb][1], cb);
          ca = mfma4(wa.z, S[kb][2], ca);
          cb = mfma4(wb.z, S[kb][2], cb);
          ca = mfma4(wa.w, S[kb][3], ca);
          cb = mfma4(wb.w, S[kb][3], cb);
          if constexpr (kb == NB - 1) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const uint32_t so = row_off(2 * p + h, r, a.ldg);
                bstore_s(rgl, vg, so, cn * (h ? cb[r] : ca[r]) + base[h][r]);
                bstore_s(rge, vg, so, gsg[h][r]);
              }
            // L_{k+1}'s blocks 2p, 2p+1 (their last read of L_k was just above)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                Lr[2 * p + h][r] = bload(rln, vo + row_off(2 * p + h, r, ld));
                pin_agpr(Lr[2 * p + h][r]);
              }
          }
          step_tail(std::integral_constant<int, s>{});
        });
      });
      if constexpr (MODE == 2) {
        const float v[4] = {col_sum(se), col_sum(sdy), col_sum(sdl), col_sum(slx)};
#pragma unroll
        for (int t = 0; t < 4; ++t)
          bstore_s(rpart, vp, (uint32_t)(((int64_t)k * 4 + t) * a.ldl * 4), v[t]);
      }
    }
    chb += CPL;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's last DMA has landed
}

template <int MP, int NP>
hipError_t launch_lena_s(const LenaArgs& a, int grid, hipStream_t s) {
  if (a.mode == 0)
    hipLaunchKernelGGL((lena_kernel<MP, NP, 0>), dim3(grid), dim3(256), 0, s, a);
  else if (a.mode == 1)
    hipLaunchKernelGGL((lena_kernel<MP, NP, 1>), dim3(grid), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((lena_kernel<MP, NP, 2>), dim3(grid), dim3(256), 0, s, a);
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

// ---------------------------------------------------------------------------------------------
// Small batches (dladmm_lena_f32 at most one 16-column workgroup per CU, the 256 x 512 shape):
// the same objective with one workgroup per 16 columns and the ROWS of each product split over
// its 4 waves (the scheme of dladmm_fused_rs.hip).  The layers' terms are independent (each reads
// only L_k, E_k and X), so every (16-column group, layer) pair is its own workgroup (grid
// ceil(B / 16) x K): at the reference loop's B = 20, 30 workgroups instead of 2.  In layer k, wave
// w loads rows 4w.. of L_k
// into LDS (G1's B operand is all of L_k), computes G1 = A^T L_k for n blocks 8w .. 8w+7 (their
// dual_gap sums and S = dual_gap'), hands S over through LDS, and computes G2 = A S for m blocks
// 4w .. 4w+3 with the gL / gE epilogue and the E / L / X sums of those rows.  Same packed
// fragments, chain orders and expressions as lena_kernel: gE, gL bit for bit; the per-column
// sums are the same terms added in another order (each wave its rows, then the 4 in wave order).
namespace dladmm {

template <int MP, int NP, int MODE>
__global__ __launch_bounds__(256, 1) void lena_rs_kernel(const LenaArgs a) {
  constexpr int MB = MP / 16, NB = NP / 16, NB4 = NB / kWaves, MB4 = MB / kWaves;
  static_assert(NB4 % 2 == 0 && MB4 % 2 == 0, "each wave computes whole pairs of blocks");
  constexpr bool GRAD = MODE >= 1, SUMS = MODE != 1;
  constexpr int S1 = (NB4 / 2) * MB, S2 = (MB4 / 2) * NB;
  __shared__ f32x4 lx[MB * 64];   // L_k of the 16 columns (G1's B operand)
  __shared__ f32x4 sx[NB * 64];   // S (G2's B operand)
  __shared__ float red[2][kWaves][4][16];  // per-wave column sums, by layer parity

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int K = a.K, m = a.m, n = a.n;
  const int64_t col = (int64_t)blockIdx.x * 16 + (lane & 15);
  const bool cv = col < a.B;
  const int b1o = w * NB4, b2o = w * MB4;
  const int64_t ld = a.ld;
  const uint32_t vo = cv ? (uint32_t)((col + (int64_t)(4 * g) * ld) * 4) : kOOB;
  const uint32_t vx = cv ? (uint32_t)((col + (int64_t)(4 * g) * a.ldx) * 4) : kOOB;
  const uint32_t mbytes = (uint32_t)((int64_t)m * ld * 4);
  auto row_off = [&](int b, int r, int64_t stride) -> uint32_t {
    uint32_t o = (uint32_t)((int64_t)(16 * b) * stride * 4);
    asm volatile("" : "+s"(o));
    return o + (uint32_t)((int64_t)r * stride * 4);
  };
  const int limm = cv ? m - 4 * g : -1, limn = cv ? n - 4 * g : -1;
  const Gap Gac{a.gc[0], a.gc[1], a.gc[2], a.gc[3]}, G1c{a.gc[4], a.gc[5], a.gc[6], a.gc[7]};
  float Xr[MB4][4];
  {
    const rsrc_t rx = mkrsrc(a.X, (uint32_t)((int64_t)m * a.ldx * 4));
#pragma unroll
    for (int b = 0; b < MB4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) Xr[b][r] = bload(rx, vx + row_off(b2o + b, r, a.ldx));
  }
  const uint32_t vf = (uint32_t)(lane * 16);
  const int64_t wl = (int64_t)MB * NB * kFrag;
  const rsrc_t rat = mkrsrc(a.Atp + (int64_t)(b1o / 2) * MB * 2 * kFrag, (uint32_t)(S1 * 2 * kFrag * 4));
  const rsrc_t ra = mkrsrc(a.Ap + (int64_t)(b2o / 2) * NB * 2 * kFrag, (uint32_t)(S2 * 2 * kFrag * 4));
  (void)wl;
  auto frag2 = [&](rsrc_t r, auto S_, f32x4& fa, f32x4& fb) {
    constexpr int s = decltype(S_)::value;
    fa = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)vf, 2 * s * 1024, 0));
    fb = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)vf, (2 * s + 1) * 1024, 0));
  };
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  const rsrc_t rpart = mkrsrc(a.part, (uint32_t)((int64_t)4 * K * a.ldl * 4));
  auto flush = [&](int k) {  // wave 0 adds the 4 waves' column sums in order
    if (w == 0 && g == 0) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float v = red[k & 1][0][t][lane];
#pragma unroll
        for (int q = 1; q < kWaves; ++q) v += red[k & 1][q][t][lane];
        bstore_s(rpart, (uint32_t)(col * 4), (uint32_t)(((int64_t)k * 4 + t) * a.ldl * 4), v);
      }
    }
  };

  {
    const int k = blockIdx.y;  // this workgroup's layer
    (void)K;
    const rsrc_t rl = mkrsrc(a.L + (int64_t)k * a.ls, mbytes);
    const rsrc_t re = mkrsrc(a.E + (int64_t)k * a.ls, mbytes);
    float Lw[MB4][4], Ew[MB4][4];
#pragma unroll
    for (int b = 0; b < MB4; ++b) {
      f32x4 lv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        Lw[b][r] = bload(rl, vo + row_off(b2o + b, r, ld));
        Ew[b][r] = bload(re, vo + row_off(b2o + b, r, ld));
        lv[r] = Lw[b][r];
      }
      lx[(b2o + b) * 64 + lane] = lv;
    }
    __syncthreads();  // L_k complete
    float se = 0.f, sdy = 0.f, sdl = 0.f, slx = 0.f;
    // ---- G1: Y = A^T L_k for this wave's n blocks
    f32x4 fa[4], fb[4];
    static_for<4>([&](auto I_) {
      constexpr int i = decltype(I_)::value;
      if constexpr (i < S1) frag2(rat, I_, fa[i], fb[i]);
    });
    static_for<NB4 / 2>([&](auto P_) {
      constexpr int pp = decltype(P_)::value;
      f32x4 ca = zero4, cb = zero4;
      static_for<MB>([&](auto J_) {
        constexpr int jb = decltype(J_)::value;
        constexpr int s = pp * MB + jb;
        const f32x4 v = lx[jb * 64 + lane];
        const f32x4 wa = fa[s % 4], wb = fb[s % 4];
        if constexpr (s + 4 < S1) frag2(rat, std::integral_constant<int, s + 4>{}, fa[s % 4], fb[s % 4]);
        ca = mfma4(wa.x, v[0], ca);
        cb = mfma4(wb.x, v[0], cb);
        ca = mfma4(wa.y, v[1], ca);
        cb = mfma4(wb.y, v[1], cb);
        ca = mfma4(wa.z, v[2], ca);
        cb = mfma4(wb.z, v[2], cb);
        ca = mfma4(wa.w, v[3], ca);
        cb = mfma4(wb.w, v[3], cb);
      });
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 s4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float y = h ? cb[r] : ca[r];
          const int rr = 16 * (b1o + 2 * pp + h) + r;
          if constexpr (MODE == 0) {
            sdy += rr < limn ? dual_gap(y, Gac) : 0.f;
            s4[r] = 0.f;
          } else if constexpr (MODE == 2) {
            float dv, dd;
            dual_gap_vd(y, Gac, dv, dd);
            sdy += rr < limn ? dv : 0.f;
            s4[r] = dd;
          } else {
            s4[r] = dual_gap_d(y, Gac);
          }
        }
        if constexpr (GRAD) sx[(b1o + 2 * pp + h) * 64 + lane] = s4;
      }
    });
    // ---- the elementwise terms of this wave's m rows (E / L / X)
    float base[MB4][4], gsg[MB4][4];
    const float c = GRAD ? a.coef[k] : 0.f;
    const float cm = c * a.inv_mb, xsg = a.xsign;
#pragma unroll
    for (int b = 0; b < MB4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float l = Lw[b][r], e = Ew[b][r], x = Xr[b][r];
        const int rr = 16 * (b2o + b) + r;
        float dl = 0.f;
        if constexpr (MODE == 0) {
          se += fabsf(e);
          sdl += rr < limm ? dual_gap(l, G1c) : 0.f;
          slx += l * x;
        } else if constexpr (MODE == 2) {
          float gv;
          dual_gap_vd(l, G1c, gv, dl);
          se += fabsf(e);
          sdl += rr < limm ? gv : 0.f;
          slx += l * x;
        } else {
          dl = dual_gap_d(l, G1c);
        }
        base[b][r] = cm * (dl + xsg * x);
        gsg[b][r] = cm * ((e > 0.f ? 1.f : 0.f) - (e < 0.f ? 1.f : 0.f));
      }
    if constexpr (SUMS) {
      const float v[4] = {col_sum(se), col_sum(sdy), col_sum(sdl), col_sum(slx)};
      if (g == 0)
#pragma unroll
        for (int t = 0; t < 4; ++t) red[k & 1][w][t][lane] = v[t];
    }
    if constexpr (GRAD) {
      __syncthreads();  // S complete
      // ---- G2: G = A S for this wave's m blocks; gL = c/(nN) G + c/(mN) (dual_gap'(L) + X)
      const float cn = c * a.inv_nb;
      const uint32_t vg = cv ? (uint32_t)((col + (int64_t)(4 * g) * a.ldg) * 4) : kOOB;
      const uint32_t gbytes = (uint32_t)((int64_t)m * a.ldg * 4);
      const rsrc_t rgl = mkrsrc(a.gL + (int64_t)k * a.gls, gbytes);
      const rsrc_t rge = mkrsrc(a.gE + (int64_t)k * a.gls, gbytes);
      static_for<4>([&](auto I_) {
        constexpr int i = decltype(I_)::value;
        if constexpr (i < S2) frag2(ra, I_, fa[i], fb[i]);
      });
      static_for<MB4 / 2>([&](auto P_) {
        constexpr int pp = decltype(P_)::value;
        f32x4 ca = zero4, cb = zero4;
        static_for<NB>([&](auto K_) {
          constexpr int kb = decltype(K_)::value;
          constexpr int s = pp * NB + kb;
          const f32x4 v = sx[kb * 64 + lane];
          const f32x4 wa = fa[s % 4], wb = fb[s % 4];
          if constexpr (s + 4 < S2) frag2(ra, std::integral_constant<int, s + 4>{}, fa[s % 4], fb[s % 4]);
          ca = mfma4(wa.x, v[0], ca);
          cb = mfma4(wb.x, v[0], cb);
          ca = mfma4(wa.y, v[1], ca);
          cb = mfma4(wb.y, v[1], cb);
          ca = mfma4(wa.z, v[2], ca);
          cb = mfma4(wb.z, v[2], cb);
          ca = mfma4(wa.w, v[3], ca);
          cb = mfma4(wb.w, v[3], cb);
        });
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int lb = 2 * pp + h;
            const uint32_t so = row_off(b2o + lb, r, a.ldg);
            bstore_s(rgl, vg, so, cn * (h ? cb[r] : ca[r]) + base[lb][r]);
            bstore_s(rge, vg, so, gsg[lb][r]);
          }
      });
    }
  }
  if constexpr (SUMS) {
    __syncthreads();
    flush(blockIdx.y);
  }
}

template <int MODE>
hipError_t launch_lena_rs_m(const LenaArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((lena_rs_kernel<kShapeMP[2], kShapeNP[2], MODE>), dim3(grid, a.K), dim3(256),
                     0, s, a);
  return hipGetLastError();
}

hipError_t launch_lena_rs(const LenaArgs& a, int grid, hipStream_t s) {
  if (a.K <= 0) return hipSuccess;           // no layer, no term
  if (a.K > 65535) return hipErrorInvalidValue;  // grid.y
  if (a.mode == 0) return launch_lena_rs_m<0>(a, grid, s);
  if (a.mode == 1) return launch_lena_rs_m<1>(a, grid, s);
  return launch_lena_rs_m<2>(a, grid, s);
}

}  // namespace dladmm
