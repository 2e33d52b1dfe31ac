// dladmm_backward.hip -- MI355X (gfx950) backward of the K-layer D-LADMM forward (SURVEY.md
// section 8 row f1): the vector-Jacobian product torch autograd computes when the reference
// training loops call total_loss.backward() (main_lena.py:229, main_syn_l1l1_scalar.py:298,
// main_syn_lasso_scalar.py:285) through DLADMMNet.forward.
//
// One reverse sweep over the layers, three GEMM kernels per layer whose epilogues carry the whole
// elementwise adjoint algebra (derivation: oracle/dladmm_oracle_grad.py, which restates it in
// numpy and is pinned against the reference's autograd gradients):
//   BK1(k)  P = A Z_k                   (m rows, contraction n)  recompute E_k, T_{k+1};
//           adjoints of L_k, T_{k+1}, E_k -> gP, adjoint of E_{k-1}, partial adjoint of L_{k-1},
//           Var_k = L_{k-1} + b1 T_k (operand of BK2/wgrad); grads of b3, b2, ss2, ss2b, theta_e
//   BK2(k)  R = A^T gP, q = W_k Var_k    (n rows, contraction m, two GEMMs)  recompute U_k;
//           gU = (adj Z_k + R) * S'(U_k) = adjoint of Z_{k-1}; grads of theta_z, s1
//   BK3(k)  gVar = M_k^T gU              (m rows, contraction n)  adjoint of L_{k-1} += gVar,
//           adjoint of T_k = b1 gVar; grad of b1
//   WG(k)   gM_k = gU Var_k^T            (n x m, contraction over the batch: split-K + fixed-order
//           reduction, so it is deterministic); gW_k = -s1 gM_k
// where M_k = -s1 W_k.  P and q are recomputed with the fragment packing / accumulation order of
// the forward kernels (U = Z_{k-1} - s1 q on both forward paths), so the shrink masks S'(.) are
// those of the forward, bit for bit.
// Parameter gradients of broadcast parameters are reduced per wave (scalars: over the wave; per
// row: over the wave's 16 columns) into partial buffers and summed in fp64 in a fixed order.
#include <array>

#include "dladmm_common.h"
#include "dladmm_internal.h"
#include "dladmm_slice.h"

namespace dladmm {

// (dS/dx, dS/dth) of S(x, th) = relu(x - th) - relu(-1.0*x - th) (main_lena.py:52-53) under
// torch's relu' = [v > 0]: dS/dx = [x-th > 0] + [-x-th > 0], dS/dth = [-x-th > 0] - [x-th > 0].
struct SD { float dx, dth; };
__device__ __forceinline__ SD shrink_d(float x, float th) {
  const float a = (x - th) > 0.0f ? 1.0f : 0.0f;
  const float b = (-x - th) > 0.0f ? 1.0f : 0.0f;
  return SD{a + b, b - a};
}

// sum over the 16 lanes that share lane>>4 (the 16 batch columns of one row)
// (the reverse sweep forms the same per-row partials with the same function, dladmm_common.h)
__device__ __forceinline__ float col16_sum(float v) { return row16_sum(v); }

#ifndef BWD_EPI_FENCE
#define BWD_EPI_FENCE 1
#endif
#ifndef BWD_MIN_WG
#define BWD_MIN_WG 2
#endif

// PH: 1 = BK1, 2 = BK2, 3 = BK3, 4 = BK1 on the forward's saved P_k = A Z_k (a.Pk; no GEMM:
// an elementwise pass over the m x B adjoints), 5 = BK2 on the saved Z_k mask only (one GEMM,
// 32-block slices; launched beside a PH 2 launch, each exits unless theta_z's sign is its case),
// 6 = BK3(k3) fused with BK1(k3 - 1) on the saved product (a.k = k3 - 1): BK3's epilogue has, per
// element, the complete adjoint of L_{k3-1} and the adjoint of T_{k3} that BK1(k3 - 1) consumes,
// so they never round-trip through HBM and BK1 needs no launch of its own
template <int EMODE, int PKIND, int PH, int NW, int SB>
__global__ __launch_bounds__(NW * 64, BWD_MIN_WG) void bwd_kernel(const BwdArgs a) {
  constexpr bool FUS = PH == 6;
  constexpr bool BK1 = PH == 1 || PH == 4 || FUS;
  constexpr bool BK2 = PH == 2 || PH == 5;
  constexpr bool PSV = PH == 4;            // no GEMM: one column per lane
  constexpr bool SAVEDP = PH == 4 || FUS;  // P = A Z_k from the forward (a.Pk)
  if constexpr (BK2 && PKIND != PK_ROW) {
    // zk_mask 2: the PH 5 launch covers theta_z >= 0 and the PH 2 launch theta_z < 0
    if (a.zk_mask == 2) {
      const bool pos = ((cfloat_p)a.scal)[a.k * DLADMM_NSCALAR + DLADMM_P_THETA_Z] >= 0.0f;
      if (pos != (PH == 5)) return;  // uniform: the whole grid exits
    }
  }
  if constexpr (BK2 && PKIND == PK_ROW) {
    // per-row theta_z (V2, V3): the PH 5 launch covers layers whose every row has theta_z >= 0,
    // the PH 2 launch the others.  With theta < 0 both relus are open on |U| < |theta| and the
    // forward's literal shrink rounds U within an ulp of -|theta| to Z = -2|theta|, the value
    // U = -|theta| gives too: the saved Z_k cannot tell the two masks apart, U can
    if (a.zk_mask == 2) {
      const float* th = a.rowp + ((int64_t)a.k * 8 + DLADMM_P_THETA_Z) * a.rstride;
      int neg = 0;
      for (int r = threadIdx.x; r < a.n; r += NW * 64) neg |= th[r] < 0.0f ? 1 : 0;
      neg = __syncthreads_or(neg);
      if ((neg == 0) != (PH == 5)) return;  // uniform over the workgroup (and the grid)
    }
  }
  // BK1 keeps 4 workgroups per CU (its latency-bound epilogue needs them): a 2-deep B ring
  constexpr int NSB = (PH == 1 || FUS) ? 2 : 3;
  __shared__ f32x4 ring[PSV ? 1 : slice_lds_f4<NW, NSB>()];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // GEMM phases: the MFMA C/D layout (lane: column l & 15, rows 16b + 4(l >> 4) + r).  PH 4 has
  // no GEMM, so a lane owns one column and a wave 64 consecutive ones: every operand access of a
  // row is one 256-byte piece (the C/D layout touches four 64-byte pieces per instruction)
  const int g = PSV ? 0 : lane >> 4;
  const int64_t col = PSV ? (int64_t)blockIdx.x * (64 * NW) + w * 64 + lane
                          : (int64_t)blockIdx.x * (16 * NW) + w * 16 + (lane & 15);
  const bool cv = col < a.B;
  const int64_t colc = cv ? col : 0;
  const int ib0 = blockIdx.y * SB;
  const int k = a.k;

  f32x4 acc[PSV ? 1 : SB];
  if constexpr (!PSV)
    slice_gemm<NW, SB, NSB>(ring, a.Wp, a.MBp, ib0, a.KB, a.S, a.ldS, a.Krows, a.B, acc);
  else
    (void)ring;
  // BK2: the shrink is monotone, so the forward's own Z_k gives S'(U) and dS/dtheta_z (and the
  // objective's sign(Z_k)) for either sign of theta_z; then q = W_k Var_k is needed only for a
  // trainable step s1 (V5).  PH 5 (one GEMM) runs the per-row kinds (V2, V3) and, with a uniform
  // theta_z >= 0, the scalar ones; a scalar layer with theta_z < 0 still goes through PH 2 (the
  // PH 2 launch of a zk_mask layer reaches here only then: it forms q)
  constexpr bool zmask = PH == 5;
  f32x4 acc2[PH == 2 ? SB : 1];
  if constexpr (PH == 5) {
    acc2[0] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else if constexpr (PH == 2) {
    slice_gemm<NW, SB, NSB>(ring, a.Wp2, a.MBp, ib0, a.KB, a.S2, a.ldS2, a.Krows, a.B, acc2);
  }

  cfloat_p sp = (cfloat_p)a.scal + k * DLADMM_NSCALAR;
  const float* rp = a.rowp ? a.rowp + (int64_t)k * 8 * a.rstride : nullptr;
  // fused training objective coefficients of layer k (0 without one)
  const float czk = a.loss_kind ? ((cfloat_p)a.lcoef)[2 * k] : 0.0f;
  const float cfk = a.loss_kind ? ((cfloat_p)a.lcoef)[2 * k + 1] : 0.0f;
  const bool lossq = a.loss_kind == DLADMM_LOSS_LASSO;
  // scalar kinds: the layer's parameters, loaded once (uniform registers)
  float spv[DLADMM_NSCALAR];
#pragma unroll
  for (int sl = 0; sl < DLADMM_NSCALAR; ++sl)
    spv[sl] = (PKIND == PK_ROW) ? 0.0f : sp[sl];
  auto pm = [&](int slot, int rowc) -> float {  // scalar or per-row parameter of layer k
    if constexpr (PKIND == PK_ROW) return rp[(int64_t)slot * a.rstride + rowc];
    else return spv[slot];
  };
  // PH 6: beta1 of the BK3 layer k3 (its only parameter)
  const int k3 = FUS ? a.k3 : k;
  const float b1s3 = (FUS && PKIND != PK_ROW && PKIND != PK_ELEM)
                         ? ((cfloat_p)a.scal)[k3 * DLADMM_NSCALAR + DLADMM_P_BETA1] : 0.0f;
  const float* rp3 = (FUS && a.rowp) ? a.rowp + (int64_t)k3 * 8 * a.rstride : nullptr;
  auto pm3_b1 = [&](int rowc) -> float {
    if constexpr (PKIND == PK_ROW) return rp3[(int64_t)DLADMM_P_BETA1 * a.rstride + rowc];
    else return b1s3;
  };
  const int64_t ldw = a.ldw;  // row stride of the adjoint / operand workspaces

  // per-slot partial sums: scalar kind over the whole wave, row kind per row (col16_sum)
  float ps[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) ps[i] = 0.0f;
  float ps3 = 0.0f;  // PH 6: the BK3 layer's beta1 partial
  const int cg = blockIdx.x * NW + w;  // column group (wave) index
  auto row_flush = [&](int row, bool rok, const float (&v)[8], unsigned mask,
                       float* part = nullptr) {
    if constexpr (PKIND == PK_ROW) {
      float* dst = part ? part : a.part;
#pragma unroll
      for (int sl = 0; sl < 8; ++sl) {
        if (!(mask & (1u << sl))) continue;
        const float s = PSV ? wave_sum(v[sl]) : col16_sum(v[sl]);
        if ((PSV ? lane == 0 : (lane & 15) == 0) && rok)
          dst[((int64_t)sl * a.rstride + row) * a.ncg + cg] = s;
      }
    }
  };

  // operand / adjoint views (uniform row part in soffset; NULL or out-of-range reads 0)
  const int m = a.m, n = a.n;
  const BView vX = make_view(a.X, m, a.ldx, g, col, cv);
  const BView vEp = make_view(a.Ep, m, a.ldep, g, col, cv);
  const BView vLp = make_view(a.Lp, m, a.ldlp, g, col, cv);
  const BView vTk = make_view(a.Tk, m, a.ldt, g, col, cv);
  const BView vPk = make_view(SAVEDP ? a.Pk : nullptr, m, a.ldt, g, col, cv);
  const BView vTk3 = make_view(FUS ? a.Tk3 : nullptr, m, a.ldt, g, col, cv);  // T_{k3}
  const BView vb13 = make_view(FUS && PKIND == PK_ELEM ? a.b1e3 : nullptr, m, a.ldb, g, col, cv);
  const BView vgb13 = make_view(FUS && PKIND == PK_ELEM ? a.gb1e3 : nullptr, m, a.ldb, g, col, cv);
  const BView vZp = make_view(a.Zp, n, a.ldzp, g, col, cv);
  const BView vZk = make_view(BK2 && zmask ? a.Zk : nullptr, n, a.ldzk, g, col, cv);
  const BView vgZ = make_view(a.gZ, n, a.ldg, g, col, cv);
  const BView vgE = make_view(a.gE, m, a.ldg, g, col, cv);
  const BView vgL = make_view(a.gL, m, a.ldg, g, col, cv);
  const BView vgT = make_view(a.gT, m, a.ldg, g, col, cv);
  const BView vAZ = make_view(a.AZ, n, ldw, g, col, cv);
  const BView vAE = make_view(a.AE, m, ldw, g, col, cv);
  const BView vAL = make_view(a.AL, m, ldw, g, col, cv);
  const BView vAT = make_view(a.AT, m, ldw, g, col, cv);
  const BView vGP = make_view(a.GP, m, ldw, g, col, cv);
  const BView vVAR = make_view(a.VAR, m, ldw, g, col, cv);
  const BView vb1 = make_view(PKIND == PK_ELEM ? a.b1e : nullptr, m, a.ldb, g, col, cv);
  const BView vb2 = make_view(PKIND == PK_ELEM ? a.b2e : nullptr, m, a.ldb, g, col, cv);
  const BView vgb1 = make_view(PKIND == PK_ELEM ? a.gb1e : nullptr, m, a.ldb, g, col, cv);
  const BView vgb2 = make_view(PKIND == PK_ELEM ? a.gb2e : nullptr, m, a.ldb, g, col, cv);

  // The epilogue is software-pipelined over output blocks: pass 1 (bload) issues every load of
  // block i + 1 before pass 2 (bfinish) computes and stores block i -- the compiler cannot move a
  // load above a store it may alias, so element order would pay one memory round trip per block.
  struct BIn { float x, ep, lp, tk, b1, b2, AL, gL, AT, gT, AE, gE, zp, AZ, gZ, gb1, P, zk,
               tk3, b13, gb13; };
  auto bload_row = [&](int i, int r) {
    const uint32_t ru = (uint32_t)(16 * (ib0 + i) + r);  // uniform part of the row
    BIn v;
    if constexpr (BK1) {
      v.x = vX.ld(ru); v.ep = vEp.ld(ru); v.lp = vLp.ld(ru); v.tk = vTk.ld(ru);
      if constexpr (SAVEDP) v.P = vPk.ld(ru);
      if constexpr (PKIND == PK_ELEM) { v.b1 = vb1.ld(ru); v.b2 = vb2.ld(ru); }
      v.AL = vAL.ld(ru); v.gL = vgL.ld(ru);
      if constexpr (!FUS) v.AT = vAT.ld(ru);  // PH 6: formed by its BK3 part
      v.gT = vgT.ld(ru);
      v.AE = vAE.ld(ru); v.gE = vgE.ld(ru);
      if constexpr (FUS) {
        v.tk3 = vTk3.ld(ru);
        if constexpr (PKIND == PK_ELEM) { v.b13 = vb13.ld(ru); v.gb13 = vgb13.ld(ru); }
      }
    } else if constexpr (BK2) {
      v.zp = vZp.ld(ru); v.AZ = vAZ.ld(ru); v.gZ = vgZ.ld(ru); v.zk = vZk.ld(ru);
    } else {
      v.tk = vTk.ld(ru);
      if constexpr (PKIND == PK_ELEM) { v.b1 = vb1.ld(ru); v.gb1 = vgb1.ld(ru); }
      v.AL = vAL.ld(ru);
    }
    return v;
  };
  auto bload = [&](auto I_) {
    constexpr int i = decltype(I_)::value;
    return std::array<BIn, 4>{bload_row(i, 0), bload_row(i, 1), bload_row(i, 2),
                              bload_row(i, 3)};
  };
  auto bfinish_row = [&](int i, int r, const BIn& v) {
    {
      const int row = 16 * (ib0 + i) + 4 * g + r;
      const uint32_t ru = (uint32_t)(16 * (ib0 + i) + r);  // uniform part of the row
      float pv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if constexpr (BK1) {
        // ---------------- BK1: rows of m.  P = A Z_k (acc, or the forward's saved product)
        const bool rok = row < m;
        const bool ok = cv && rok;
        const int rowc = rok ? row : 0;
        float P;
        if constexpr (SAVEDP) P = v.P;
        else P = acc[i][r];
        // PH 6: BK3 of layer k3 first -- gVar = M_k3^T gU; its outputs (the complete adjoint of
        // L_{k3-1} and the adjoint of T_{k3}) are this BK1's incoming adjoints
        float aLin = v.AL, aTin = v.AT;
        if constexpr (FUS) {
          const float gVar = acc[i][r];
          const float b13 = (PKIND == PK_ELEM) ? v.b13 : pm3_b1(rowc);
          float pb1 = gVar * v.tk3;
          if constexpr (PKIND == PK_ELEM) vgb13.st(ru, v.gb13 + pb1);
          aLin = v.AL + gVar;
          aTin = b13 * gVar;   // adjoint of T_k3 (main_lena.py:85)
          if (!ok) pb1 = 0.f;
          if constexpr (PKIND == PK_ROW) {
            float pv3[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            pv3[DLADMM_P_BETA1] = pb1;
            row_flush(row, rok, pv3, 1u << DLADMM_P_BETA1, a.part3);
          } else {
            ps3 += pb1;
            asm volatile("" : "+v"(ps3));
          }
        }
        const float x = v.x;
        const float ep = v.ep;
        const float lp = v.lp;
        const float tk = v.tk;
        float b1, b2 = 0.f, b3;
        if constexpr (PKIND == PK_ELEM) {
          b1 = v.b1;
          b2 = v.b2;
          b3 = b1;  // main_lena.py:85,89: beta1 serves Var and L
        } else {
          b1 = pm(DLADMM_P_BETA1, rowc);
          b3 = pm(DLADMM_P_BETA3, rowc);
          if constexpr (EMODE != EM_LASSO) b2 = pm(DLADMM_P_BETA2, rowc);
        }
        // incoming adjoints of L_k, T_{k+1}, E_k
        const float aL = aLin + v.gL;
        const float aT = aTin + v.gT;
        const float aE = v.AE + v.gE;
        // recompute the forward's E_k and T_{k+1} (same expressions as the forward kernels)
        float e, gP, gEp = 0.f, gLp;
        float t;
        if constexpr (EMODE == EM_V1) {
          const float u = (x - P) - b2 * lp;                                  // main_lena.py:87
          const float the = pm(DLADMM_P_THETA_E, rowc);
          e = shrink(u, the);
          t = (P + e) - x;
          const float gTn = aT + b3 * aL;
          pv[DLADMM_P_BETA3] = aL * t;
          const float gEt = aE + gTn;
          const SD d = shrink_d(u, the);
          const float gEh = gEt * d.dx;
          pv[DLADMM_P_THETA_E] = gEt * d.dth;
          gP = gTn - gEh;
          pv[DLADMM_P_BETA2] = -gEh * lp;
          gLp = aL - b2 * gEh;
        } else if constexpr (EMODE == EM_VVAR) {
          const float ss2 = pm(DLADMM_P_SS2, rowc), the = pm(DLADMM_P_THETA_E, rowc);
          const float r0 = (P + ep) - x;
          const float vv = lp + b2 * r0;                                      // scalar.py:114
          const float eh = ep - ss2 * vv;                                     // scalar.py:115
          e = shrink(eh, the);
          t = (P + e) - x;
          const float gTn = aT + b3 * aL;
          pv[DLADMM_P_BETA3] = aL * t;
          const float gEt = aE + gTn;
          const SD d = shrink_d(eh, the);
          const float gEh = gEt * d.dx;
          pv[DLADMM_P_THETA_E] = gEt * d.dth;
          const float gVV = -ss2 * gEh;
          pv[DLADMM_P_SS2] = -gEh * vv;
          gLp = aL + gVV;
          pv[DLADMM_P_BETA2] = gVV * r0;
          gP = gTn + b2 * gVV;
          gEp = gEh + b2 * gVV;
        } else {
          const float ss2 = pm(DLADMM_P_SS2, rowc), ss2b = pm(DLADMM_P_SS2B, rowc);
          e = ss2 * (x - P) - ss2b * lp;                                      // lasso.py:102-103
          t = (P + e) - x;
          const float gTn = aT + b3 * aL;
          pv[DLADMM_P_BETA3] = aL * t;
          const float gEt = aE + gTn;
          pv[DLADMM_P_SS2] = gEt * (x - P);
          gP = gTn - ss2 * gEt;
          pv[DLADMM_P_SS2B] = -gEt * lp;
          gLp = aL - ss2b * gEt;
        }
        (void)e;
        {
          // d/dP of cf_k * fit_k: fit = sum|X - P| (torch sgn(0) = 0) or 0.5 sum (X - P)^2.
          // Branch-free (cf = 0 without a fused loss: gP - 0 * finite = gP exactly); a per-row
          // branch here splits the unrolled epilogue and the compiler hoists whole rows.
          const float res = x - P;
          const float dfit = lossq ? res : (res > 0.f ? 1.f : (res < 0.f ? -1.f : 0.f));
          gP = gP - cfk * dfit;
        }
        // out-of-range rows / columns: the stores are dropped by the buffer bounds
        vGP.st(ru, gP);
        vAE.st(ru, gEp);
        vAL.st(ru, gLp);
        vVAR.st(ru, lp + b1 * tk);  // Var_k = L_{k-1} + b1 T_k (main_lena.py:71,85)
        if constexpr (PKIND == PK_ELEM) {
          vgb1.st(ru, pv[DLADMM_P_BETA3]);  // BK3 adds gVar*T_k
          vgb2.st(ru, pv[DLADMM_P_BETA2]);
        }
        if (!ok) {
#pragma unroll
          for (int sl = 0; sl < 8; ++sl) pv[sl] = 0.f;
        }
        row_flush(row, rok, pv, (1u << DLADMM_P_BETA3) | (1u << DLADMM_P_BETA2) |
                                    (1u << DLADMM_P_THETA_E) | (1u << DLADMM_P_SS2) |
                                    (1u << DLADMM_P_SS2B));
      } else if constexpr (BK2) {
        // ---------------- BK2: rows of n.  acc = R = A^T gP, acc2 = q = W_k Var_k
        const bool rok = row < n;
        const bool ok = cv && rok;
        const int rowc = rok ? row : 0;
        const float R = acc[i][r];
        const float q = PH == 5 ? 0.0f : acc2[PH == 5 ? 0 : i][r];
        const float zp = v.zp;
        float s1 = 1.0f;
        if constexpr (PKIND == PK_SCALAR) s1 = spv[DLADMM_P_S1];
        // U exactly as the forward kernels formed it: Z_{k-1} - s1 (W_k Var_k)
        const float U = zp - ((PKIND == PK_SCALAR) ? s1 * q : q);
        const float thz = pm(DLADMM_P_THETA_Z, rowc);
        float gZt = (v.AZ + v.gZ) + R;
        // Z_k = S(U, theta_z): the forward's (zmask) or recomputed as the forward formed it
        const float z = zmask ? v.zk : shrink(U, thz);
        // d/dZ_k of cz_k * sum|Z_k|
        gZt = gZt + czk * (z > 0.f ? 1.f : (z < 0.f ? -1.f : 0.f));
        SD d = shrink_d(U, thz);
        if (zmask) {
          // S is monotone: [U - th > 0] = [Z_k > -c], [-U - th > 0] = [Z_k < c] with c = 0 for
          // th >= 0 and c = 2|th| for th < 0 (both relus open, Z = 2U, where |Z_k| < 2|th|).
          // Both kinds reach PH 5 only with th >= 0 on every row (c = 0: exact); the c > 0
          // branch serves the DLADMM_BWD_ZMASK experiments.
          const float c = thz >= 0.f ? 0.f : -2.0f * thz;
          const float zp1 = z > -c ? 1.f : 0.f, zn1 = z < c ? 1.f : 0.f;
          d = SD{zp1 + zn1, zn1 - zp1};
        }
        const float gU = gZt * d.dx;
        pv[DLADMM_P_THETA_Z] = gZt * d.dth;
        if constexpr (PKIND == PK_SCALAR) {
          pv[DLADMM_P_S1] = -gU * q;  // dU/ds1 = -W Var
        }
        vAZ.st(ru, gU);  // adjoint of Z_{k-1}; also BK3's operand and wgrad's gM rows
        if (!ok) {
#pragma unroll
          for (int sl = 0; sl < 8; ++sl) pv[sl] = 0.f;
        }
        row_flush(row, rok, pv, 1u << DLADMM_P_THETA_Z);
      } else {
        // ---------------- BK3: rows of m.  acc = gVar = M_k^T gU
        const bool rok = row < m;
        const bool ok = cv && rok;
        const int rowc = rok ? row : 0;
        const float gVar = acc[i][r];
        const float tk = v.tk;
        float b1;
        if constexpr (PKIND == PK_ELEM) b1 = v.b1;
        else b1 = pm(DLADMM_P_BETA1, rowc);
        pv[DLADMM_P_BETA1] = gVar * tk;
        vAL.st(ru, v.AL + gVar);
        vAT.st(ru, b1 * gVar);  // adjoint of T_k (main_lena.py:85)
        if constexpr (PKIND == PK_ELEM) vgb1.st(ru, v.gb1 + pv[DLADMM_P_BETA1]);
        if (!ok) pv[DLADMM_P_BETA1] = 0.f;
        row_flush(row, rok, pv, 1u << DLADMM_P_BETA1);
      }
#pragma unroll
      for (int sl = 0; sl < 8; ++sl) {
        ps[sl] += pv[sl];
        // materialise the running sum here: otherwise the scheduler sinks the whole serial
        // chain below the last row and keeps every row's terms live (hundreds of registers)
        if constexpr (PKIND != PK_ROW) asm volatile("" : "+v"(ps[sl]));
      }
    }
  };
  auto bfinish = [&](auto I_, const std::array<BIn, 4>& in) {
    constexpr int i = decltype(I_)::value;
#pragma unroll
    for (int r = 0; r < 4; ++r) bfinish_row(i, r, in[r]);
  };
  // BK1 loads up to 12 operands per element: pipelined it needs > 128 registers and loses the
  // 4-workgroups-per-CU occupancy that hides its latency better, so it runs block by block
  constexpr bool kPipe = !BK1;
  std::array<BIn, 4> cur;
  if constexpr (kPipe) cur = bload(std::integral_constant<int, 0>{});
  static_for<SB>([&](auto I_) {
    constexpr int i = decltype(I_)::value;
    if constexpr (!kPipe) {
#pragma unroll
      for (int r = 0; r < (PSV ? 16 : 4); r += 2) {  // two rows' loads, then their stores
        const BIn v0 = bload_row(i, r), v1 = bload_row(i, r + 1);
        bfinish_row(i, r, v0);
        bfinish_row(i, r + 1, v1);
      }
      asm volatile("" ::: "memory");  // no load of the next block moves above this one's stores
    } else if constexpr (i + 1 < SB) {
      const auto nxt = bload(std::integral_constant<int, i + 1>{});
      asm volatile("" ::: "memory");  // block i+1's loads stay above block i's stores
      bfinish(I_, cur);
      cur = nxt;
    } else {
      bfinish(I_, cur);
    }
    if constexpr (BWD_EPI_FENCE) __builtin_amdgcn_sched_barrier(0);
  });
  if constexpr (PKIND == PK_SCALAR) {
    // PH 5 slices span two 16-block slices: the partial goes to the first one's slot and the
    // second one's slot is zeroed (the reduction sums the 16-block slot count)
    const int sy = PH == 5 ? 2 * (int)blockIdx.y : (int)blockIdx.y;
    const int slot = sy * gridDim.x * NW + cg;
    auto flush = [&](int sl) {
      const float s = wave_sum(ps[sl]);
      if (lane == 0) {
        a.part[(int64_t)sl * a.nslots + slot] = s;
        if (PH == 5) a.part[(int64_t)sl * a.nslots + slot + gridDim.x * NW] = 0.0f;
      }
    };
    if constexpr (FUS) {
      const float s = wave_sum(ps3);
      if (lane == 0) a.part3[(int64_t)DLADMM_P_BETA1 * a.nslots + slot] = s;
    }
    if constexpr (BK1) {
      flush(DLADMM_P_BETA3);
      if constexpr (EMODE == EM_VVAR) { flush(DLADMM_P_BETA2); flush(DLADMM_P_SS2); flush(DLADMM_P_THETA_E); }
      if constexpr (EMODE == EM_V1) { flush(DLADMM_P_BETA2); flush(DLADMM_P_THETA_E); }
      if constexpr (EMODE == EM_LASSO) { flush(DLADMM_P_SS2); flush(DLADMM_P_SS2B); }
    } else if constexpr (BK2) {
      flush(DLADMM_P_THETA_Z);
      flush(DLADMM_P_S1);
    } else {
      flush(DLADMM_P_BETA1);
    }
  }
}

// ------------------------------------------------------------------------ weight gradient
// part[c][i][j] = sum_{b in chunk c} G[i][b] * V[j][b]   (G: n x ld, V: m x ld; both zero-padded
// to whole 128-row tiles and whole 16-column steps, so no masks).  One workgroup = 4 waves in a
// 2 x 2 grid over a 128 x 128 output tile; a wave keeps 4 x 4 16x16 accumulators.
// Operands stream by LDS-DMA through a 4-stage ring: a stage is one 16-column step of the tile,
// 16 fragments of 1 KiB (G row blocks 0..7, V row blocks 0..7), each in the MFMA operand layout
// (lane l: row 16 a + (l & 15), columns 16 s + 4 (l >> 4) .. +3), so every operand read is one
// conflict-free ds_read_b128; wave w DMAs fragments 4w .. 4w+3, three steps ahead.  Per step and
// block pair, 4 MFMAs whose k-index is the batch column 16 s + 4 (l >> 4) + q -- the same
// permutation for both operands, so the contraction is exact.  ~110 registers: two workgroups
// per CU.  (The previous form loaded the operands into registers one step ahead: 178 us per
// layer at B = 65,536, latency-bound.)
constexpr int kWgStages = 4;
//
// 1-D grid over (tile, chunk, layer).  Workgroups reach the 8 XCDs round-robin by linear id; with
// xcd set the tiles of one (chunk, layer) run on one XCD back to back, so its L2 serves the G and
// V row blocks they share (each V block is read by every G tile, each G block by every V tile)
// once from HBM.  Without it, consecutive ids spread a chunk's tiles over the XCDs.
// Iteration s issues the LDS-DMA of step s + 3 right after the barrier, beside the fragment reads
// (issued after the first quarter of the MFMAs, or one piece after each quarter, it measured no
// faster: round-5 A/B)
__global__ __launch_bounds__(256, 2) void wgrad_kernel(const WgradArgs a, int xcd) {
  __shared__ f32x4 ring[kWgStages * 16 * 64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tiles_m = a.MBp16 / 8;  // 128-column tiles (of V rows)
  const int ntiles = (a.NBp16 / 8) * tiles_m;
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
  const int64_t zl = grp / a.nchunks;  // layer of a batched launch
  const int cy = grp % a.nchunks;
  const int ti = tile / tiles_m, tj = tile % tiles_m;
  const int64_t b0 = (int64_t)cy * a.chunk;
  int64_t b1 = b0 + a.chunk;
  if (b1 > a.Bpad) b1 = a.Bpad;
  const int steps = b1 > b0 ? (int)((b1 - b0) / 16) : 0;
  const int r = lane & 15, g = lane >> 4;

  f32x4 acc[4][4];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};

  // this wave's DMA share: waves 0, 1 the G row blocks 4w .. 4w+3, waves 2, 3 the V row blocks
  // 4(w-2) .. +3 of the tile; lane offset of row 16 f + r, column 4 g (bytes, < 2^31: host)
  const float* src = w < 2 ? a.G + zl * a.gls + (int64_t)(ti * 128 + 64 * w) * a.ld
                           : a.V + zl * a.vls + (int64_t)(tj * 128 + 64 * (w - 2)) * a.ld;
  src += b0;
  const uint32_t vl = (uint32_t)(((int64_t)r * a.ld + 4 * g) * 4);
  const uint32_t rs16 = (uint32_t)(16 * a.ld * 4);
  auto issue_f = [&](int s, int stage, int f) {
    uint64_t sb = (uint64_t)(src + 16 * (int64_t)s);
    asm volatile("" : "+s"(sb));
    glds16((const float*)sb, vl + f * rs16, ring + (stage * 16 + 4 * w + f) * 64);
  };
  auto issue = [&](int s, int stage) {
#pragma unroll
    for (int f = 0; f < 4; ++f) issue_f(s, stage, f);
  };
#pragma unroll
  for (int s = 0; s < kWgStages - 1; ++s)
    if (s < steps) issue(s, s);
  const int gf = 4 * (w >> 1), vf = 8 + 4 * (w & 1);  // this wave's operand fragments
  for (int s = 0; s < steps; ++s) {
    // stage s landed for every wave (the DMAs of the steps after it may stay in flight), and
    // every wave is done reading stage s - 1, which the issue below overwrites
    if (s + kWgStages - 2 < steps) ring_barrier_n<4 * (kWgStages - 2)>();
    else ring_barrier_n<0>();
    const bool more = s + kWgStages - 1 < steps;
    const int ns = s + kWgStages - 1, nst = (s + kWgStages - 1) % kWgStages;
    if (more) issue(ns, nst);
    const f32x4* st = ring + (s % kWgStages) * 16 * 64;
    f32x4 ga[4], va[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      ga[x] = st[(gf + x) * 64 + lane];
      va[x] = st[(vf + x) * 64 + lane];
    }
    auto quarter = [&](int q) {
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) acc[x][y] = mfma4(ga[x][q], va[y][q], acc[x][y]);
    };
#pragma unroll
    for (int q = 0; q < 4; ++q) quarter(q);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA in flight when the LDS is released
  // C/D layout: lane holds column (l & 15) = V row j, rows 4g + r' = G rows
  const int i0 = ti * 128 + (w >> 1) * 64, j0 = tj * 128 + (w & 1) * 64;
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

// gW[i][j] (+)= scale * sum_c part[c][i][j], c in fixed order; scale = -s1_k (or -1)
// gW = -s1_k * sum of the chunk partials G = gU_k Var_k^T (accumulate: tied V5 sums layers).
// Wd (V5): also the block's share of <W, G> in fp64 -> dotp[block]: ss1_k's gradient is
// sum_b sum_i gU_ib * dU_ib/dss1 = -sum_ij W_ij G_ij, the inner product of the tied weight with
// the same sums the weight gradient forms (no q = W Var_k product needed)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* part, int nchunks,
                                                           int64_t nm, const float* scal, int k,
                                                           int accumulate, float* gW,
                                                           int64_t ldgw, int m, const float* Wd,
                                                           int64_t ldwd, double* dotp) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  double dv = 0.0;
  if (e < nm) {
    float s = 0.0f;
    for (int c = 0; c < nchunks; ++c) s += part[(int64_t)c * nm + e];
    const float scale = -(scal ? scal[k * DLADMM_NSCALAR + DLADMM_P_S1] : 1.0f);
    const int64_t i = e / m, j = e % m;
    float* dst = gW + i * ldgw + j;
    *dst = accumulate ? *dst + scale * s : scale * s;
    if (Wd) dv = (double)Wd[i * ldwd + j] * (double)s;
  }
  if (Wd) {  // uniform: fixed-order block sum
    __shared__ double red[256];
    red[threadIdx.x] = dv;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) dotp[blockIdx.x] = red[0];
  }
}

// The same reduction for the nl layers of a batched weight-gradient launch (WredArgs): per
// element, each layer's chunk sum in the chunk order of wgrad_reduce_kernel; tied: added into
// one gW in descending layer order, as the per-layer launches did
__global__ __launch_bounds__(256) void wgrad_reduce_layers_kernel(const WredArgs a) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int i = (int)(e / a.m), j = (int)(e % a.m);  // used for e < nm only
  __shared__ double red[256];
  auto layer_sum = [&](int y) -> float {
    float s = 0.0f;
    const float* pp = a.part + (int64_t)y * a.pls;
    for (int c = 0; c < a.nchunks; ++c) s += pp[(int64_t)c * a.nm + e];
    return s;
  };
  auto dot_flush = [&](int k, double dv) {  // uniform: fixed-order block sum
    red[threadIdx.x] = dv;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) a.dotp[(int64_t)k * a.nbd + blockIdx.x] = red[0];
    __syncthreads();
  };
  if (!a.tied) {
    const int y = blockIdx.y, k = a.klo + y;
    double dv = 0.0;
    if (e < a.nm) {
      const float s = layer_sum(y);
      const float scale = -(a.scal ? a.scal[k * DLADMM_NSCALAR + DLADMM_P_S1] : 1.0f);
      a.gW[(int64_t)k * a.gls + (int64_t)i * a.ldgw + j] = scale * s;
      if (a.Wd) dv = (double)a.Wd[(int64_t)i * a.ldwd + j] * (double)s;
    }
    if (a.Wd) dot_flush(k, dv);
    return;
  }
  for (int y = a.nl - 1; y >= 0; --y) {
    const int k = a.klo + y;
    double dv = 0.0;
    if (e < a.nm) {
      const float s = layer_sum(y);
      const float scale = -(a.scal ? a.scal[k * DLADMM_NSCALAR + DLADMM_P_S1] : 1.0f);
      float* dst = a.gW + (int64_t)i * a.ldgw + j;
      *dst = *dst + scale * s;
      if (a.Wd) dv = (double)a.Wd[(int64_t)i * a.ldwd + j] * (double)s;
    }
    if (a.Wd) dot_flush(k, dv);
  }
}

hipError_t launch_wgrad_reduce_layers(const WredArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(wgrad_reduce_layers_kernel, dim3((unsigned)((a.nm + 255) / 256),
                                                      a.tied ? 1 : a.nl), dim3(256), 0, s, a);
  return hipGetLastError();
}

// g_s1 = -sum_b dotp[b] (fixed order) -> the layer's ss1 slot of the scalar gradients
__global__ __launch_bounds__(256) void s1_dot_finish_kernel(const double* dotp, int nb,
                                                            double* out) {
  __shared__ double red[256];
  double s = 0.0;
  for (int b = threadIdx.x; b < nb; b += 256) s += dotp[b];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = -red[0];
}

// ------------------------------------------------------------------------ dispatch
template <int EM, int PK, int PH>
hipError_t launch_bwd_v(const BwdArgs& a, dim3 grid, int sb, hipStream_t s) {
  constexpr int NW = kBwdWaves;
  // 16 output blocks per slice (with 32 the epilogue's operand loads spill: PH 1, scalar kind);
  // PH 5 (one GEMM, light epilogue) runs 32
  constexpr int SB = PH == 5 ? 32 : 16;
  if (sb != SB) return hipErrorInvalidValue;
  hipLaunchKernelGGL((bwd_kernel<EM, PK, PH, NW, SB>), grid, dim3(NW * 64), 0, s, a);
  return hipGetLastError();
}

template <int PH>
hipError_t launch_bwd_ph(int variant, const BwdArgs& a, dim3 grid, int sb, hipStream_t s) {
  switch (variant) {
    case DLADMM_V1_LENA: return launch_bwd_v<EM_V1, PK_ELEM, PH>(a, grid, sb, s);
    case DLADMM_V2_LTHETA: return launch_bwd_v<EM_V1, PK_ROW, PH>(a, grid, sb, s);
    case DLADMM_V3_FULL: return launch_bwd_v<EM_VVAR, PK_ROW, PH>(a, grid, sb, s);
    case DLADMM_V4_SCALAR:
    case DLADMM_V5_TIED: return launch_bwd_v<EM_VVAR, PK_SCALAR, PH>(a, grid, sb, s);
    case DLADMM_V6_LASSO: return launch_bwd_v<EM_LASSO, PK_SCALAR, PH>(a, grid, sb, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_bwd(int phase, int variant, const BwdArgs& a, dim3 grid, int sb,
                      hipStream_t s) {
  switch (phase) {
    case 1: return launch_bwd_ph<1>(variant, a, grid, sb, s);
    case 4: return launch_bwd_ph<4>(variant, a, grid, sb, s);
    case 5: return launch_bwd_ph<5>(variant, a, grid, sb, s);
    case 2: return launch_bwd_ph<2>(variant, a, grid, sb, s);
    case 3: return launch_bwd_ph<3>(variant, a, grid, sb, s);
    case 6: return launch_bwd_ph<6>(variant, a, grid, sb, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_wgrad(const WgradArgs& a, int tiles, hipStream_t s, int layers) {
  // XCD-grouped tiles where the (chunk, layer) count is a multiple of 8
  const int groups = a.nchunks * layers;
  const int xcd = groups % 8 == 0 ? 1 : 0;
  if (tiles != (a.NBp16 / 8) * (a.MBp16 / 8)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wgrad_kernel, dim3(tiles * groups), dim3(256), 0, s, a, xcd);
  return hipGetLastError();
}

hipError_t launch_wgrad_reduce(const float* part, int nchunks, int n, int m, const float* scal,
                               int k, int accumulate, float* gW, int64_t ldgw, hipStream_t s,
                               const float* Wd, int64_t ldwd, double* dotp) {
  const int64_t nm = (int64_t)n * m;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((nm + 255) / 256)), dim3(256), 0, s,
                     part, nchunks, nm, scal, k, accumulate, gW, ldgw, m, Wd, ldwd, dotp);
  return hipGetLastError();
}

int s1_dot_blocks(int n, int m) { return (int)(((int64_t)n * m + 255) / 256); }

hipError_t launch_s1_dot_finish(const double* dotp, int n, int m, double* out, hipStream_t s) {
  hipLaunchKernelGGL(s1_dot_finish_kernel, dim3(1), dim3(256), 0, s, dotp, s1_dot_blocks(n, m),
                     out);
  return hipGetLastError();
}

}  // namespace dladmm
