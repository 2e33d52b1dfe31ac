// dladmm_eval.hip -- per-column evaluation objectives over a forward's saved layers (SURVEY.md
// section 8 row f3): the per-sample sums the reference test scripts reduce into NMSE, L1L1,
// Normalized-L1L1, GT and Normalized-GT (test_syn_l1l1_scalar.py:436-489,
// test_syn_lasso_scalar.py:491-503).
//
// One thread per batch column (a wave's loads are coalesced across its 64 columns), one grid row
// per layer, fp64 accumulation:
//   reg[k][b] = sum_i |Z_k[i,b]|
//   fit[k][b] = sum_i |E_k - T_{k+1}|[i,b]  (L1L1)   or  0.5 sum_i (E_k - T_{k+1})^2  (LASSO)
//               -- X - A Z_k = E_k - T_{k+1} exactly in real arithmetic (T_{k+1} = A Z_k + E_k - X,
//               main_lena.py:88), so no product A Z_k is formed again
//   dz[k][b]  = sum_i (Z_k - Zref)^2[i,b],  de[k][b] = sum_i (E_k - Eref)^2[i,b]   (refs given)
#include "dladmm_common.h"

namespace dladmm {

struct ColObjArgs {
  int m, n, B, K;
  const float* Z; int64_t zls, ldz;   // layer k: Z + k*zls, row stride ldz
  const float* E; int64_t els, lde;
  const float* T; int64_t tls, ldt;   // layer k uses T_{k+1} = T + (k+1)*tls (may be NULL)
  const float* Zref; int64_t ldzr;
  const float* Eref; int64_t lder;
  int fit_kind;                       // dladmm_loss_kind
  double *reg, *fit, *dz, *de;        // [K][B] each, NULL = not wanted
};

__global__ __launch_bounds__(256) void colobj_kernel(const ColObjArgs a) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int k = blockIdx.y;
  if (b >= a.B) return;
  const float* Zk = a.Z + k * a.zls;
  const float* Ek = a.E ? a.E + k * a.els : nullptr;
  const int64_t o = (int64_t)k * a.B + b;
  if (a.reg || a.dz) {
    double r = 0.0, dz = 0.0;
    for (int i = 0; i < a.n; ++i) {
      const float z = Zk[i * a.ldz + b];
      r += fabs((double)z);
      if (a.Zref) {
        const double d = (double)(a.Zref[i * a.ldzr + b] - z);  // fp32 difference, as torch
        dz += d * d;
      }
    }
    if (a.reg) a.reg[o] = r;
    if (a.dz) a.dz[o] = dz;
  }
  if (Ek && (a.fit || a.de)) {
    const float* Tn = a.T ? a.T + (k + 1) * a.tls : nullptr;
    double f = 0.0, de = 0.0;
    for (int i = 0; i < a.m; ++i) {
      const float e = Ek[i * a.lde + b];
      if (Tn) {
        const double res = (double)(e - Tn[i * a.ldt + b]);
        f += a.fit_kind == DLADMM_LOSS_LASSO ? 0.5 * res * res : fabs(res);
      }
      if (a.Eref) {
        const double d = (double)(a.Eref[i * a.lder + b] - e);
        de += d * d;
      }
    }
    if (a.fit) a.fit[o] = f;
    if (a.de) a.de[o] = de;
  }
}

}  // namespace dladmm

extern "C" int dladmm_colobj_f32(const dladmm_colobj_desc* d, void* stream) {
  using namespace dladmm;
  if (!d) return DLADMM_E_NULL;
  if (d->abi_version != DLADMM_ABI_VERSION) return DLADMM_E_ABI_VERSION;
  if (d->m < 1 || d->n < 1 || d->batch < 1 || d->layers < 1) return DLADMM_E_SHAPE;
  if (!d->Z) return DLADMM_E_NULL;
  if ((d->fit || d->de) && !d->E) return DLADMM_E_NULL;
  if (d->fit && !d->T) return DLADMM_E_NULL;
  if (d->dz && !d->Zref) return DLADMM_E_NULL;
  if (d->de && !d->Eref) return DLADMM_E_NULL;
  if (d->fit_kind != DLADMM_LOSS_L1L1 && d->fit_kind != DLADMM_LOSS_LASSO && d->fit)
    return DLADMM_E_UNSUPPORTED;
  ColObjArgs a{};
  a.m = d->m; a.n = d->n; a.B = d->batch; a.K = d->layers;
  a.Z = d->Z; a.zls = d->z_layer_stride; a.ldz = d->ld_z;
  a.E = d->E; a.els = d->e_layer_stride; a.lde = d->ld_e;
  a.T = d->T; a.tls = d->t_layer_stride; a.ldt = d->ld_t;
  a.Zref = d->Zref; a.ldzr = d->ld_zref;
  a.Eref = d->Eref; a.lder = d->ld_eref;
  a.fit_kind = d->fit_kind;
  a.reg = d->reg; a.fit = d->fit; a.dz = d->dz; a.de = d->de;
  hipLaunchKernelGGL(colobj_kernel, dim3((unsigned)((d->batch + 255) / 256), d->layers),
                     dim3(256), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
