// dladmm_lskm.hip -- the safeguard step of learned + safeguarded KM (LSKM), SURVEY.md section 8
// row f2: test_syn_l1l1_scalar.py:227-266 and mu_updater.py:18-116.
//
// Per layer the LSKM forward evaluates, from the same state, a classic KM/LADMM step and a
// learned (L2O) step, then one more KM step from the L2O candidate to form the fixed-point
// residual S (test_syn_l1l1_scalar.py:160-178); those three steps are 1-layer calls of the fused
// forward kernel.  This kernel does the rest.  A workgroup owns 16 batch columns and splits
// their rows over 16 row lanes (256 threads; a wave covers 16 columns x 4 rows, 64-B segments):
// each lane sums every 16th row of its column, the 16 partial sums are added in lane order (a
// fixed order: deterministic), one lane per column decides, and all 256 threads copy the chosen
// candidate.  (Round 6: one thread per column walked all rows alone -- 494 us per call at
// B = 1,000, half of the LSKM forward's GPU time; tools/prof_lskm.py.)
//   |S|   = sqrt( sum_i (beta Ts_i)^2 + (c ((Es_i - 2 El_i) + Ep_i))^2 )      (:173-175, :124-126)
//   keep  = |S| < (1 - delta) mu                                            (:232)
//   mu    = updater(|S|, keep)                                              (mu_updater.py)
//   out   = keep ? L2O candidate : KM candidate   for Z, E, L, T            (:251-259)
//   count += !keep                                                          (:283)
// The norm is accumulated in fp64 (the reference's fp32 reduction order is torch's own).
#include "dladmm_common.h"

namespace dladmm {

struct SafeguardArgs {
  int m, n, B;
  int64_t ld;  // common row stride of every matrix
  const float *Zl, *El, *Ll, *Tl;   // L2O candidate
  const float *Zk, *Ek, *Lk, *Tk;   // KM candidate
  const float *Es, *Ts;             // KM step from the L2O candidate
  const float* Ep;                  // E of the state both steps started from
  float *Zo, *Eo, *Lo, *To;         // selected outputs
  float* mu;                        // [B] in/out
  float* norm_out;                  // [B] |S| (optional)
  int* count;                       // number of safeguarded columns (atomic, integer)
  float beta, c, thresh;            // thresh = 1 - delta
  int updater;                      // enum dladmm_mu_updater
  float param;
};

constexpr int kSgCols = 16, kSgRows = 16;  // columns x row lanes of a workgroup (256 threads)

__global__ __launch_bounds__(256) void safeguard_kernel(const SafeguardArgs a) {
  __shared__ double part[kSgRows][kSgCols];
  __shared__ int keep_s[kSgCols];
  const int tc = threadIdx.x % kSgCols, tr = threadIdx.x / kSgCols;
  const int64_t col = (int64_t)blockIdx.x * kSgCols + tc;
  const bool cv = col < a.B;
  double s = 0.0;
  if (cv) {
    for (int i = tr; i < a.m; i += kSgRows) {
      const int64_t o = (int64_t)i * a.ld + col;
      const float t = a.beta * a.Ts[o];
      const float e = a.c * ((a.Es[o] - 2.0f * a.El[o]) + a.Ep[o]);
      s += (double)t * t + (double)e * e;
    }
  }
  part[tr][tc] = s;
  __syncthreads();
  int flag = 0;
  if (tr == 0) {
    double t = 0.0;
    for (int j = 0; j < kSgRows; ++j) t += part[j][tc];
    bool keep = false;
    if (cv) {
      const float nrm = (float)sqrt(t);
      const float mu0 = a.mu[col];
      keep = nrm < a.thresh * mu0;
      float mu1 = mu0;
      switch (a.updater) {
        case DLADMM_MU_EMA: mu1 = keep ? a.param * nrm + (1.0f - a.param) * mu0 : mu0; break;
        case DLADMM_MU_GS: mu1 = keep ? (1.0f - a.param) * mu0 : mu0; break;
        case DLADMM_MU_RT: mu1 = keep ? nrm : mu0; break;
        default: mu1 = 1e10f; break;  // BlankUpdater.step returns 10**10 (mu_updater.py:108-110)
      }
      if (a.norm_out) a.norm_out[col] = nrm;
      // initialisation (no outputs): mu_0 = |S_0| (test_syn_l1l1_scalar.py:190-197)
      a.mu[col] = a.Zo ? mu1 : nrm;
      flag = keep ? 0 : 1;
    }
    keep_s[tc] = keep ? 1 : 0;
  }
  if (!a.Zo) return;  // whole-grid uniform
  __syncthreads();
  // one atomic per workgroup (integer: order-independent); the deciding lanes are wave 0's
  // first 16 threads
  const unsigned long long bal = __ballot(flag);
  if (threadIdx.x == 0 && bal) atomicAdd(a.count, (int)__popcll(bal));
  if (!cv) return;
  const bool keep = keep_s[tc] != 0;
  const float* zs = keep ? a.Zl : a.Zk;
  const float* es = keep ? a.El : a.Ek;
  const float* ls = keep ? a.Ll : a.Lk;
  const float* ts = keep ? a.Tl : a.Tk;
  for (int i = tr; i < a.n; i += kSgRows) {
    const int64_t o = (int64_t)i * a.ld + col;
    a.Zo[o] = zs[o];
  }
  for (int i = tr; i < a.m; i += kSgRows) {
    const int64_t o = (int64_t)i * a.ld + col;
    a.Eo[o] = es[o];
    a.Lo[o] = ls[o];
    a.To[o] = ts[o];
  }
}

}  // namespace dladmm

extern "C" int dladmm_safeguard_f32(const dladmm_safeguard_desc* d, void* stream) {
  using namespace dladmm;
  if (!d) return DLADMM_E_NULL;
  if (d->abi_version != DLADMM_ABI_VERSION) return DLADMM_E_ABI_VERSION;
  if (d->m < 1 || d->n < 1 || d->batch < 1 || d->ld < d->batch) return DLADMM_E_SHAPE;
  if (d->updater < DLADMM_MU_NONE || d->updater > DLADMM_MU_RT) return DLADMM_E_UNSUPPORTED;
  const void* req[] = {d->El, d->Es, d->Ts, d->Ep, d->mu};
  for (const void* p : req)
    if (!p) return DLADMM_E_NULL;
  if (d->Zo) {  // select mode (otherwise: mu = |S| only)
    const void* sel[] = {d->Zl, d->Ll, d->Tl, d->Zk, d->Ek, d->Lk, d->Tk, d->Eo, d->Lo, d->To,
                         d->count};
    for (const void* p : sel)
      if (!p) return DLADMM_E_NULL;
  }
  SafeguardArgs a{};
  a.m = d->m; a.n = d->n; a.B = d->batch; a.ld = d->ld;
  a.Zl = d->Zl; a.El = d->El; a.Ll = d->Ll; a.Tl = d->Tl;
  a.Zk = d->Zk; a.Ek = d->Ek; a.Lk = d->Lk; a.Tk = d->Tk;
  a.Es = d->Es; a.Ts = d->Ts; a.Ep = d->Ep;
  a.Zo = d->Zo; a.Eo = d->Eo; a.Lo = d->Lo; a.To = d->To;
  a.mu = d->mu; a.norm_out = d->norm_out; a.count = d->count;
  a.beta = d->beta; a.c = d->c; a.thresh = (float)(1.0 - d->delta);  // python (1.0-delta)
  a.updater = d->updater; a.param = d->mu_param;
  hipLaunchKernelGGL(safeguard_kernel, dim3((unsigned)((d->batch + kSgCols - 1) / kSgCols)),
                     dim3(256), 0,
                     (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
