// dladmm_tile_bf16_queue.hip -- the bf16 mode's forward (BASELINE config 5) as ONE persistent
// launch: workgroups pull tile units (phase, column tile, row tile) from work queues in dependency
// order, so that at any time some CUs run main loops (MFMA, L2 -> LDS operand stream) while
// others run epilogues (HBM), instead of every CU passing through the two in the same phase, as
// the one-launch-per-product sequence does.
//
// Units and dependencies.  Phase q: 0 = prologue (T_0, Var_0), 2k+1 = G1(k), 2k+2 = G2(k); a
// unit is one 256 x 256 output tile of its phase, the wide tile body of the one-phase kernel
// (dladmm_tile_bf16_body.h, 8 waves, 128 KiB ring, one workgroup per CU), so every element is the
// same chain and the outputs are bit-identical to it.  Unit (q, c, r) reads what phase q - 1
// wrote for column tile c (all its row tiles: the packed B operand spans the contraction) and
// nothing of another column; the buffers a later phase rewrites (packed Var / Z, the lean-mode
// state) were last read by units this one transitively waits for.  So a unit waits for exactly
// one count, done[q - 1][c] = rows(q - 1).
//
// Queues.  Column tile c belongs to queue c % 8; a workgroup serves the queue of its own XCD
// first (HW_REG_XCC_ID: a column's state and packed operands then stay in one L2; speed only),
// then helps the others.  A queue's tickets run along diagonals: step t holds, for each lag class
// l (columns (c / 8) % lags == l), the units of phase t - l -- G1 and G2 units interleaved, so
// the workgroups drift out of phase.  A ticket's dependencies have smaller tickets of the same
// queue, claimed by running workgroups, so the schedule cannot deadlock whatever the residency;
// every wait is bounded anyway (err word, results then invalid).
//
// Hand-off (cdna_hip_programming.md section 6, Guideline 16): the producing workgroup's waves
// drain their stores, barrier, one lane releases at agent scope and adds to the count; the
// consumer polls it with sc1 loads, acquires at agent scope, waits, barriers, then loads.
#include "dladmm_queue.h"
#include "dladmm_tile_bf16_body.h"

#ifndef DLADMM_QUEUE_EXP
#define DLADMM_QUEUE_EXP 0  // timing experiments (results may be WRONG): 1 no acquire / release
                            // fences, 2 no dependency waits
#endif

namespace dladmm {

namespace {

constexpr int kLaChunk = 12;
struct LayerChunk {
  LayerArgs a[kLaChunk];
  LayerArgs* dst;
  int n;
};
static_assert(sizeof(LayerChunk) <= 4000, "kernel argument limit");

__global__ __launch_bounds__(64) void layer_table_kernel(const LayerChunk c) {
  // one dword per lane at a time: the table is read by scalar loads of the queue kernel
  const int words = (int)(sizeof(LayerArgs) / 4);
  for (int i = 0; i < c.n; ++i) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(&c.a[i]);
    uint32_t* d = reinterpret_cast<uint32_t*>(c.dst + i);
    for (int w = threadIdx.x; w < words; w += 64) d[w] = s[w];
  }
}

constexpr int kSpinLimit = 1 << 20;  // polls of one dependency (~1 s) before giving up

__device__ __forceinline__ int q_rows(const QueueArgs& qa, int q) {
  return q == 0 ? qa.rows2 : ((q & 1) ? qa.rows1 : qa.rows2);
}

template <int EMODE, int PKIND>
__global__ __launch_bounds__(512, 1) void tile_bf16_queue_kernel(const QueueArgs qa) {
  using G = TileG<8>;
  __shared__ f32x4 ring[G::NST * G::SF * 64];
  __shared__ int sh_ticket;
  static_assert(sizeof(LayerArgs) % 4 == 0, "table words");

  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const int nph = qa.nph, gx = qa.gx, lags = qa.lags;
  const int last_step = nph + lags - 1;  // steps 0 .. last_step - 1

  for (int qi = 0; qi < 8; ++qi) {
    const int x = (int)((xcc + qi) & 7);
    const int ncx = x < gx ? (gx - x + 7) / 8 : 0;  // column tiles of queue x
    if (ncx == 0) continue;
    // columns of lag class l in queue x
    auto n_l = [&](int l) { return l < ncx ? (ncx - l + lags - 1) / lags : 0; };
    auto step_units = [&](int t) {
      int u = 0;
      for (int l = 0; l < lags; ++l) {
        const int q = t - l;
        if (q >= 0 && q < nph) u += n_l(l) * q_rows(qa, q);
      }
      return u;
    };
    int t = 0, base = 0, tsz = step_units(0);  // this workgroup's cursor in queue x
    for (;;) {
      if (threadIdx.x == 0) sh_ticket = atomicAdd(&qa.tickets[32 * x], 1);
      __syncthreads();
      const int T = __builtin_amdgcn_readfirstlane(sh_ticket);
      __syncthreads();  // every wave has read the ticket before the next one overwrites it
      while (t < last_step && T >= base + tsz) {
        base += tsz;
        ++t;
        tsz = t < last_step ? step_units(t) : 0;
      }
      if (t >= last_step) break;  // queue x is exhausted
      int rem = T - base, q = 0, c = 0, r = 0;
      for (int l = 0; l < lags; ++l) {
        const int ql = t - l;
        const int sz = (ql >= 0 && ql < nph) ? n_l(l) * q_rows(qa, ql) : 0;
        if (rem < sz) {
          const int rows = q_rows(qa, ql);
          q = ql;
          c = 8 * (l + lags * (rem / rows)) + x;
          r = rem % rows;
          break;
        }
        rem -= sz;
      }
      q = __builtin_amdgcn_readfirstlane(q);
      c = __builtin_amdgcn_readfirstlane(c);
      r = __builtin_amdgcn_readfirstlane(r);
      // wait for phase q - 1 of column tile c, then acquire its writes
      if (q > 0 && threadIdx.x == 0 && !(DLADMM_QUEUE_EXP & 2)) {
        const int need = q_rows(qa, q - 1);
        int* cnt = qa.done + (int64_t)(q - 1) * gx + c;
        int it = 0;
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
          __builtin_amdgcn_s_sleep(4);
          if ((++it & 255) == 0 &&
              (it >= kSpinLimit ||
               __hip_atomic_load(qa.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            __hip_atomic_store(qa.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
        if (!(DLADMM_QUEUE_EXP & 1)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      // the phase's arguments through the constant address space: scalar loads (a generic read
      // would be vector loads, whose waits drain the ring's DMA)
      typedef const uint32_t __attribute__((address_space(4)))* cword_t;
      LayerArgs a;
      {
        const cword_t src = (cword_t)(qa.ph + q);
        uint32_t* dst = reinterpret_cast<uint32_t*>(&a);
#pragma unroll
        for (int i = 0; i < (int)(sizeof(LayerArgs) / 4); ++i) dst[i] = src[i];
      }
      const int ph = q == 0 ? 2 : ((q & 1) ? 0 : 1);
      if (ph == 0) tile_body<EMODE, PKIND, 0, 8>(a, ring, c, r);
      else if (ph == 1) tile_body<EMODE, PKIND, 1, 8>(a, ring, c, r);
      else tile_body<EMODE, PKIND, 2, 8>(a, ring, c, r);
      // release: every wave's stores drained, then one lane publishes the unit
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        if (!(DLADMM_QUEUE_EXP & 1)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(qa.done + (int64_t)q * gx + c, 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// a timed-out dependency wait (err set) poisons the results instead of passing silently: the
// first element of the last layer's Z and every (layer, term) row of the loss partials
__global__ __launch_bounds__(64) void queue_err_kernel(const int* err, float* z, float* lossp,
                                                       int rows, int64_t stride) {
  if (*err == 0) return;
  const float nan = __builtin_nanf("");
  if (threadIdx.x == 0 && z) z[0] = nan;
  if (lossp)
    for (int i = threadIdx.x; i < rows; i += 64) lossp[(int64_t)i * stride] = nan;
}

template <int EMODE, int PKIND>
hipError_t launch_q(const QueueArgs& q, int grid, hipStream_t s) {
  hipLaunchKernelGGL((tile_bf16_queue_kernel<EMODE, PKIND>), dim3(grid), dim3(512), 0, s, q);
  return hipGetLastError();
}

}  // namespace

hipError_t write_layer_table(const LayerArgs* host, int n, LayerArgs* dst, hipStream_t s) {
  for (int b = 0; b < n; b += kLaChunk) {
    LayerChunk c{};
    c.n = n - b < kLaChunk ? n - b : kLaChunk;
    for (int i = 0; i < c.n; ++i) c.a[i] = host[b + i];
    c.dst = dst + b;
    hipLaunchKernelGGL(layer_table_kernel, dim3(1), dim3(64), 0, s, c);
    if (hipError_t e = hipGetLastError()) return e;
  }
  return hipSuccess;
}

hipError_t launch_queue_check(const QueueArgs& q, float* z_last, float* lossp, int rows,
                              int64_t stride, hipStream_t s) {
  hipLaunchKernelGGL(queue_err_kernel, dim3(1), dim3(64), 0, s, (const int*)q.err, z_last, lossp,
                     rows, stride);
  return hipGetLastError();
}

hipError_t launch_tile_bf16_queue(int variant, const QueueArgs& q, int grid, hipStream_t s) {
  switch (variant) {
    case DLADMM_V1_LENA: return launch_q<EM_V1, PK_ELEM>(q, grid, s);
    case DLADMM_V2_LTHETA: return launch_q<EM_V1, PK_ROW>(q, grid, s);
    case DLADMM_V3_FULL: return launch_q<EM_VVAR, PK_ROW>(q, grid, s);
    case DLADMM_V4_SCALAR:
    case DLADMM_V5_TIED: return launch_q<EM_VVAR, PK_SCALAR>(q, grid, s);
    case DLADMM_V6_LASSO: return launch_q<EM_LASSO, PK_SCALAR>(q, grid, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace dladmm
