// bf16_tile256.hip -- probe for VERDICT r05 item 3 (BASELINE config 5): a 256 x 256 output tile
// per workgroup whose main loop runs at ONE wave per SIMD -- 4 waves of 128 x 128 (64 f32x4
// accumulators = 256 AGPRs each), the fragments of k-block kb + 1 read from LDS into a second
// register set while the 64 MFMAs of k-block kb run, the operands LDS-DMA'd through a 4-stage
// ring (32 KiB per stage: 16 A + 16 B fragments of 1 KiB, the product's packed fragment
// layout).  No epilogue: it times the main loop the product would need for the
// "larger tiles, one wave per SIMD" lever of DESIGN.md section 12 and shows where it stops.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/probe/bf16_tile256.hip \
//         -o tools/probe/bf16_tile256
//   tools/probe/bf16_tile256            # correctness at 512 x 512 x 256, then the two config-5
//                                       # products: G1 4096 x 16384 x 1024, G2 1024 x 16384 x 4096
//
// Output (one JSON line per shape): us per GEMM (median of 20 after 5 warmup launches), TF/s,
// fraction of the 2.5 PF/s dense bf16 peak.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int kNST = 4;   // ring stages (4 x 32 KiB)
constexpr int kSF = 32;   // fragments per stage: 16 A row blocks + 16 B column blocks
constexpr int kPW = 8;    // DMA pieces per wave per stage

__device__ __forceinline__ void glds16(const void* sbase, uint32_t voff, const void* ldst) {
  unsigned keep;
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ldst);
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(dst)
      : "memory");
}

struct Args {
  const char* A;  // packed [KB][MB16] fragments of 1 KiB (lane l: row l & 15, k 8 (l >> 4) ..)
  const char* B;  // packed [KB][NB16] fragments (lane l: column l & 15, k 8 (l >> 4) ..)
  float* C;       // M x N fp32 (store mode) or null
  int M, N, KB;
  int store;
};

// Workgroup = 4 waves (2 x 2) of 128 x 128.  blockIdx -> tile: consecutive workgroups go to the
// 8 XCDs round-robin; tile = xcd-major so that one XCD's workgroups walk the row tiles of a few
// column strips (their B strip stays in that XCD's L2).
template <bool STORE>
__global__ __launch_bounds__(256, 1) void tile256(const Args a) {
  __shared__ f32x4 ring[kNST * kSF * 64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int mt = a.M / 256, nt = a.N / 256, ntile = mt * nt;
  const int L = blockIdx.x;
  const int per = ntile / 8;
  const int t = (L % 8) * per + L / 8;
  const int ti = t % mt, tj = t / mt;
  const int MB16 = a.M / 16, NB16 = a.N / 16;
  const int KB = a.KB;

  // wave w DMAs stage fragments f = 8 w .. 8 w + 7: waves 0, 1 the 16 A row blocks, waves 2, 3
  // the 16 B column blocks (a wave-uniform base and k-block stride, no per-piece select)
  const char* dbase = w < 2 ? a.A + ((int64_t)ti * 16 + 8 * w) * 1024
                            : a.B + ((int64_t)tj * 16 + 8 * (w - 2)) * 1024;
  const int64_t kstride = (int64_t)(w < 2 ? MB16 : NB16) * 1024;
  auto issue1 = [&](int kb, int slot, int q) {
    glds16(dbase + kb * kstride + q * 1024, lane * 16, ring + (slot * kSF + 8 * w + q) * 64);
  };
  auto issue = [&](int kb, int slot) {
#pragma unroll
    for (int q = 0; q < kPW; ++q) issue1(kb, slot, q);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: stages 0 .. NST-1 issued (past the end: k-block 0 again, never consumed)
#pragma unroll
  for (int st = 0; st < kNST; ++st) issue(st < KB ? st : 0, st);
  bf16x8 fa[2][8], fb[2][8];
  // stage 0 landed (the NST - 1 younger stages may be in flight)
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(kPW * (kNST - 1)) : "memory");
  {
    const bf16x8* st = reinterpret_cast<const bf16x8*>(ring);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[0][i] = st[(8 * wr + i) * 64 + lane];
#pragma unroll
    for (int j = 0; j < 8; ++j) fb[0][j] = st[(16 + 8 * wc + j) * 64 + lane];
  }
  // iteration kb: registers hold k-block kb (set c); stage kb + 1 must have landed for every
  // wave, and every wave has read stage kb out of the ring (its slot then takes kb + NST).
  // While the 64 MFMAs of kb run: 16 fragment reads of kb + 1 (one per 4 MFMAs) and this wave's
  // 8 DMA pieces of kb + NST (one per 8 MFMAs).
  // one body per k-block: the next k-block's fragments land in (fa[1], fb[1]) and are copied
  // into set 0 at the end of the iteration (loop-carried registers stay fixed)
  for (int kb = 0; kb < KB; ++kb) {
    // stage kb + 1 landed: the younger NST - 2 stages' pieces may stay in flight
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(kPW * (kNST - 2)) : "memory");
    const int nk = kb + kNST < KB ? kb + kNST : 0;
    const int slot = kb % kNST, nslot = (kb + 1) % kNST;
    const bf16x8* st = reinterpret_cast<const bf16x8*>(ring + nslot * kSF * 64);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int j = 4 * h; j < 4 * h + 4; ++j) acc[i][j] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0][i], fb[0][j], acc[i][j], 0, 0, 0);
        const int r = 2 * i + h;  // read r of 16: A fragments first, then B
        __builtin_amdgcn_sched_barrier(0);
        // (the last k-block reads a slot it never uses: in range, harmless, branch-free)
        if (r < 8) fa[1][r] = st[(8 * wr + r) * 64 + lane];
        else fb[1][r - 8] = st[(16 + 8 * wc + r - 8) * 64 + lane];
        if (h == 1) issue1(nk, slot, i);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      fa[0][i] = fa[1][i];
      fb[0][i] = fb[1][i];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if constexpr (STORE) {
    // lane: column l & 15 of block j, rows 4 (l >> 4) + q of block i
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = ti * 256 + wr * 128 + 16 * i + 4 * (lane >> 4) + q;
          const int col = tj * 256 + wc * 128 + 16 * j + (lane & 15);
          a.C[(int64_t)row * a.N + col] = acc[i][j][q];
        }
  } else {
    float s = 0.f;  // keep every accumulator live
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (s == 1234.5f) a.C[0] = s;
  }
}

static uint16_t f2bf(float x) {  // RNE
  uint32_t u;
  memcpy(&u, &x, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float x;
  memcpy(&x, &u, 4);
  return x;
}

// pack a rows x K row-major bf16 matrix into [K/32][rows/16] fragments
static void pack(const std::vector<uint16_t>& m, int rows, int K, std::vector<uint16_t>& out) {
  out.assign((size_t)rows * K, 0);
  const int RB = rows / 16;
  for (int kb = 0; kb < K / 32; ++kb)
    for (int rb = 0; rb < RB; ++rb)
      for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 8; ++e) {
          const size_t o = (((size_t)kb * RB + rb) * 64 + l) * 8 + e;
          out[o] = m[(size_t)(16 * rb + (l & 15)) * K + 32 * kb + 8 * (l >> 4) + e];
        }
}

static double run(int M, int N, int K, bool check) {
  std::vector<uint16_t> A((size_t)M * K), Bt((size_t)N * K), Ap, Bp;
  uint32_t s = 12345u;
  auto rnd = [&]() {
    s = s * 1664525u + 1013904223u;
    return ((s >> 8) & 0xffff) / 65536.0f - 0.5f;
  };
  for (auto& x : A) x = f2bf(rnd());
  for (auto& x : Bt) x = f2bf(rnd());
  pack(A, M, K, Ap);
  pack(Bt, N, K, Bp);
  char *dA, *dB;
  float* dC;
  CHECK(hipMalloc(&dA, Ap.size() * 2));
  CHECK(hipMalloc(&dB, Bp.size() * 2));
  CHECK(hipMalloc(&dC, (size_t)M * N * 4));
  CHECK(hipMemcpy(dA, Ap.data(), Ap.size() * 2, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dB, Bp.data(), Bp.size() * 2, hipMemcpyHostToDevice));
  Args a{dA, dB, dC, M, N, K / 32, check ? 1 : 0};
  const int grid = (M / 256) * (N / 256);
  if (grid % 8) { fprintf(stderr, "tile count must be a multiple of 8\n"); exit(1); }
  if (check) {
    hipLaunchKernelGGL(tile256<true>, dim3(grid), dim3(256), 0, 0, a);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    std::vector<float> C((size_t)M * N);
    CHECK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
    double maxe = 0, maxr = 0;
    for (int i = 0; i < M; ++i)
      for (int j = 0; j < N; ++j) {
        double r = 0;
        for (int k = 0; k < K; ++k) r += (double)bf2f(A[(size_t)i * K + k]) * bf2f(Bt[(size_t)j * K + k]);
        maxe = std::max(maxe, std::fabs(r - C[(size_t)i * N + j]));
        maxr = std::max(maxr, std::fabs(r));
      }
    printf("{\"check\": \"%dx%dx%d\", \"max_abs_err\": %.3e, \"max_abs\": %.3e}\n", M, N, K, maxe,
           maxr);
    CHECK(hipFree(dA)); CHECK(hipFree(dB)); CHECK(hipFree(dC));
    return maxe / maxr;
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int it = 0; it < 25; ++it) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(tile256<false>, dim3(grid), dim3(256), 0, 0, a);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (it >= 5) ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  const double us = 1e3 * ts[ts.size() / 2];
  const double tf = 2.0 * M * N * (double)K / (us * 1e-6) / 1e12;
  printf("{\"shape\": \"%dx%dx%d\", \"grid\": %d, \"us_median\": %.1f, \"us_min\": %.1f, "
         "\"tflops\": %.1f, \"frac_bf16_2.5PF\": %.3f}\n",
         M, N, K, grid, us, 1e3 * ts[0], tf, tf / 2500.0);
  CHECK(hipFree(dA)); CHECK(hipFree(dB)); CHECK(hipFree(dC));
  return us;
}

int main() {
  const double rel = run(512, 1024, 256, true);
  if (!(rel < 1e-3)) { fprintf(stderr, "probe: wrong result (rel %.3e)\n", rel); return 1; }
  run(4096, 16384, 1024, false);   // config 5 G1: W_k (n x m) . Var_k (m x B)
  run(1024, 16384, 4096, false);   // config 5 G2: A (m x n) . Z_k (n x B)
  return 0;
}
