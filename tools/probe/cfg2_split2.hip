// Probe (timing only, results meaningless), second form: the row-split skeleton for BASELINE
// config 2 (V4, m=256 n=512 K=15, B = 10,000) with the weight stream the real kernel would use.
// cfg2_split.hip streamed each wave's fragments into registers 8 ahead, which is latency-bound
// on its own; here every wave streams ITS quarter of each weight by LDS-DMA into a private ring
// (4-KiB chunks = 2 MFMA steps, SLOTS chunks, SLOTS - 1 in flight; a wave only reads what it
// DMA'd itself, so the ring needs vmcnt waits, no workgroup barrier), and the B operands come
// from the workgroup's LDS exchange images (Z: 32 KB, Var: 16 KB), two barriers per layer:
//   G1: wave w = output blocks 8w..8w+7 of Z (4 pairs) x 16 Var blocks: 128 fragments
//   G2: wave w = output blocks 4w..4w+3 of P (2 pairs) x 32 Z blocks:   128 fragments
// STORES adds the per-element output stores of the real kernel (Z rows after G1, E / L / T
// rows after G2: one dword per lane and row, 64-B row segments) to a scratch buffer.
// Prints per-variant kernel milliseconds (median of 7) as one JSON line.
//   hipcc -O3 --offload-arch=gfx950 -I d-ladmm_amd/csrc tools/probe/cfg2_split2.hip \
//         -o tools/probe/cfg2_split2
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#include "dladmm_common.h"

using namespace dladmm;

constexpr int kLayerFloats = 2 * 128 * 1024;  // W_k and A, 512 KiB each (1,024 fragments total)

template <int SLOTS, int OCC, bool STORES>
__global__ __launch_bounds__(256, OCC) void split2(const float* __restrict__ W, int layers, int B,
                                                   float* __restrict__ out) {
  __shared__ f32x4 ring[4 * SLOTS * 4 * 64];
  __shared__ f32x4 zimg[32 * 64];
  __shared__ f32x4 vimg[16 * 64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  for (int i = threadIdx.x; i < 32 * 64; i += 256) zimg[i] = f32x4{1e-3f, 0.5f, 0.25f, 0.125f};
  for (int i = threadIdx.x; i < 16 * 64; i += 256) vimg[i] = f32x4{1e-3f, 0.5f, 0.25f, 0.125f};
  __syncthreads();
  f32x4* my = ring + w * SLOTS * 4 * 64;
  const int64_t col = (int64_t)blockIdx.x * 16 + (lane & 15);
  const uint32_t vo = col < B ? (uint32_t)((col + (int64_t)(4 * g) * B) * 4) : kOOB;
  const rsrc_t ro = mkrsrc(out, (uint32_t)(512 * (int64_t)B * 4));
  float sink = 0.f;

  // one GEMM pass: NS = 64 steps over this wave's 128 fragments (src: 128 KiB contiguous);
  // NK contraction blocks per pair, B operand blocks from img
  auto pass = [&](const float* src, const f32x4* img, int NK, f32x4* dst, int dst0) {
#pragma unroll
    for (int c = 0; c < SLOTS - 1; ++c) glds16x4(src + c * 4 * kFrag, lane * 16, my + c * 256);
    f32x4 ca = {0.f, 0.f, 0.f, 0.f}, cb = ca;
    int pr = 0;
#pragma unroll 1
    for (int c = 0; c < 32; ++c) {  // chunk c = steps 2c, 2c+1
      // chunk c landed (the SLOTS - 2 newer chunks stay in flight); slot of chunk c-1 is free
      if (c + SLOTS - 1 <= 32 + SLOTS - 2) {
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(4 * (SLOTS - 2)) : "memory");
      }
      if (c + SLOTS - 1 < 32)
        glds16x4(src + (c + SLOTS - 1) * 4 * kFrag, lane * 16, my + ((c + SLOTS - 1) % SLOTS) * 256);
      else  // keep the count: a DMA of the chunk again (harmless, same data)
        glds16x4(src + c * 4 * kFrag, lane * 16, my + ((c + SLOTS - 1) % SLOTS) * 256);
      const f32x4* sl = my + (c % SLOTS) * 256;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int s = 2 * c + h;
        const int kb = s % NK;
        const f32x4 wa = sl[(2 * h) * 64 + lane], wb = sl[(2 * h + 1) * 64 + lane];
        const f32x4 bv = img[kb * 64 + lane];
        ca = mfma4(wa.x, bv.x, ca);
        cb = mfma4(wb.x, bv.x, cb);
        ca = mfma4(wa.y, bv.y, ca);
        cb = mfma4(wb.y, bv.y, cb);
        ca = mfma4(wa.z, bv.z, ca);
        cb = mfma4(wb.z, bv.z, cb);
        ca = mfma4(wa.w, bv.w, ca);
        cb = mfma4(wb.w, bv.w, cb);
        if (kb == NK - 1) {  // pair done: its two blocks go to the exchange image (+ stores)
          dst[(dst0 + 2 * pr) * 64 + lane] = ca;
          dst[(dst0 + 2 * pr + 1) * 64 + lane] = cb;
          if constexpr (STORES) {
            const int nst = dst == zimg ? 1 : 3;  // Z; or E, L, T
#pragma unroll
            for (int r = 0; r < 4; ++r)
              for (int q = 0; q < nst; ++q) {
                const uint32_t so = (uint32_t)(((dst0 + 2 * pr) * 16 + r + 128 * q) * (int64_t)B * 4);
                bstore_s(ro, vo, so, ca[r]);
                bstore_s(ro, vo, so + 16 * B * 4, cb[r]);
              }
          }
          sink += ca.x + cb.y;
          ca = f32x4{0.f, 0.f, 0.f, 0.f};
          cb = ca;
          ++pr;
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  };
  for (int k = 0; k < layers; ++k) {
    const float* lw = W + (int64_t)k * kLayerFloats;
    pass(lw + w * 128 * kFrag, vimg, 16, zimg, 8 * w);                        // G1
    __syncthreads();
    pass(lw + 128 * 1024 + w * 128 * kFrag, zimg, 32, vimg, 4 * w);           // G2
    __syncthreads();
  }
  if (sink == 12345.f) out[threadIdx.x] = sink;
}

template <int SLOTS, int OCC, bool STORES>
float run(const float* W, int grid, int layers, int B, float* out, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((split2<SLOTS, OCC, STORES>), dim3(grid), dim3(256), 0, 0, W, layers, B, out);
  hipDeviceSynchronize();
  std::vector<float> t;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(a);
    hipLaunchKernelGGL((split2<SLOTS, OCC, STORES>), dim3(grid), dim3(256), 0, 0, W, layers, B, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  const int layers = 15, reps = 7, B = 10000, grid = (B + 15) / 16;
  float* W;
  float* out;
  hipMalloc(&W, (size_t)layers * kLayerFloats * 4);
  hipMalloc(&out, (size_t)512 * B * 4);
  hipMemset(W, 0x3c, (size_t)layers * kLayerFloats * 4);
  const float s4 = run<4, 1, false>(W, grid, layers, B, out, reps);
  const float s6 = run<6, 1, false>(W, grid, layers, B, out, reps);
  const float s2o2 = run<2, 2, false>(W, grid, layers, B, out, reps);
  const float s4st = run<4, 1, true>(W, grid, layers, B, out, reps);
  const float s6st = run<6, 1, true>(W, grid, layers, B, out, reps);
  const double flop = 2.0 * 2 * 256 * 512 * (double)B * layers;
  printf("{\"slots4_ms\": %.4f, \"slots6_ms\": %.4f, \"slots2_two_per_cu_ms\": %.4f, "
         "\"slots4_stores_ms\": %.4f, \"slots6_stores_ms\": %.4f, \"fused_kernel_ms_ref\": 1.046, "
         "\"best_frac_of_157TF\": %.3f}\n",
         s4, s6, s2o2, s4st, s6st,
         flop / (std::min(std::min(s4, s6), s2o2) * 1e-3) / 157.3e12);
  return 0;
}
