// Probe (timing only, results meaningless): can BASELINE config 2 (V4, m=256 n=512 K=15,
// B = 10,000) beat the fused kernel's one-workgroup-per-CU shape by splitting each 16-column
// group's rows over the four waves of a workgroup?  DESIGN.md section 12 argued it on paper;
// this measures the two skeletons the argument compares, MFMAs + weight streaming + the
// exchange barriers, no epilogue:
//   shared: 157 workgroups x 4 waves, a wave = 16 columns x ALL rows: 4,096 v_mfma_f32_16x16x4
//           per layer, every wave reading all 1,024 weight fragments (1 MB per layer; the four
//           waves read the same ones, so the CU fetches them once)  -- today's fused kernel
//   split:  625 workgroups x 4 waves, a wave = 16 columns x a quarter of the rows: 1,024 MFMAs
//           per layer on ITS OWN 256 fragments (the workgroup still streams 1 MB per layer);
//           B operands from LDS (48 KB per workgroup, the Z / Var exchange image), two
//           workgroup barriers per layer; at most three workgroups per CU
// Fragments go straight to registers, D ahead.  Prints per-layer microseconds of each.
//   hipcc -O3 --offload-arch=gfx950 tools/probe/cfg2_split.hip -o tools/probe/cfg2_split
#include <hip/hip_runtime.h>
#include <cstdio>
#include <algorithm>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NFRAG, bool SPLIT>
__global__ __launch_bounds__(256, SPLIT ? 3 : 1) void probe(const f32x4* __restrict__ W,
                                                            int layers, float* out) {
  constexpr int D = 8;                     // fragments in flight per wave
  __shared__ f32x4 bimg[SPLIT ? 3072 : 64];  // 48 KB exchange image (split), else a token
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < (SPLIT ? 3072 : 64); i += 256)
    bimg[i] = f32x4{1e-3f * i, 0.5f, 0.25f, 0.125f};
  __syncthreads();
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  f32x4 breg = bimg[lane];
  for (int k = 0; k < layers; ++k) {
    // split: wave w streams its own quarter; shared: every wave streams the whole layer
    const f32x4* src = W + ((size_t)k * (SPLIT ? 4 : 1) + (SPLIT ? w : 0)) * NFRAG * 64 + lane;
    f32x4 f[D];
#pragma unroll
    for (int d = 0; d < D; ++d) f[d] = __builtin_nontemporal_load(src + d * 64);
#pragma unroll 1
    for (int i0 = 0; i0 < NFRAG; i0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const f32x4 cur = f[d];
        if (i0 + d + D < NFRAG) f[d] = src[(i0 + d + D) * 64];
        if constexpr (SPLIT) breg = bimg[((i0 + d) & 31) * 64 + lane];  // B from the LDS image
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.x, breg.x, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.y, breg.y, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.z, breg.z, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.w, breg.w, acc1, 0, 0, 0);
      }
    }
    if constexpr (SPLIT) {  // the two exchange points of a layer (Z after G1, Var after G2)
      __syncthreads();
      __syncthreads();
    }
  }
  const f32x4 s = acc0 + acc1;
  if (s.x + s.y + s.z + s.w == 12345.f) out[threadIdx.x] = s.x;
}

template <int NFRAG, bool SPLIT>
float run(const f32x4* W, int grid, int layers, float* out, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((probe<NFRAG, SPLIT>), dim3(grid), dim3(256), 0, 0, W, layers, out);
  hipDeviceSynchronize();
  std::vector<float> t;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(a);
    hipLaunchKernelGGL((probe<NFRAG, SPLIT>), dim3(grid), dim3(256), 0, 0, W, layers, out);
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
  const int layers = 15, reps = 7;
  // 1 MB of fp32 fragments per layer (W_k and A of 256 x 512), layers of them
  const size_t nf4 = (size_t)layers * 1024 * 64;
  f32x4* W;
  float* out;
  hipMalloc(&W, nf4 * sizeof(f32x4));
  hipMalloc(&out, 4096);
  hipMemset(W, 0x3c, nf4 * sizeof(f32x4));  // nonzero operands (clock under load)
  const float ts = run<1024, false>(W, 157, layers, out, reps);
  const float t1 = run<256, true>(W, 256, layers, out, reps);   // one split workgroup per CU
  const float tp = run<256, true>(W, 625, layers, out, reps);   // config 2's 625 groups
  const double flop = 2.0 * 2 * 256 * 512 * 10000.0 * layers;   // the 2 K products
  printf("{\"shared_157wg_ms\": %.4f, \"shared_us_per_layer\": %.2f, "
         "\"split_256wg_ms\": %.4f, \"split_625wg_ms\": %.4f, \"split_us_per_layer\": %.2f, "
         "\"split_over_shared\": %.3f, \"shared_frac_of_157TF\": %.3f, "
         "\"split_frac_of_157TF\": %.3f}\n",
         ts, 1e3 * ts / layers, t1, tp, 1e3 * tp / layers, tp / ts,
         flop / (ts * 1e-3) / 157.3e12, flop / (tp * 1e-3) / 157.3e12);
  return 0;
}
