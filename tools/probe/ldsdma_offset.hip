// Probe: does the instruction offset of global_load_lds_dwordx4 / buffer_load_dwordx4 lds also
// advance the LDS destination?  Each of 4 DMAs copies 1 KiB; print where each KiB landed.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* src, float* out) {
  __shared__ float lds[4 * 256 + 256];
  for (int i = threadIdx.x; i < 5 * 256; i += 64) lds[i] = -1.0f;
  __syncthreads();
  unsigned keep;
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds);
  const unsigned voff = threadIdx.x * 16;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "global_load_lds_dwordx4 %1, %2 offset:1024\n\t"
      "global_load_lds_dwordx4 %1, %2 offset:2048\n\t"
      "global_load_lds_dwordx4 %1, %2 offset:3072\n\t"
      "s_mov_b32 m0, %0\n\ts_waitcnt vmcnt(0)"
      : "=&s"(keep) : "v"(voff), "s"(src), "s"(dst) : "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 5 * 256; i += 64) out[i] = lds[i];
}
int main() {
  float *s, *o; float h[5 * 256];
  hipMalloc(&s, 4096 * 4); hipMalloc(&o, 5 * 256 * 4);
  float init[4096]; for (int i = 0; i < 4096; ++i) init[i] = i;
  hipMemcpy(s, init, sizeof(init), hipMemcpyHostToDevice);
  k<<<1, 64>>>(s, o);
  hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
  for (int q = 0; q < 5; ++q) printf("LDS KiB %d: first %g last %g\n", q, h[q * 256], h[q * 256 + 255]);
  printf("%s\n", hipGetErrorString(hipDeviceSynchronize()));
}
