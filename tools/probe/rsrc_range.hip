// Probe: which offsets does the raw-buffer range check (num_records) cover on gfx950?
// store through a 1024-byte descriptor at (voffset, soffset) pairs; print which landed.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(float* buf, int voff, int soff) {
  if (threadIdx.x != 0) return;
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, (short)0, 1024, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(0x3f800000u, r, voff, soff, 0);
}

int main() {
  float* d;
  hipMalloc(&d, 8192);
  const int cases[][2] = {{0, 0}, {2048, 0}, {0, 2048}, {1020, 0}, {0, 1020}, {512, 508}, {512, 512}};
  for (auto& c : cases) {
    hipMemset(d, 0, 8192);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, c[0], c[1]);
    float h[2048];
    hipMemcpy(h, d, 8192, hipMemcpyDeviceToHost);
    const int idx = (c[0] + c[1]) / 4;
    printf("voff %5d soff %5d -> element %4d %s\n", c[0], c[1], idx, h[idx] == 1.0f ? "STORED" : "dropped");
  }
  return 0;
}
