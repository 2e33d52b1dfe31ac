// Probe: accuracy of v_mfma_f32_16x16x32_f16 accumulation (products exact in f32) against an
// exact fp64 sum, and of the 3-product split (hi*hi + hi*lo + lo*hi) for f32 dot products.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <random>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// A: [16][K] f16 row-major, B: [K][16] f16; one wave; D[16][16]
__global__ void mm(const _Float16* A, const _Float16* B, float* D, int K) {
  int l = threadIdx.x, r = l & 15, g = l >> 4;
  f32x4 acc = {0, 0, 0, 0};
  for (int k0 = 0; k0 < K; k0 += 32) {
    f16x8 a, b;
    for (int j = 0; j < 8; ++j) {
      a[j] = A[r * K + k0 + 8 * g + j];
      b[j] = B[(k0 + 8 * g + j) * 16 + r];
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
  }
  for (int i = 0; i < 4; ++i) D[(4 * g + i) * 16 + r] = acc[i];
}

// split test: f32 A [16][K], B [K][16]; per-tensor pow2 scale for A, per-column for B
__global__ void split_mm(const float* A, const float* B, float* D, int K, float sa, const float* sb) {
  int l = threadIdx.x, r = l & 15, g = l >> 4;
  f32x4 acc = {0, 0, 0, 0};
  float s = sb[r];
  for (int k0 = 0; k0 < K; k0 += 32) {
    f16x8 ah, al, bh, bl;
    for (int j = 0; j < 8; ++j) {
      float av = A[r * K + k0 + 8 * g + j] * sa;
      _Float16 h = (_Float16)av;
      ah[j] = h; al[j] = (_Float16)(av - (float)h);
      float bv = B[(k0 + 8 * g + j) * 16 + r] * s;
      _Float16 hb = (_Float16)bv;
      bh[j] = hb; bl[j] = (_Float16)(bv - (float)hb);
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc, 0, 0, 0);
  }
  for (int i = 0; i < 4; ++i) D[(4 * g + i) * 16 + r] = acc[i];
}

// native f32 MFMA chain for comparison
__global__ void f32_mm(const float* A, const float* B, float* D, int K) {
  int l = threadIdx.x, r = l & 15, g = l >> 4;
  f32x4 acc = {0, 0, 0, 0};
  for (int k0 = 0; k0 < K; k0 += 4)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[r * K + k0 + g], B[(k0 + g) * 16 + r], acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) D[(4 * g + i) * 16 + r] = acc[i];
}

int main() {
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0, 1);
  const int K = 512;
  // (1) exact f16 inputs: MFMA accumulation error vs exact
  {
    std::vector<_Float16> A(16 * K), B(K * 16);
    for (auto& x : A) x = (_Float16)nd(rng);
    for (auto& x : B) x = (_Float16)nd(rng);
    _Float16 *dA, *dB; float* dD;
    hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2); hipMalloc(&dD, 256 * 4);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    mm<<<1, 64>>>(dA, dB, dD, K);
    std::vector<float> D(256);
    hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost);
    double maxrel = 0, sumerr = 0, sumabs = 0; int exact = 0;
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
      double s = 0, sa = 0; float fchain = 0;
      for (int k = 0; k < K; ++k) { double p = (double)A[i * K + k] * (double)B[k * 16 + j]; s += p; sa += fabs(p); fchain = fmaf((float)A[i*K+k], (float)B[k*16+j], fchain); }
      double e = fabs(D[i * 16 + j] - s);
      maxrel = fmax(maxrel, e / sa); sumerr += e; sumabs += sa;
      exact += (D[i * 16 + j] == (float)s);
    }
    printf("f16 MFMA K=%d: max err/sum|p| = %.3e, mean err/sum|p| = %.3e, %d/256 == f32(exact)\n", K, maxrel, sumerr / sumabs, exact);
  }
  // (2) f32 inputs via 3-product split vs native f32 MFMA, both vs fp64
  {
    std::vector<float> A(16 * K), B(K * 16), sb(16);
    for (auto& x : A) x = nd(rng) * 0.05f;
    for (int j = 0; j < 16; ++j) {
      float mx = 0;
      float colscale = powf(10.f, (float)(j % 8) - 4.f);  // columns from 1e-4 to 1e3
      for (int k = 0; k < K; ++k) { float v = nd(rng) * colscale; if (k % 3 == 0) v = 0; B[k * 16 + j] = v; mx = fmaxf(mx, fabsf(v)); }
      int e; frexpf(mx, &e); sb[j] = ldexpf(1.f, 15 - e);
    }
    float amx = 0; for (auto x : A) amx = fmaxf(amx, fabsf(x));
    int ea; frexpf(amx, &ea); float sa = ldexpf(1.f, 15 - ea);
    float *dA, *dB, *dD, *dS;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dD, 1024); hipMalloc(&dS, 64);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dS, sb.data(), 64, hipMemcpyHostToDevice);
    std::vector<float> D1(256), D2(256);
    split_mm<<<1, 64>>>(dA, dB, dD, K, sa, dS);
    hipMemcpy(D1.data(), dD, 1024, hipMemcpyDeviceToHost);
    f32_mm<<<1, 64>>>(dA, dB, dD, K);
    hipMemcpy(D2.data(), dD, 1024, hipMemcpyDeviceToHost);
    double e1 = 0, e2 = 0, n = 0, m1 = 0, m2 = 0;
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
      double s = 0, sa2 = 0;
      for (int k = 0; k < K; ++k) { double p = (double)A[i * K + k] * B[k * 16 + j]; s += p; sa2 += fabs(p); }
      double d1 = D1[i * 16 + j] / ((double)sa * sb[j]);
      e1 += (d1 - s) * (d1 - s); e2 += (D2[i * 16 + j] - s) * (D2[i * 16 + j] - s); n += s * s;
      m1 = fmax(m1, fabs(d1 - s) / sa2); m2 = fmax(m2, fabs(D2[i * 16 + j] - s) / sa2);
    }
    printf("split f16x3: nrel %.3e  max err/sum|p| %.3e\nnative f32 : nrel %.3e  max err/sum|p| %.3e\n",
           sqrt(e1 / n), m1, sqrt(e2 / n), m2);
  }
  hipError_t err = hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(err));
  return 0;
}
