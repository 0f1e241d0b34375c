// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o probe_bf16 tools/probe_bf16.hip
// (1) bf16 MFMA / VALU co-issue: one v_mfma_f32_32x32x16_bf16 chain + M VALU fmas per MFMA.
// (2) accuracy of a 32x32 (K=128) product on f32 MFMA vs split-bf16 (3 and 6 products) vs fp64.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int M>
__global__ __launch_bounds__(256) void cobf(float* out, int iters) {
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(threadIdx.x * 1e-3f + i); b[i] = (__bf16)(1.0f + i * 1e-2f); }
  float v[8], s = 1.0001f, c = threadIdx.x * 1e-3f;
  for (int i = 0; i < 8; ++i) v[i] = threadIdx.x * (i + 1) * 1e-4f;
  for (int it = 0; it < iters; ++it) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < M; ++j) v[j % 8] = __builtin_fmaf(v[j % 8], s, c);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, M, 0);
  }
  float r = 0.f;
  for (int i = 0; i < 16; ++i) r += acc[i];
  for (int i = 0; i < 8; ++i) r += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__device__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  float r = x - (float)h;
  m = (__bf16)r;
  r = r - (float)m;
  l = (__bf16)r;
}

// C(32x32) = A(32xK) B(Kx32), K = 128; mode 0 f32 MFMA, 3 = bf16x3, 6 = bf16x6
__global__ __launch_bounds__(64) void gemm(const float* A, const float* B, float* C, int mode) {
  const int l = threadIdx.x, half = l >> 5, l32 = l & 31;
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  if (mode == 0) {
    for (int k = 0; k < 128; k += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[l32 * 128 + k + half], B[(k + half) * 32 + l32], acc, 0, 0, 0);
  } else {
    for (int k0 = 0; k0 < 128; k0 += 16) {
      bf16x8 ah, am, al, bh, bm, bl;
      for (int j = 0; j < 8; ++j) {
        __bf16 h, m, lo;
        split3(A[l32 * 128 + k0 + 8 * half + j], h, m, lo);
        ah[j] = h; am[j] = m; al[j] = lo;
        split3(B[(k0 + 8 * half + j) * 32 + l32], h, m, lo);
        bh[j] = h; bm[j] = m; bl[j] = lo;
      }
      if (mode == 6) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
    }
  }
  for (int e = 0; e < 16; ++e) C[((e & 3) + 8 * (e >> 2) + 4 * half) * 32 + l32] = acc[e];
}

template <int M>
void run(float* out, int iters) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  cobf<M><<<1024, 256>>>(out, 100);
  (void)hipEventRecord(e0);
  cobf<M><<<1024, 256>>>(out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  // 1024 blocks x 4 waves = one wave per SIMD
  printf("bf16 mfma + %2d valu: %.2f ns/iter = %.1f cyc @2.4GHz\n", M, ms * 1e6 / iters, ms * 1e6 / iters * 2.4);
}

int main() {
  float* out;
  (void)hipMalloc(&out, 1024 * 256 * 4);
  const int iters = 200000;
  run<0>(out, iters);
  run<4>(out, iters);
  run<8>(out, iters);
  run<12>(out, iters);
  run<16>(out, iters);
  run<24>(out, iters);
  // accuracy
  std::vector<float> A(32 * 128), B(128 * 32), C(32 * 32);
  srand(1);
  for (int trial = 0; trial < 3; ++trial) {
    for (auto& x : A) x = (rand() / (float)RAND_MAX - 0.5f) * (trial == 2 ? 1000.f : 2.f);
    for (auto& x : B) x = (rand() / (float)RAND_MAX - 0.5f) * 2.f;
    std::vector<double> R(32 * 32, 0.0);
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j)
        for (int k = 0; k < 128; ++k) R[i * 32 + j] += (double)A[i * 128 + k] * B[k * 32 + j];
    double mx = 0;
    for (double r : R) mx = fmax(mx, fabs(r));
    float *dA, *dB, *dC;
    (void)hipMalloc(&dA, A.size() * 4);
    (void)hipMalloc(&dB, B.size() * 4);
    (void)hipMalloc(&dC, C.size() * 4);
    (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    for (int mode : {0, 3, 6}) {
      gemm<<<1, 64>>>(dA, dB, dC, mode);
      (void)hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
      double err = 0, rel = 0;
      for (int i = 0; i < 32 * 32; ++i) {
        err = fmax(err, fabs(C[i] - R[i]));
        rel = fmax(rel, fabs(C[i] - R[i]) / fmax(fabs(R[i]), 1e-30));
      }
      printf("trial %d mode %d: max abs err / max|ref| = %.3e, max elementwise rel %.3e\n", trial, mode, err / mx, rel);
    }
  }
  return 0;
}
