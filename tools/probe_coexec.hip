// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o probe_coexec tools/probe_coexec.hip
// f32 MFMA / VALU co-execution probe: per iteration one v_mfma_f32_32x32x2_f32 (dependent
// chain) and M independent VALU fmas in the same wave (mode 0), or MFMA-only waves 0-3 and
// VALU-only waves 4-7 of one 512-thread block (mode 1).  Prints ns per iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int M, int MODE>
__global__ __launch_bounds__(512) void probe(float* out, int iters) {
  f32x16 acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = threadIdx.x * (i + 1) * 1e-4f;
  const int wv = threadIdx.x >> 6;
  const bool do_mfma = MODE == 0 || (MODE == 1 && wv < 4);
  const bool do_valu = MODE == 0 || wv >= 4;
  if (MODE == 0 && wv >= 4) return;
  if (MODE == 2 && wv < 4) return;
  if (do_mfma && do_valu) {
    for (int it = 0; it < iters; ++it) {
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < M; ++j) v[j % 8] = __builtin_fmaf(v[j % 8], b, a);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, M, 0);
    }
  } else if (do_mfma) {
    for (int it = 0; it < iters; ++it) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  } else {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < M; ++j) v[j % 8] = __builtin_fmaf(v[j % 8], b, a);
    }
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += acc[i];
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int M, int MODE>
void run(float* out, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<M, MODE><<<256, 512>>>(out, 100);
  hipEventRecord(e0);
  probe<M, MODE><<<256, 512>>>(out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("mode %d M %3d: %.2f ns/iter\n", MODE, M, ms * 1e6 / iters);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 512 * 4);
  const int iters = 200000;
  run<0, 0>(out, iters);
  run<4, 0>(out, iters);
  run<8, 0>(out, iters);
  run<16, 0>(out, iters);
  run<24, 0>(out, iters);
  run<32, 0>(out, iters);
  run<0, 1>(out, iters);
  run<8, 1>(out, iters);
  run<16, 1>(out, iters);
  run<32, 1>(out, iters);
  run<8, 2>(out, iters);
  run<16, 2>(out, iters);
  run<32, 2>(out, iters);
  // VALU-only reference: MODE 1 with MFMA waves doing 0 iterations is not expressible; M-only
  hipFree(out);
  return 0;
}
