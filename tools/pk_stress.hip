// Packed-f32 stress kernel (diagnostic, never product).  Every lane runs
// the same chain of dependent fmas three ways and compares them bit for bit:
//   form 0: packed f32 (f32x2 fma / mul / add) with the second operand a broadcast scalar --
//           the compiler encodes it with op_sel (the pattern of the failing kNN distances);
//   form 1: packed f32 with the second operand a genuine register pair (its two halves are
//           equal but opaque to the compiler: no op_sel);
//   form 2: the scalar chain (v_fma_f32), the reference.
// n must be a power of two.  mism[f] counts lanes whose form-f result differs from form 2 (global atomics, vector path).
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -shared -fPIC \
//     tools/pk_stress.hip -o tools/pk_stress.so
#include <hip/hip_runtime.h>

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float opaque(float v) {
  float r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

template <int FORM>
__global__ __launch_bounds__(256) void pk_stress_kernel(const float* __restrict__ x, int n,
                                                        int iters,
                                                        unsigned long long* __restrict__ mism) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const float a0 = x[(2 * t) & (n - 1)], a1 = x[(2 * t + 1) & (n - 1)];
  const float w = x[(t * 7 + 3) & (n - 1)];
  f32x2 acc = {a0, a1};
  float s0 = a0, s1 = a1;
  const f32x2 wb = FORM == 0 ? f32x2{w, w} : f32x2{w, opaque(w)};
  const f32x2 hb = FORM == 0 ? f32x2{0.5f, 0.5f} : f32x2{opaque(0.5f), opaque(0.5f)};
  for (int i = 0; i < iters; ++i) {
    const float q = x[(t + i * 977) & (n - 1)];
    const float q2 = FORM == 0 ? q : opaque(q);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      // d = (fma(acc, w, acc * q) + q) * 0.5  (mul / fma / add, as in the distance chains)
      const float qj = __fadd_rn(q, 0.015625f * j), qj2 = __fadd_rn(q2, 0.015625f * j);
      if (FORM < 2) {
        const f32x2 qq = f32x2{qj, qj2};
        const f32x2 m = acc * qq;
        const f32x2 f = __builtin_elementwise_fma(acc, wb, m);
        acc = (f + qq) * hb;
      }
      s0 = __fmul_rn(__fadd_rn(__builtin_fmaf(s0, w, __fmul_rn(s0, qj)), qj), 0.5f);
      s1 = __fmul_rn(__fadd_rn(__builtin_fmaf(s1, w, __fmul_rn(s1, qj)), qj), 0.5f);
    }
  }
  if (FORM < 2) {
    if (__float_as_uint(acc[0]) != __float_as_uint(s0) || __float_as_uint(acc[1]) != __float_as_uint(s1))
      atomicAdd(&mism[FORM], 1ull);
  }
  if (FORM == 2 && s0 == 12345.f) atomicAdd(&mism[2], 1ull);  // keep the scalar chain live
}

extern "C" __attribute__((visibility("default"))) int pk_stress(int form, const float* x, int n,
                                                                int iters, int blocks,
                                                                unsigned long long* mism,
                                                                void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (form == 0)
    hipLaunchKernelGGL(pk_stress_kernel<0>, dim3(blocks), dim3(256), 0, st, x, n, iters, mism);
  else if (form == 1)
    hipLaunchKernelGGL(pk_stress_kernel<1>, dim3(blocks), dim3(256), 0, st, x, n, iters, mism);
  else
    hipLaunchKernelGGL(pk_stress_kernel<2>, dim3(blocks), dim3(256), 0, st, x, n, iters, mism);
  return (int)hipGetLastError();
}
