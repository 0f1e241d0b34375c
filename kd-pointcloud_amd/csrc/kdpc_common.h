// Shared device helpers for the gfx950 kernels of kd-pointcloud_amd.
// Wave64 only: every cross-lane helper below assumes 64 lanes (CDNA4).
//
// No packed f32 VALU anywhere (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32, from f32x2
// arithmetic or from the SLP vectoriser): measured on the MI355X, their results were now and
// then wrong while another kernel's waves (the KD teacher's forward on its own stream) ran
// beside them -- the culled kNN's seed distances came out low, so whole neighbours went
// missing -- and the same kernels built with scalar f32 ops never were (DESIGN.md section 5,
// tools/knn_race.py).  Every source is built with -fno-slp-vectorize -fno-vectorize (build_native.py) and
// tests/test_native_lib.py disassembles the library to check that none is left.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kdpc.h"  // C ABI declarations (include/kdpc.h): definitions must match

#define KDPC_API extern "C" __attribute__((visibility("default")))

namespace kdpc {

constexpr int kWave = 64;

__host__ __device__ inline int divup(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ inline long long divupll(long long a, long long b) { return (a + b - 1) / b; }

// nvcc -O2 (fmad=true) contraction of (x2-x1)^2 + (y2-y1)^2 + (z2-z1)^2, as used by the
// reference kernels (sampling_gpu.cu:130, ball_query_gpu.cu:33, interpolate_gpu.cu:36).
// Written with explicit fmas so the compiler cannot re-contract or SLP-pack it.
__device__ __forceinline__ float dist3(float x1, float y1, float z1, float x2, float y2,
                                       float z2) {
  const float dx = x2 - x1, dy = y2 - y1, dz = z2 - z1;
  return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
}

// pointconv_util.py:73-94 square_distance, expanded form, exactly as torch evaluates it:
//   dot = fma(z,z', fma(y,y', x*x'));  d = -2*dot;  d += |q|^2;  d += |r|^2
// with |p|^2 = (x*x + y*y) + z*z separately rounded.
__device__ __forceinline__ float sqnorm3(float x, float y, float z) {
  return __fadd_rn(__fadd_rn(__fmul_rn(x, x), __fmul_rn(y, y)), __fmul_rn(z, z));
}
__device__ __forceinline__ float sqdist_expanded(float qx, float qy, float qz, float sq, float rx,
                                                 float ry, float rz, float sr) {
  const float dot = __builtin_fmaf(qz, rz, __builtin_fmaf(qy, ry, __fmul_rn(qx, rx)));
  return __fadd_rn(__fadd_rn(-2.0f * dot, sq), sr);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// Intra-wave LDS hand-off (this wave's lanes wrote, other lanes of the same wave read next):
// a compiler memory barrier -- no LDS access is moved across it, whatever the types or
// addresses -- plus wave_barrier (which alone orders no memory).  The hardware keeps one
// wave's LDS accesses in order, so no s_barrier is needed.
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// Full-wave butterfly reductions (every lane ends with the result).
__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    unsigned w = __shfl_xor(v, o, kWave);
    v = w > v ? w : v;
  }
  return v;
}
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    unsigned w = __shfl_xor(v, o, kWave);
    v = w < v ? w : v;
  }
  return v;
}

// lane l receives lane l-1's value; lane 0 receives `fill` (DPP wave_shr:1, gfx9).
__device__ __forceinline__ float wave_shr1(float v, float fill) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(fill), __float_as_int(v),
                                                    0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ int wave_shr1(int v, int fill) {
  return __builtin_amdgcn_update_dpp(fill, v, 0x138, 0xf, 0xf, false);
}

__device__ __forceinline__ unsigned long long lanemask_lt() {
  const int l = lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Deterministic column sums of partial slabs (csrc/colsum.hip): dst[i] = sum_s slab[s][i]
// for s < nrows, i < len, summed in fixed-size chunks (fixed order); scratch holds
// colsum_scratch_floats(nrows, len) floats.
size_t colsum_scratch_floats(int nrows, long long len);
hipError_t colsum(int nrows, long long len, const float* slab, float* dst, float* scratch,
                  hipStream_t st);

// Fused wide cost volume (csrc/cost_volume_wide.hip): Din = Dout = d in {128, 256}, K <= 32;
// dispatched by kdpc_cost_volume_fwd / _bwd (csrc/cost_volume.hip).
bool cost_volume_wide_fused_supported(int din, int dout, int k);
hipError_t cost_volume_wide_fused_fwd(int b, int n1, int n2, int k, int d, const float* x1,
                                      const float* x2, const int* idx, const float* p1,
                                      const float* p2, const float* wpos, const float* bpos,
                                      const float* w1, const float* b1, float* out,
                                      unsigned char* amax, hipStream_t st);
size_t cost_volume_wide_fused_bwd_workspace_floats(int b, int n1, int d);
hipError_t cost_volume_wide_fused_bwd(int b, int n1, int n2, int k, int d, const float* x1,
                                      const float* x2, const int* idx, const float* p1,
                                      const float* p2, const float* wpos, const float* bpos,
                                      const float* w1, const float* out,
                                      const unsigned char* amax, const unsigned char* slope0,
                                      const float* dout, float* dp1, float* dp2_rows, float* dx1,
                                      float* ddir_rows, const int* rank, float* rows, float* ws,
                                      float* dparams, hipStream_t st);

}  // namespace kdpc

// Argument validation shared by every C entry point: a bad size is an error code,
// never a launch (reference launchers printed and exit(-1)ed on failure).
#define KDPC_CHECK_ARG(cond)                       \
  do {                                             \
    if (!(cond)) return (int)hipErrorInvalidValue; \
  } while (0)

#define KDPC_RETURN_LAUNCH() return (int)hipGetLastError()
