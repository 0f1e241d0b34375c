// Weight gradients of the network's skinny 1x1 layers: out (O x I) = A^T B for A (R x O),
// B (R x I) with a tiny O x I (the xyz -> 32 input convs, the 3-channel flow heads).
//
// dense.splitk_tn runs these as a chunked batched GEMM; with O or I <= 4 the BLAS library
// picks 16x16 / 16x32 tiles and ran them at ~0.5 GFLOP per 50 us (rocprofv3, round 2: ~0.45
// ms per step over ~15 such GEMMs) for a few MB of operands.  Here: one workgroup per slab of
// rows stages 16-row tiles of A and B in LDS and accumulates its O x I partial (each thread
// owns up to 4 outputs, rows ascending), the slab partials are summed by the fixed-order
// column sum.  Deterministic: the result depends only on the shape.
#include "kdpc_common.h"

#include <algorithm>

using namespace kdpc;

namespace {

constexpr int kTile = 16;       // rows staged per step
constexpr int kPer = 4;         // outputs per thread
constexpr int kMaxOut = 256 * kPer;
constexpr int kMaxWidth = 512;  // O + I staged per row

inline void plan(int r, int* slabs, int* rpw) {
  int s = std::max(1, std::min(1024, divup(r, 256)));
  *rpw = divup(r, s);
  *slabs = divup(r, *rpw);
}

__global__ __launch_bounds__(256) void dense_tn_small_kernel(int r, int o, int in, int rpw,
                                                             const float* __restrict__ a,
                                                             const float* __restrict__ b,
                                                             float* __restrict__ slab) {
  __shared__ float sa[kTile * kMaxWidth];
  float* sb = sa + kTile * o;
  const int t = threadIdx.x;
  const int nout = o * in;
  const int r0 = blockIdx.x * rpw, r1 = min(r, r0 + rpw);
  float acc[kPer];
  int oo[kPer], ii[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    acc[q] = 0.f;
    const int e = t + 256 * q;
    oo[q] = e < nout ? e / in : 0;
    ii[q] = e < nout ? e - (e / in) * in : 0;
  }
  for (int rt = r0; rt < r1; rt += kTile) {
    const int nr = min(kTile, r1 - rt);
    for (int e = t; e < nr * o; e += 256) sa[e] = a[(long long)rt * o + e];
    for (int e = t; e < nr * in; e += 256) sb[e] = b[(long long)rt * in + e];
    __syncthreads();
    for (int k = 0; k < nr; ++k) {
#pragma unroll
      for (int q = 0; q < kPer; ++q)
        acc[q] = __builtin_fmaf(sa[k * o + oo[q]], sb[k * in + ii[q]], acc[q]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int e = t + 256 * q;
    if (e < nout) slab[(long long)blockIdx.x * nout + e] = acc[q];
  }
}

}  // namespace

KDPC_API size_t kdpc_dense_tn_small_workspace_bytes(int r, int o, int i) {
  if (r <= 0 || o <= 0 || i <= 0 || o * i > kMaxOut || o + i > kMaxWidth) return 0;
  int slabs, rpw;
  plan(r, &slabs, &rpw);
  const long long len = (long long)o * i;
  return (size_t)(slabs * len + colsum_scratch_floats(slabs, len)) * sizeof(float);
}

KDPC_API int kdpc_dense_tn_small(int r, int o, int i, const float* a, const float* b, float* out,
                                 void* workspace, size_t workspace_bytes, void* stream) {
  KDPC_CHECK_ARG(r > 0 && o > 0 && i > 0 && o * i <= kMaxOut && o + i <= kMaxWidth);
  KDPC_CHECK_ARG(a && b && out && workspace &&
                 workspace_bytes >= kdpc_dense_tn_small_workspace_bytes(r, o, i));
  int slabs, rpw;
  plan(r, &slabs, &rpw);
  float* slab = reinterpret_cast<float*>(workspace);
  const long long len = (long long)o * i;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(dense_tn_small_kernel, dim3(slabs), dim3(256), 0, st, r, o, i, rpw, a, b,
                     slab);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return (int)colsum(slabs, len, slab, out, slab + (size_t)slabs * len, st);
}
