// Weight gradients of the network's skinny 1x1 layers: out (O x I) = A^T B for A (R x O),
// B (R x I) with a tiny O x I (the xyz -> 32 input convs, the 3-channel flow heads).
//
// dense.splitk_tn runs these as a chunked batched GEMM; with O or I <= 4 the BLAS library
// picks 16x16 / 16x32 tiles and ran them at ~0.5 GFLOP per 50 us (rocprofv3, round 2: ~0.45
// ms per step over ~15 such GEMMs) for a few MB of operands.  Here: one workgroup per slab of
// rows; each thread owns 4 entries of the wide side x the whole narrow side (<= 4) in
// registers and walks its row group with 8 rows of loads in flight; the row groups' partials
// are summed in order through LDS, the slab partials by the fixed-order column sum.
// Deterministic: the result depends only on the shape.  (An LDS-staged first version read
// two LDS words per fma and ran ~30 us per call.)
#include "kdpc_common.h"

#include <algorithm>

using namespace kdpc;

namespace {

constexpr int kNarrow = 4;      // the narrow side (min(O, I)) held whole per thread
constexpr int kMaxOut = 1024;
constexpr int kMaxWidth = 512;  // O + I

inline void plan(int r, int* slabs, int* rpw) {
  int s = std::max(1, std::min(1024, divup(r, 512)));
  *rpw = divup(r, s);
  *slabs = divup(r, *rpw);
}

// W = the wide side, n = the narrow side (<= 4).  Thread t: wide block wb = t % WB (4 wide
// entries), row group rg = t / WB; it walks rows r0 + rg, r0 + rg + RG, ... (8 rows in flight)
// accumulating its 4 x n outputs from registers, then the RG row-group partials are summed
// in order through LDS.  A_IS_WIDE: A (R x O) is the wide operand (out[o][i], o wide).
template <bool A_IS_WIDE>
__global__ __launch_bounds__(256) void dense_tn_small_kernel(int r, int o, int in, int rpw,
                                                             const float* __restrict__ a,
                                                             const float* __restrict__ b,
                                                             float* __restrict__ slab) {
  __shared__ float part[4096];
  const int w = A_IS_WIDE ? o : in, n = A_IS_WIDE ? in : o;
  const float* wide = A_IS_WIDE ? a : b;
  const float* nar = A_IS_WIDE ? b : a;
  const int wbn = (w + 3) / 4;         // wide blocks
  const int rg_n = max(1, 256 / wbn);  // row groups
  const int t = threadIdx.x;
  const int wb = t % wbn, rg = t / wbn;
  const bool act = rg < rg_n && t < rg_n * wbn;
  const int r0 = blockIdx.x * rpw, r1 = min(r, r0 + rpw);
  float acc[4][kNarrow];
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < kNarrow; ++y) acc[x][y] = 0.f;
  if (act) {
    constexpr int U = 8;
    for (int rr = r0 + rg; rr < r1; rr += U * rg_n) {
      float wv[U][4], nv[U][kNarrow];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int row = rr + u * rg_n;
        const bool ok = row < r1;
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          const int c = 4 * wb + x;
          wv[u][x] = ok && c < w ? wide[(long long)row * w + c] : 0.f;
        }
#pragma unroll
        for (int y = 0; y < kNarrow; ++y) nv[u][y] = ok && y < n ? nar[(long long)row * n + y] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < kNarrow; ++y) acc[x][y] = __builtin_fmaf(wv[u][x], nv[u][y], acc[x][y]);
    }
  }
  // partials part[rg][wide entry][narrow entry], summed over the row groups in order
  const int len = w * n;
  if (act) {
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int c = 4 * wb + x;
      if (c < w)
#pragma unroll
        for (int y = 0; y < kNarrow; ++y)
          if (y < n) part[rg * len + c * n + y] = acc[x][y];
    }
  }
  __syncthreads();
  for (int e = t; e < len; e += 256) {
    float s = part[e];
    for (int g = 1; g < rg_n; ++g) s = __fadd_rn(s, part[g * len + e]);
    const int c = e / n, y = e - (e / n) * n;  // wide entry c, narrow entry y
    const int oi = A_IS_WIDE ? c * in + y : y * in + c;
    slab[(long long)blockIdx.x * len + oi] = s;
  }
}

// y (R x N) = x (R x K) m (K x N) [+ bias] with min(K, N) <= 4: the skinny forward / input-
// gradient GEMMs of the same layers (BLAS: 16-wide tiles, 20-50 us each; memory-bound here).
// N <= 4: four lanes per row split K (float4 steps, lane q takes k = 4q + 16s), partial dot
// products summed by a fixed butterfly.  K <= 4: one thread per (row, 4 outputs).
template <bool NARROW_OUT>
__global__ __launch_bounds__(256) void dense_small_kernel(int r, int k, int n,
                                                          const float* __restrict__ x,
                                                          const float* __restrict__ m,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ y) {
  __shared__ float ms[4096];
  for (int e = threadIdx.x; e < k * n; e += 256) ms[e] = m[e];
  __syncthreads();
  if (NARROW_OUT) {
    const long long total = (long long)r * 4;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {  // every lane of a row group iterates alike
      const long long row = e >> 2;
      const int q = (int)(e & 3);
      const float* xr = x + row * k;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      if ((k & 3) == 0) {
        for (int c = 4 * q; c < k; c += 16) {
          const float4 v = *reinterpret_cast<const float4*>(xr + c);
          const float xv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (j < n) acc[j] = __builtin_fmaf(xv[u], ms[(c + u) * n + j], acc[j]);
        }
      } else {
        for (int c = q; c < k; c += 4)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (j < n) acc[j] = __builtin_fmaf(xr[c], ms[c * n + j], acc[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[j] += __shfl_xor(acc[j], 1);
        acc[j] += __shfl_xor(acc[j], 2);
      }
      if (q == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (j < n) y[row * n + j] = bias ? __fadd_rn(acc[j], bias[j]) : acc[j];
      }
    }
  } else {
    const int nv = (n + 3) / 4;
    const long long total = (long long)r * nv;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
      const long long row = e / nv;
      const int c0 = 4 * (int)(e - row * nv);
      float xv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) xv[u] = u < k ? x[row * k + u] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = c0 + j;
        if (c >= n) break;
        float acc = 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (u < k) acc = __builtin_fmaf(xv[u], ms[u * n + c], acc);
        y[row * n + c] = bias ? __fadd_rn(acc, bias[c]) : acc;
      }
    }
  }
}

}  // namespace

KDPC_API size_t kdpc_dense_tn_small_workspace_bytes(int r, int o, int i) {
  if (r <= 0 || o <= 0 || i <= 0 || std::min(o, i) > kNarrow || o * i > kMaxOut ||
      o + i > kMaxWidth)
    return 0;
  int slabs, rpw;
  plan(r, &slabs, &rpw);
  const long long len = (long long)o * i;
  return (size_t)(slabs * len + colsum_scratch_floats(slabs, len)) * sizeof(float);
}

KDPC_API int kdpc_dense_tn_small(int r, int o, int i, const float* a, const float* b, float* out,
                                 void* workspace, size_t workspace_bytes, void* stream) {
  KDPC_CHECK_ARG(r > 0 && o > 0 && i > 0 && std::min(o, i) <= kNarrow && o * i <= kMaxOut &&
                 o + i <= kMaxWidth);
  KDPC_CHECK_ARG(a && b && out && workspace &&
                 workspace_bytes >= kdpc_dense_tn_small_workspace_bytes(r, o, i));
  int slabs, rpw;
  plan(r, &slabs, &rpw);
  float* slab = reinterpret_cast<float*>(workspace);
  const long long len = (long long)o * i;
  hipStream_t st = (hipStream_t)stream;
  if (o >= i)
    hipLaunchKernelGGL(dense_tn_small_kernel<true>, dim3(slabs), dim3(256), 0, st, r, o, i, rpw,
                       a, b, slab);
  else
    hipLaunchKernelGGL(dense_tn_small_kernel<false>, dim3(slabs), dim3(256), 0, st, r, o, i, rpw,
                       a, b, slab);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return (int)colsum(slabs, len, slab, out, slab + (size_t)slabs * len, st);
}

KDPC_API int kdpc_dense_small(int r, int k, int n, const float* x, const float* m,
                              const float* bias, float* y, void* stream) {
  KDPC_CHECK_ARG(r >= 0 && k > 0 && n > 0 && std::min(k, n) <= 4 && k * n <= 4096);
  if (r == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(x && m && y);
  hipStream_t st = (hipStream_t)stream;
  if (n <= 4) {
    const long long work = (long long)r * 4;
    const int grid = (int)std::min<long long>(divupll(work, 256), 1 << 16);
    hipLaunchKernelGGL(dense_small_kernel<true>, dim3(grid), dim3(256), 0, st, r, k, n, x, m,
                       bias, y);
  } else {
    const long long work = (long long)r * ((n + 3) / 4);
    const int grid = (int)std::min<long long>(divupll(work, 256), 1 << 16);
    hipLaunchKernelGGL(dense_small_kernel<false>, dim3(grid), dim3(256), 0, st, r, k, n, x, m,
                       bias, y);
  }
  return (int)hipGetLastError();
}
