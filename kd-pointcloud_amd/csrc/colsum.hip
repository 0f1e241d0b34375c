// Deterministic column sums of per-workgroup partial slabs: dst[i] = sum_s slab[s][i].
//
// Every parameter-gradient reduction here ends with such a sum over hundreds to thousands
// of slab rows.  One thread walking all rows of one column serialises thousands of
// dependent loads (~110 us for 512 x 248); instead the rows are summed in chunks of 64 by
// a 2-D grid, and the chunk partials again, each level in a fixed order (ascending rows
// within a chunk, ascending chunks), so the result depends only on the shape.
#include <algorithm>

#include "kdpc_common.h"

namespace {

constexpr int kCols = 64;     // columns per workgroup
constexpr int kGroups = 4;    // row groups per workgroup (256 threads)
constexpr int kChunk = 64;    // rows per workgroup

// out[blockIdx.y][c] = sum of rows [blockIdx.y*kChunk, +kChunk) of column c (in order:
// rows within each of the kGroups interleaved sub-chunks ascending, sub-chunks ascending)
__global__ __launch_bounds__(256) void colsum_kernel(int nrows, long long len,
                                                     const float* __restrict__ src,
                                                     float* __restrict__ dst) {
  __shared__ float part[kGroups][kCols];
  const int cx = threadIdx.x % kCols, g = threadIdx.x / kCols;
  const long long c = (long long)blockIdx.x * kCols + cx;
  const int r0 = blockIdx.y * kChunk + g * (kChunk / kGroups);
  const int r1 = min(nrows, r0 + kChunk / kGroups);
  float a = 0.f;
  if (c < len) {
#pragma unroll 4
    for (int r = r0; r < r1; ++r) a = __fadd_rn(a, src[(long long)r * len + c]);
  }
  part[g][cx] = a;
  __syncthreads();
  if (g == 0 && c < len) {
    float s = part[0][cx];
#pragma unroll
    for (int q = 1; q < kGroups; ++q) s = __fadd_rn(s, part[q][cx]);
    dst[(long long)blockIdx.y * len + c] = s;
  }
}

}  // namespace

namespace kdpc {

size_t colsum_scratch_floats(int nrows, long long len) {
  size_t total = 0;
  int n = nrows;
  while (n > kChunk) {
    n = divup(n, kChunk);
    total += (size_t)n * len;
  }
  return total;
}

hipError_t colsum(int nrows, long long len, const float* slab, float* dst, float* scratch,
                  hipStream_t st) {
  const float* src = slab;
  int n = nrows;
  while (true) {
    const int out_rows = divup(n, kChunk);
    float* out = out_rows == 1 ? dst : scratch;
    dim3 grid((unsigned)divupll(len, kCols), (unsigned)out_rows);
    hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, st, n, len, src, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || out_rows == 1) return e;
    src = out;
    scratch += (size_t)out_rows * len;
    n = out_rows;
  }
}

}  // namespace kdpc

// ------------------------------------------------------------------------------ C ABI
KDPC_API size_t kdpc_colsum_workspace_bytes(int nrows, int len) {
  if (nrows <= 0 || len <= 0) return 0;
  return kdpc::colsum_scratch_floats(nrows, len) * sizeof(float);
}

// dst[i] = sum over rows r of src[r][i] (row-major (nrows, len)), fixed summation order.
KDPC_API int kdpc_colsum(int nrows, int len, const float* src, float* dst, void* workspace,
                         size_t workspace_bytes, void* stream) {
  KDPC_CHECK_ARG(nrows >= 0 && len >= 0);
  if (len == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(dst);
  if (nrows == 0) return (int)hipMemsetAsync(dst, 0, sizeof(float) * len, (hipStream_t)stream);
  KDPC_CHECK_ARG(src && workspace_bytes >= kdpc_colsum_workspace_bytes(nrows, len));
  KDPC_CHECK_ARG(workspace_bytes == 0 || workspace);
  return (int)kdpc::colsum(nrows, len, src, dst, reinterpret_cast<float*>(workspace),
                           (hipStream_t)stream);
}
