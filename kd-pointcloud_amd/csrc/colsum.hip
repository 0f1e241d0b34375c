// Deterministic column sums of per-workgroup partial slabs: dst[i] = sum_s slab[s][i].
//
// Every parameter-gradient reduction here ends with such a sum over hundreds to millions
// of rows.  One thread walking all rows of one column serialises thousands of dependent
// loads (~110 us for 512 x 248); instead a 2-D grid sums row slabs (level 1: about 1024
// workgroups over the whole matrix, each 64 columns x one contiguous slab of rows) and one
// more launch sums the slab partials (level 2); matrices of <= 256 rows take one launch.
// Inside a workgroup the 4 row groups each sum a contiguous quarter of the slab ascending
// and the quarters are added in order, so the result depends only on the shape.  (Round 1
// used fixed 64-row chunks and as many levels as needed: 3-4 launches for the 2^16-2^21
// row gradients, 215 launches per training step.)
#include <algorithm>

#include "kdpc_common.h"

namespace {

using kdpc::divupll;

constexpr int kCols = 64;        // columns per workgroup
constexpr int kGroups = 4;       // row groups per workgroup (256 threads)
constexpr int kOneLevel = 256;   // rows summed in a single launch
// level-1 workgroups aimed for: 512 (round-4 whole-step A/B, six runs each: 16.04 vs 16.15 ms
// mean at 1024; 2048 in between)
constexpr int kLevel1WG = 512;
inline int level1_wg() { return kLevel1WG; }

// out[blockIdx.y][c] = sum of rows [blockIdx.y*rpw, +rpw) of column c: row group g sums the
// g-th contiguous quarter ascending, the quarters are added in order
__global__ __launch_bounds__(256) void colsum_kernel(int nrows, long long len, int rpw,
                                                     const float* __restrict__ src,
                                                     float* __restrict__ dst) {
  __shared__ float part[kGroups][kCols];
  const int cx = threadIdx.x % kCols, g = threadIdx.x / kCols;
  const long long c = (long long)blockIdx.x * kCols + cx;
  const int q = (rpw + kGroups - 1) / kGroups;
  const int r0 = blockIdx.y * rpw + g * q;
  const int r1 = min(min(nrows, blockIdx.y * rpw + rpw), r0 + q);
  float a = 0.f;
  if (c < len) {
#pragma unroll 8
    for (int r = r0; r < r1; ++r) a = __fadd_rn(a, src[(long long)r * len + c]);
  }
  part[g][cx] = a;
  __syncthreads();
  if (g == 0 && c < len) {
    float s = part[0][cx];
#pragma unroll
    for (int k = 1; k < kGroups; ++k) s = __fadd_rn(s, part[k][cx]);
    dst[(long long)blockIdx.y * len + c] = s;
  }
}

// level-1 slab count and rows per slab for an (nrows, len) matrix (1 slab: single launch)
inline void colsum_plan(int nrows, long long len, int* slabs, int* rpw) {
  if (nrows <= kOneLevel) {
    *slabs = 1;
    *rpw = nrows;
    return;
  }
  const long long cb = divupll(len, kCols);
  long long g = std::max(2ll, divupll(level1_wg(), cb));
  g = std::min(g, divupll(nrows, 64));
  g = std::max(1ll, std::min(g, 1024ll));
  *rpw = (int)divupll(nrows, g);
  *slabs = (int)divupll(nrows, *rpw);
}

}  // namespace

namespace kdpc {

size_t colsum_scratch_floats(int nrows, long long len) {
  int slabs, rpw;
  colsum_plan(nrows, len, &slabs, &rpw);
  return slabs > 1 ? (size_t)slabs * len : 0;
}

hipError_t colsum(int nrows, long long len, const float* slab, float* dst, float* scratch,
                  hipStream_t st) {
  int slabs, rpw;
  colsum_plan(nrows, len, &slabs, &rpw);
  const unsigned cb = (unsigned)divupll(len, kCols);
  if (slabs == 1) {
    hipLaunchKernelGGL(colsum_kernel, dim3(cb, 1), dim3(256), 0, st, nrows, len, nrows, slab, dst);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(colsum_kernel, dim3(cb, (unsigned)slabs), dim3(256), 0, st, nrows, len, rpw,
                     slab, scratch);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(colsum_kernel, dim3(cb, 1), dim3(256), 0, st, slabs, len, slabs, scratch, dst);
  return hipGetLastError();
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

// ------------------------------------------------------------------------------------------
// out[i][c] = -sum_{j<k} in[i][j][c] (ascending j): the center gradient of a grouped
// relative-offset layer, dcenter = -sum_k drel (WeightNet backward), in one launch (torch's
// `-x.sum(2)` was a strided reduction plus a negation: two launches per layer).
namespace {
__global__ __launch_bounds__(256) void neg_sum_k_kernel(long long m, int k, int c,
                                                        const float* __restrict__ in,
                                                        float* __restrict__ out) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= m * c) return;
  const long long i = e / c;
  const int ch = (int)(e - i * c);
  const float* p = in + i * k * c + ch;
  float s = 0.f;
  for (int j = 0; j < k; ++j) s = __fadd_rn(s, p[(long long)j * c]);
  out[e] = -s;
}
}  // namespace

KDPC_API int kdpc_neg_sum_k(int m, int k, int c, const float* in, float* out,
                            void* stream) {
  KDPC_CHECK_ARG(m >= 0 && k >= 1 && c >= 1);
  if (m == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(in && out);
  hipLaunchKernelGGL(neg_sum_k_kernel, dim3((unsigned)divupll((long long)m * c, 256)), dim3(256),
                     0, (hipStream_t)stream, (long long)m, k, c, in, out);
  KDPC_RETURN_LAUNCH();
}

// ------------------------------------------------------------------------------------------
// Many small copies in one launch: dst[i] <- src[i] (byte segments, each a multiple of 4
// bytes).  The graphed step packs ~240 parameter gradients into its flat gradient buffer
// and hands the ~70 prefetched plan tensors to the next replay every step; torch's
// _foreach_copy_ ran the first as 4 launches at ~0.6 TB/s (112 us for 32 MB, round-4
// trace).  Here a launch takes up to kSegs segments by value (the pointers are baked into a
// captured graph; segments < 2 GiB, < 32 GiB per launch), a thread copies one 16-byte chunk of the concatenation (4-byte words
// where a segment or its pointers are not 16-byte aligned), segment found by binary search
// over the chunk prefix sums.
namespace {
constexpr int kSegs = 128;  // 3 KiB of kernel arguments
struct Segs {
  const char* src[kSegs];
  char* dst[kSegs];
  int bytes[kSegs];
  int off[kSegs + 1];  // prefix sums of 16-byte chunks
  int n;
};

__global__ __launch_bounds__(256) void copy_segments_kernel(Segs s) {
  const int total = s.off[s.n];
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < total; c += gridDim.x * blockDim.x) {
    int lo = 0, hi = s.n - 1;  // the segment i with off[i] <= c < off[i+1]
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s.off[mid] <= c) lo = mid; else hi = mid - 1;
    }
    const long long b = (long long)(c - s.off[lo]) * 16;
    const char* src = s.src[lo] + b;
    char* dst = s.dst[lo] + b;
    const long long left = s.bytes[lo] - b;
    const bool vec = left >= 16 && ((reinterpret_cast<unsigned long long>(src) |
                                     reinterpret_cast<unsigned long long>(dst)) & 15ull) == 0;
    if (vec) {
      *reinterpret_cast<int4*>(dst) = *reinterpret_cast<const int4*>(src);
    } else {
      const int words = (int)(left < 16 ? left : 16) / 4;
      for (int w = 0; w < words; ++w)
        reinterpret_cast<int*>(dst)[w] = reinterpret_cast<const int*>(src)[w];
    }
  }
}
}  // namespace

KDPC_API int kdpc_copy_segments(int n, const void* const* src, void* const* dst,
                                const long long* bytes, void* stream) {
  KDPC_CHECK_ARG(n >= 0);
  if (n == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(src && dst && bytes);
  for (int i = 0; i < n; ++i)
    KDPC_CHECK_ARG(bytes[i] >= 0 && bytes[i] % 4 == 0 && (bytes[i] == 0 || (src[i] && dst[i])) &&
                   (reinterpret_cast<unsigned long long>(src[i]) & 3ull) == 0 &&
                   (reinterpret_cast<unsigned long long>(dst[i]) & 3ull) == 0);
  hipStream_t st = (hipStream_t)stream;
  for (int g0 = 0; g0 < n;) {
    Segs s{};
    s.off[0] = 0;
    int i = 0;
    for (; i < kSegs && g0 + i < n; ++i) {
      const long long chunks = (bytes[g0 + i] + 15) / 16;
      KDPC_CHECK_ARG(chunks < (1ll << 27));  // one segment < 2 GiB
      if ((long long)s.off[i] + chunks >= (1ll << 31)) break;  // next launch
      s.src[i] = static_cast<const char*>(src[g0 + i]);
      s.dst[i] = static_cast<char*>(dst[g0 + i]);
      s.bytes[i] = (int)bytes[g0 + i];
      s.off[i + 1] = s.off[i] + (int)chunks;
    }
    s.n = i;
    g0 += i;
    const int total = s.off[s.n];
    if (total == 0) continue;
    const int grid = (int)std::min<long long>(divupll(total, 256), 4096);
    hipLaunchKernelGGL(copy_segments_kernel, dim3(grid), dim3(256), 0, st, s);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return (int)hipSuccess;
}
