// Deterministic scatter-add (backward) kernels and point-major row gathers.
//
// The reference backward kernels (sampling_gpu.cu:46-63, group_points_gpu.cu:8-25,
// interpolate_gpu.cu:120-142) scatter with float atomicAdd: run-to-run nondeterministic,
// and on MI355X a lane-per-row f32 atomic pattern runs ~17x below the chip's atomic rate.
// Here every scatter-add is a gather-sum over an inverted index (CSR):
//   keys   = b*N + idx[b,p]   (p = flat position within batch b)
//   perm   = positions sorted by key, ascending position inside a key (stable radix sort)
//   offsets[key] = first slot of key in perm
// so grad[b,..,n] = sum of grad_out over perm[offsets[b*N+n] .. offsets[b*N+n+1]) in
// ascending position order — bit-identical to a sequential CPU accumulation, independent of
// scheduling.  One CSR serves every gradient that scatters through the same index.
#include <hipcub/hipcub.hpp>

#include "kdpc_common.h"

using namespace kdpc;

namespace {

__global__ void csr_keys_kernel(int b, int n, int p, const int* __restrict__ idx,
                                unsigned* __restrict__ keys, int* __restrict__ vals) {
  const long long total = (long long)b * p;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int bi = (int)(e / p);
    keys[e] = (unsigned)bi * (unsigned)n + (unsigned)idx[e];
    vals[e] = (int)e;
  }
}

// offsets[k] = first sorted slot with key >= k, for k in [0, B*N]
__global__ void csr_offsets_kernel(long long total, unsigned nkeys,
                                   const unsigned* __restrict__ keys_sorted,
                                   int* __restrict__ offsets) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i <= total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long kprev = i == 0 ? -1 : (long long)keys_sorted[i - 1];
    const long long kcur = i == total ? (long long)nkeys : (long long)keys_sorted[i];
    for (long long k = kprev + 1; k <= kcur; ++k) offsets[k] = (int)i;
  }
}

inline int grid_for(long long total, int block) {
  long long g = divupll(total, block);
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

inline int bits_for(unsigned long long v) {
  int bits = 1;
  while (bits < 32 && (1ull << bits) <= v) ++bits;
  return bits;
}

struct CsrLayout {
  size_t keys_in, keys_out, vals_in, cub, total;
};

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

hipError_t csr_layout(int b, int n, int p, CsrLayout* L) {
  const long long items = (long long)b * p;
  size_t cub_bytes = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(
      nullptr, cub_bytes, (const unsigned*)nullptr, (unsigned*)nullptr, (const int*)nullptr,
      (int*)nullptr, (int)items, 0, bits_for((unsigned long long)b * n), (hipStream_t)0);
  if (e != hipSuccess) return e;
  L->keys_in = 0;
  L->keys_out = align256(sizeof(unsigned) * items);
  L->vals_in = L->keys_out + align256(sizeof(unsigned) * items);
  L->cub = L->vals_in + align256(sizeof(int) * items);
  L->total = L->cub + align256(cub_bytes);
  return hipSuccess;
}

hipError_t csr_build(int b, int n, int p, const int* idx, void* ws, size_t ws_bytes, int* offsets,
                     int* perm, hipStream_t st) {
  CsrLayout L;
  hipError_t e = csr_layout(b, n, p, &L);
  if (e != hipSuccess) return e;
  if (ws_bytes < L.total) return hipErrorInvalidValue;
  char* base = (char*)ws;
  unsigned* keys_in = (unsigned*)(base + L.keys_in);
  unsigned* keys_out = (unsigned*)(base + L.keys_out);
  int* vals_in = (int*)(base + L.vals_in);
  void* cub_tmp = base + L.cub;
  size_t cub_bytes = L.total - L.cub;
  const long long items = (long long)b * p;
  hipLaunchKernelGGL(csr_keys_kernel, dim3(grid_for(items, 256)), dim3(256), 0, st, b, n, p, idx,
                     keys_in, vals_in);
  e = hipcub::DeviceRadixSort::SortPairs(cub_tmp, cub_bytes, keys_in, keys_out, vals_in, perm,
                                         (int)items, 0, bits_for((unsigned long long)b * n), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(csr_offsets_kernel, dim3(grid_for(items + 1, 256)), dim3(256), 0, st, items,
                     (unsigned)((unsigned long long)b * n), keys_out, offsets);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// channel-major gather-sums, one thread per (b, c, n), n fastest.
// grad[b,c,n] = sum_{j in seg(b,n)} src[b, c, pos(perm[j])]
__global__ __launch_bounds__(256) void csr_sum_cm_kernel(int b, int c, int n, int p,
                                                         const float* __restrict__ src,
                                                         const int* __restrict__ offsets,
                                                         const int* __restrict__ perm,
                                                         float* __restrict__ dst) {
  const long long total = (long long)b * c * n;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int ni = (int)(e % n);
    const long long bc = e / n;
    const int bi = (int)(bc / c);
    const long long key = (long long)bi * n + ni;
    const int j0 = offsets[key], j1 = offsets[key + 1];
    const float* s = src + bc * p - (long long)bi * p;  // src row (b,c) minus batch offset
    float acc = 0.f;
    for (int j = j0; j < j1; ++j) acc = __fadd_rn(acc, s[perm[j]]);
    dst[e] = acc;
  }
}

// LDS-staged channel-major gather-sum for P <= 40960: one workgroup per (b, c) stages the
// whole gradient row src[b,c,:] (coalesced float4, read exactly once from HBM) and then
// walks the CSR segments of every n reading LDS; the result row is written coalesced.
// Same ascending-position summation order as csr_sum_cm_kernel (bit-identical results).
constexpr int kSumRowLdsBytes = 160 * 1024;

__global__ __launch_bounds__(256) void csr_sum_cm_lds_kernel(int c, int n, int p,
                                                             const float* __restrict__ src,
                                                             const int* __restrict__ offsets,
                                                             const int* __restrict__ perm,
                                                             float* __restrict__ dst) {
  extern __shared__ __attribute__((aligned(16))) float row[];  // [p]
  const int ci = blockIdx.x;
  const int bi = blockIdx.y;
  const float* s = src + ((long long)bi * c + ci) * p;
  if ((p & 3) == 0) {
    for (int e = threadIdx.x * 4; e < p; e += 256 * 4)
      *reinterpret_cast<float4*>(row + e) = *reinterpret_cast<const float4*>(s + e);
  } else {
    for (int e = threadIdx.x; e < p; e += 256) row[e] = s[e];
  }
  __syncthreads();
  const int* off = offsets + (long long)bi * n;
  const int base = bi * p;
  float* d = dst + ((long long)bi * c + ci) * n;
  for (int ni = threadIdx.x; ni < n; ni += 256) {
    const int j0 = off[ni], j1 = off[ni + 1];
    float acc = 0.f;
    for (int j = j0; j < j1; ++j) acc = __fadd_rn(acc, row[perm[j] - base]);
    d[ni] = acc;
  }
}

// three_interpolate_grad: positions are (n,t) of idx (B,N,3); contribution g[b,c,n]*w[b,n,t]
__global__ __launch_bounds__(256) void csr_sum_interp_kernel(int b, int c, int n, int m,
                                                             const float* __restrict__ grad_out,
                                                             const float* __restrict__ weight,
                                                             const int* __restrict__ offsets,
                                                             const int* __restrict__ perm,
                                                             float* __restrict__ dst) {
  const long long total = (long long)b * c * m;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int mi = (int)(e % m);
    const long long bc = e / m;
    const int bi = (int)(bc / c);
    const long long key = (long long)bi * m + mi;
    const int j0 = offsets[key], j1 = offsets[key + 1];
    const float* g = grad_out + bc * n;
    float acc = 0.f;
    for (int j = j0; j < j1; ++j) {
      const int gp = perm[j];                    // global position b*3N + n*3 + t
      const int local = gp - bi * 3 * n;
      acc = __fadd_rn(acc, __fmul_rn(g[local / 3], weight[gp]));
    }
    dst[e] = acc;
  }
}

// ---------------------------------------------------------------------------------------
// point-major rows: out[b,p,:] = points[b, idx[b,p], :]   (B,N,C) -> (B,P,C)
template <int V>
__global__ __launch_bounds__(256) void group_rows_kernel(int b, int n, int c, int p,
                                                         const float* __restrict__ points,
                                                         const int* __restrict__ idx,
                                                         float* __restrict__ out) {
  const int cv = c / V;
  const long long total = (long long)b * p * cv;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % cv);
    const long long row = e / cv;  // b*p + pos
    const int bi = (int)(row / p);
    const long long src_row = (long long)bi * n + idx[row];
    if (V == 4) {
      reinterpret_cast<float4*>(out)[e] =
          reinterpret_cast<const float4*>(points)[src_row * cv + ch];
    } else {
      out[e] = points[src_row * c + ch];
    }
  }
}

// grad_points[b,n,:] = sum over seg(b,n) of grad_out[pos,:]  (rows, ascending position)
template <int V>
__global__ __launch_bounds__(256) void csr_sum_rows_kernel(int b, int n, int c,
                                                           const float* __restrict__ grad_out,
                                                           const int* __restrict__ offsets,
                                                           const int* __restrict__ perm,
                                                           float* __restrict__ dst) {
  const int cv = c / V;
  const long long total = (long long)b * n * cv;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % cv);
    const long long key = e / cv;  // b*n + ni
    const int j0 = offsets[key], j1 = offsets[key + 1];
    if (V == 4) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int j = j0; j < j1; ++j) {
        const float4 v = reinterpret_cast<const float4*>(grad_out)[(long long)perm[j] * cv + ch];
        acc.x = __fadd_rn(acc.x, v.x);
        acc.y = __fadd_rn(acc.y, v.y);
        acc.z = __fadd_rn(acc.z, v.z);
        acc.w = __fadd_rn(acc.w, v.w);
      }
      reinterpret_cast<float4*>(dst)[e] = acc;
    } else {
      float acc = 0.f;
      for (int j = j0; j < j1; ++j) acc = __fadd_rn(acc, grad_out[(long long)perm[j] * c + ch]);
      dst[e] = acc;
    }
  }
}

// Workspace of the reference-shaped grad entry points: [CSR build scratch | offsets (B*N+1)
// | perm (B*P)].  The *_ws variants take it from the caller; the reference-signature ones
// (no workspace argument) take it from the stream-ordered allocator on their own stream
// (hipMallocAsync / hipFreeAsync): no library-global state, safe across threads and
// streams, and the allocation is ordered with the kernels that use it.
struct GradWs {
  size_t csr, off, perm, total;
};

hipError_t grad_ws_layout(int b, int n, int p, GradWs* L) {
  CsrLayout C;
  hipError_t e = csr_layout(b, n, p, &C);
  if (e != hipSuccess) return e;
  L->csr = C.total;
  L->off = align256(sizeof(int) * ((size_t)b * n + 1));
  L->perm = align256(sizeof(int) * (size_t)b * p);
  L->total = L->csr + L->off + L->perm;
  return hipSuccess;
}

// builds the CSR of idx (B,P) over [0,N) inside ws; -> offsets / perm pointers into ws
hipError_t ws_csr(int b, int n, int p, const int* idx, void* ws, size_t ws_bytes, hipStream_t st,
                  int** offsets, int** perm) {
  GradWs L;
  hipError_t e = grad_ws_layout(b, n, p, &L);
  if (e != hipSuccess) return e;
  if (!ws || ws_bytes < L.total) return hipErrorInvalidValue;
  *offsets = (int*)((char*)ws + L.csr);
  *perm = (int*)((char*)ws + L.csr + L.off);
  return csr_build(b, n, p, idx, ws, L.csr, *offsets, *perm, st);
}

}  // namespace

// ----------------------------------------------------------------------------- CSR API
KDPC_API size_t kdpc_csr_workspace_bytes(int b, int n, int p) {
  if (b <= 0 || n <= 0 || p <= 0) return 0;
  CsrLayout L;
  if (csr_layout(b, n, p, &L) != hipSuccess) return 0;
  return L.total;
}

// Build the inverted index of idx (B,P) with values in [0,N): offsets (B*N+1), perm (B*P).
KDPC_API int kdpc_csr_build(int b, int n, int p, const int* idx, void* workspace,
                            size_t workspace_bytes, int* offsets, int* perm, void* stream) {
  KDPC_CHECK_ARG(b > 0 && n > 0 && p > 0 && idx && workspace && offsets && perm);
  KDPC_CHECK_ARG((unsigned long long)b * n < (1ull << 31) && (long long)b * p < (1ll << 31));
  return (int)csr_build(b, n, p, idx, workspace, workspace_bytes, offsets, perm,
                        (hipStream_t)stream);
}

// (B,C,P) channel-major source -> (B,C,N): serves group_points_grad and gather_points_grad
KDPC_API int kdpc_csr_sum_channels(int b, int c, int n, int p, const float* src,
                                   const int* offsets, const int* perm, float* dst,
                                   void* stream) {
  KDPC_CHECK_ARG(b >= 0 && c >= 0 && n > 0 && p >= 0);
  const long long total = (long long)b * c * n;
  if (total == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(dst && offsets && (p == 0 || (src && perm)));
  if (p > 0 && (size_t)p * sizeof(float) <= kSumRowLdsBytes && c <= 65535 && b <= 65535) {
    // once per process (thread-safe static initialisation)
    static const hipError_t attr = hipFuncSetAttribute(
        (const void*)csr_sum_cm_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
        kSumRowLdsBytes);
    if (attr != hipSuccess) return (int)attr;
    hipLaunchKernelGGL(csr_sum_cm_lds_kernel, dim3(c, b), dim3(256), (size_t)p * sizeof(float),
                       (hipStream_t)stream, c, n, p, src, offsets, perm, dst);
    KDPC_RETURN_LAUNCH();
  }
  hipLaunchKernelGGL(csr_sum_cm_kernel, dim3(grid_for(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, b, c, n, p, src, offsets, perm, dst);
  KDPC_RETURN_LAUNCH();
}

KDPC_API int kdpc_three_interpolate_grad_csr(int b, int c, int n, int m, const float* grad_out,
                                             const float* weight, const int* offsets,
                                             const int* perm, float* grad_points, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && c >= 0 && n >= 0 && m > 0);
  const long long total = (long long)b * c * m;
  if (total == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(grad_points && offsets && (n == 0 || (grad_out && weight && perm)));
  hipLaunchKernelGGL(csr_sum_interp_kernel, dim3(grid_for(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, b, c, n, m, grad_out, weight, offsets, perm,
                     grad_points);
  KDPC_RETURN_LAUNCH();
}

// Point-major row gather (B,N,C) x (B,P) -> (B,P,C): the layout pointconv_util's
// index_points_group returns, produced directly (no permute/contiguous round trips).
KDPC_API int kdpc_group_rows(int b, int n, int c, int p, const float* points, const int* idx,
                             float* out, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n > 0 && c >= 0 && p >= 0);
  if ((long long)b * p * c == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(points && idx && out);
  hipStream_t st = (hipStream_t)stream;
  const bool v4 = (c % 4) == 0 && ((uintptr_t)points % 16) == 0 && ((uintptr_t)out % 16) == 0;
  if (v4) {
    const long long total = (long long)b * p * (c / 4);
    hipLaunchKernelGGL(group_rows_kernel<4>, dim3(grid_for(total, 256)), dim3(256), 0, st, b, n,
                       c, p, points, idx, out);
  } else {
    const long long total = (long long)b * p * c;
    hipLaunchKernelGGL(group_rows_kernel<1>, dim3(grid_for(total, 256)), dim3(256), 0, st, b, n,
                       c, p, points, idx, out);
  }
  KDPC_RETURN_LAUNCH();
}

KDPC_API int kdpc_group_rows_grad_csr(int b, int n, int c, const float* grad_out,
                                      const int* offsets, const int* perm, float* grad_points,
                                      void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n > 0 && c >= 0);
  if ((long long)b * n * c == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(grad_out && offsets && perm && grad_points);
  hipStream_t st = (hipStream_t)stream;
  const bool v4 =
      (c % 4) == 0 && ((uintptr_t)grad_out % 16) == 0 && ((uintptr_t)grad_points % 16) == 0;
  if (v4) {
    const long long total = (long long)b * n * (c / 4);
    hipLaunchKernelGGL(csr_sum_rows_kernel<4>, dim3(grid_for(total, 256)), dim3(256), 0, st, b, n,
                       c, grad_out, offsets, perm, grad_points);
  } else {
    const long long total = (long long)b * n * c;
    hipLaunchKernelGGL(csr_sum_rows_kernel<1>, dim3(grid_for(total, 256)), dim3(256), 0, st, b, n,
                       c, grad_out, offsets, perm, grad_points);
  }
  KDPC_RETURN_LAUNCH();
}

// ------------------------------------------- reference-shaped grad entry points (no CSR arg)
KDPC_API size_t kdpc_grad_workspace_bytes(int b, int n, int p) {
  if (b <= 0 || n <= 0 || p <= 0) return 0;
  GradWs L;
  return grad_ws_layout(b, n, p, &L) == hipSuccess ? L.total : 0;
}

KDPC_API int kdpc_gather_points_grad_ws(int b, int c, int n, int npoints, const float* grad_out,
                                        const int* idx, float* grad_points, void* workspace,
                                        size_t workspace_bytes, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && c >= 0 && n > 0 && npoints >= 0);
  if ((long long)b * c * n == 0) return (int)hipSuccess;
  hipStream_t st = (hipStream_t)stream;
  if (npoints == 0) return (int)hipMemsetAsync(grad_points, 0, sizeof(float) * b * c * n, st);
  KDPC_CHECK_ARG(grad_out && idx && grad_points);
  int *offsets, *perm;
  hipError_t e = ws_csr(b, n, npoints, idx, workspace, workspace_bytes, st, &offsets, &perm);
  if (e != hipSuccess) return (int)e;
  return kdpc_csr_sum_channels(b, c, n, npoints, grad_out, offsets, perm, grad_points, stream);
}

KDPC_API int kdpc_group_points_grad_ws(int b, int c, int n, int npoints, int nsample,
                                       const float* grad_out, const int* idx, float* grad_points,
                                       void* workspace, size_t workspace_bytes, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && c >= 0 && n > 0 && npoints >= 0 && nsample >= 0);
  if ((long long)b * c * n == 0) return (int)hipSuccess;
  hipStream_t st = (hipStream_t)stream;
  const int p = npoints * nsample;
  if (p == 0) return (int)hipMemsetAsync(grad_points, 0, sizeof(float) * b * c * n, st);
  KDPC_CHECK_ARG(grad_out && idx && grad_points);
  int *offsets, *perm;
  hipError_t e = ws_csr(b, n, p, idx, workspace, workspace_bytes, st, &offsets, &perm);
  if (e != hipSuccess) return (int)e;
  return kdpc_csr_sum_channels(b, c, n, p, grad_out, offsets, perm, grad_points, stream);
}

KDPC_API int kdpc_three_interpolate_grad_ws(int b, int c, int n, int m, const float* grad_out,
                                            const int* idx, const float* weight,
                                            float* grad_points, void* workspace,
                                            size_t workspace_bytes, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && c >= 0 && n >= 0 && m > 0);
  if ((long long)b * c * m == 0) return (int)hipSuccess;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) return (int)hipMemsetAsync(grad_points, 0, sizeof(float) * b * c * m, st);
  KDPC_CHECK_ARG(grad_out && idx && weight && grad_points);
  int *offsets, *perm;
  hipError_t e = ws_csr(b, m, n * 3, idx, workspace, workspace_bytes, st, &offsets, &perm);
  if (e != hipSuccess) return (int)e;
  return kdpc_three_interpolate_grad_csr(b, c, n, m, grad_out, weight, offsets, perm, grad_points,
                                         stream);
}

namespace {
// run fn(workspace, bytes) with a stream-ordered temporary of `bytes` on st
template <class F>
int with_stream_ws(size_t bytes, hipStream_t st, F fn) {
  void* ws = nullptr;
  hipError_t e = hipMallocAsync(&ws, bytes, st);
  if (e != hipSuccess) return (int)e;
  const int r = fn(ws, bytes);
  e = hipFreeAsync(ws, st);
  return r != 0 ? r : (int)e;
}
}  // namespace

// Reference: gather_points_grad_wrapper(b, c, n, npoints, grad_out, idx, grad_points)
KDPC_API int kdpc_gather_points_grad(int b, int c, int n, int npoints, const float* grad_out,
                                     const int* idx, float* grad_points, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && c >= 0 && n > 0 && npoints >= 0);
  if ((long long)b * c * n * npoints == 0)
    return kdpc_gather_points_grad_ws(b, c, n, npoints, grad_out, idx, grad_points, nullptr, 0,
                                      stream);
  return with_stream_ws(kdpc_grad_workspace_bytes(b, n, npoints), (hipStream_t)stream,
                        [&](void* ws, size_t nb) {
                          return kdpc_gather_points_grad_ws(b, c, n, npoints, grad_out, idx,
                                                            grad_points, ws, nb, stream);
                        });
}

// Reference: group_points_grad_wrapper(b, c, n, npoints, nsample, grad_out, idx, grad_points)
KDPC_API int kdpc_group_points_grad(int b, int c, int n, int npoints, int nsample,
                                    const float* grad_out, const int* idx, float* grad_points,
                                    void* stream) {
  KDPC_CHECK_ARG(b >= 0 && c >= 0 && n > 0 && npoints >= 0 && nsample >= 0);
  const long long p = (long long)npoints * nsample;
  if ((long long)b * c * n * p == 0)
    return kdpc_group_points_grad_ws(b, c, n, npoints, nsample, grad_out, idx, grad_points,
                                     nullptr, 0, stream);
  return with_stream_ws(kdpc_grad_workspace_bytes(b, n, (int)p), (hipStream_t)stream,
                        [&](void* ws, size_t nb) {
                          return kdpc_group_points_grad_ws(b, c, n, npoints, nsample, grad_out,
                                                           idx, grad_points, ws, nb, stream);
                        });
}

// Reference: three_interpolate_grad_wrapper(b, c, n, m, grad_out, idx, weight, grad_points)
KDPC_API int kdpc_three_interpolate_grad(int b, int c, int n, int m, const float* grad_out,
                                         const int* idx, const float* weight, float* grad_points,
                                         void* stream) {
  KDPC_CHECK_ARG(b >= 0 && c >= 0 && n >= 0 && m > 0);
  if ((long long)b * c * m * n == 0)
    return kdpc_three_interpolate_grad_ws(b, c, n, m, grad_out, idx, weight, grad_points,
                                          nullptr, 0, stream);
  return with_stream_ws(kdpc_grad_workspace_bytes(b, m, n * 3), (hipStream_t)stream,
                        [&](void* ws, size_t nb) {
                          return kdpc_three_interpolate_grad_ws(b, c, n, m, grad_out, idx, weight,
                                                                grad_points, ws, nb, stream);
                        });
}
