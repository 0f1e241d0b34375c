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
#include <type_traits>

#include "kdpc_common.h"

using namespace kdpc;

namespace {

__device__ __forceinline__ float vadd(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float4 vadd(float4 a, float4 b) {
  return make_float4(__fadd_rn(a.x, b.x), __fadd_rn(a.y, b.y), __fadd_rn(a.z, b.z),
                     __fadd_rn(a.w, b.w));
}

// CSR build = a counting sort by key (b*N + idx) that keeps ascending position inside a key:
//   memset (two count arrays) -> count (integer atomics) -> exclusive scan (hipcub,
//   single-pass decoupled look-back) -> fill (slot = offset + an atomic per-key counter:
//   every position lands in its key's segment, in arbitrary order) -> segment rank sort
//   (one wave per key), which restores ascending position order.
// ~6 launches and ~3 passes over the index, against ~10 launches of rocprim's radix /
// merge sort (round 1: 19 builds per training step, 1.5 ms).  The result is exactly the
// stable sort's, so every gather-sum through it is bit-identical to before.  Indices
// outside [0, N) are left out of every segment (the reference had no bounds check).
// grid (position blocks, batch): no per-element division
__global__ __launch_bounds__(256) void csr_count_kernel(int n, int p, const int* __restrict__ idx,
                                                        int* __restrict__ cnt) {
  const int b = blockIdx.y;
  const int* row = idx + (long long)b * p;
  int* c = cnt + (long long)b * n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < p; i += gridDim.x * blockDim.x) {
    const int v = row[i];
    if ((unsigned)v < (unsigned)n) atomicAdd(&c[v], 1);
  }
}

__global__ __launch_bounds__(256) void csr_fill_kernel(int n, int p, const int* __restrict__ idx,
                                                       const int* __restrict__ offsets,
                                                       int* __restrict__ fill,
                                                       int* __restrict__ perm) {
  const int b = blockIdx.y;
  const int* row = idx + (long long)b * p;
  const long long kb = (long long)b * n;
  const int e0 = b * p;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < p; i += gridDim.x * blockDim.x) {
    const int v = row[i];
    if ((unsigned)v < (unsigned)n) perm[offsets[kb + v] + atomicAdd(&fill[kb + v], 1)] = e0 + i;
  }
}

// one wave per key (grid-stride): put the key's segment of perm in ascending order.
//  * up to 64 * kHold entries: positions are distinct, so slot(x) = #{y in segment : y < x};
//    each lane holds up to kHold entries and every entry is broadcast once (readlane): a
//    segment of L entries costs L steps.  All entries are in registers before any store, so
//    the segment is rewritten in place.
//  * longer segments (in-degree > 256: a hub point, or degenerate input such as duplicated
//    points): the wave scans its batch's index row in order and appends every position that
//    maps to the key (ballot + popcount), P / 64 steps whatever L is.
constexpr int kHold = 4;
__global__ __launch_bounds__(256) void csr_segsort_kernel(long long m, int n, int p,
                                                          const int* __restrict__ idx,
                                                          const int* __restrict__ offsets,
                                                          int* __restrict__ perm) {
  const int lane = threadIdx.x & 63;
  const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long long nwaves = ((long long)gridDim.x * blockDim.x) >> 6;
  for (long long key = wave; key < m; key += nwaves) {
    const int o0 = offsets[key], len = offsets[key + 1] - o0;
    if (len <= 1) continue;
    int* seg = perm + o0;
    if (len <= 64 * kHold) {
      int x[kHold], rank[kHold];
#pragma unroll
      for (int h = 0; h < kHold; ++h) {
        const int i = lane + 64 * h;
        x[h] = i < len ? seg[i] : 0x7fffffff;
        rank[h] = 0;
      }
#pragma unroll
      for (int h2 = 0; h2 < kHold; ++h2) {
        if (64 * h2 >= len) break;
        const int lim = min(64, len - 64 * h2);
        for (int j = 0; j < lim; ++j) {
          const int y = __builtin_amdgcn_readlane(x[h2], j);
#pragma unroll
          for (int h = 0; h < kHold; ++h) rank[h] += y < x[h] ? 1 : 0;
        }
      }
#pragma unroll
      for (int h = 0; h < kHold; ++h)
        if (lane + 64 * h < len) seg[rank[h]] = x[h];
    } else {
      const long long b = key / n;
      const int v = (int)(key - b * n);
      const long long e0 = b * p;
      int out = 0;
      for (int i0 = 0; i0 < p; i0 += 64) {
        const int i = i0 + lane;
        const bool hit = i < p && idx[e0 + i] == v;
        const unsigned long long mask = __ballot(hit);
        if (hit) {
          const int before = __popcll(mask & ((1ull << lane) - 1ull));
          seg[out + before] = (int)(e0 + i);
        }
        out += __popcll(mask);
      }
    }
  }
}

// CSR build for key spaces that fit in LDS (n <= kLdsKeys per batch): one 1024-thread
// workgroup per batch element counts its index row into an LDS histogram (LDS atomics:
// no device-scope atomics, which ran at ~27 G/s for the 4.2 M-entry cost-volume index),
// scans it in LDS, and later fills the segments from LDS cursors.  Two launches replace the
// memset / count / scan (2) / fill chain; the segment rank sort stays (LDS cursors hand out
// slots in arbitrary order inside a key, exactly like the global-atomic fill).
constexpr int kLdsKeys = 15872;  // histogram ints per workgroup (<= 62 KiB of LDS)
constexpr int kLdsThreads = 1024;

// inclusive block scan of one int per thread (1024 threads = 16 waves); -> block total
__device__ __forceinline__ int block_incl_scan(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  if (lane == 63) wsum[wv] = v;
  __syncthreads();
  if (wv == 0) {
    int w = lane < kLdsThreads / 64 ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int u = __shfl_up(w, o, 64);
      if (lane >= o) w += u;
    }
    if (lane < kLdsThreads / 64) wsum[lane] = w;
  }
  __syncthreads();
  const int add = wv > 0 ? wsum[wv - 1] : 0;
  *total = wsum[kLdsThreads / 64 - 1];
  return v + add;
}

// per batch b: histogram of idx[b,:] over [0,n), its exclusive scan -> offsets[b*n + k]
// (batch-local; csr_lds_fill adds the batch's base), and the batch's valid count -> tot[b]
__global__ __launch_bounds__(kLdsThreads) void csr_lds_count_kernel(int n, int p,
                                                                    const int* __restrict__ idx,
                                                                    int* __restrict__ offsets,
                                                                    int* __restrict__ tot) {
  extern __shared__ int h[];  // n histogram ints + 16 wave sums
  int* wsum = h + n;
  const int b = blockIdx.x, t = threadIdx.x;
  const int* row = idx + (long long)b * p;
  for (int k = t; k < n; k += kLdsThreads) h[k] = 0;
  __syncthreads();
  int i = t;
  for (; i + 3 * kLdsThreads < p; i += 4 * kLdsThreads) {  // four loads in flight
    int v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = row[i + u * kLdsThreads];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if ((unsigned)v[u] < (unsigned)n) atomicAdd(&h[v[u]], 1);
  }
  for (; i < p; i += kLdsThreads) {
    const int v = row[i];
    if ((unsigned)v < (unsigned)n) atomicAdd(&h[v], 1);
  }
  __syncthreads();
  // thread t owns keys [t*E, t*E + E): its block sum, the block scan, then the running sum
  const int E = (n + kLdsThreads - 1) / kLdsThreads;
  const int k0 = t * E, k1 = min(n, k0 + E);
  int s = 0;
  for (int k = k0; k < k1; ++k) s += h[k];
  int total;
  int run = block_incl_scan(s, wsum, &total) - s;
  int* off = offsets + (long long)b * n;
  for (int k = k0; k < k1; ++k) {
    const int c = h[k];
    off[k] = run;
    run += c;
  }
  if (t == 0) tot[b] = total;
}

// per batch b: base = valid positions of batches < b; final offsets; fill from LDS cursors
__global__ __launch_bounds__(kLdsThreads) void csr_lds_fill_kernel(int n, int p, int nb,
                                                                   const int* __restrict__ idx,
                                                                   int* __restrict__ offsets,
                                                                   const int* __restrict__ tot,
                                                                   int* __restrict__ perm) {
  extern __shared__ int cur[];  // n cursors + 16 wave sums
  int* wsum = cur + n;
  const int b = blockIdx.x, t = threadIdx.x;
  int part = 0;
  for (int j = t; j < b; j += kLdsThreads) part += tot[j];
  int base;
  block_incl_scan(part, wsum, &base);
  int* off = offsets + (long long)b * n;
  for (int k = t; k < n; k += kLdsThreads) {
    const int o = off[k] + base;
    off[k] = o;
    cur[k] = o;
  }
  if (b == nb - 1 && t == 0) offsets[(long long)nb * n] = base + tot[b];
  __syncthreads();
  const int* row = idx + (long long)b * p;
  const int e0 = b * p;
  for (int i = t; i < p; i += kLdsThreads) {
    const int v = row[i];
    if ((unsigned)v < (unsigned)n) perm[atomicAdd(&cur[v], 1)] = e0 + i;
  }
}

// rank[i] = the CSR slot of position i (perm[rank[i]] == i), -1 for an index outside
// [0, n) (in no segment).  One thread per position: the slots in [0, offsets[b*n]) scatter
// their position, the out-of-range positions mark themselves.
__global__ __launch_bounds__(256) void csr_rank_kernel(long long total, int n,
                                                       const int* __restrict__ idx,
                                                       const int* __restrict__ perm,
                                                       const int* __restrict__ end,
                                                       int* __restrict__ rank) {
  const long long valid = *end;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    if (i < valid) rank[perm[i]] = (int)i;
    if ((unsigned)idx[i] >= (unsigned)n) rank[i] = -1;
  }
}

inline int grid_for(long long total, int block) {
  long long g = divupll(total, block);
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

struct CsrLayout {
  size_t cnt, fill, scan, scan_bytes, total;  // byte offsets into the workspace
};

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

hipError_t csr_layout(int b, int n, int p, CsrLayout* L) {
  (void)p;
  const long long m = (long long)b * n;
  size_t scan_bytes = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, (const int*)nullptr,
                                                  (int*)nullptr, (int)(m + 1), (hipStream_t)0);
  if (e != hipSuccess) return e;
  L->cnt = 0;                                  // m + 1 counts (the last stays 0)
  L->fill = (size_t)(m + 1) * sizeof(int);     // m per-key fill counters
  L->scan = align256(L->fill + (size_t)m * sizeof(int));
  L->scan_bytes = scan_bytes;
  L->total = L->scan + align256(scan_bytes);
  return hipSuccess;
}

hipError_t csr_build(int b, int n, int p, const int* idx, void* ws, size_t ws_bytes, int* offsets,
                     int* perm, hipStream_t st) {
  CsrLayout L;
  hipError_t e = csr_layout(b, n, p, &L);
  if (e != hipSuccess) return e;
  if (ws_bytes < L.total) return hipErrorInvalidValue;
  char* base = reinterpret_cast<char*>(ws);
  int* cnt = reinterpret_cast<int*>(base + L.cnt);
  int* fill = reinterpret_cast<int*>(base + L.fill);
  const long long m = (long long)b * n;
  const int sgrid = (int)std::min<long long>(divupll(m, 4), 8192);  // 4 waves per workgroup
  if (n <= kLdsKeys) {  // LDS histogram path (cnt holds the per-batch totals)
    const size_t lds = (size_t)(n + 16) * sizeof(int);
    hipLaunchKernelGGL(csr_lds_count_kernel, dim3(b), dim3(kLdsThreads), lds, st, n, p, idx,
                       offsets, cnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(csr_lds_fill_kernel, dim3(b), dim3(kLdsThreads), lds, st, n, p, b, idx,
                       offsets, cnt, perm);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(csr_segsort_kernel, dim3(sgrid), dim3(256), 0, st, m, n, p, idx, offsets,
                       perm);
    return hipGetLastError();
  }
  if ((e = hipMemsetAsync(cnt, 0, L.fill + sizeof(int) * m, st)) != hipSuccess) return e;
  const dim3 pgrid((unsigned)std::min(divup(p, 256), std::max(1, 4096 / b)), (unsigned)b);
  hipLaunchKernelGGL(csr_count_kernel, pgrid, dim3(256), 0, st, n, p, idx, cnt);
  size_t scan_bytes = L.scan_bytes;
  e = hipcub::DeviceScan::ExclusiveSum(base + L.scan, scan_bytes, cnt, offsets, (int)(m + 1), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(csr_fill_kernel, pgrid, dim3(256), 0, st, n, p, idx, offsets, fill, perm);
  hipLaunchKernelGGL(csr_segsort_kernel, dim3(sgrid), dim3(256), 0, st, m, n, p, idx, offsets,
                     perm);
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
// The segment walk is unrolled kU wide: the kU perm entries, then the kU rows, are loaded
// before the adds (which stay in ascending order), so a segment of L rows costs ~2 L / kU
// dependent memory latencies instead of 2 L (round 1: one perm load -> one row load -> add
// per neighbour, latency-bound at ~40 us for the level-0 gradients).
constexpr int kU = 8;

template <int V>
__global__ __launch_bounds__(256) void csr_sum_rows_kernel(int b, int n, int c,
                                                           const float* __restrict__ grad_out,
                                                           const int* __restrict__ offsets,
                                                           const int* __restrict__ perm,
                                                           float* __restrict__ dst) {
  using vec = typename std::conditional<V == 4, float4, float>::type;
  const int cv = c / V;
  const long long total = (long long)b * n * cv;
  const vec* src = reinterpret_cast<const vec*>(grad_out);
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long key = e / cv;  // b*n + ni
    const int ch = (int)(e - key * cv);
    const int j0 = offsets[key], j1 = offsets[key + 1];
    vec acc{};
    int j = j0;
    for (; j + kU <= j1; j += kU) {
      int pj[kU];
      vec v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) pj[u] = perm[j + u];
#pragma unroll
      for (int u = 0; u < kU; ++u) v[u] = src[(long long)pj[u] * cv + ch];
#pragma unroll
      for (int u = 0; u < kU; ++u) acc = vadd(acc, v[u]);
    }
    for (; j < j1; ++j) acc = vadd(acc, src[(long long)perm[j] * cv + ch]);
    reinterpret_cast<vec*>(dst)[e] = acc;
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
  KDPC_CHECK_ARG(b > 0 && b <= 65535 && n > 0 && p > 0 && idx && workspace && offsets && perm);
  KDPC_CHECK_ARG((unsigned long long)b * n < (1ull << 31) && (long long)b * p < (1ll << 31));
  return (int)csr_build(b, n, p, idx, workspace, workspace_bytes, offsets, perm,
                        (hipStream_t)stream);
}

// (B,C,P) channel-major source -> (B,C,N): serves group_points_grad and gather_points_grad
// Inverse of the CSR permutation: rank (B*P) with perm[rank[i]] == i, -1 where idx[i] is
// outside [0, n).  offsets / perm from kdpc_csr_build of the same idx.
KDPC_API int kdpc_csr_rank(int b, int n, int p, const int* idx, const int* offsets,
                           const int* perm, int* rank, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n > 0 && p >= 0);
  const long long total = (long long)b * p;
  if (total == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(idx && offsets && perm && rank);
  hipLaunchKernelGGL(csr_rank_kernel, dim3(grid_for(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, total, n, idx, perm, offsets + (long long)b * n, rank);
  KDPC_RETURN_LAUNCH();
}

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
