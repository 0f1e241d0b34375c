// Forward kernels behind the reference's pointnet2_cuda API (channel-major (B,C,N)
// features, point-major (B,N,3) xyz, int32 indices).  Backward kernels live in
// scatter.hip (deterministic CSR reductions instead of the reference's float atomics).
#include "kdpc_common.h"

using namespace kdpc;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------
// gather_points: out[b,c,m] = points[b,c,idx[b,m]]        (reference sampling_gpu.cu:8-24)
//
// LDS-staged (kGatherRowLds: rows of N <= 20480): a workgroup owns ONE channel row of one
// cloud.  It issues its output indices (int4) first, then stages the whole row in LDS by
// direct global -> LDS loads, every one in flight at once (a row is read from HBM exactly
// once, as coalesced 16-byte loads: with M/N = 1/4 every cache line of the row holds an
// index anyway), and writes its M outputs as nontemporal float4 stores from random LDS reads.
// The random 4-byte global gathers of the direct kernel (one L2 request per output) are gone.
// Workgroups walk (cloud, channel) with the channel fastest, so the C rows that share one
// index slice run back to back and re-read it from L2.
constexpr int kGatherOut = 4;     // int4 index loads (16 outputs) in flight per thread
constexpr int kGatherRowLds = 80 * 1024;

__global__ __launch_bounds__(256) void gather_points_lds_kernel(int c, int n, int m,
                                                                const float* __restrict__ points,
                                                                const int* __restrict__ idx,
                                                                float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float row[];
  const long long bc = blockIdx.x;             // b * c + channel
  const int bi = (int)(bc / c);
  const int* ib = idx + (long long)bi * m;     // m % 4 == 0 (host-checked)
  float* ob = out + bc * m;
  const int t = threadIdx.x;
  int4 q[kGatherOut];
#pragma unroll
  for (int u = 0; u < kGatherOut; ++u) {
    const int p = (t + u * 256) * 4;
    q[u] = p < m ? *reinterpret_cast<const int4*>(ib + p) : make_int4(0, 0, 0, 0);
  }
  const f32x4* src = reinterpret_cast<const f32x4*>(points + bc * n);  // n % 4 == 0
  f32x4* dst = reinterpret_cast<f32x4*>(row);
  const int n4 = n >> 2;
  // the row goes straight from memory into LDS (global_load_lds, 16 bytes per lane: a wave's
  // 64 lanes fill 1 KB at the wave's LDS base): no register round trip and no ds_write pass
  // (gather C=64 standalone 3.21 -> 2.72 us per launch)
  const int wbase = t & ~63;
  for (int base = 0; base < n4; base += 256) {
    if (base + t < n4)
      __builtin_amdgcn_global_load_lds(static_cast<const void*>(src + base + t),
                                       (__attribute__((address_space(3))) void*)(dst + base + wbase),
                                       16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int p0 = 0; p0 < m; p0 += kGatherOut * 1024) {
    // every LDS read first (indices of unused slots are 0: row[0] is staged), then the
    // stores: one wait for the index loads, none between the stores
    f32x4 v[kGatherOut];
#pragma unroll
    for (int u = 0; u < kGatherOut; ++u)
      v[u] = f32x4{row[q[u].x], row[q[u].y], row[q[u].z], row[q[u].w]};
#pragma unroll
    for (int u = 0; u < kGatherOut; ++u) {
      const int p = p0 + (t + u * 256) * 4;
      if (p < m) __builtin_nontemporal_store(v[u], reinterpret_cast<f32x4*>(ob + p));
    }
    const int pn = p0 + kGatherOut * 1024;
#pragma unroll
    for (int u = 0; u < kGatherOut; ++u) {
      const int p = pn + (t + u * 256) * 4;
      if (p < m) q[u] = *reinterpret_cast<const int4*>(ib + p);
    }
  }
}

// Direct kernel (rows too long for LDS, or n / m not multiples of 4): a thread owns 4
// consecutive outputs of kGatherCG channels (one index load serves all of them).
constexpr int kGatherCG = 4;

__global__ __launch_bounds__(256) void gather_points_kernel(int c, int n, int m,
                                                            const float* __restrict__ points,
                                                            const int* __restrict__ idx,
                                                            float* __restrict__ out) {
  const int bi = blockIdx.z;
  const int c0 = blockIdx.y * kGatherCG;
  const int p4 = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (p4 >= m) return;
  const int* ib = idx + (long long)bi * m;
  const float* pb = points + ((long long)bi * c + c0) * n;
  float* ob = out + ((long long)bi * c + c0) * m;
  const int cg = min(kGatherCG, c - c0);
  const int np = min(4, m - p4);
  int q[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) q[j] = j < np ? ib[p4 + j] : 0;
  for (int cc = 0; cc < cg; ++cc) {
    const float* r = pb + (long long)cc * n;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < np) ob[(long long)cc * m + p4 + j] = r[q[j]];
  }
}

// ---------------------------------------------------------------------------------------
// group_points: out[b,c,s,k] = points[b,c,idx[b,s,k]]   (reference group_points_gpu.cu:47-66)
// A thread owns 4 consecutive (s,k) positions (one int4 idx load reused for CG channels,
// one float4 store per channel); blockIdx.y walks channel groups.  The index tile is read
// once per channel group instead of once per channel.
constexpr int kGroupCG = 8;

__global__ __launch_bounds__(256) void group_points_kernel(int c, int n, int p_total,
                                                           const float* __restrict__ points,
                                                           const int* __restrict__ idx,
                                                           float* __restrict__ out) {
  const int bi = blockIdx.z;
  const int c0 = blockIdx.y * kGroupCG;
  const int p4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (p4 >= p_total) return;
  const int* ib = idx + (long long)bi * p_total;
  const float* pb = points + ((long long)bi * c + c0) * n;
  float* ob = out + ((long long)bi * c + c0) * p_total;
  const int cg = min(kGroupCG, c - c0);
  if (p4 + 3 < p_total && (p_total & 3) == 0) {
    const int4 q = *reinterpret_cast<const int4*>(ib + p4);
    for (int cc = 0; cc < cg; ++cc) {
      const float* row = pb + (long long)cc * n;
      float4 v;
      v.x = row[q.x];
      v.y = row[q.y];
      v.z = row[q.z];
      v.w = row[q.w];
      *reinterpret_cast<float4*>(ob + (long long)cc * p_total + p4) = v;
    }
  } else {
    for (int t = 0; t < 4 && p4 + t < p_total; ++t) {
      const int q = ib[p4 + t];
      for (int cc = 0; cc < cg; ++cc) ob[(long long)cc * p_total + p4 + t] = pb[(long long)cc * n + q];
    }
  }
}

// LDS-staged variant: a workgroup owns CG whole channel rows of one cloud (CG*N*4 <= 80 KiB,
// so two workgroups share a CU; loaded once with coalesced float4 reads) and a slice of the
// S*K positions.  Every output is a random LDS read instead of a random 4-byte global
// gather; the HBM streams are the coalesced float4 stores and the int4 index reads.  A
// thread keeps kGU int4 index loads in flight (the loop would otherwise wait one L2/MALL
// round trip per 1024 positions), and the first batch is issued before the row staging so
// the two overlap.  Work units (cloud, slice) are spread so that the C/CG channel groups
// reading the same index slice run on one XCD (`xcd_units`), keeping those re-reads in its L2.
constexpr int kRowLdsBytes = 80 * 1024;
constexpr int kGU = 4;

template <int CG>
__global__ __launch_bounds__(256) void group_points_lds_kernel(int c, int n, int p_total,
                                                               int p_slice, int nslice,
                                                               int groups, int xcd_units,
                                                               const float* __restrict__ points,
                                                               const int* __restrict__ idx,
                                                               float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float rows[];  // [CG][n]
  int unit, grp;
  const int id = blockIdx.x;
  if (xcd_units > 0) {  // units % 8 == 0: XCD x (= id % 8) owns units [x*xcd_units, ...)
    const int j = id >> 3;
    unit = (id & 7) * xcd_units + j / groups;
    grp = j % groups;
  } else {
    unit = id / groups;
    grp = id % groups;
  }
  const int bi = unit / nslice;
  const int slice = unit % nslice;
  const int c0 = grp * CG;
  const int cg = min(CG, c - c0);
  const int pbeg = slice * p_slice;
  const int pend = min(p_total, pbeg + p_slice);
  const int* ib = idx + (long long)bi * p_total;
  float* ob = out + ((long long)bi * c + c0) * p_total;

  // first index batch in flight while the rows are staged
  int4 q[kGU];
  int p4 = pbeg + threadIdx.x * 4;
#pragma unroll
  for (int u = 0; u < kGU; ++u) {
    const int pu = p4 + u * 1024;
    q[u] = pu + 3 < pend ? *reinterpret_cast<const int4*>(ib + pu) : make_int4(0, 0, 0, 0);
  }
  const float* pb = points + ((long long)bi * c + c0) * n;
  if ((n & 3) == 0) {  // straight from memory into LDS (as gather_points_lds_kernel)
    const int tot4 = cg * (n >> 2), wbase = threadIdx.x & ~63;
    const f32x4* src = reinterpret_cast<const f32x4*>(pb);
    f32x4* dst = reinterpret_cast<f32x4*>(rows);
    for (int base = 0; base < tot4; base += 256) {
      if (base + (int)threadIdx.x < tot4)
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(src + base + threadIdx.x),
                                         (__attribute__((address_space(3))) void*)(dst + base + wbase),
                                         16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    for (int e = threadIdx.x; e < cg * n; e += 256) rows[e] = pb[e];
  }
  __syncthreads();

  for (; p4 < pend; p4 += kGU * 1024) {
#pragma unroll
    for (int u = 0; u < kGU; ++u) {
      const int pu = p4 + u * 1024;
      if (pu + 3 < pend) {
#pragma unroll
        for (int cc = 0; cc < CG; ++cc) {
          if (cc < cg) {
            const float* r = rows + cc * n;
            const f32x4 v = {r[q[u].x], r[q[u].y], r[q[u].z], r[q[u].w]};
            __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(ob + (long long)cc * p_total + pu));
          }
        }
      } else {
        for (int t = pu; t < pend; ++t) {
          const int qq = ib[t];
          for (int cc = 0; cc < cg; ++cc) ob[(long long)cc * p_total + t] = rows[cc * n + qq];
        }
      }
    }
    // next batch
    const int pn = p4 + kGU * 1024;
#pragma unroll
    for (int u = 0; u < kGU; ++u) {
      const int pu = pn + u * 1024;
      if (pu + 3 < pend) q[u] = *reinterpret_cast<const int4*>(ib + pu);
    }
  }
}

// ---------------------------------------------------------------------------------------
// ball_query (reference ball_query_gpu.cu:9-45): the first nsample k (ascending) with
// d2 < r^2; if any hit, the remaining slots repeat the first hit; no hit -> zeros.
// One wave per query: lanes test 64 consecutive candidates, ballot + popcount give each
// hit its slot in ascending-k order, and the wave stops as soon as nsample hits exist —
// identical output to the reference's serial scan.
__global__ __launch_bounds__(256) void ball_query_kernel(int b, int n, int m, float radius2,
                                                         int nsample,
                                                         const float* __restrict__ new_xyz,
                                                         const float* __restrict__ xyz,
                                                         int* __restrict__ idx) {
  const int wave_global = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = lane_id();
  if (wave_global >= b * m) return;
  const int bi = wave_global / m;
  const float* q = new_xyz + (long long)wave_global * 3;
  const float qx = q[0], qy = q[1], qz = q[2];
  const float* xb = xyz + (long long)bi * n * 3;
  int* out = idx + (long long)wave_global * nsample;
  int cnt = 0;
  int first = 0;
  for (int base = 0; base < n && cnt < nsample; base += kWave) {
    const int k = base + lane;
    bool hit = false;
    if (k < n) {
      const float d2 = dist3(xb[k * 3 + 0], xb[k * 3 + 1], xb[k * 3 + 2], qx, qy, qz);
      hit = d2 < radius2;
    }
    const unsigned long long mask = __ballot(hit);
    if (mask == 0ull) continue;
    if (cnt == 0) first = base + __ffsll((long long)mask) - 1;
    const int slot = cnt + __popcll(mask & lanemask_lt());
    if (hit && slot < nsample) out[slot] = k;
    cnt += __popcll(mask);
  }
  // slots past the hit count: first hit (reference fill loop, :36-39) or zero
  for (int s = cnt + lane; s < nsample; s += kWave) out[s] = cnt > 0 ? first : 0;
}

// ---------------------------------------------------------------------------------------
// three_nn (reference interpolate_gpu.cu:9-52): 3 smallest d2 per unknown point, strict <
// so the earlier known index wins ties (the reference's double running bests compare the
// same float values).  One thread per unknown point; known points staged through LDS in
// tiles and read as broadcasts.
constexpr int kNNTile = 1024;

__global__ __launch_bounds__(256) void three_nn_kernel(int b, int n, int m,
                                                       const float* __restrict__ unknown,
                                                       const float* __restrict__ known,
                                                       float* __restrict__ dist2,
                                                       int* __restrict__ idx) {
  __shared__ float sk[kNNTile * 3];
  const int bi = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = p < n;
  float ux = 0.f, uy = 0.f, uz = 0.f;
  if (active) {
    const float* u = unknown + ((long long)bi * n + p) * 3;
    ux = u[0]; uy = u[1]; uz = u[2];
  }
  const float* kb = known + (long long)bi * m * 3;
  float b1 = INFINITY, b2 = INFINITY, b3 = INFINITY;
  int i1 = 0, i2 = 0, i3 = 0;
  for (int t0 = 0; t0 < m; t0 += kNNTile) {
    const int tn = min(kNNTile, m - t0);
    __syncthreads();
    for (int e = threadIdx.x; e < tn * 3; e += blockDim.x) sk[e] = kb[(long long)t0 * 3 + e];
    __syncthreads();
    if (active) {
      for (int j = 0; j < tn; ++j) {
        const float d = dist3(sk[j * 3 + 0], sk[j * 3 + 1], sk[j * 3 + 2], ux, uy, uz);
        const int k = t0 + j;
        if (d < b1) {
          b3 = b2; i3 = i2; b2 = b1; i2 = i1; b1 = d; i1 = k;
        } else if (d < b2) {
          b3 = b2; i3 = i2; b2 = d; i2 = k;
        } else if (d < b3) {
          b3 = d; i3 = k;
        }
      }
    }
  }
  if (active) {
    float* o = dist2 + ((long long)bi * n + p) * 3;
    int* oi = idx + ((long long)bi * n + p) * 3;
    // reference initial best is 1e40 in double, stored as (float)1e40 == +inf
    o[0] = b1; o[1] = b2; o[2] = b3;
    oi[0] = i1; oi[1] = i2; oi[2] = i3;
  }
}

// ---------------------------------------------------------------------------------------
// three_interpolate (reference interpolate_gpu.cu:77-97), n fastest.
__global__ __launch_bounds__(256) void three_interpolate_kernel(int b, int c, int m, int n,
                                                                const float* __restrict__ points,
                                                                const int* __restrict__ idx,
                                                                const float* __restrict__ weight,
                                                                float* __restrict__ out) {
  const long long total = (long long)b * c * n;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int p = (int)(e % n);
    const long long bc = e / n;
    const int bi = (int)(bc / c);
    const float* row = points + bc * m;
    const long long o3 = ((long long)bi * n + p) * 3;
    const float w0 = weight[o3 + 0], w1 = weight[o3 + 1], w2 = weight[o3 + 2];
    const float v0 = row[idx[o3 + 0]], v1 = row[idx[o3 + 1]], v2 = row[idx[o3 + 2]];
    out[e] = __builtin_fmaf(w2, v2, __builtin_fmaf(w1, v1, __fmul_rn(w0, v0)));
  }
}

// Point-major path for clouds whose channel rows do not fit in LDS (N > 20480 at CG = 1,
// e.g. BASELINE configs[4]: N = 65536): the (B,C,N) table is first transposed to (B,N,C) in
// a stream-ordered scratch, then a thread gathers its 4 positions' whole rows (C floats, one
// or two cache lines each, every byte used) and writes each channel's 4 values as one float4
// -- a wave's stores to a channel row are 1 KiB contiguous.  The direct kernel above reads
// one 4-byte value per cache line it brings in.
template <int C4>
__global__ __launch_bounds__(256) void transpose_cn_kernel(int n, const float* __restrict__ src,
                                                           float* __restrict__ dst) {
  constexpr int C = 4 * C4;
  __shared__ float tile[C][65];
  const int bi = blockIdx.y;
  const int n0 = blockIdx.x * 64;
  const float* sb = src + (long long)bi * C * n;
  for (int e = threadIdx.x; e < C * 64; e += 256) {
    const int c = e / 64, j = e % 64;
    tile[c][j] = n0 + j < n ? sb[(long long)c * n + n0 + j] : 0.f;
  }
  __syncthreads();
  float* db = dst + ((long long)bi * n + n0) * C;
  for (int e = threadIdx.x; e < C * 64; e += 256) {
    const int j = e / C, c = e % C;
    if (n0 + j < n) db[(long long)j * C + c] = tile[c][j];
  }
}

template <int C4>
__global__ __launch_bounds__(256) void group_points_pm_kernel(int n, int p_total,
                                                              const float* __restrict__ pt,
                                                              const int* __restrict__ idx,
                                                              float* __restrict__ out) {
  constexpr int C = 4 * C4;
  const int bi = blockIdx.y;
  const int p4 = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (p4 >= p_total) return;  // p_total % 4 == 0 (checked by the caller)
  const int4 q = *reinterpret_cast<const int4*>(idx + (long long)bi * p_total + p4);
  const float4* rb = reinterpret_cast<const float4*>(pt + (long long)bi * n * C);
  float* ob = out + (long long)bi * C * p_total + p4;
#pragma unroll 2
  for (int c4 = 0; c4 < C4; ++c4) {
    const float4 a = rb[(long long)q.x * C4 + c4];
    const float4 b = rb[(long long)q.y * C4 + c4];
    const float4 c = rb[(long long)q.z * C4 + c4];
    const float4 d = rb[(long long)q.w * C4 + c4];
    const f32x4 o0 = {a.x, b.x, c.x, d.x}, o1 = {a.y, b.y, c.y, d.y};
    const f32x4 o2 = {a.z, b.z, c.z, d.z}, o3 = {a.w, b.w, c.w, d.w};
    float* o = ob + (long long)(4 * c4) * p_total;
    __builtin_nontemporal_store(o0, reinterpret_cast<f32x4*>(o));
    __builtin_nontemporal_store(o1, reinterpret_cast<f32x4*>(o + p_total));
    __builtin_nontemporal_store(o2, reinterpret_cast<f32x4*>(o + 2ll * p_total));
    __builtin_nontemporal_store(o3, reinterpret_cast<f32x4*>(o + 3ll * p_total));
  }
}

template <int C4>
hipError_t group_pm_launch(int b, int n, int p_total, const float* points, const int* idx,
                           float* out, hipStream_t st) {
  void* pt = nullptr;
  const size_t bytes = (size_t)b * n * 4 * C4 * sizeof(float);
  hipError_t e = hipMallocAsync(&pt, bytes, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(transpose_cn_kernel<C4>, dim3(divup(n, 64), b), dim3(256), 0, st, n, points,
                     (float*)pt);
  e = hipGetLastError();
  if (e == hipSuccess) {
    hipLaunchKernelGGL(group_points_pm_kernel<C4>, dim3(divup(p_total / 4, 256), b), dim3(256), 0,
                       st, n, p_total, (const float*)pt, idx, out);
    e = hipGetLastError();
  }
  const hipError_t f = hipFreeAsync(pt, st);
  return e != hipSuccess ? e : f;
}

template <int CG>
hipError_t launch_group_lds(dim3 grid, size_t lds, hipStream_t st, int c, int n, int p_total,
                            int p_slice, int nslice, int groups, int xcd_units,
                            const float* points, const int* idx, float* out) {
  auto k = group_points_lds_kernel<CG>;
  // once per process and instantiation (thread-safe static initialisation)
  static const hipError_t attr = hipFuncSetAttribute(
      (const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, kRowLdsBytes);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(k, grid, dim3(256), lds, st, c, n, p_total, p_slice, nslice, groups,
                     xcd_units, points, idx, out);
  return hipGetLastError();
}

inline int grid_for(long long total, int block) {
  long long g = divupll(total, block);
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

// Reference: gather_points_wrapper(b, c, n, npoints, points, idx, out)  (sampling.cpp:11-22)
KDPC_API int kdpc_gather_points(int b, int c, int n, int npoints, const float* points,
                                const int* idx, float* out, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && c >= 0 && n > 0 && npoints >= 0);
  const long long total = (long long)b * c * npoints;
  if (total == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(points && idx && out);
  hipStream_t st = (hipStream_t)stream;
  if ((n & 3) == 0 && (npoints & 3) == 0 && (size_t)n * sizeof(float) <= (size_t)kGatherRowLds &&
      (long long)b * c < (1ll << 31)) {
    static const hipError_t attr = hipFuncSetAttribute(
        (const void*)gather_points_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
        kGatherRowLds);
    if (attr != hipSuccess) return (int)attr;
    hipLaunchKernelGGL(gather_points_lds_kernel, dim3((unsigned)(b * c)), dim3(256),
                       (size_t)n * sizeof(float), st, c, n, npoints, points, idx, out);
    KDPC_RETURN_LAUNCH();
  }
  KDPC_CHECK_ARG(b <= 65535 && divup(c, kGatherCG) <= 65535);
  hipLaunchKernelGGL(gather_points_kernel, dim3(divup(divup(npoints, 4), 256), divup(c, kGatherCG), b),
                     dim3(256), 0, st, c, n, npoints, points, idx, out);
  KDPC_RETURN_LAUNCH();
}

// Reference: group_points_wrapper(b, c, n, npoints, nsample, points, idx, out)
// (group_points.cpp:27-38)
KDPC_API int kdpc_group_points(int b, int c, int n, int npoints, int nsample, const float* points,
                               const int* idx, float* out, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && c >= 0 && n > 0 && npoints >= 0 && nsample >= 0);
  const long long p_total = (long long)npoints * nsample;
  if ((long long)b * c * p_total == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(points && idx && out && p_total < (1ll << 31));
  KDPC_CHECK_ARG(b <= 65535);
  hipStream_t st = (hipStream_t)stream;
  const int cg = kRowLdsBytes / (4 * n);
  if (cg >= 1 && (p_total % 4) == 0) {
    // channel groups of CG rows; slices so that the grid covers >= ~512 workgroups
    const int CG = cg >= 8 ? 8 : (cg >= 4 ? 4 : (cg >= 2 ? 2 : 1));
    const int groups = divup(c, CG);
    int nslice = divup(512, b * groups);
    const int min_slice = 4096;
    nslice = max(1, min(nslice, (int)divupll(p_total, min_slice)));
    int p_slice = (int)divupll(divupll(p_total, nslice), 4) * 4;
    nslice = (int)divupll(p_total, p_slice);
    const long long units = (long long)b * nslice;
    const long long wgs = units * groups;
    KDPC_CHECK_ARG(wgs < (1ll << 31));
    const int xcd_units = (units % 8 == 0) ? (int)(units / 8) : 0;
    const size_t lds = (size_t)CG * n * sizeof(float);
    const dim3 grid((unsigned)wgs);
    const int pt = (int)p_total;
    hipError_t e;
    switch (CG) {
      case 8: e = launch_group_lds<8>(grid, lds, st, c, n, pt, p_slice, nslice, groups, xcd_units, points, idx, out); break;
      case 4: e = launch_group_lds<4>(grid, lds, st, c, n, pt, p_slice, nslice, groups, xcd_units, points, idx, out); break;
      case 2: e = launch_group_lds<2>(grid, lds, st, c, n, pt, p_slice, nslice, groups, xcd_units, points, idx, out); break;
      default: e = launch_group_lds<1>(grid, lds, st, c, n, pt, p_slice, nslice, groups, xcd_units, points, idx, out);
    }
    return (int)e;
  }
  if ((p_total % 4) == 0 && (c == 16 || c == 32 || c == 64)) {
    const int pt = (int)p_total;
    switch (c) {
      case 16: return (int)group_pm_launch<4>(b, n, pt, points, idx, out, st);
      case 32: return (int)group_pm_launch<8>(b, n, pt, points, idx, out, st);
      default: return (int)group_pm_launch<16>(b, n, pt, points, idx, out, st);
    }
  }
  dim3 grid(divup((int)divupll(p_total, 4), 256), divup(c, kGroupCG), b);
  KDPC_CHECK_ARG(grid.y <= 65535);
  hipLaunchKernelGGL(group_points_kernel, grid, dim3(256), 0, st, c, n, (int)p_total, points, idx,
                     out);
  KDPC_RETURN_LAUNCH();
}

// Reference: ball_query_wrapper(b, n, m, radius, nsample, new_xyz, xyz, idx)
// (ball_query.cpp:16-28).  idx is fully written (zeros where the reference relied on the
// caller's .zero_()).
KDPC_API int kdpc_ball_query(int b, int n, int m, float radius, int nsample, const float* new_xyz,
                             const float* xyz, int* idx, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n >= 0 && m >= 0 && nsample >= 0);
  if ((long long)b * m * nsample == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(new_xyz && idx && (n == 0 || xyz));
  const long long waves = (long long)b * m;
  KDPC_CHECK_ARG(waves * kWave < (1ll << 31));
  const float r2 = radius * radius;
  hipLaunchKernelGGL(ball_query_kernel, dim3((int)divupll(waves * kWave, 256)), dim3(256), 0,
                     (hipStream_t)stream, b, n, m, r2, nsample, new_xyz, xyz, idx);
  KDPC_RETURN_LAUNCH();
}

// Reference: three_nn_wrapper(b, n, m, unknown, known, dist2, idx)  (interpolate.cpp:14-24).
// dist2 holds squared distances (the Python wrapper takes the sqrt).
KDPC_API int kdpc_three_nn(int b, int n, int m, const float* unknown, const float* known,
                           float* dist2, int* idx, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n >= 0 && m >= 0 && b <= 65535);
  if ((long long)b * n == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(unknown && dist2 && idx && (m == 0 || known));
  hipLaunchKernelGGL(three_nn_kernel, dim3(divup(n, 256), b), dim3(256), 0, (hipStream_t)stream,
                     b, n, m, unknown, known, dist2, idx);
  KDPC_RETURN_LAUNCH();
}

// Reference: three_interpolate_wrapper(b, c, m, n, points, idx, weight, out)
// (interpolate.cpp:27-41)
KDPC_API int kdpc_three_interpolate(int b, int c, int m, int n, const float* points,
                                    const int* idx, const float* weight, float* out,
                                    void* stream) {
  KDPC_CHECK_ARG(b >= 0 && c >= 0 && m > 0 && n >= 0);
  const long long total = (long long)b * c * n;
  if (total == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(points && idx && weight && out);
  hipLaunchKernelGGL(three_interpolate_kernel, dim3(grid_for(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, b, c, m, n, points, idx, weight, out);
  KDPC_RETURN_LAUNCH();
}
