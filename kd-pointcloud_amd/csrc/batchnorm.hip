// Train-mode BatchNorm1d over the rows of a point-major (R, C) tensor, fused with the
// LeakyReLU that follows it in every scene-flow estimator PointConv (reference
// pointconv_util.py:217-258 with bn=True: Linear -> BatchNorm1d -> LeakyReLU(0.1)).
//
// The reference normalises a (B, C, N) tensor: per-channel statistics over B and N.  On the
// point-major layout the same statistics are column statistics of (R = B*N, C); torch's
// channels-last BatchNorm kernels took ~150 us per (65536, 128) pass on MI355X, ~10x the
// bytes-moved bound.  Here:
//   forward : bn_stats (per-block Welford partials, fixed block -> slab order)
//             bn_finalize (Chan merges of the slabs in a fixed order: one wave per channel;
//                          mean, invstd, running stats)
//             bn_apply  (y = act((x - mean) * invstd * w + b), float4 rows)
//   backward: bn_bwd_reduce (per-block sums of dy and dy*xhat, dy = dy_act * slope(y))
//             colsum (slab column sums, fixed order -> dbias, dweight)
//             bn_bwd_apply (dx = w * invstd * (dy - sum(dy)/R - xhat * sum(dy*xhat)/R))
// Every reduction has a fixed order (no atomics): results depend only on the shape.
#include <algorithm>

#include "kdpc_common.h"

using namespace kdpc;

namespace {

constexpr int kBlock = 256;
constexpr int kMaxSlabs = 256;

// block b of `nblk` covers rows [b*rpb, min(R, (b+1)*rpb))
inline int rows_per_block(long long r) {
  const long long nb = std::min<long long>(kMaxSlabs, std::max<long long>(1, divupll(r, 256)));
  return (int)divupll(r, nb);
}
// the backward reduction: up to 2048 blocks of >= 64 rows (round 4: 256 blocks of 256 rows
// left one workgroup per CU walking 32 dependent row steps -- ~1.2 TB/s at R = 65536; the
// order of the sums changes with the block size, the backward makes no discrete choice)
constexpr int kMaxSlabsBwd = 2048;
inline int rows_per_block_bwd(long long r) {
  const long long nb = std::min<long long>(kMaxSlabsBwd, std::max<long long>(1, divupll(r, 64)));
  return (int)divupll(r, nb);
}

// thread layout inside a block: channel group cg (4 channels), row lane rl
struct Lay {
  int cv, lanes, cg, rl;
};
__device__ __forceinline__ Lay lay_of(int c) {
  Lay l;
  l.cv = c / 4;
  l.lanes = kBlock / l.cv;
  l.cg = threadIdx.x % l.cv;
  l.rl = threadIdx.x / l.cv;
  return l;
}

__device__ __forceinline__ void welford_merge(float& n, float& m, float& m2, float nb, float mb,
                                              float m2b) {
  if (nb == 0.f) return;
  if (n == 0.f) {
    n = nb;
    m = mb;
    m2 = m2b;
    return;
  }
  const float nn = n + nb;
  const float d = mb - m;
  m = m + d * (nb / nn);
  m2 = m2 + m2b + d * d * (n * nb / nn);
  n = nn;
}

// slab: (nblk, 3, C) = count, mean, M2
__global__ __launch_bounds__(kBlock) void bn_stats_kernel(int r, int c, int rpb,
                                                          const float* __restrict__ x,
                                                          float* __restrict__ slab) {
  extern __shared__ float sh[];  // [lanes][3][C]
  const Lay L = lay_of(c);
  const int r0 = blockIdx.x * rpb, r1 = min(r, r0 + rpb);
  float n[4] = {0, 0, 0, 0}, m[4] = {0, 0, 0, 0}, m2[4] = {0, 0, 0, 0};
  if (L.rl < L.lanes) {
    for (int row = r0 + L.rl; row < r1; row += L.lanes) {
      const float4 v = reinterpret_cast<const float4*>(x + (long long)row * c)[L.cg];
      const float xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        n[i] += 1.f;
        const float d = xs[i] - m[i];
        m[i] += d / n[i];
        m2[i] = __builtin_fmaf(d, xs[i] - m[i], m2[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float* p = sh + (L.rl * 3) * c + 4 * L.cg + i;
      p[0] = n[i];
      p[c] = m[i];
      p[2 * c] = m2[i];
    }
  }
  __syncthreads();
  for (int ch = threadIdx.x; ch < c; ch += kBlock) {
    float N = 0.f, M = 0.f, M2 = 0.f;
    for (int l = 0; l < L.lanes; ++l) {
      const float* p = sh + (l * 3) * c + ch;
      welford_merge(N, M, M2, p[0], p[c], p[2 * c]);
    }
    float* o = slab + (long long)blockIdx.x * 3 * c + ch;
    o[0] = N;
    o[c] = M;
    o[2 * c] = M2;
  }
}

// one wave per channel: lane l merges slabs l, l+64, ... in order, then a fixed xor
// butterfly merges the lanes (deterministic)
__global__ __launch_bounds__(kBlock) void bn_finalize_kernel(int r, int c, int nslab,
                                                             const float* __restrict__ slab,
                                                             float eps, float momentum,
                                                             float* __restrict__ mean,
                                                             float* __restrict__ invstd,
                                                             float* __restrict__ run_mean,
                                                             float* __restrict__ run_var) {
  const int ch = (blockIdx.x * kBlock + threadIdx.x) / kWave;
  const int lane = lane_id();
  if (ch >= c) return;  // wave-uniform
  float N = 0.f, M = 0.f, M2 = 0.f;
  for (int s = lane; s < nslab; s += kWave) {
    const float* p = slab + (long long)s * 3 * c + ch;
    welford_merge(N, M, M2, p[0], p[c], p[2 * c]);
  }
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const float nb = __shfl_xor(N, o, kWave), mb = __shfl_xor(M, o, kWave);
    const float m2b = __shfl_xor(M2, o, kWave);
    // merge in lane order so both partners compute the identical result
    if (lane & o) {
      float n2 = nb, mm = mb, mq = m2b;
      welford_merge(n2, mm, mq, N, M, M2);
      N = n2;
      M = mm;
      M2 = mq;
    } else {
      welford_merge(N, M, M2, nb, mb, m2b);
    }
  }
  if (lane != 0) return;
  const float var = M2 / N;  // biased (normalisation)
  mean[ch] = M;
  invstd[ch] = 1.f / sqrtf(var + eps);
  if (run_mean) {
    const float unbiased = r > 1 ? M2 / (N - 1.f) : var;
    run_mean[ch] = (1.f - momentum) * run_mean[ch] + momentum * M;
    run_var[ch] = (1.f - momentum) * run_var[ch] + momentum * unbiased;
  }
}

__global__ __launch_bounds__(kBlock) void bn_apply_kernel(long long n4, int cv, float slope,
                                                          const float* __restrict__ x,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ b,
                                                          float* __restrict__ y) {
  for (long long e = (long long)blockIdx.x * kBlock + threadIdx.x; e < n4;
       e += (long long)gridDim.x * kBlock) {
    const int c4 = (int)(e % cv) * 4;
    const float4 v = reinterpret_cast<const float4*>(x)[e];
    const float xs[4] = {v.x, v.y, v.z, v.w};
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float h = (xs[i] - mean[c4 + i]) * invstd[c4 + i] * w[c4 + i] + b[c4 + i];
      o[i] = h > 0.f ? h : h * slope;
    }
    reinterpret_cast<float4*>(y)[e] = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// slab: (nblk, 2, C) = sum dy, sum dy*xhat
__global__ __launch_bounds__(kBlock) void bn_bwd_reduce_kernel(int r, int c, int rpb, float slope,
                                                               const float* __restrict__ dya,
                                                               const float* __restrict__ ya,
                                                               const float* __restrict__ x,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               float* __restrict__ slab) {
  extern __shared__ float sh[];  // [lanes][2][C]
  const Lay L = lay_of(c);
  const int r0 = blockIdx.x * rpb, r1 = min(r, r0 + rpb);
  float s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  if (L.rl < L.lanes) {
    float mu[4], is[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      mu[i] = mean[4 * L.cg + i];
      is[i] = invstd[4 * L.cg + i];
    }
    // kU rows' loads issued together, then accumulated in row order (same sums as one row
    // at a time)
    constexpr int kU = 4;
    for (int row0 = r0 + L.rl; row0 < r1; row0 += kU * L.lanes) {
      float4 g[kU], a[kU], v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int row = row0 + u * L.lanes;
        const long long o = (long long)(row < r1 ? row : r0) * c;
        g[u] = reinterpret_cast<const float4*>(dya + o)[L.cg];
        a[u] = reinterpret_cast<const float4*>(ya + o)[L.cg];
        v[u] = reinterpret_cast<const float4*>(x + o)[L.cg];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (row0 + u * L.lanes >= r1) break;
        const float gs[4] = {g[u].x, g[u].y, g[u].z, g[u].w};
        const float as[4] = {a[u].x, a[u].y, a[u].z, a[u].w};
        const float xs[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float dy = as[i] > 0.f ? gs[i] : gs[i] * slope;
          s1[i] += dy;
          s2[i] = __builtin_fmaf(dy, (xs[i] - mu[i]) * is[i], s2[i]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float* p = sh + (L.rl * 2) * c + 4 * L.cg + i;
      p[0] = s1[i];
      p[c] = s2[i];
    }
  }
  __syncthreads();
  for (int ch = threadIdx.x; ch < c; ch += kBlock) {
    float a = 0.f, b2 = 0.f;
    for (int l = 0; l < L.lanes; ++l) {
      a += sh[(l * 2) * c + ch];
      b2 += sh[(l * 2 + 1) * c + ch];
    }
    float* o = slab + (long long)blockIdx.x * 2 * c + ch;
    o[0] = a;
    o[c] = b2;
  }
}

__global__ void bn_bwd_copy_kernel(int c, const float* __restrict__ sums,
                                   float* __restrict__ dbias, float* __restrict__ dweight) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  dbias[ch] = sums[ch];
  dweight[ch] = sums[c + ch];
}

__global__ __launch_bounds__(kBlock) void bn_bwd_apply_kernel(long long n4, int cv, float rinv,
                                                              float slope,
                                                              const float* __restrict__ dya,
                                                              const float* __restrict__ ya,
                                                              const float* __restrict__ x,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ dbias,
                                                              const float* __restrict__ dweight,
                                                              float* __restrict__ dx) {
  for (long long e = (long long)blockIdx.x * kBlock + threadIdx.x; e < n4;
       e += (long long)gridDim.x * kBlock) {
    const int c4 = (int)(e % cv) * 4;
    const float4 g = reinterpret_cast<const float4*>(dya)[e];
    const float4 a = reinterpret_cast<const float4*>(ya)[e];
    const float4 v = reinterpret_cast<const float4*>(x)[e];
    const float gs[4] = {g.x, g.y, g.z, g.w}, as[4] = {a.x, a.y, a.z, a.w};
    const float xs[4] = {v.x, v.y, v.z, v.w};
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = c4 + i;
      const float dy = as[i] > 0.f ? gs[i] : gs[i] * slope;
      const float xh = (xs[i] - mean[ch]) * invstd[ch];
      o[i] = w[ch] * invstd[ch] * (dy - dbias[ch] * rinv - xh * dweight[ch] * rinv);
    }
    reinterpret_cast<float4*>(dx)[e] = make_float4(o[0], o[1], o[2], o[3]);
  }
}

inline int ew_grid(long long n4) {
  return (int)std::min<long long>(std::max<long long>(1, divupll(n4, kBlock)), 8192);
}

}  // namespace

KDPC_API size_t kdpc_batchnorm_workspace_bytes(int r, int c) {
  if (r <= 0 || c <= 0) return 0;
  const long long nblk = divupll(r, rows_per_block(r));
  const long long nbb = divupll(r, rows_per_block_bwd(r));
  // forward: slab (nblk, 3, C); backward: slab (nbb, 2, C) | column sums (2C) | colsum scratch
  const long long fwd = nblk * 3 * c;
  const long long bwd = nbb * 2 * c + 2 * c + colsum_scratch_floats((int)nbb, 2 * c);
  return (size_t)std::max(fwd, bwd) * sizeof(float);
}

// Train-mode forward.  x, y (R, C) row-major; C % 4 == 0 and C <= 1024; mean/invstd (C)
// outputs (saved for backward); run_mean/run_var (C) updated in place (NULL: not tracked).
KDPC_API int kdpc_batchnorm_lrelu_fwd(int r, int c, const float* x, const float* weight,
                                      const float* bias, float eps, float momentum, float slope,
                                      float* run_mean, float* run_var, float* mean, float* invstd,
                                      float* y, void* workspace, size_t workspace_bytes,
                                      void* stream) {
  KDPC_CHECK_ARG(r > 0 && c > 0 && c % 4 == 0 && c / 4 <= kBlock);
  KDPC_CHECK_ARG(x && weight && bias && mean && invstd && y && workspace);
  KDPC_CHECK_ARG(workspace_bytes >= kdpc_batchnorm_workspace_bytes(r, c));
  KDPC_CHECK_ARG((run_mean == nullptr) == (run_var == nullptr));
  hipStream_t st = (hipStream_t)stream;
  const int rpb = rows_per_block(r);
  const int nblk = (int)divupll(r, rpb);
  const int lanes = kBlock / (c / 4);
  float* slab = reinterpret_cast<float*>(workspace);
  hipLaunchKernelGGL(bn_stats_kernel, dim3(nblk), dim3(kBlock), (size_t)lanes * 3 * c * 4, st, r,
                     c, rpb, x, slab);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(divup(c * kWave, kBlock)), dim3(kBlock), 0, st, r,
                     c, nblk, slab, eps, momentum, mean, invstd, run_mean, run_var);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  const long long n4 = (long long)r * c / 4;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(ew_grid(n4)), dim3(kBlock), 0, st, n4, c / 4, slope, x,
                     mean, invstd, weight, bias, y);
  KDPC_RETURN_LAUNCH();
}

// y = act((x - mean) * invstd * w + b) with given statistics (eval mode: running stats).
KDPC_API int kdpc_batchnorm_lrelu_apply(int r, int c, const float* x, const float* mean,
                                        const float* invstd, const float* weight,
                                        const float* bias, float slope, float* y, void* stream) {
  KDPC_CHECK_ARG(r >= 0 && c > 0 && c % 4 == 0);
  if (r == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(x && mean && invstd && weight && bias && y);
  const long long n4 = (long long)r * c / 4;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(ew_grid(n4)), dim3(kBlock), 0, (hipStream_t)stream,
                     n4, c / 4, slope, x, mean, invstd, weight, bias, y);
  KDPC_RETURN_LAUNCH();
}

// Backward of kdpc_batchnorm_lrelu_fwd: dy_act, y_act (the forward's output), x (its input)
// -> dx, dweight, dbias.
KDPC_API int kdpc_batchnorm_lrelu_bwd(int r, int c, const float* dy_act, const float* y_act,
                                      const float* x, const float* weight, const float* mean,
                                      const float* invstd, float slope, float* dx,
                                      float* dweight, float* dbias, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  KDPC_CHECK_ARG(r > 0 && c > 0 && c % 4 == 0 && c / 4 <= kBlock);
  KDPC_CHECK_ARG(dy_act && y_act && x && weight && mean && invstd && dx && dweight && dbias &&
                 workspace);
  KDPC_CHECK_ARG(workspace_bytes >= kdpc_batchnorm_workspace_bytes(r, c));
  hipStream_t st = (hipStream_t)stream;
  const int rpb = rows_per_block_bwd(r);
  const int nblk = (int)divupll(r, rpb);
  const int lanes = kBlock / (c / 4);
  float* slab = reinterpret_cast<float*>(workspace);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(nblk), dim3(kBlock), (size_t)lanes * 2 * c * 4, st,
                     r, c, rpb, slope, dy_act, y_act, x, mean, invstd, slab);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  float* sums = slab + (size_t)nblk * 2 * c;  // [sum dy (C) | sum dy*xhat (C)]
  if ((e = colsum(nblk, 2 * c, slab, sums, sums + 2 * c, st)) != hipSuccess) return (int)e;
  const long long n4 = (long long)r * c / 4;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(ew_grid(n4)), dim3(kBlock), 0, st, n4, c / 4,
                     1.f / (float)r, slope, dy_act, y_act, x, mean, invstd, weight, sums,
                     sums + c, dx);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  hipLaunchKernelGGL(bn_bwd_copy_kernel, dim3(divup(c, 256)), dim3(256), 0, st, c, sums, dbias,
                     dweight);
  KDPC_RETURN_LAUNCH();
}
