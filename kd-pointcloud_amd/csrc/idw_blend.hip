// 3-NN inverse-distance blend of UpsampleFlow / PointWarping (reference pointconv_util.py:
// 2130-2139 and 2165-2170), fused:
//
//   g_k = ref[idx_k] - q,  d_k = max(||g_k||, 1e-10),  r_k = 1 / d_k,
//   w_k = r_k / (r_0 + r_1 + r_2),  blend = sum_k w_k vals[idx_k]
//   out = blend  (UpsampleFlow)   or   out = q - blend  (PointWarping, C = 3)
//
// The reference evaluates this as ~10 broadcast torch kernels forward (norm, clamp, two
// reciprocals, sum, div, mul, sum, sub) and ~15 backward, each a full pass over (B,N,3[,C]):
// here one pass forward, and backward one CSR gather-sum for the values plus one per-query
// pass for the coordinate gradient (only PointWarping needs it: its reference points are
// xyz1 + flow).  Arithmetic follows the torch expression's order (products rounded, then
// summed in k order; no contraction: the library is built with -ffp-contract=off).
//
// Layout (point-major): ref (B,S,3), qry (B,N,3), vals (B,S,C), idx (B,N,3) int32 in [0,S),
// out (B,N,C), w (B,N,3).  No float atomics: the scatter of the values / reference-point
// gradients goes through the CSR of idx (ascending (n, k) position per reference point).
#include "kdpc_common.h"

#include <algorithm>

using namespace kdpc;

namespace {

constexpr float kMinDist = 1e-10f;  // .clamp(min=1e-10) of the reference

struct Geo3 {
  float g[3][3];  // g_k = ref[idx_k] - q
  float len[3];   // ||g_k||
  float r[3];     // 1 / max(||g_k||, 1e-10)
  float w[3];     // r_k / sum r
  float sum;      // r_0 + r_1 + r_2
  int nb[3];      // global reference rows b*S + idx_k
};

__device__ __forceinline__ void idw_geometry(const float* __restrict__ ref,
                                             const float* __restrict__ qry,
                                             const int* __restrict__ idx, long long row, int s,
                                             int bi, Geo3& o) {
  const float qx = qry[row * 3 + 0], qy = qry[row * 3 + 1], qz = qry[row * 3 + 2];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int nb = bi * s + idx[row * 3 + k];
    o.nb[k] = nb;
    const float gx = ref[(long long)nb * 3 + 0] - qx;
    const float gy = ref[(long long)nb * 3 + 1] - qy;
    const float gz = ref[(long long)nb * 3 + 2] - qz;
    o.g[k][0] = gx;
    o.g[k][1] = gy;
    o.g[k][2] = gz;
    const float len = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(gx, gx), __fmul_rn(gy, gy)),
                                           __fmul_rn(gz, gz)));
    o.len[k] = len;
    o.r[k] = __fdiv_rn(1.0f, fmaxf(len, kMinDist));
  }
  o.sum = __fadd_rn(__fadd_rn(o.r[0], o.r[1]), o.r[2]);
#pragma unroll
  for (int k = 0; k < 3; ++k) o.w[k] = __fdiv_rn(o.r[k], o.sum);
}

// one thread per (query row, 4 channels)
__global__ __launch_bounds__(256) void idw_fwd_kernel(int b, int n, int s, int c,
                                                      const float* __restrict__ ref,
                                                      const float* __restrict__ qry,
                                                      const float* __restrict__ vals,
                                                      const int* __restrict__ idx,
                                                      float* __restrict__ out,
                                                      float* __restrict__ wout, int warp) {
  const int cv = (c + 3) / 4;
  const long long total = (long long)b * n * cv;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long row = e / cv;
    const int v = (int)(e - row * cv);
    const int bi = (int)(row / n);
    Geo3 o;
    idw_geometry(ref, qry, idx, row, s, bi, o);
    if (v == 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) wout[row * 3 + k] = o.w[k];
    }
    if ((c & 3) == 0) {  // 16-byte value rows (warp implies c = 3: never here)
      float4 x[3];
#pragma unroll
      for (int k = 0; k < 3; ++k)
        x[k] = *reinterpret_cast<const float4*>(vals + (long long)o.nb[k] * c + 4 * v);
      auto blend = [&](float a0, float a1, float a2) {
        return __fadd_rn(__fadd_rn(__fmul_rn(o.w[0], a0), __fmul_rn(o.w[1], a1)),
                         __fmul_rn(o.w[2], a2));
      };
      *reinterpret_cast<float4*>(out + row * c + 4 * v) =
          make_float4(blend(x[0].x, x[1].x, x[2].x), blend(x[0].y, x[1].y, x[2].y),
                      blend(x[0].z, x[1].z, x[2].z), blend(x[0].w, x[1].w, x[2].w));
      continue;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = 4 * v + i;
      if (ch >= c) break;
      float acc = __fmul_rn(o.w[0], vals[(long long)o.nb[0] * c + ch]);
      acc = __fadd_rn(acc, __fmul_rn(o.w[1], vals[(long long)o.nb[1] * c + ch]));
      acc = __fadd_rn(acc, __fmul_rn(o.w[2], vals[(long long)o.nb[2] * c + ch]));
      out[row * c + ch] = warp ? __fsub_rn(qry[row * 3 + ch], acc) : acc;
    }
  }
}

// dvals[b,j,ch] = sum over the CSR entries p = (n*3 + k) of reference point j of
// w[p] * dblend[n, ch] (dblend = -dout for PointWarping), ascending p.  One thread per
// (reference point, V channels): the segment's perm / w entries are read once per V channels
// (V = 4 with 16-byte dout rows when C % 4 == 0), in the same per-channel order.
template <int V>
__global__ __launch_bounds__(256) void idw_bwd_vals_kernel(int b, int s, int c,
                                                           const float* __restrict__ dout,
                                                           const float* __restrict__ w,
                                                           const int* __restrict__ offsets,
                                                           const int* __restrict__ perm,
                                                           float* __restrict__ dvals, int warp) {
  const int cv = c / V;
  const long long total = (long long)b * s * cv;
  const float sg = warp ? -1.f : 1.f;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long key = e / cv;
    const int v = (int)(e - key * cv);
    const int j0 = offsets[key], j1 = offsets[key + 1];
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
    for (int j = j0; j < j1; ++j) {
      const int p = perm[j];
      const float wp = w[p];
      const float* g = dout + (long long)(p / 3) * c + V * v;
      float gv[V];
      if constexpr (V == 4) {
        const float4 x = *reinterpret_cast<const float4*>(g);
        gv[0] = x.x, gv[1] = x.y, gv[2] = x.z, gv[3] = x.w;
      } else {
        gv[0] = g[0];
      }
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] = __fadd_rn(acc[i], __fmul_rn(wp, sg * gv[i]));
    }
#pragma unroll
    for (int i = 0; i < V; ++i) dvals[key * c + V * v + i] = acc[i];
  }
}

// one thread per query row: the gradient of the blend weights with respect to the
// coordinates.  drow (B,N,3,3) = d loss / d ref[idx_k] contributions (sum them per reference
// point through the CSR), dqry (B,N,3) (may be null).  Follows torch's chain: blend ->
// weight = a / norm (a = 1/dist, norm = sum 1/dist) -> dist = clamp(norm(g), 1e-10) -> g.
__global__ __launch_bounds__(256) void idw_bwd_coords_kernel(
    int b, int n, int s, int c, const float* __restrict__ ref, const float* __restrict__ qry,
    const float* __restrict__ vals, const int* __restrict__ idx, const float* __restrict__ dout,
    float* __restrict__ drow, float* __restrict__ dqry, int warp) {
  const long long total = (long long)b * n;
  for (long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x; row < total;
       row += (long long)gridDim.x * blockDim.x) {
    const int bi = (int)(row / n);
    Geo3 o;
    idw_geometry(ref, qry, idx, row, s, bi, o);
    // dw_k = <dblend, vals[idx_k]>
    float dw[3] = {0.f, 0.f, 0.f};
    for (int ch = 0; ch < c; ++ch) {
      const float g0 = dout[row * c + ch];
      const float g = warp ? -g0 : g0;
#pragma unroll
      for (int k = 0; k < 3; ++k)
        dw[k] = __fadd_rn(dw[k], __fmul_rn(g, vals[(long long)o.nb[k] * c + ch]));
    }
    // weight_k = a_k / norm: da_k = dw_k / norm; dnorm = -sum_k dw_k a_k / norm^2
    const float inv = __fdiv_rn(1.0f, o.sum);
    float dnorm = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) dnorm = __fadd_rn(dnorm, __fmul_rn(dw[k], o.r[k]));
    dnorm = -__fmul_rn(dnorm, __fmul_rn(inv, inv));
    float dq[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      // both 1/dist uses: d(1/d)/dd = -1/d^2; clamp passes the gradient where ||g|| >= 1e-10;
      // d||g||/dg = g / ||g||
      const float dr = __fadd_rn(__fmul_rn(dw[k], inv), dnorm);
      const float dd = -__fmul_rn(dr, __fmul_rn(o.r[k], o.r[k]));
      const bool pass = o.len[k] >= kMinDist;
      const float sc = pass ? __fdiv_rn(dd, o.len[k]) : 0.f;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const float gi = __fmul_rn(sc, o.g[k][i]);
        drow[(row * 3 + k) * 3 + i] = gi;
        dq[i] = __fsub_rn(dq[i], gi);
      }
    }
    if (dqry) {
#pragma unroll
      for (int i = 0; i < 3; ++i)
        dqry[row * 3 + i] = warp ? __fadd_rn(dq[i], dout[row * c + i]) : dq[i];
    }
  }
}

inline int grid_of(long long work) {
  return (int)std::min<long long>(std::max<long long>(divupll(work, 256), 1), 1 << 20);
}

}  // namespace

KDPC_API int kdpc_idw_blend_fwd(int b, int n, int s, int c, const float* ref, const float* qry,
                                const float* vals, const int* idx, float* out, float* w,
                                int warp, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n >= 0 && s > 0 && c > 0 && (!warp || c == 3));
  if ((long long)b * n == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(ref && qry && vals && idx && out && w);
  const long long work = (long long)b * n * ((c + 3) / 4);
  hipLaunchKernelGGL(idw_fwd_kernel, dim3(grid_of(work)), dim3(256), 0, (hipStream_t)stream, b,
                     n, s, c, ref, qry, vals, idx, out, w, warp);
  return (int)hipGetLastError();
}

KDPC_API int kdpc_idw_blend_bwd_vals(int b, int n, int s, int c, const float* dout,
                                     const float* w, const int* offsets, const int* perm,
                                     float* dvals, int warp, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n >= 0 && s > 0 && c > 0 && (!warp || c == 3));
  if ((long long)b * s == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(offsets && perm && dvals && ((long long)b * n == 0 || (dout && w)));
  if (c % 4 == 0)
    hipLaunchKernelGGL(idw_bwd_vals_kernel<4>, dim3(grid_of((long long)b * s * c / 4)), dim3(256),
                       0, (hipStream_t)stream, b, s, c, dout, w, offsets, perm, dvals, warp);
  else
    hipLaunchKernelGGL(idw_bwd_vals_kernel<1>, dim3(grid_of((long long)b * s * c)), dim3(256), 0,
                       (hipStream_t)stream, b, s, c, dout, w, offsets, perm, dvals, warp);
  return (int)hipGetLastError();
}

KDPC_API int kdpc_idw_blend_bwd_coords(int b, int n, int s, int c, const float* ref,
                                       const float* qry, const float* vals, const int* idx,
                                       const float* dout, float* drow, float* dqry, int warp,
                                       void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n >= 0 && s > 0 && c > 0 && (!warp || c == 3));
  if ((long long)b * n == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(ref && qry && vals && idx && dout && drow);
  hipLaunchKernelGGL(idw_bwd_coords_kernel, dim3(grid_of((long long)b * n)), dim3(256), 0,
                     (hipStream_t)stream, b, n, s, c, ref, qry, vals, idx, dout, drow, dqry, warp);
  return (int)hipGetLastError();
}
