// Fused WeightNet-weighted neighbour sums: PointConvFlow's two cost sums (reference
// pointconv_util.py:2039-2112):
//
//   w[q,k,:]  = ReLU(W2 ReLU(W1 ReLU(W0 dir[q,k] + b0) + b1) + b2)        (C channels)
//   out[q,c]  = sum_k w[q,k,c] * v(q,k,c)
//   v(q,k,c)  = v[q,k,c]                  dense     (point-to-patch: the MLP'd patch)
//             = v[b, idx[q,k], c]         gathered  (patch-to-patch: the cost of neighbours)
//
// The reference materialises w (B,C,K,N) with three 1x1 convs, the product w * v and, for the
// patch-to-patch sum, the gathered (B,N,K,C) copy of the point-to-patch cost -- four
// K-times-larger tensors per sum.  Here one wave owns one query: lanes k < K run the row's
// 3 -> 8 -> 8 hidden layers once, the 8 hidden values are broadcast per neighbour (readlane),
// and each lane computes its channel's weight and accumulates the product in a register; only
// (B,N,C) leaves the chip.
//
// Backward (same layout): dv rows (B,N,K,C) = w * dout (the dense case's gradient; for the
// gathered case the caller sums them per point through the kNN CSR), the W2 / b2 gradients in
// per-lane registers, dh1 = W2^T d2 by a butterfly over the channel lanes, and the 3 -> 8 -> 8
// layers' backward row-parallel (lanes k) from per-wave LDS factors; the 104 small parameter
// gradients are then reduced over the query's rows by lane-owned entries.  Every workgroup
// writes one slab row; colsum adds the slabs in slab order (no float atomics).
#include <algorithm>

#include "kdpc_common.h"

using namespace kdpc;

namespace {

constexpr int kH = 8;        // hidden width (WeightNet hidden_unit [8, 8])
constexpr int kMaxK = 64;    // neighbours per query (one lane each in the hidden pass)
constexpr int kWaves = 4;    // per workgroup
constexpr int kSmall = 3 * kH + kH + kH * kH + kH;  // W0 | b0 | W1 | b1 = 104
// packed parameter layout (floats): W0 8x3 | b0 8 | W1 8x8 | b1 8 | W2 Cx8 | b2 C
constexpr int oW0 = 0, oB0 = 24, oW1 = 32, oB1 = 96, oW2 = 104;

struct Prm {
  const float *w0, *b0, *w1, *b1, *w2, *b2;  // nn.Conv2d tensors, row-major
};

__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }

// y = W x + b with W (O x I): ascending-i fma chain, then the bias (as weightnet.hip)
template <int O, int I>
__device__ __forceinline__ void dense(const float* w, const float* b, const float (&x)[I],
                                      float (&y)[O]) {
#pragma unroll
  for (int o = 0; o < O; ++o) {
    float a = __fmul_rn(w[o * I], x[0]);
#pragma unroll
    for (int i = 1; i < I; ++i) a = __builtin_fmaf(w[o * I + i], x[i], a);
    y[o] = __fadd_rn(a, b[o]);
  }
}

// lane k < K: the row's direction and hidden layers (zeros elsewhere)
__device__ __forceinline__ void hidden(const Prm& p, const float* dir, long long row, bool live,
                                       float (&d)[3], float (&h0)[kH], float (&h1)[kH]) {
#pragma unroll
  for (int i = 0; i < 3; ++i) d[i] = live ? dir[row * 3 + i] : 0.f;
  dense<kH, 3>(p.w0, p.b0, d, h0);
#pragma unroll
  for (int i = 0; i < kH; ++i) h0[i] = relu(h0[i]);
  dense<kH, kH>(p.w1, p.b1, h0, h1);
#pragma unroll
  for (int i = 0; i < kH; ++i) h1[i] = relu(h1[i]);
}

__device__ __forceinline__ float bcast(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// channel lane c's pre-activation of neighbour row kk: W2[c] . h1 + b2[c]
__device__ __forceinline__ float z2_of(const float (&w2r)[kH], float b2r, const float (&hs)[kH]) {
  float a = __fmul_rn(w2r[0], hs[0]);
#pragma unroll
  for (int j = 1; j < kH; ++j) a = __builtin_fmaf(w2r[j], hs[j], a);
  return __fadd_rn(a, b2r);
}

template <int CB>
__global__ __launch_bounds__(256) void wsum_fwd_kernel(int nq, int n, int m, int k, int c,
                                                       int qpw, const float* __restrict__ dir,
                                                       const int* __restrict__ idx,
                                                       const float* __restrict__ v, Prm p,
                                                       float* __restrict__ out) {
  const int lane = lane_id();
  const int q0 = (blockIdx.x * kWaves + (threadIdx.x >> 6)) * qpw;
  float w2r[CB][kH], b2r[CB];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const int cc = lane + 64 * cb;
#pragma unroll
    for (int j = 0; j < kH; ++j) w2r[cb][j] = cc < c ? p.w2[cc * kH + j] : 0.f;
    b2r[cb] = cc < c ? p.b2[cc] : 0.f;
  }
  for (int q = q0; q < min(nq, q0 + qpw); ++q) {
    const long long qk = (long long)q * k;
    const bool live = lane < k;
    float d[3], h0[kH], h1[kH];
    hidden(p, dir, qk + lane, live, d, h0, h1);
    const long long vb = (long long)(q / n) * m;  // gathered table rows of q's batch
    const int nb = (idx && live) ? idx[qk + lane] : 0;
    float acc[CB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) acc[cb] = 0.f;
    for (int kk = 0; kk < k; ++kk) {
      float hs[kH];
#pragma unroll
      for (int j = 0; j < kH; ++j) hs[j] = bcast(h1[j], kk);
      const long long vrow = idx ? vb + __builtin_amdgcn_readlane(nb, kk) : qk + kk;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        const int cc = lane + 64 * cb;
        if (cc < c) {
          const float w = relu(z2_of(w2r[cb], b2r[cb], hs));
          acc[cb] = __fadd_rn(acc[cb], __fmul_rn(w, v[vrow * c + cc]));
        }
      }
    }
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      const int cc = lane + 64 * cb;
      if (cc < c) out[(long long)q * c + cc] = acc[cb];
    }
  }
}

// per-row factor layout of the hidden-layer backward (LDS, one row per neighbour)
constexpr int fH0 = 0, fD1 = kH, fD0 = 2 * kH, fDir = 3 * kH, kFS = 3 * kH + 4;  // 28

template <int CB>
__global__ __launch_bounds__(256) void wsum_bwd_kernel(
    int nq, int n, int m, int k, int c, int qpw, const float* __restrict__ dir,
    const int* __restrict__ idx, const float* __restrict__ v, Prm p,
    const float* __restrict__ dout, float* __restrict__ dv_rows, float* __restrict__ ddir,
    float* __restrict__ slab) {
  __shared__ float fac_all[kWaves][kMaxK * kFS];
  __shared__ float dh1_all[kWaves][kMaxK * kH];
  __shared__ float red[kSmall + 9 * 256];  // workgroup partials (up to C = 256)
  const int wave = threadIdx.x >> 6, lane = lane_id();
  float* fac = fac_all[wave];
  float* dh1s = dh1_all[wave];
  const int q0 = (blockIdx.x * kWaves + wave) * qpw;
  float w2r[CB][kH], b2r[CB], gw2[CB][kH], gb2[CB];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) {
    const int cc = lane + 64 * cb;
#pragma unroll
    for (int j = 0; j < kH; ++j) {
      w2r[cb][j] = cc < c ? p.w2[cc * kH + j] : 0.f;
      gw2[cb][j] = 0.f;
    }
    b2r[cb] = cc < c ? p.b2[cc] : 0.f;
    gb2[cb] = 0.f;
  }
  // the two small-parameter entries this lane owns: gradient = sum over rows of
  // fac[fa] * fac[fb] (fb < 0: bias, fac[fa] alone)
  int fa[2], fb[2];
  float ge[2] = {0.f, 0.f};
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int e = lane + 64 * s2;
    fa[s2] = -1;
    fb[s2] = -1;
    if (e < oB0) { fa[s2] = fD0 + e / 3; fb[s2] = fDir + e % 3; }
    else if (e < oW1) { fa[s2] = fD0 + (e - oB0); }
    else if (e < oB1) { fa[s2] = fD1 + (e - oW1) / kH; fb[s2] = fH0 + (e - oW1) % kH; }
    else if (e < kSmall) { fa[s2] = fD1 + (e - oB1); }
  }
  for (int q = q0; q < min(nq, q0 + qpw); ++q) {
    const long long qk = (long long)q * k;
    const bool live = lane < k;
    float d[3], h0[kH], h1[kH];
    hidden(p, dir, qk + lane, live, d, h0, h1);
    const long long vb = (long long)(q / n) * m;
    const int nb = (idx && live) ? idx[qk + lane] : 0;
    float dq[CB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) {
      const int cc = lane + 64 * cb;
      dq[cb] = cc < c ? dout[(long long)q * c + cc] : 0.f;
    }
    for (int kk = 0; kk < k; ++kk) {
      float hs[kH];
#pragma unroll
      for (int j = 0; j < kH; ++j) hs[j] = bcast(h1[j], kk);
      const long long vrow = idx ? vb + __builtin_amdgcn_readlane(nb, kk) : qk + kk;
      float pj[kH];
#pragma unroll
      for (int j = 0; j < kH; ++j) pj[j] = 0.f;
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        const int cc = lane + 64 * cb;
        if (cc < c) {
          const float z = z2_of(w2r[cb], b2r[cb], hs);
          const float w = relu(z);
          dv_rows[(qk + kk) * c + cc] = __fmul_rn(w, dq[cb]);
          const float d2 = z > 0.f ? __fmul_rn(dq[cb], v[vrow * c + cc]) : 0.f;
#pragma unroll
          for (int j = 0; j < kH; ++j) {
            gw2[cb][j] = __builtin_fmaf(d2, hs[j], gw2[cb][j]);
            pj[j] = __builtin_fmaf(w2r[cb][j], d2, pj[j]);
          }
          gb2[cb] = __fadd_rn(gb2[cb], d2);
        }
      }
      // dh1[kk][j] = sum over the channel lanes (butterfly; every lane ends with the sum)
#pragma unroll
      for (int j = 0; j < kH; ++j) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) pj[j] = __fadd_rn(pj[j], __shfl_xor(pj[j], o, kWave));
      }
      if (lane == 0) {
#pragma unroll
        for (int j = 0; j < kH; ++j) dh1s[kk * kH + j] = pj[j];
      }
    }
    // hidden layers' backward, row-parallel (lane = neighbour row; LDS ops of one wave are
    // ordered, so lane 0's dh1 stores above are visible)
    if (live) {
      float dz1[kH], dz0[kH];
#pragma unroll
      for (int i = 0; i < kH; ++i) dz1[i] = h1[i] > 0.f ? dh1s[lane * kH + i] : 0.f;
#pragma unroll
      for (int j = 0; j < kH; ++j) {
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < kH; ++i) a = __builtin_fmaf(p.w1[i * kH + j], dz1[i], a);
        dz0[j] = h0[j] > 0.f ? a : 0.f;
      }
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < kH; ++i) a = __builtin_fmaf(p.w0[i * 3 + t], dz0[i], a);
        ddir[(qk + lane) * 3 + t] = a;
      }
      float* f = fac + lane * kFS;
#pragma unroll
      for (int i = 0; i < kH; ++i) {
        f[fH0 + i] = h0[i];
        f[fD1 + i] = dz1[i];
        f[fD0 + i] = dz0[i];
      }
#pragma unroll
      for (int t = 0; t < 3; ++t) f[fDir + t] = d[t];
    }
    // small-parameter gradients: lane-owned entries over the query's rows, ascending row
    for (int kk = 0; kk < k; ++kk) {
      const float* f = fac + kk * kFS;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        if (fa[s2] >= 0)
          ge[s2] = fb[s2] >= 0 ? __builtin_fmaf(f[fa[s2]], f[fb[s2]], ge[s2]) : __fadd_rn(ge[s2], f[fa[s2]]);
      }
    }
  }
  // workgroup partial: waves add into one LDS row in wave order, then one slab row
  const int np = kSmall + 9 * c;
  for (int w = 0; w < kWaves; ++w) {
    if (wave == w) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int e = lane + 64 * s2;
        if (e < kSmall) red[e] = w ? __fadd_rn(red[e], ge[s2]) : ge[s2];
      }
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) {
        const int cc = lane + 64 * cb;
        if (cc < c) {
#pragma unroll
          for (int j = 0; j < kH; ++j) {
            float* e = red + oW2 + cc * kH + j;
            *e = w ? __fadd_rn(*e, gw2[cb][j]) : gw2[cb][j];
          }
          float* e = red + oW2 + kH * c + cc;
          *e = w ? __fadd_rn(*e, gb2[cb]) : gb2[cb];
        }
      }
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < np; e += blockDim.x) slab[(long long)blockIdx.x * np + e] = red[e];
}

inline int qpw_of(long long nq) { return (int)std::max(1ll, divupll(nq, 256ll * 8 * kWaves)); }
inline int grid_of(long long nq) { return (int)divupll(nq, (long long)kWaves * qpw_of(nq)); }

bool wsum_ok(int b, int n, int m, int k, int c) {
  return b > 0 && n > 0 && m > 0 && k >= 1 && k <= kMaxK && c >= 1 && c <= 256 &&
         (long long)b * n * k * c < (1ll << 31) && (long long)b * m * c < (1ll << 31);
}


}  // namespace

KDPC_API int kdpc_wn_wsum_param_count(int c) { return kSmall + 9 * c; }

// Forward.  dir (B,N,K,3); idx (B,N,K) int32 in [0,M) or null (dense); v (B,N,K,C) dense or
// (B,M,C) gathered; W0 (8,3) b0 (8) W1 (8,8) b1 (8) W2 (C,8) b2 (C) (the WeightNet's
// nn.Conv2d tensors, row-major); out (B,N,C).
KDPC_API int kdpc_wn_wsum_fwd(int b, int n, int m, int k, int c, const float* dir, const int* idx,
                              const float* v, const float* w0, const float* b0, const float* w1,
                              const float* b1, const float* w2, const float* b2, float* out,
                              void* stream) {
  KDPC_CHECK_ARG(wsum_ok(b, n, idx ? m : 1, k, c) && dir && v && out);
  KDPC_CHECK_ARG(w0 && b0 && w1 && b1 && w2 && b2);
  const long long nq = (long long)b * n;
  const int qpw = qpw_of(nq);
  const Prm p{w0, b0, w1, b1, w2, b2};
  hipStream_t st = (hipStream_t)stream;
#define KDPC_WS_FWD(CB)                                                                       \
  hipLaunchKernelGGL(wsum_fwd_kernel<CB>, dim3(grid_of(nq)), dim3(256), 0, st, (int)nq, n, m, k, \
                     c, qpw, dir, idx, v, p, out)
  if (c <= 64) KDPC_WS_FWD(1);
  else if (c <= 128) KDPC_WS_FWD(2);
  else KDPC_WS_FWD(4);
#undef KDPC_WS_FWD
  KDPC_RETURN_LAUNCH();
}

KDPC_API size_t kdpc_wn_wsum_bwd_workspace_bytes(int b, int n, int c) {
  if (b <= 0 || n <= 0 || c < 1 || c > 256) return 0;
  const long long nslabs = grid_of((long long)b * n);
  const int np = kSmall + 9 * c;
  return (size_t)(nslabs * np + colsum_scratch_floats((int)nslabs, np)) * sizeof(float);
}

// Backward.  dout (B,N,C) -> dv_rows (B,N,K,C) = w * dout (the dense v's gradient; for a
// gathered v the caller sums the rows per point through the CSR of idx), ddir (B,N,K,3),
// dparams = packed [W0 | b0 | W1 | b1 | W2 | b2] gradients.
KDPC_API int kdpc_wn_wsum_bwd(int b, int n, int m, int k, int c, const float* dir, const int* idx,
                              const float* v, const float* w0, const float* b0, const float* w1,
                              const float* b1, const float* w2, const float* b2,
                              const float* dout, float* dv_rows, float* ddir, float* dparams,
                              void* workspace, size_t workspace_bytes, void* stream) {
  KDPC_CHECK_ARG(wsum_ok(b, n, idx ? m : 1, k, c) && dir && v && dout && dv_rows && ddir &&
                 workspace && dparams);
  KDPC_CHECK_ARG(w0 && b0 && w1 && b1 && w2 && b2);
  KDPC_CHECK_ARG(workspace_bytes >= kdpc_wn_wsum_bwd_workspace_bytes(b, n, c));
  const long long nq = (long long)b * n;
  const int qpw = qpw_of(nq);
  const int grid = grid_of(nq);
  const Prm p{w0, b0, w1, b1, w2, b2};
  hipStream_t st = (hipStream_t)stream;
  float* slab = (float*)workspace;
#define KDPC_WS_BWD(CB)                                                                       \
  hipLaunchKernelGGL(wsum_bwd_kernel<CB>, dim3(grid), dim3(256), 0, st, (int)nq, n, m, k, c, \
                     qpw, dir, idx, v, p, dout, dv_rows, ddir, slab)
  if (c <= 64) KDPC_WS_BWD(1);
  else if (c <= 128) KDPC_WS_BWD(2);
  else KDPC_WS_BWD(4);
#undef KDPC_WS_BWD
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const int np = kSmall + 9 * c;
  return (int)colsum(grid, np, slab, dparams, slab + (size_t)grid * np, st);
}
