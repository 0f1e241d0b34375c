// Wide cost volume: CrossLayerLight.cross / FlowEmbeddingLayer (reference
// pointconv_util.py:1826-1850, :1497-1517) at the levels whose channel widths (Din, Dout >=
// 128) are too wide for the one-wave-per-query kernel of cost_volume.hip (its W1 fragments
// would need 256+ VGPRs).  Same math:
//     h0[n,k,:] = LeakyReLU((P2[j_k] + P1[n]) + (Wpos (x2[j_k] - x1[n]) + bpos))
//     z1 = h0 W1^T + b1 (a plain GEMM: stays on the BLAS library),  out[n,:] = max_k LReLU(z1)
// Everything around the GEMM is fused instead of materialised op by op (gather, broadcast
// add, K=3 position GEMM, add, activation, activation, max, and the same again backward):
//   cvw_h0_kernel        gather + position transform + add + LeakyReLU -> h0 (rows, Din)
//   cvw_max_kernel       LeakyReLU + max over K + first argmax (u8)     -> out, amax
//   cvw_max_bwd_kernel   dense dz1 (the max routes each channel to one row) and the
//                        per-query activation-scaled gradient (for db1)
//   cvw_h0_bwd_kernel    dz0 = dh0 * LReLU'(h0) in place, dP1 = sum_k dz0, and per-wave dWpos
//                        partials (fixed assignment, summed by colsum: no float atomics)
// LeakyReLU' is read from the sign of the activation output (slope 0.1 > 0: h > 0 <=> z > 0,
// and z = 0 takes the slope as torch's leaky_relu_backward does).
#include <algorithm>

#include "kdpc_common.h"

using namespace kdpc;

namespace {

constexpr float kSlope = 0.1f;
constexpr int kBlock = 256;
constexpr int kBwdWgs = 1024;  // h0 backward: fixed grid (4 waves each) -> dWpos slab rows

__device__ __forceinline__ float lrelu(float x) { return x > 0.f ? x : x * kSlope; }

// one thread per (row, 4 channels); rows = (b, n, k) flattened
__global__ __launch_bounds__(kBlock) void cvw_h0_kernel(long long rows, int n1, int n2, int k,
                                                        int d, const float* __restrict__ x1,
                                                        const float* __restrict__ x2,
                                                        const int* __restrict__ idx,
                                                        const float* __restrict__ p1,
                                                        const float* __restrict__ p2,
                                                        const float* __restrict__ wpos,
                                                        const float* __restrict__ bpos,
                                                        float* __restrict__ h0) {
  const int d4 = d >> 2;
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  const long long row = t / d4;
  if (row >= rows) return;
  const int c0 = (int)(t - row * d4) * 4;
  const long long bn = row / k;  // b * n1 + n
  const long long b = bn / n1;
  const int j = idx[row];
  const float* q = x1 + bn * 3;
  const float* r = x2 + (b * n2 + j) * 3;
  const float dx = r[0] - q[0], dy = r[1] - q[1], dz = r[2] - q[2];
  const float4 g2 = *reinterpret_cast<const float4*>(p2 + (b * n2 + j) * d + c0);
  const float4 g1 = *reinterpret_cast<const float4*>(p1 + bn * d + c0);
  const float gv[4] = {g2.x, g2.y, g2.z, g2.w}, pv[4] = {g1.x, g1.y, g1.z, g1.w};
  float h[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = c0 + i;
    const float pos = __fadd_rn(
        __builtin_fmaf(wpos[c * 3 + 2], dz,
                       __builtin_fmaf(wpos[c * 3 + 1], dy, __fmul_rn(wpos[c * 3], dx))),
        bpos[c]);
    h[i] = lrelu(__fadd_rn(__fadd_rn(gv[i], pv[i]), pos));
  }
  *reinterpret_cast<float4*>(h0 + row * d + c0) = make_float4(h[0], h[1], h[2], h[3]);
}

// one thread per (query, output channel): out = LReLU(max_k z1), amax = first maximal k
__global__ __launch_bounds__(kBlock) void cvw_max_kernel(long long nq, int k, int dout,
                                                         const float* __restrict__ z1,
                                                         float* __restrict__ out,
                                                         unsigned char* __restrict__ amax) {
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (t >= nq * dout) return;
  const long long q = t / dout;
  const int c = (int)(t - q * dout);
  const float* z = z1 + q * k * dout + c;
  float m = z[0];
  int a = 0;
#pragma unroll 8
  for (int kk = 1; kk < k; ++kk) {
    const float v = z[(long long)kk * dout];
    if (v > m) {
      m = v;
      a = kk;
    }
  }
  out[t] = lrelu(m);
  amax[t] = (unsigned char)a;
}

// dz1 (rows, Dout) dense: g at (argmax row, c), 0 elsewhere; gsc (nq, Dout) = g
__global__ __launch_bounds__(kBlock) void cvw_max_bwd_kernel(long long nq, int k, int dout,
                                                             const float* __restrict__ gout,
                                                             const float* __restrict__ out,
                                                             const unsigned char* __restrict__ amax,
                                                             float* __restrict__ dz1,
                                                             float* __restrict__ gsc) {
  const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (t >= nq * dout) return;
  const long long q = t / dout;
  const int c = (int)(t - q * dout);
  const float g = out[t] > 0.f ? gout[t] : gout[t] * kSlope;
  gsc[t] = g;
  const int a = amax[t];
  float* dz = dz1 + q * k * dout + c;
#pragma unroll 8
  for (int kk = 0; kk < k; ++kk) dz[(long long)kk * dout] = kk == a ? g : 0.f;
}

// One wave per query (grid-stride over queries, fixed grid): lane l owns channels
// l + 64 i.  dz (rows, D) holds dh0 on entry and dz0 on exit.
template <int D>
__global__ __launch_bounds__(256) void cvw_h0_bwd_kernel(int nq, int n1, int n2, int k,
                                                         const float* __restrict__ x1,
                                                         const float* __restrict__ x2,
                                                         const int* __restrict__ idx,
                                                         const float* __restrict__ h0,
                                                         float* __restrict__ dz,
                                                         float* __restrict__ dp1,
                                                         float* __restrict__ slab) {
  constexpr int CPL = D / kWave;
  const int lane = lane_id();
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nw = gridDim.x * 4;
  float aw[CPL][3];
#pragma unroll
  for (int i = 0; i < CPL; ++i) aw[i][0] = aw[i][1] = aw[i][2] = 0.f;
  for (int q = wid; q < nq; q += nw) {
    const long long b = q / n1;
    const float qx = x1[(long long)q * 3], qy = x1[(long long)q * 3 + 1],
                qz = x1[(long long)q * 3 + 2];
    float acc[CPL];
#pragma unroll
    for (int i = 0; i < CPL; ++i) acc[i] = 0.f;
#pragma unroll 8
    for (int kk = 0; kk < k; ++kk) {
      const long long row = (long long)q * k + kk;
      const int j = idx[row];
      const float* r = x2 + (b * n2 + j) * 3;
      const float dx = r[0] - qx, dy = r[1] - qy, dzz = r[2] - qz;
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        const long long o = row * D + lane + kWave * i;
        const float g = dz[o];
        const float z = h0[o] > 0.f ? g : g * kSlope;
        dz[o] = z;
        acc[i] = __fadd_rn(acc[i], z);
        aw[i][0] = __builtin_fmaf(z, dx, aw[i][0]);
        aw[i][1] = __builtin_fmaf(z, dy, aw[i][1]);
        aw[i][2] = __builtin_fmaf(z, dzz, aw[i][2]);
      }
    }
#pragma unroll
    for (int i = 0; i < CPL; ++i) dp1[(long long)q * D + lane + kWave * i] = acc[i];
  }
  float* sl = slab + (long long)wid * D * 3;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + kWave * i;
    sl[c * 3 + 0] = aw[i][0];
    sl[c * 3 + 1] = aw[i][1];
    sl[c * 3 + 2] = aw[i][2];
  }
}

}  // namespace

// ------------------------------------------------------------------------------ C ABI
KDPC_API int kdpc_cost_volume_wide_supported(int din, int dout, int k) {
  return (din == 64 || din == 128 || din == 256 || din == 512) && dout >= 1 && k >= 1 &&
         k <= 255;
}

KDPC_API int kdpc_cost_volume_wide_h0(int b, int n1, int n2, int k, int din, const float* x1,
                                      const float* x2, const int* idx, const float* p1,
                                      const float* p2, const float* wpos, const float* bpos,
                                      float* h0, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n1 >= 0 && n2 > 0 && k >= 1 && din > 0 && din % 4 == 0);
  const long long rows = (long long)b * n1 * k;
  if (rows == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(x1 && x2 && idx && p1 && p2 && wpos && bpos && h0);
  const long long threads = rows * (din / 4);
  hipLaunchKernelGGL(cvw_h0_kernel, dim3((unsigned)divupll(threads, kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, rows, n1, n2, k, din, x1, x2, idx, p1, p2, wpos, bpos,
                     h0);
  KDPC_RETURN_LAUNCH();
}

KDPC_API int kdpc_cost_volume_wide_max(int b, int n1, int k, int dout, const float* z1,
                                       float* out, unsigned char* amax, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n1 >= 0 && k >= 1 && k <= 255 && dout > 0);
  const long long nq = (long long)b * n1;
  if (nq == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(z1 && out && amax);
  hipLaunchKernelGGL(cvw_max_kernel, dim3((unsigned)divupll(nq * dout, kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, nq, k, dout, z1, out, amax);
  KDPC_RETURN_LAUNCH();
}

KDPC_API int kdpc_cost_volume_wide_max_bwd(int b, int n1, int k, int dout, const float* gout,
                                           const float* out, const unsigned char* amax,
                                           float* dz1, float* gsc, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n1 >= 0 && k >= 1 && k <= 255 && dout > 0);
  const long long nq = (long long)b * n1;
  if (nq == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(gout && out && amax && dz1 && gsc);
  hipLaunchKernelGGL(cvw_max_bwd_kernel, dim3((unsigned)divupll(nq * dout, kBlock)), dim3(kBlock),
                     0, (hipStream_t)stream, nq, k, dout, gout, out, amax, dz1, gsc);
  KDPC_RETURN_LAUNCH();
}

// Rows of the dWpos slab written by kdpc_cost_volume_wide_h0_bwd (each din*3 floats).
KDPC_API int kdpc_cost_volume_wide_slab_rows(void) { return kBwdWgs * 4; }

KDPC_API int kdpc_cost_volume_wide_h0_bwd(int b, int n1, int n2, int k, int din,
                                          const float* x1, const float* x2, const int* idx,
                                          const float* h0, float* dz, float* dp1, float* slab,
                                          void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n1 >= 0 && n2 > 0 && k >= 1 &&
                 kdpc_cost_volume_wide_supported(din, 4, k));
  KDPC_CHECK_ARG(slab && ((long long)b * n1 == 0 || (x1 && x2 && idx && h0 && dz && dp1)));
  KDPC_CHECK_ARG((long long)b * n1 < (1ll << 31));
  const int nq = b * n1;
  hipStream_t st = (hipStream_t)stream;
  // every slab row is written (nq == 0 -> zero partials)
  switch (din) {
    case 64:
      hipLaunchKernelGGL(cvw_h0_bwd_kernel<64>, dim3(kBwdWgs), dim3(256), 0, st, nq, n1, n2, k,
                         x1, x2, idx, h0, dz, dp1, slab);
      break;
    case 128:
      hipLaunchKernelGGL(cvw_h0_bwd_kernel<128>, dim3(kBwdWgs), dim3(256), 0, st, nq, n1, n2, k,
                         x1, x2, idx, h0, dz, dp1, slab);
      break;
    case 256:
      hipLaunchKernelGGL(cvw_h0_bwd_kernel<256>, dim3(kBwdWgs), dim3(256), 0, st, nq, n1, n2, k,
                         x1, x2, idx, h0, dz, dp1, slab);
      break;
    default:
      hipLaunchKernelGGL(cvw_h0_bwd_kernel<512>, dim3(kBwdWgs), dim3(256), 0, st, nq, n1, n2, k,
                         x1, x2, idx, h0, dz, dp1, slab);
      break;
  }
  KDPC_RETURN_LAUNCH();
}
