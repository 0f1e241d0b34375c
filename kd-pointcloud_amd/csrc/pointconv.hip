// Fused PointConv neighbourhood contraction (reference pointconv_util.py:217-258, 401-446):
//
//   G[r,k,:]  = cat(xyz[idx[r,k]] - center[r], feats[idx[r,k]])        (C = 3 + D)
//   A[r, c*W + w] = sum_k G[r,k,c] * Wt[r,k,w]                          (c-major, W = 16)
//
// which the reference evaluates as group -> cat -> permute -> batched (C x K)(K x W) matmul
// over B*S tiny matrices (rocBLAS runs that at a few % of the chip, profiles/round01).
// Here a workgroup takes RB rows: the K gathered neighbour rows (coalesced row reads of the
// point-major feature table) and the K x W weights go to LDS, and every thread produces
// consecutive A elements of the row (coalesced stores).  Summation over k is in ascending
// order, one fma per term, like the reference's k-ordered product.
//
// Backward, same staging plus the row of dA:
//   dG[r,k,c]  = sum_w dA[r, c*W+w] * Wt[r,k,w]      -> per-(r,k) rows, summed per point by
//                                                        the caller through the kNN CSR
//   dWt[r,k,w] = sum_c dA[r, c*W+w] * G[r,k,c]
//   dcenter[r] = -sum_k dG[r,k,0:3]
#include "kdpc_common.h"

using namespace kdpc;

namespace {

constexpr int kW = 16;          // WeightNet output width (weightnet=16 in every model layer)
constexpr int kLdsBudget = 48 * 1024;

// stage G (K x C, padded row LDC) and Wt (K x W) of row r into LDS
__device__ __forceinline__ void stage_row(int r, int k, int d, int ldc, const float* __restrict__ xyz_b,
                                          const float* __restrict__ center,
                                          const float* __restrict__ feats_b,
                                          const int* __restrict__ idx, const float* __restrict__ wt,
                                          float* g, float* w, int tid, int nthr) {
  const int c = 3 + d;
  const float cx = center[(long long)r * 3 + 0], cy = center[(long long)r * 3 + 1],
              cz = center[(long long)r * 3 + 2];
  for (int e = tid; e < k * c; e += nthr) {
    const int kk = e / c, cc = e - kk * c;
    const int j = idx[(long long)r * k + kk];
    float v;
    if (cc < 3) {
      const float ctr = cc == 0 ? cx : (cc == 1 ? cy : cz);
      v = xyz_b[(long long)j * 3 + cc] - ctr;
    } else {
      v = feats_b[(long long)j * d + (cc - 3)];
    }
    g[kk * ldc + cc] = v;
  }
  for (int e = tid; e < k * kW; e += nthr) w[e] = wt[(long long)r * k * kW + e];
}

__global__ __launch_bounds__(256) void pointconv_contract_fwd_kernel(
    int n, int s, int k, int d, int rb, const float* __restrict__ xyz,
    const float* __restrict__ center, const float* __restrict__ feats,
    const int* __restrict__ idx, const float* __restrict__ wt, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int b = blockIdx.y;
  const int c = 3 + d;
  const int ldc = c + 1;
  const int row_floats = k * ldc + k * kW;
  const int r0 = blockIdx.x * rb;
  const float* xyz_b = xyz + (long long)b * n * 3;
  const float* feats_b = feats + (long long)b * n * d;
  const float* cen = center + (long long)b * s * 3;
  const int* ib = idx + (long long)b * s * k;
  const float* wb = wt + (long long)b * s * k * kW;
  const int rows = min(rb, s - r0);
  for (int q = 0; q < rows; ++q) {
    float* g = lds + q * row_floats;
    stage_row(r0 + q, k, d, ldc, xyz_b, cen, feats_b, ib, wb, g, g + k * ldc, threadIdx.x,
              blockDim.x);
  }
  __syncthreads();
  const int cw = c * kW;
  for (int q = 0; q < rows; ++q) {
    const float* g = lds + q * row_floats;
    const float* w = g + k * ldc;
    float* o = out + ((long long)b * s + r0 + q) * cw;
    for (int e = threadIdx.x; e < cw; e += blockDim.x) {
      const int cc = e >> 4, ww = e & (kW - 1);
      float acc = 0.f;
      for (int kk = 0; kk < k; ++kk) acc = __builtin_fmaf(g[kk * ldc + cc], w[kk * kW + ww], acc);
      o[e] = acc;
    }
  }
}

__global__ __launch_bounds__(256) void pointconv_contract_bwd_kernel(
    int n, int s, int k, int d, int rb, const float* __restrict__ xyz,
    const float* __restrict__ center, const float* __restrict__ feats,
    const int* __restrict__ idx, const float* __restrict__ wt, const float* __restrict__ dout,
    float* __restrict__ dg_rows, float* __restrict__ dwt, float* __restrict__ dcenter) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int b = blockIdx.y;
  const int c = 3 + d;
  const int ldc = c + 1;
  const int cw = c * kW;
  const int row_floats = k * ldc + k * kW + cw;
  const int r0 = blockIdx.x * rb;
  const float* xyz_b = xyz + (long long)b * n * 3;
  const float* feats_b = feats + (long long)b * n * d;
  const float* cen = center + (long long)b * s * 3;
  const int* ib = idx + (long long)b * s * k;
  const float* wb = wt + (long long)b * s * k * kW;
  const int rows = min(rb, s - r0);
  for (int q = 0; q < rows; ++q) {
    float* g = lds + q * row_floats;
    stage_row(r0 + q, k, d, ldc, xyz_b, cen, feats_b, ib, wb, g, g + k * ldc, threadIdx.x,
              blockDim.x);
    float* da = g + k * ldc + k * kW;
    const float* src = dout + ((long long)b * s + r0 + q) * cw;
    for (int e = threadIdx.x; e < cw; e += blockDim.x) da[e] = src[e];
  }
  __syncthreads();
  for (int q = 0; q < rows; ++q) {
    const float* g = lds + q * row_floats;
    const float* w = g + k * ldc;
    const float* da = w + k * kW;
    const long long rr = (long long)b * s + r0 + q;
    // dG[k][c] = sum_w dA[c*W+w] * Wt[k][w]
    float* dgr = dg_rows + rr * k * c;
    for (int e = threadIdx.x; e < k * c; e += blockDim.x) {
      const int kk = e / c, cc = e - kk * c;
      float acc = 0.f;
#pragma unroll
      for (int ww = 0; ww < kW; ++ww) acc = __builtin_fmaf(da[cc * kW + ww], w[kk * kW + ww], acc);
      dgr[e] = acc;
    }
    // dWt[k][w] = sum_c dA[c*W+w] * G[k][c]
    float* dw = dwt + rr * k * kW;
    for (int e = threadIdx.x; e < k * kW; e += blockDim.x) {
      const int kk = e >> 4, ww = e & (kW - 1);
      float acc = 0.f;
      for (int cc = 0; cc < c; ++cc) acc = __builtin_fmaf(da[cc * kW + ww], g[kk * ldc + cc], acc);
      dw[e] = acc;
    }
  }
  __syncthreads();
  // dcenter[r][i] = -sum_k dG[r,k,i]  (ascending k), recomputed from LDS
  for (int e = threadIdx.x; e < rows * 3; e += blockDim.x) {
    const int q = e / 3, i = e - q * 3;
    const float* g = lds + q * row_floats;
    const float* w = g + k * ldc;
    const float* da = w + k * kW;
    float sum = 0.f;
    for (int kk = 0; kk < k; ++kk) {
      float acc = 0.f;
#pragma unroll
      for (int ww = 0; ww < kW; ++ww) acc = __builtin_fmaf(da[i * kW + ww], w[kk * kW + ww], acc);
      sum = __fadd_rn(sum, acc);
    }
    dcenter[((long long)b * s + r0 + q) * 3 + i] = -sum;
  }
}

constexpr size_t kMaxLds = 160 * 1024;

inline void allow_lds(const void* fn) {
  // one-time opt-in to the full 160 KiB of gfx950 LDS for the wide (C=515) levels
  static const void* done[4] = {nullptr, nullptr, nullptr, nullptr};
  for (auto& d : done) {
    if (d == fn) return;
    if (d == nullptr) {
      hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLds);
      d = fn;
      return;
    }
  }
}

inline int rows_per_block(int k, int c, bool bwd) {
  const int row_floats = k * (c + 1) + k * kW + (bwd ? c * kW : 0);
  const int rb = kLdsBudget / (row_floats * 4);
  return rb < 1 ? 1 : (rb > 8 ? 8 : rb);
}

}  // namespace

// A (B,S,16*(3+D)) from xyz (B,N,3), center (B,S,3), feats (B,N,D) point-major,
// idx (B,S,K), wt (B,S,K,16).  One row's K x (4+D) + K x 16 floats must fit the 160 KiB LDS.
KDPC_API int kdpc_pointconv_contract_fwd(int b, int n, int s, int k, int d, const float* xyz,
                                         const float* center, const float* feats, const int* idx,
                                         const float* wt, float* out, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n > 0 && s >= 0 && k >= 1 && d >= 0 && b <= 65535);
  if ((long long)b * s == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(xyz && center && idx && wt && out && (d == 0 || feats));
  const int c = 3 + d;
  const int rb = rows_per_block(k, c, false);
  const size_t lds = (size_t)rb * (k * (c + 1) + k * kW) * sizeof(float);
  KDPC_CHECK_ARG(lds <= kMaxLds);
  allow_lds((const void*)pointconv_contract_fwd_kernel);
  hipLaunchKernelGGL(pointconv_contract_fwd_kernel, dim3(divup(s, rb), b), dim3(256), lds,
                     (hipStream_t)stream, n, s, k, d, rb, xyz, center, feats, idx, wt, out);
  KDPC_RETURN_LAUNCH();
}

// dout (B,S,16*(3+D)) -> dg_rows (B,S,K,3+D) (per-neighbour rows of dG: sum them per point
// with kdpc_group_rows_grad_csr; columns 0..2 are d(xyz), 3.. are d(feats)),
// dwt (B,S,K,16), dcenter (B,S,3).
KDPC_API int kdpc_pointconv_contract_bwd(int b, int n, int s, int k, int d, const float* xyz,
                                         const float* center, const float* feats, const int* idx,
                                         const float* wt, const float* dout, float* dg_rows,
                                         float* dwt, float* dcenter, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n > 0 && s >= 0 && k >= 1 && d >= 0 && b <= 65535);
  if ((long long)b * s == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(xyz && center && idx && wt && dout && dg_rows && dwt && dcenter &&
                 (d == 0 || feats));
  const int c = 3 + d;
  const int rb = rows_per_block(k, c, true);
  const size_t lds = (size_t)rb * (k * (c + 1) + k * kW + c * kW) * sizeof(float);
  KDPC_CHECK_ARG(lds <= kMaxLds);
  allow_lds((const void*)pointconv_contract_bwd_kernel);
  hipLaunchKernelGGL(pointconv_contract_bwd_kernel, dim3(divup(s, rb), b), dim3(256), lds,
                     (hipStream_t)stream, n, s, k, d, rb, xyz, center, feats, idx, wt, dout,
                     dg_rows, dwt, dcenter);
  KDPC_RETURN_LAUNCH();
}
