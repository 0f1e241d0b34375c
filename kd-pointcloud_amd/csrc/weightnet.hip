// Fused WeightNet over grouped neighbour offsets (reference pointconv_util.py:184-215, as
// used by PointConv / PointConvD :217-258, :401-446 with weightnet=16, hidden [8, 8], no BN).
//
//   rel[r]  = xyz[b, idx[r]] - center[b, s]                  r = (b, s, k) row
//   h0 = ReLU(W0 rel + b0)   (8)
//   h1 = ReLU(W1 h0  + b1)   (8)
//   wt = ReLU(W2 h1  + b2)   (16)                            -> wt (B,S,K,16)
//
// The reference runs this as three 1x1 Conv2d on a (B,3,K,S) tensor: 3 GEMMs whose inner
// dims are 3 and 8 over up to 590K rows, plus the grouping and three ReLUs, and in backward
// three weight-gradient GEMMs that reduce 590K rows into 8x3 / 8x8 / 16x8 outputs (a few
// workgroups each) plus three more elementwise passes.  Here one thread owns one row: the
// whole MLP is ~220 fmas in registers, the weights sit in LDS (broadcast reads), and the
// only HBM traffic is the idx/xyz gather and the 64-byte output row.
//
// Backward recomputes the row's forward, back-propagates through the three ReLUs, and
// accumulates the 248 parameter-gradient terms in registers over a fixed grid-stride set
// of rows; each workgroup reduces its threads in a fixed tree order into one slab row, and
// a second kernel sums the slabs in slab order.  No float atomics: the result depends only
// on the problem size, never on scheduling.  Optional drel (B,S,K,3) for inputs that need
// a gradient (the caller scatters it through the kNN CSR).
#include <algorithm>

#include "kdpc_common.h"

using namespace kdpc;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kIn = 3, kH0 = 8, kH1 = 8, kOut = 16;
// packed parameter layout (floats): W0 8x3 | b0 8 | W1 8x8 | b1 8 | W2 16x8 | b2 16
constexpr int oW0 = 0, oB0 = oW0 + kH0 * kIn, oW1 = oB0 + kH0, oB1 = oW1 + kH1 * kH0,
              oW2 = oB1 + kH1, oB2 = oW2 + kOut * kH1, kNP = oB2 + kOut;  // 248
constexpr int kBlock = 256;
constexpr int kBwdGrid = 512;  // fixed: the reduction order depends on nothing else

// relative offset of row r (fp32, same subtraction as the reference's grouped - center)
__device__ __forceinline__ void rel_of(int r, int s, int k, int n, const float* xyz,
                                       const float* center, const int* idx, float (&rel)[3]) {
  const unsigned bs = (unsigned)r / (unsigned)k;  // b*S + s
  const unsigned b = bs / (unsigned)s;
  const int j = idx[r];
  const float* p = xyz + ((long long)b * n + j) * 3;
  const float* c = center + (long long)bs * 3;
#pragma unroll
  for (int i = 0; i < 3; ++i) rel[i] = __fsub_rn(p[i], c[i]);
}

// y[o] = sum_i W[o,i] x[i] (ascending i, fma chain) + b[o]
template <int O, int I>
__device__ __forceinline__ void dense(const float* sp_w, const float* sp_b, const float (&x)[I],
                                      float (&y)[O]) {
#pragma unroll
  for (int o = 0; o < O; ++o) {
    float a = __fmul_rn(sp_w[o * I], x[0]);
#pragma unroll
    for (int i = 1; i < I; ++i) a = __builtin_fmaf(sp_w[o * I + i], x[i], a);
    y[o] = __fadd_rn(a, sp_b[o]);
  }
}

template <int O>
__device__ __forceinline__ void relu(float (&y)[O]) {
#pragma unroll
  for (int o = 0; o < O; ++o) y[o] = y[o] > 0.f ? y[o] : 0.f;
}

// The six parameter tensors (nn.Conv2d weights/biases, row-major).  Their addresses are
// uniform, so the compiler reads them with scalar loads into SGPRs: no VGPRs are held for
// the 248 weights, and no packing copy is needed on the host side.
struct Params {
  const float *w0, *b0, *w1, *b1, *w2, *b2;
};
__global__ __launch_bounds__(kBlock) void wn_fwd_kernel(int rows, int s, int k, int n,
                                                        const float* __restrict__ xyz,
                                                        const float* __restrict__ center,
                                                        const int* __restrict__ idx,
                                                        Params sp, float* __restrict__ wt) {
  const int r = blockIdx.x * kBlock + threadIdx.x;
  if (r >= rows) return;
  float rel[3], h0[kH0], h1[kH1], o[kOut];
  rel_of(r, s, k, n, xyz, center, idx, rel);
  dense<kH0, kIn>(sp.w0, sp.b0, rel, h0);
  relu(h0);
  dense<kH1, kH0>(sp.w1, sp.b1, h0, h1);
  relu(h1);
  dense<kOut, kH1>(sp.w2, sp.b2, h1, o);
  relu(o);
  float4* dst = reinterpret_cast<float4*>(wt + (long long)r * kOut);
#pragma unroll
  for (int v = 0; v < kOut / 4; ++v)
    dst[v] = make_float4(o[4 * v], o[4 * v + 1], o[4 * v + 2], o[4 * v + 3]);
}

// One row's forward recomputed and back-propagated through the three ReLUs: the factors
// both backward kernels start from (one definition, so their drel rows are bit-identical).
struct RowGrad {
  float rel[3], h0[kH0], h1[kH1], d2[kOut], d1[kH1], d0[kH0];
};
__device__ __forceinline__ void row_grad(int r, int s, int k, int n, const float* xyz,
                                         const float* center, const int* idx, const Params& sp,
                                         const float* dwt, RowGrad& t) {
  float o[kOut];
  rel_of(r, s, k, n, xyz, center, idx, t.rel);
  dense<kH0, kIn>(sp.w0, sp.b0, t.rel, t.h0);
  relu(t.h0);
  dense<kH1, kH0>(sp.w1, sp.b1, t.h0, t.h1);
  relu(t.h1);
  dense<kOut, kH1>(sp.w2, sp.b2, t.h1, o);
  const float4* src = reinterpret_cast<const float4*>(dwt + (long long)r * kOut);
#pragma unroll
  for (int v = 0; v < kOut / 4; ++v) {
    const float4 x = src[v];
    t.d2[4 * v] = x.x;
    t.d2[4 * v + 1] = x.y;
    t.d2[4 * v + 2] = x.z;
    t.d2[4 * v + 3] = x.w;
  }
#pragma unroll
  for (int q = 0; q < kOut; ++q) t.d2[q] = o[q] > 0.f ? t.d2[q] : 0.f;
#pragma unroll
  for (int i = 0; i < kH1; ++i) {
    float a = 0.f;
#pragma unroll
    for (int q = 0; q < kOut; ++q) a = __builtin_fmaf(sp.w2[q * kH1 + i], t.d2[q], a);
    t.d1[i] = t.h1[i] > 0.f ? a : 0.f;
  }
#pragma unroll
  for (int i = 0; i < kH0; ++i) {
    float a = 0.f;
#pragma unroll
    for (int q = 0; q < kH1; ++q) a = __builtin_fmaf(sp.w1[q * kH0 + i], t.d1[q], a);
    t.d0[i] = t.h0[i] > 0.f ? a : 0.f;
  }
}

__device__ __forceinline__ void store_drel(int r, const Params& sp, const RowGrad& t,
                                           float* __restrict__ drel) {
#pragma unroll
  for (int i = 0; i < kIn; ++i) {
    float a = 0.f;
#pragma unroll
    for (int q = 0; q < kH0; ++q) a = __builtin_fmaf(sp.w0[q * kIn + i], t.d0[q], a);
    drel[(long long)r * 3 + i] = a;
  }
}

// drel only (one thread per row): the half of the backward the upstream layers wait for;
// the parameter half (wn_bwd_mfma_kernel<false>) can then run on another stream.
__global__ __launch_bounds__(kBlock) void wn_bwd_rel_kernel(int rows, int s, int k, int n,
                                                            const float* __restrict__ xyz,
                                                            const float* __restrict__ center,
                                                            const int* __restrict__ idx,
                                                            Params sp,
                                                            const float* __restrict__ dwt,
                                                            float* __restrict__ drel) {
  const int r = blockIdx.x * kBlock + threadIdx.x;
  if (r >= rows) return;
  RowGrad t;
  row_grad(r, s, k, n, xyz, center, idx, sp, dwt, t);
  store_drel(r, sp, t, drel);
}

// Parameter half on the f32 matrix cores (round 6; replaces round 5's wn_bwd_kernel, which
// summed per-row factor products from an LDS tile one parameter per thread).  Every parameter gradient is one entry of
//   P = sum_r D_r H_r^T,  D_r = [d0 (8) | d1 (8) | d2 (16)],  H_r = [rel (3) | h0 (8) | h1 (8) | 1]
// (dW0 = the d0 x rel block, db0 = d0 x 1, dW1 = d1 x h0, db1 = d1 x 1, dW2 = d2 x h1,
// db2 = d2 x 1), i.e. a 32 x 32 x rows product: a wave takes 64 rows (one per lane: the
// row's forward and backward as row_grad), transposes D and H through its own LDS tile and
// runs 32 v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulation in the matrix core's
// fixed order) per 64 rows.  A workgroup's 4 waves take 4 consecutive 64-row tiles per
// grid-stride step; at the end their 4 accumulators are summed in wave order into the block's
// slab row, and the kBwdGrid slab rows are summed in slab order by colsum.  Deterministic: the
// result depends only on the problem size.  Product alone (tools/bench_wn.py, 589,824 rows):
// 39.6 us against 54.8 us for round 5's kernel.
constexpr int kWaveTile = 64;
constexpr int kBwdWaves = kBwdGrid;  // slab rows: one per workgroup
constexpr int kDS = 33, kHS = 21;  // LDS row strides of the D / H tiles (bank spread)

// REL: also store drel (kdpc_weightnet_bwd with drel)
template <bool REL>
__global__ __launch_bounds__(kBlock) void wn_bwd_mfma_kernel(int rows, int s, int k, int n,
                                                            const float* __restrict__ xyz,
                                                            const float* __restrict__ center,
                                                            const int* __restrict__ idx,
                                                            Params sp,
                                                            const float* __restrict__ dwt,
                                                            float* __restrict__ drel,
                                                            float* __restrict__ slab) {
  __shared__ float tiles[kBlock / 64][kWaveTile * (kDS + kHS)];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* Dt = tiles[wv];
  float* Ht = Dt + kWaveTile * kDS;
    f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  // block-uniform trip count (the block's 4 waves take 4 consecutive 64-row tiles per step),
  // so the loop can hold a workgroup barrier: with it the 248 weights are re-read per step
  // with scalar loads (SGPR operands) instead of being hoisted out of the loop into VGPRs
  for (long long tb = (long long)blockIdx.x * kBlock; tb < rows; tb += (long long)kBwdGrid * kBlock) {
    __syncthreads();
    const long long r = tb + wv * kWaveTile + lane;
    float* dl = Dt + lane * kDS;
    float* hl = Ht + lane * kHS;
    if (r < rows) {
      RowGrad t;
      row_grad((int)r, s, k, n, xyz, center, idx, sp, dwt, t);
      if (REL) store_drel((int)r, sp, t, drel);
#pragma unroll
      for (int q = 0; q < kH0; ++q) dl[q] = t.d0[q];
#pragma unroll
      for (int q = 0; q < kH1; ++q) dl[kH0 + q] = t.d1[q];
#pragma unroll
      for (int q = 0; q < kOut; ++q) dl[kH0 + kH1 + q] = t.d2[q];
#pragma unroll
      for (int q = 0; q < kIn; ++q) hl[q] = t.rel[q];
#pragma unroll
      for (int q = 0; q < kH0; ++q) hl[kIn + q] = t.h0[q];
#pragma unroll
      for (int q = 0; q < kH1; ++q) hl[kIn + kH0 + q] = t.h1[q];
      hl[19] = 1.f;
    } else {  // rows past the end add nothing
#pragma unroll
      for (int q = 0; q < 32; ++q) dl[q] = 0.f;
#pragma unroll
      for (int q = 0; q < 20; ++q) hl[q] = 0.f;
    }
    __syncthreads();  // (not wave_lds_sync: its asm memory clobber turns the weights' scalar
                      // loads into vector loads held in VGPRs)
    // K-step st: rows 2 st (lanes 0-31) and 2 st + 1 (lanes 32-63); A[i][.] = D[row][i],
    // B[.][j] = H[row][j] (0 past column 20)
    const int i = lane & 31, rr = lane >> 5;
#pragma unroll 4
    for (int st = 0; st < kWaveTile / 2; ++st) {
      const int row = 2 * st + rr;
      const float a = Dt[row * kDS + i];
      const float bv = i < 20 ? Ht[row * kHS + i] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, acc, 0, 0, 0);
    }
    // (the next step's __syncthreads orders these reads before the tile is rewritten)
  }
  // acc register e of lane l = P[(e & 3) + 8 (e >> 2) + 4 (l >> 5)][l & 31]; the block's 4
  // waves leave their parameter vectors in LDS and are summed in wave order into one slab row
  __syncthreads();  // every wave is done reading its tiles
  float* red = &tiles[0][0];  // [kBlock / 64][kNP]
  const int j = lane & 31;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int i = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
    int pi = -1;
    if (i < kH0) {
      if (j < kIn) pi = oW0 + i * kIn + j;
      else if (j == 19) pi = oB0 + i;
    } else if (i < kH0 + kH1) {
      if (j >= kIn && j < kIn + kH0) pi = oW1 + (i - kH0) * kH0 + (j - kIn);
      else if (j == 19) pi = oB1 + (i - kH0);
    } else {
      if (j >= kIn + kH0 && j < kIn + kH0 + kH1) pi = oW2 + (i - kH0 - kH1) * kH1 + (j - kIn - kH0);
      else if (j == 19) pi = oB2 + (i - kH0 - kH1);
    }
    if (pi >= 0) red[wv * kNP + pi] = acc[e];
  }
  __syncthreads();
  if (threadIdx.x < kNP) {
    float v = red[threadIdx.x];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) v += red[w * kNP + threadIdx.x];
    slab[(long long)blockIdx.x * kNP + threadIdx.x] = v;
  }
}

}  // namespace

KDPC_API int kdpc_weightnet_param_count(void) { return kNP; }

KDPC_API size_t kdpc_weightnet_bwd_workspace_bytes(void) {
  return ((size_t)kBwdWaves * kNP + colsum_scratch_floats(kBwdWaves, kNP)) * sizeof(float);
}

KDPC_API int kdpc_weightnet_fwd(int b, int n, int s, int k, const float* xyz, const float* center,
                                const int* idx, const float* w0, const float* b0, const float* w1,
                                const float* b1, const float* w2, const float* b2, float* wt,
                                void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n > 0 && s >= 0 && k >= 1);
  const long long rows = (long long)b * s * k;
  if (rows == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(xyz && center && idx && w0 && b0 && w1 && b1 && w2 && b2 && wt &&
                 rows < (1ll << 31) - kBlock);
  const Params p{w0, b0, w1, b1, w2, b2};
  hipLaunchKernelGGL(wn_fwd_kernel, dim3((unsigned)divupll(rows, kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, (int)rows, s, k, n, xyz, center, idx, p, wt);
  KDPC_RETURN_LAUNCH();
}

KDPC_API int kdpc_weightnet_bwd_rel(int b, int n, int s, int k, const float* xyz,
                                    const float* center, const int* idx, const float* w0,
                                    const float* b0, const float* w1, const float* b1,
                                    const float* w2, const float* b2, const float* dwt,
                                    float* drel, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n > 0 && s >= 0 && k >= 1);
  const long long rows = (long long)b * s * k;
  if (rows == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(xyz && center && idx && w0 && b0 && w1 && b1 && w2 && b2 && dwt && drel &&
                 rows < (1ll << 31) - kBlock);
  const Params p{w0, b0, w1, b1, w2, b2};
  hipLaunchKernelGGL(wn_bwd_rel_kernel, dim3((unsigned)divupll(rows, kBlock)), dim3(kBlock), 0,
                     (hipStream_t)stream, (int)rows, s, k, n, xyz, center, idx, p, dwt, drel);
  KDPC_RETURN_LAUNCH();
}

KDPC_API int kdpc_weightnet_bwd(int b, int n, int s, int k, const float* xyz,
                                const float* center, const int* idx, const float* w0,
                                const float* b0, const float* w1, const float* b1,
                                const float* w2, const float* b2, const float* dwt, float* drel,
                                float* dparams, void* workspace, size_t workspace_bytes,
                                void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n > 0 && s >= 0 && k >= 1);
  const long long rows = (long long)b * s * k;
  KDPC_CHECK_ARG(dparams && workspace && workspace_bytes >= kdpc_weightnet_bwd_workspace_bytes());
  KDPC_CHECK_ARG(rows == 0 ||
                 (xyz && center && idx && w0 && b0 && w1 && b1 && w2 && b2 && dwt));
  KDPC_CHECK_ARG(rows < (1ll << 31) - (long long)kBwdGrid * kBlock);
  hipStream_t st = (hipStream_t)stream;
  const Params p{w0, b0, w1, b1, w2, b2};
  float* slab = reinterpret_cast<float*>(workspace);
  // every slab row is written (rows == 0 -> all-zero partials)
  if (drel)
    hipLaunchKernelGGL(wn_bwd_mfma_kernel<true>, dim3(kBwdGrid), dim3(kBlock), 0, st, (int)rows, s,
                       k, n, xyz, center, idx, p, dwt, drel, slab);
  else
    hipLaunchKernelGGL(wn_bwd_mfma_kernel<false>, dim3(kBwdGrid), dim3(kBlock), 0, st, (int)rows, s,
                       k, n, xyz, center, idx, p, dwt, drel, slab);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return (int)colsum(kBwdWaves, kNP, slab, dparams, slab + (size_t)kBwdWaves * kNP, st);
}
