// Fused PointConv layer on the f32 matrix cores (reference pointconv_util.py:217-258 and
// 401-446: group -> cat -> (C x K)(K x 16) matmul per point -> Linear(16C -> O)).
//
//   G[r,k,c] = cat(xyz[idx[r,k]] - center[r], feats[idx[r,k]])         c < C = 3 + D
//   A[r, c*16+w] = sum_k G[r,k,c] * wt[r,k,w]                           (never stored)
//   y[r, o]  = sum_j A[r,j] * wl[o,j] + bias[o]
//
// The reference materialises A (R x 16C: 549 MB for the level-0 scene-flow estimator at
// batch 8) and runs the Linear as a separate GEMM.  Here a workgroup owns 32 rows and walks
// the channels in chunks of 8 (128 columns of A): it gathers the chunk's neighbour
// channels into LDS, forms the 32 x 128 block of A on the VALU (K fmas per element, the
// WeightNet weights held in registers), and multiplies it into the 32 x O output tile with
// v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulation; the Linear weight streams
// from L2).  A never touches HBM.
//
// Backward (two kernels + deterministic reductions, no float atomics):
//   data:   dA = dy wl per chunk (MFMA), then per (row, neighbour) on the VALU
//             dG[r,k,c]  = sum_w dA[r,c*16+w] wt[r,k,w]   -> chunk-major rows, summed per
//                                                          point through the kNN CSR
//             dwt[r,k,w] = sum_c dA[r,c*16+w] G[r,k,c]
//             dcenter[r] = -sum_k dG[r,k,0:3]
//   weight: dwl[o, j] = sum_r dy[r,o] A[r,j]  with A recomputed per (chunk, row split),
//           per-split partial tiles summed in split order.
//
// MFMA operand mapping (v_mfma_f32_32x32x2_f32, wave64): lane l supplies A[l&31][l>>5] and
// B[l>>5][l&31]; the result register i of lane l is D[(i&3) + 8*(i>>2) + 4*(l>>5)][l&31].
// The GEMM's inner index is walked in blocks of 8: MFMA step j of block b uses inner
// indices 8b+j (lanes 0-31) and 8b+4+j (lanes 32-63), so every lane's operands for four
// steps are one float4 (LDS: ds_read_b128; global: one 16-byte load).
#include <algorithm>

#include "kdpc_common.h"

using namespace kdpc;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kW = 16;              // WeightNet width (weightnet=16 in every model layer)
constexpr int kTM = 32;             // rows per tile (one MFMA M tile)
constexpr int kCC = 8;              // channels per chunk
constexpr int kNC = kCC * kW;       // A columns per chunk (128)
constexpr int kKMax = 16;           // neighbours per row supported
constexpr int kThreads = 256;
constexpr int kBlk = kTM * 4 + 16;  // floats per 4-column block of an MFMA-A-layout tile
constexpr int kTS = kTM + 4;        // row stride of transposed (inner = row) tiles
constexpr int kDaS = kNC + 4;       // row stride of the dA chunk
constexpr int kTargetWG = 512;      // grid size the split heuristics aim for

struct Geo {
  int n, s, k, d, c, r, nch;  // c = 3 + d, r = B*S rows, nch = ceil(c / kCC)
  const float* xyz;           // (B,N,3)
  const float* center;        // (B,S,3)
  const float* feats;         // (B,N,D)
  const int* idx;             // (B,S,K)
};

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 mfma4(float4 a, float4 b, f32x16 c) {
  c = mfma(a.x, b.x, c);
  c = mfma(a.y, b.y, c);
  c = mfma(a.z, b.z, c);
  return mfma(a.w, b.w, c);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// per-tile row metadata: batch offset (b*N, -1 for rows past the end) and center
__device__ __forceinline__ void load_rows(const Geo& g, int row0, int* rbase, float* rctr) {
  const int t = threadIdx.x;
  if (t < kTM) {
    const int row = row0 + t;
    const bool ok = row < g.r;
    rbase[t] = ok ? (row / g.s) * g.n : -1;
    rctr[t * 3 + 0] = ok ? g.center[(long long)row * 3 + 0] : 0.f;
    rctr[t * 3 + 1] = ok ? g.center[(long long)row * 3 + 1] : 0.f;
    rctr[t * 3 + 2] = ok ? g.center[(long long)row * 3 + 2] : 0.f;
  }
}

// G[row, k, cg] for neighbour point j of a batch whose first point is `base`
__device__ __forceinline__ float g_value(const Geo& g, int base, const float* ctr, int j, int cg) {
  if (cg < 3) return g.xyz[(long long)(base + j) * 3 + cg] - ctr[cg];
  if (cg < g.c) return g.feats[(long long)(base + j) * g.d + (cg - 3)];
  return 0.f;
}

// gl[(r*K + k)*kCC + c] = G[row0+r, k, c0+c]  (0 past the last row / channel)
__device__ __forceinline__ void stage_g(const Geo& g, int row0, int c0, const int* rbase,
                                        const float* rctr, float* gl) {
  const int c = threadIdx.x & (kCC - 1);
  const int total = kTM * g.k;
  for (int rk = threadIdx.x / kCC; rk < total; rk += kThreads / kCC) {
    const int r = rk / g.k;
    const int kk = rk - r * g.k;
    const int base = rbase[r];
    float v = 0.f;
    if (base >= 0) {
      const int j = g.idx[(long long)(row0 + r) * g.k + kk];
      v = g_value(g, base, rctr + r * 3, j, c0 + c);
    }
    gl[rk * kCC + c] = v;
  }
}

// builder thread (w = t & 15, rows rr = t >> 4 and rr + 16): its WeightNet weights
__device__ __forceinline__ void load_wt(const Geo& g, const float* __restrict__ wt, int row0,
                                        float (&wr)[2][kKMax]) {
  const int w = threadIdx.x & (kW - 1), rr = threadIdx.x >> 4;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int row = row0 + rr + 16 * q;
#pragma unroll
    for (int k = 0; k < kKMax; ++k)
      wr[q][k] = (row < g.r && k < g.k) ? wt[((long long)row * g.k + k) * kW + w] : 0.f;
  }
}

// a[q][cl] = A[row0 + rr + 16q, (c0 + cl)*16 + w] = sum_k G * wt  (ascending k, one fma each)
__device__ __forceinline__ void build_a(const Geo& g, const float* gl, const float (&wr)[2][kKMax],
                                        float (&a)[2][kCC]) {
  const int rr = threadIdx.x >> 4;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = rr + 16 * q;
#pragma unroll
    for (int c = 0; c < kCC; ++c) a[q][c] = 0.f;
#pragma unroll
    for (int k = 0; k < kKMax; ++k) {
      if (k < g.k) {
        const float4 lo = *reinterpret_cast<const float4*>(gl + (r * g.k + k) * kCC);
        const float4 hi = *reinterpret_cast<const float4*>(gl + (r * g.k + k) * kCC + 4);
        const float wk = wr[q][k];
        a[q][0] = __builtin_fmaf(lo.x, wk, a[q][0]);
        a[q][1] = __builtin_fmaf(lo.y, wk, a[q][1]);
        a[q][2] = __builtin_fmaf(lo.z, wk, a[q][2]);
        a[q][3] = __builtin_fmaf(lo.w, wk, a[q][3]);
        a[q][4] = __builtin_fmaf(hi.x, wk, a[q][4]);
        a[q][5] = __builtin_fmaf(hi.y, wk, a[q][5]);
        a[q][6] = __builtin_fmaf(hi.z, wk, a[q][6]);
        a[q][7] = __builtin_fmaf(hi.w, wk, a[q][7]);
      }
    }
  }
}

// ------------------------------------------------------------------------------ forward
// grid (row tiles, channel splits).  A split > 1 writes a partial tile to slab[split].
template <int O>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2)))
void pc_fwd_kernel(Geo g, const float* __restrict__ wt, const float* __restrict__ wl,
                   const float* __restrict__ bias, float* __restrict__ y,
                   float* __restrict__ slab, int chunks_per_split) {
  __shared__ int rbase[kTM];
  __shared__ float rctr[kTM * 3];
  __shared__ __attribute__((aligned(16))) float gl[kTM * kKMax * kCC];
  __shared__ __attribute__((aligned(16))) float al[(kNC / 4) * kBlk];
  constexpr int NT = O / 32;                  // output column tiles
  constexpr int TPW = NT >= 4 ? NT / 4 : 1;   // tiles per wave
  constexpr int KG = NT >= 4 ? 1 : 4 / NT;    // waves splitting a chunk's inner index
  constexpr int GB = 16 / KG;                 // 8-column blocks per wave and chunk
  const int row0 = blockIdx.x * kTM;
  const int split = blockIdx.y;
  const int ch0 = split * chunks_per_split;
  const int ch1 = min(g.nch, ch0 + chunks_per_split);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, half = lane >> 5, l32 = lane & 31;
  const int w = t & (kW - 1), rr = t >> 4;
  const int tile0 = (wv % (4 / KG)) * TPW;
  const int kgrp = wv / (4 / KG);
  const long long c16 = (long long)g.c * kW;

  load_rows(g, row0, rbase, rctr);
  float wr[2][kKMax];
  load_wt(g, wt, row0, wr);
  f32x16 acc[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) acc[i] = zero16();

  for (int ch = ch0; ch < ch1; ++ch) {
    const int c0 = ch * kCC;
    __syncthreads();  // row metadata ready / previous chunk's MFMAs done with `al`
    stage_g(g, row0, c0, rbase, rctr, gl);
    __syncthreads();
    float a[2][kCC];
    build_a(g, gl, wr, a);
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int cl = 0; cl < kCC; ++cl) {
        const int col = cl * kW + w;
        al[(col >> 2) * kBlk + (rr + 16 * q) * 4 + (col & 3)] = a[q][cl];
      }
    __syncthreads();
#pragma unroll 4
    for (int gb = kgrp * GB; gb < (kgrp + 1) * GB; ++gb) {
      const float4 av = *reinterpret_cast<const float4*>(al + (2 * gb + half) * kBlk + l32 * 4);
      const int col = c0 * kW + 8 * gb + 4 * half;  // this lane's 4 inner indices
      const bool ok = (col >> 4) < g.c;
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        const int n = (tile0 + i) * 32 + l32;
        const float4 bv = ok ? *reinterpret_cast<const float4*>(wl + n * c16 + col)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
        acc[i] = mfma4(av, bv, acc[i]);
      }
    }
  }

  if (KG > 1) {  // fold the inner-index groups (fixed order: group 0 + group 1 + ...)
    __syncthreads();
    float* red = gl;  // 16 KB: (KG-1) * (4/KG) waves * 16 regs * 64 lanes floats
    if (kgrp > 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        red[(((kgrp - 1) * (4 / KG) + (wv % (4 / KG))) * 16 + i) * 64 + lane] = acc[0][i];
    }
    __syncthreads();
    if (kgrp == 0) {
      for (int k2 = 1; k2 < KG; ++k2)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          acc[0][i] = __fadd_rn(acc[0][i], red[(((k2 - 1) * (4 / KG) + wv) * 16 + i) * 64 + lane]);
    }
  }
  if (kgrp != 0) return;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int n = (tile0 + i) * 32 + l32;
    const float bn = slab ? 0.f : bias[n];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = row0 + (e & 3) + 8 * (e >> 2) + 4 * half;
      if (row < g.r) {
        if (slab)
          slab[((long long)split * g.r + row) * O + n] = acc[i][e];
        else
          y[(long long)row * O + n] = __fadd_rn(acc[i][e], bn);
      }
    }
  }
}

// dst[e] = sum_s slab[s][e] (+ bias[e % O]), ascending s
__global__ __launch_bounds__(256) void pc_slab_sum_kernel(int nslabs, long long len,
                                                          const float* __restrict__ slab,
                                                          const float* __restrict__ bias, int o,
                                                          float* __restrict__ dst) {
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < len;
       e += (long long)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int s = 0; s < nslabs; ++s) v = __fadd_rn(v, slab[(long long)s * len + e]);
    if (bias) v = __fadd_rn(v, bias[e % o]);
    dst[e] = v;
  }
}

// -------------------------------------------------------------------- backward: data
// grid (row tiles, channel splits).  dgc: chunk-major dG rows [nch][R*K][kCC].
template <int O>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2)))
void pc_bwd_data_kernel(Geo g, const float* __restrict__ wt, const float* __restrict__ wl,
                        const float* __restrict__ dy, float* __restrict__ dgc,
                        float* __restrict__ dwt, float* __restrict__ dcenter,
                        int chunks_per_split) {
  __shared__ int rbase[kTM];
  __shared__ float rctr[kTM * 3];
  __shared__ __attribute__((aligned(16))) float dyl[(O / 4) * kBlk];
  __shared__ __attribute__((aligned(16))) float dal[kTM * kDaS];
  __shared__ float dcl[kTM * kKMax * 3];
  const int row0 = blockIdx.x * kTM;
  const int split = blockIdx.y;
  const int ch0 = split * chunks_per_split;
  const int ch1 = min(g.nch, ch0 + chunks_per_split);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, half = lane >> 5, l32 = lane & 31;
  const long long c16 = (long long)g.c * kW;
  const long long rk_total = (long long)g.r * g.k;

  load_rows(g, row0, rbase, rctr);
  for (int e = t; e < kTM * O; e += kThreads) {
    const int r = e / O, o = e % O;
    const int row = row0 + r;
    dyl[(o >> 2) * kBlk + r * 4 + (o & 3)] = row < g.r ? dy[(long long)row * O + o] : 0.f;
  }
  // (row, neighbour) pairs owned by this thread: p = t and t + 256
  const int P = kTM * g.k;
  float wp[2][kW], dw[2][kW];
  int pr[2], pk[2];
  bool pv[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = t + kThreads * q;
    pr[q] = p / g.k;
    pk[q] = p - pr[q] * g.k;
    pv[q] = p < P && row0 + pr[q] < g.r;
    const long long pos = (long long)(row0 + pr[q]) * g.k + pk[q];
#pragma unroll
    for (int v = 0; v < kW / 4; ++v) {
      const float4 x = pv[q] ? reinterpret_cast<const float4*>(wt + pos * kW)[v]
                             : make_float4(0.f, 0.f, 0.f, 0.f);
      wp[q][4 * v + 0] = x.x;
      wp[q][4 * v + 1] = x.y;
      wp[q][4 * v + 2] = x.z;
      wp[q][4 * v + 3] = x.w;
    }
#pragma unroll
    for (int w = 0; w < kW; ++w) dw[q][w] = 0.f;
  }
  __syncthreads();

  const int n0 = wv * 32;  // this wave's 32 dA columns of the chunk
  for (int ch = ch0; ch < ch1; ++ch) {
    const int c0 = ch * kCC;
    const int colg = c0 * kW + n0 + l32;
    const bool ok = (colg >> 4) < g.c;
    f32x16 acc = zero16();
#pragma unroll 4
    for (int og = 0; og < O / 8; ++og) {
      const float4 av = *reinterpret_cast<const float4*>(dyl + (2 * og + half) * kBlk + l32 * 4);
      const int ob = 8 * og + 4 * half;
      float4 bv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ok) {
        bv.x = wl[(ob + 0) * c16 + colg];
        bv.y = wl[(ob + 1) * c16 + colg];
        bv.z = wl[(ob + 2) * c16 + colg];
        bv.w = wl[(ob + 3) * c16 + colg];
      }
      acc = mfma4(av, bv, acc);
    }
#pragma unroll
    for (int e = 0; e < 16; ++e)
      dal[((e & 3) + 8 * (e >> 2) + 4 * half) * kDaS + n0 + l32] = acc[e];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (!pv[q]) continue;
      const int r = pr[q];
      const int base = rbase[r];
      const int j = g.idx[(long long)(row0 + r) * g.k + pk[q]];
      float gv[kCC];
#pragma unroll
      for (int c = 0; c < kCC; ++c) gv[c] = g_value(g, base, rctr + r * 3, j, c0 + c);
      const long long pos = (long long)(row0 + r) * g.k + pk[q];
      float* dgo = dgc + ((long long)ch * rk_total + pos) * kCC;
#pragma unroll 2
      for (int cl = 0; cl < kCC; ++cl) {
        float da[kW];
#pragma unroll
        for (int v = 0; v < kW / 4; ++v) {
          const float4 x = *reinterpret_cast<const float4*>(dal + r * kDaS + cl * kW + 4 * v);
          da[4 * v + 0] = x.x;
          da[4 * v + 1] = x.y;
          da[4 * v + 2] = x.z;
          da[4 * v + 3] = x.w;
        }
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < kW; ++w) s = __builtin_fmaf(da[w], wp[q][w], s);
        dgo[cl] = s;
        if (c0 == 0 && cl < 3) dcl[(r * g.k + pk[q]) * 3 + cl] = s;
        const float gc = gv[cl];
#pragma unroll
        for (int w = 0; w < kW; ++w) dw[q][w] = __builtin_fmaf(da[w], gc, dw[q][w]);
      }
    }
    __syncthreads();
  }
  if (ch0 == 0 && t < kTM * 3) {
    const int r = t / 3, i = t - (t / 3) * 3;
    const int row = row0 + r;
    if (row < g.r) {
      float s = 0.f;
      for (int k = 0; k < g.k; ++k) s = __fadd_rn(s, dcl[(r * g.k + k) * 3 + i]);
      dcenter[(long long)row * 3 + i] = -s;
    }
  }
  float* dwt_dst = dwt + (long long)split * rk_total * kW;  // slab when split > 0 exists
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (!pv[q]) continue;
    const long long pos = (long long)(row0 + pr[q]) * g.k + pk[q];
    float4* dst = reinterpret_cast<float4*>(dwt_dst + pos * kW);
#pragma unroll
    for (int v = 0; v < kW / 4; ++v)
      dst[v] = make_float4(dw[q][4 * v], dw[q][4 * v + 1], dw[q][4 * v + 2], dw[q][4 * v + 3]);
  }
}

// per point (one wave each): d_xyz / d_feats = sum of its dG rows in CSR (ascending position)
__global__ __launch_bounds__(256) void pc_csr_sum_kernel(long long npts, int c, int d,
                                                         long long rk_total,
                                                         const float* __restrict__ dgc,
                                                         const int* __restrict__ offsets,
                                                         const int* __restrict__ perm,
                                                         float* __restrict__ dxyz,
                                                         float* __restrict__ dfeats) {
  const long long key = (long long)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
  if (key >= npts) return;
  const int lane = threadIdx.x & (kWave - 1);
  const int j0 = offsets[key], j1 = offsets[key + 1];
  for (int ch = dxyz ? lane : 3 + lane; ch < c; ch += kWave) {
    const float* src = dgc + (long long)(ch / kCC) * rk_total * kCC + (ch % kCC);
    float s = 0.f;
    for (int j = j0; j < j1; ++j) s = __fadd_rn(s, src[(long long)perm[j] * kCC]);
    if (ch < 3)
      dxyz[key * 3 + ch] = s;
    else
      dfeats[key * d + (ch - 3)] = s;
  }
}

// ------------------------------------------------------------------ backward: weight
// grid (channel chunks, row splits); dwl tile (O x 128) of this chunk over the split's rows
template <int O>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2)))
void pc_bwd_weight_kernel(Geo g, const float* __restrict__ wt, const float* __restrict__ dy,
                          float* __restrict__ dwl, int rows_per_split) {
  __shared__ int rbase[kTM];
  __shared__ float rctr[kTM * 3];
  __shared__ __attribute__((aligned(16))) float gl[kTM * kKMax * kCC];
  __shared__ __attribute__((aligned(16))) float dyt[O * kTS];
  __shared__ __attribute__((aligned(16))) float at[kNC * kTS];
  constexpr int MT = O / 32;
  constexpr int MPW = MT >= 4 ? MT / 4 : 1;
  constexpr int NPW = MT >= 4 ? 4 : 2;
  const int ch = blockIdx.x, split = blockIdx.y;
  const int c0 = ch * kCC;
  const int rbeg = split * rows_per_split;
  const int rend = min(g.r, rbeg + rows_per_split);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, half = lane >> 5, l32 = lane & 31;
  const int w = t & (kW - 1), rr = t >> 4;
  const int m0 = MT >= 4 ? wv * MPW : (wv & 1);
  const int nb0 = MT >= 4 ? 0 : (wv >> 1) * 2;
  const long long c16 = (long long)g.c * kW;

  f32x16 acc[MPW][NPW];
#pragma unroll
  for (int i = 0; i < MPW; ++i)
#pragma unroll
    for (int j = 0; j < NPW; ++j) acc[i][j] = zero16();

  for (int row0 = rbeg; row0 < rend; row0 += kTM) {
    __syncthreads();  // previous tile's MFMAs done with dyt / at
    load_rows(g, row0, rbase, rctr);
    float wr[2][kKMax];
    load_wt(g, wt, row0, wr);
    for (int e = t; e < kTM * O; e += kThreads) {
      const int r = e / O, o = e % O;
      const int row = row0 + r;
      dyt[o * kTS + r] = row < rend ? dy[(long long)row * O + o] : 0.f;
    }
    __syncthreads();
    stage_g(g, row0, c0, rbase, rctr, gl);
    __syncthreads();
    float a[2][kCC];
    build_a(g, gl, wr, a);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const bool live = row0 + rr + 16 * q < rend;
#pragma unroll
      for (int cl = 0; cl < kCC; ++cl) at[(cl * kW + w) * kTS + rr + 16 * q] = live ? a[q][cl] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int gb = 0; gb < kTM / 8; ++gb) {
      float4 av[MPW], bv[NPW];
#pragma unroll
      for (int i = 0; i < MPW; ++i)
        av[i] = *reinterpret_cast<const float4*>(dyt + ((m0 + i) * 32 + l32) * kTS + 8 * gb + 4 * half);
#pragma unroll
      for (int j = 0; j < NPW; ++j)
        bv[j] = *reinterpret_cast<const float4*>(at + ((nb0 + j) * 32 + l32) * kTS + 8 * gb + 4 * half);
#pragma unroll
      for (int i = 0; i < MPW; ++i)
#pragma unroll
        for (int j = 0; j < NPW; ++j) acc[i][j] = mfma4(av[i], bv[j], acc[i][j]);
    }
  }
  float* dst = dwl + (long long)split * O * c16;  // slab when the rows are split
#pragma unroll
  for (int i = 0; i < MPW; ++i)
#pragma unroll
    for (int j = 0; j < NPW; ++j) {
      const long long col = (long long)c0 * kW + (nb0 + j) * 32 + l32;
      if (col >= c16) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int o = (m0 + i) * 32 + (e & 3) + 8 * (e >> 2) + 4 * half;
        dst[o * c16 + col] = acc[i][j][e];
      }
    }
}

// ------------------------------------------------------------------------------- host
struct Plan {
  int r, c, nch, rt;
  int ks, cps;   // channel splits (fwd and bwd-data) and chunks per split
  int rs, rps;   // row splits (bwd-weight) and rows per split
  size_t fwd_slab, dgc, dwt_slab, dwl_slab;  // bytes
};

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

bool plan_of(int b, int s, int k, int d, int o, Plan* p) {
  if (b < 0 || s < 0 || k < 1 || k > kKMax || d < 0 || !(o == 64 || o == 128 || o == 256))
    return false;
  const long long r = (long long)b * s;
  if (r > (1ll << 26) || (long long)(3 + d) * kW * o > (1ll << 30)) return false;
  p->r = (int)r;
  p->c = 3 + d;
  p->nch = divup(p->c, kCC);
  p->rt = divup(p->r, kTM);
  int ks = p->rt > 0 ? std::min(p->nch, std::max(1, divup(kTargetWG, p->rt))) : 1;
  p->cps = divup(p->nch, ks);
  p->ks = divup(p->nch, p->cps);
  int rs = std::max(1, std::min(std::max(p->rt, 1), divup(kTargetWG, p->nch)));
  p->rps = divup(std::max(p->rt, 1), rs) * kTM;
  p->rs = std::max(1, divup(p->r, p->rps));
  const size_t c16 = (size_t)p->c * kW;
  p->fwd_slab = p->ks > 1 ? align256((size_t)p->ks * p->r * o * 4) : 0;
  p->dgc = align256((size_t)p->nch * p->r * k * kCC * 4);
  p->dwt_slab = p->ks > 1 ? align256((size_t)p->ks * p->r * k * kW * 4) : 0;
  p->dwl_slab = p->rs > 1 ? align256((size_t)p->rs * o * c16 * 4) : 0;
  return true;
}

hipError_t slab_sum(int nslabs, long long len, const float* slab, const float* bias, int o,
                    float* dst, hipStream_t st) {
  const int grid = (int)std::min<long long>(divupll(len, 256), 4096);
  hipLaunchKernelGGL(pc_slab_sum_kernel, dim3(grid), dim3(256), 0, st, nslabs, len, slab, bias, o,
                     dst);
  return hipGetLastError();
}

template <int O>
hipError_t fwd_launch(const Geo& g, const Plan& p, const float* wt, const float* wl,
                      const float* bias, float* y, float* slab, hipStream_t st) {
  hipLaunchKernelGGL((pc_fwd_kernel<O>), dim3(p.rt, p.ks), dim3(kThreads), 0, st, g, wt, wl, bias,
                     y, p.ks > 1 ? slab : nullptr, p.cps);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || p.ks == 1) return e;
  return slab_sum(p.ks, (long long)p.r * O, slab, bias, O, y, st);
}

template <int O>
hipError_t bwd_launch(const Geo& g, const Plan& p, int b, const float* wt, const float* wl,
                      const float* dy, const int* offsets, const int* perm, float* dxyz,
                      float* dfeats, float* dcenter, float* dwt, float* dwl, char* ws,
                      hipStream_t st) {
  float* dgc = reinterpret_cast<float*>(ws);
  float* dwt_slab = reinterpret_cast<float*>(ws + p.dgc);
  float* dwl_slab = reinterpret_cast<float*>(ws + p.dgc + p.dwt_slab);
  const long long rk = (long long)p.r * g.k;
  hipLaunchKernelGGL((pc_bwd_data_kernel<O>), dim3(p.rt, p.ks), dim3(kThreads), 0, st, g, wt, wl,
                     dy, dgc, p.ks > 1 ? dwt_slab : dwt, dcenter, p.cps);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (p.ks > 1 && (e = slab_sum(p.ks, rk * kW, dwt_slab, nullptr, 1, dwt, st)) != hipSuccess)
    return e;
  const long long npts = (long long)b * g.n;
  hipLaunchKernelGGL(pc_csr_sum_kernel, dim3((unsigned)divupll(npts, 4)), dim3(256), 0, st, npts,
                     g.c, g.d, rk, dgc, offsets, perm, dxyz, dfeats);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL((pc_bwd_weight_kernel<O>), dim3(p.nch, p.rs), dim3(kThreads), 0, st, g, wt,
                     dy, p.rs > 1 ? dwl_slab : dwl, p.rps);
  if ((e = hipGetLastError()) != hipSuccess || p.rs == 1) return e;
  return slab_sum(p.rs, (long long)O * g.c * kW, dwl_slab, nullptr, 1, dwl, st);
}

Geo geo_of(int n, int s, int k, int d, const Plan& p, const float* xyz, const float* center,
           const float* feats, const int* idx) {
  Geo g;
  g.n = n;
  g.s = s;
  g.k = k;
  g.d = d;
  g.c = p.c;
  g.r = p.r;
  g.nch = p.nch;
  g.xyz = xyz;
  g.center = center;
  g.feats = feats;
  g.idx = idx;
  return g;
}

}  // namespace

KDPC_API int kdpc_pointconv_supported(int k, int d, int o) {
  Plan p;
  return plan_of(1, 1, k, d, o, &p) ? 1 : 0;
}

KDPC_API size_t kdpc_pointconv_fwd_workspace_bytes(int b, int s, int k, int d, int o) {
  Plan p;
  return plan_of(b, s, k, d, o, &p) ? p.fwd_slab : 0;
}

KDPC_API int kdpc_pointconv_fwd(int b, int n, int s, int k, int d, int o, const float* xyz,
                                const float* center, const float* feats, const int* idx,
                                const float* wt, const float* wl, const float* bias, float* y,
                                void* workspace, size_t workspace_bytes, void* stream) {
  Plan p;
  KDPC_CHECK_ARG(n > 0 && b <= 65535 && plan_of(b, s, k, d, o, &p));
  if (p.r == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(xyz && center && idx && wt && wl && bias && y && (d == 0 || feats));
  KDPC_CHECK_ARG(workspace_bytes >= p.fwd_slab && (p.fwd_slab == 0 || workspace));
  const Geo g = geo_of(n, s, k, d, p, xyz, center, feats, idx);
  float* slab = reinterpret_cast<float*>(workspace);
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = o == 64    ? fwd_launch<64>(g, p, wt, wl, bias, y, slab, st)
                 : o == 128 ? fwd_launch<128>(g, p, wt, wl, bias, y, slab, st)
                            : fwd_launch<256>(g, p, wt, wl, bias, y, slab, st);
  return (int)e;
}

KDPC_API size_t kdpc_pointconv_bwd_workspace_bytes(int b, int s, int k, int d, int o) {
  Plan p;
  return plan_of(b, s, k, d, o, &p) ? p.dgc + p.dwt_slab + p.dwl_slab : 0;
}

KDPC_API int kdpc_pointconv_bwd(int b, int n, int s, int k, int d, int o, const float* xyz,
                                const float* center, const float* feats, const int* idx,
                                const float* wt, const float* wl, const float* dy,
                                const int* offsets, const int* perm, float* dxyz, float* dfeats,
                                float* dcenter, float* dwt, float* dwl, void* workspace,
                                size_t workspace_bytes, void* stream) {
  Plan p;
  KDPC_CHECK_ARG(n > 0 && b <= 65535 && plan_of(b, s, k, d, o, &p));
  hipStream_t st = (hipStream_t)stream;
  if (p.r == 0) {
    hipError_t e = hipSuccess;
    if (dxyz) e = hipMemsetAsync(dxyz, 0, sizeof(float) * b * n * 3, st);
    if (e == hipSuccess && d > 0) e = hipMemsetAsync(dfeats, 0, sizeof(float) * b * n * d, st);
    if (e == hipSuccess) e = hipMemsetAsync(dwl, 0, sizeof(float) * o * p.c * kW, st);
    return (int)e;
  }
  KDPC_CHECK_ARG(xyz && center && idx && wt && wl && dy && offsets && perm && dcenter && dwt &&
                 dwl && (d == 0 || (feats && dfeats)));
  KDPC_CHECK_ARG(workspace && workspace_bytes >= p.dgc + p.dwt_slab + p.dwl_slab);
  const Geo g = geo_of(n, s, k, d, p, xyz, center, feats, idx);
  char* ws = reinterpret_cast<char*>(workspace);
  hipError_t e =
      o == 64    ? bwd_launch<64>(g, p, b, wt, wl, dy, offsets, perm, dxyz, dfeats, dcenter, dwt, dwl, ws, st)
      : o == 128 ? bwd_launch<128>(g, p, b, wt, wl, dy, offsets, perm, dxyz, dfeats, dcenter, dwt, dwl, ws, st)
                 : bwd_launch<256>(g, p, b, wt, wl, dy, offsets, perm, dxyz, dfeats, dcenter, dwt, dwl, ws, st);
  return (int)e;
}
