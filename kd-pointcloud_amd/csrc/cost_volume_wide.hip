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
#include "split_bf16.h"

using namespace kdpc;
using namespace kdpc_x6;

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

// ===================================================================================
// Fused wide cost volume, Din = Dout = D in {128, 256}, K <= 32: the whole
//   gather -> position transform -> add -> LeakyReLU -> W1 (MFMA) -> LeakyReLU -> max over K
// in one kernel, and the backward in one kernel, so neither h0 (rows x D) nor z1 ever
// reaches HBM (the unfused path above writes and re-reads both, around two BLAS GEMMs).
//
// Workgroup = D/32 waves; wave w owns the 32-column block [32w, 32w+32) of the D x D MLP.
// Queries are walked in a software pipeline: query q's 32 neighbour rows of h0 sit in one
// of two LDS tiles while the next query's gathers (issued at the top of the iteration) land
// and are turned into the other tile.  The 32 rows of the v_mfma_f32_32x32x2_f32 tile ARE
// the query's neighbours: the max over K is a column reduction of the accumulator.
// -----------------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr unsigned kOOB = 0x80000000u;  // out-of-range buffer offset: loads read 0, stores drop

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float bld(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
__device__ __forceinline__ float4 bld4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

template <int D>
struct WideGeo {
  static constexpr int NW = D / 32;      // waves per workgroup
  static constexpr int NT = NW * 64;     // threads = 2D
  static constexpr int LD = D + 4;       // LDS row stride (floats)
  static constexpr int C4 = D / 4;       // float4 column groups
  static constexpr int RG = NT / C4;     // row groups of the build / column passes (8)
  static constexpr int RPT = 32 / RG;    // rows per thread (4)
  static_assert(RG * RPT == 32, "build mapping");
};

// The gathered inputs of one query for this thread's build slots (rows rg + RG*i,
// channels 4 c4 .. +3), loaded one query ahead.
template <int D>
struct WideLoads {
  float4 p2[WideGeo<D>::RPT];
  float x2[WideGeo<D>::RPT][3];
  float4 p1;
  float x1[3];
};

// Buffers over whole tensors (batch offsets folded into the byte offsets).
struct WideSrc {
  __amdgpu_buffer_rsrc_t x1, x2, idx, p1, p2;
  int n1, n2, k, nq;
};

template <int D>
__device__ __forceinline__ void wide_load_idx(const WideSrc& s, int q, int (&j)[WideGeo<D>::RPT],
                                              int rg) {
  using G = WideGeo<D>;
  const bool live = q < s.nq;
#pragma unroll
  for (int i = 0; i < G::RPT; ++i) {
    const int r = rg + G::RG * i;
    const unsigned off = (live && r < s.k) ? ((unsigned)q * (unsigned)s.k + r) * 4u : kOOB;
    j[i] = (int)__builtin_amdgcn_raw_buffer_load_b32(s.idx, (int)off, 0, 0);
  }
}

template <int D>
__device__ __forceinline__ void wide_load(const WideSrc& s, int q, const int (&j)[WideGeo<D>::RPT],
                                          int rg, int c4, WideLoads<D>& L) {
  using G = WideGeo<D>;
  const bool live = q < s.nq;
  const int b = live ? q / s.n1 : 0;
#pragma unroll
  for (int i = 0; i < G::RPT; ++i) {
    const int r = rg + G::RG * i;
    const bool ok = live && r < s.k;
    const unsigned pt = (unsigned)b * (unsigned)s.n2 + (unsigned)j[i];
    const unsigned po = ok ? (pt * D + 4u * c4) * 4u : kOOB;
    L.p2[i] = bld4(s.p2, po);
    const unsigned xo = ok ? pt * 12u : kOOB;
    L.x2[i][0] = bld(s.x2, xo);
    L.x2[i][1] = bld(s.x2, xo == kOOB ? kOOB : xo + 4u);
    L.x2[i][2] = bld(s.x2, xo == kOOB ? kOOB : xo + 8u);
  }
  L.p1 = bld4(s.p1, live ? ((unsigned)q * D + 4u * c4) * 4u : kOOB);
  const unsigned qo = live ? (unsigned)q * 12u : kOOB;
  L.x1[0] = bld(s.x1, qo);
  L.x1[1] = bld(s.x1, qo == kOOB ? kOOB : qo + 4u);
  L.x1[2] = bld(s.x1, qo == kOOB ? kOOB : qo + 8u);
}

// h0 rows of the staged query into the LDS tile H (rows >= K are zero), same arithmetic as
// cvw_h0_kernel / cost_volume.hip build_h0; directions into dirs[32] when asked.
template <int D>
__device__ __forceinline__ void wide_build(const WideLoads<D>& L, int k, int rg, int c4,
                                           const float4* wposT, float* H, float4* dirs) {
  using G = WideGeo<D>;
  float wp[4][3], bp[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float4 v = wposT[4 * c4 + e];
    wp[e][0] = v.x;
    wp[e][1] = v.y;
    wp[e][2] = v.z;
    bp[e] = v.w;
  }
#pragma unroll
  for (int i = 0; i < G::RPT; ++i) {
    const int r = rg + G::RG * i;
    const float dx = L.x2[i][0] - L.x1[0], dy = L.x2[i][1] - L.x1[1], dz = L.x2[i][2] - L.x1[2];
    const float g[4] = {L.p2[i].x, L.p2[i].y, L.p2[i].z, L.p2[i].w};
    const float p[4] = {L.p1.x, L.p1.y, L.p1.z, L.p1.w};
    float h[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float pos = __fadd_rn(
          __builtin_fmaf(wp[e][2], dz, __builtin_fmaf(wp[e][1], dy, __fmul_rn(wp[e][0], dx))), bp[e]);
      h[e] = r < k ? lrelu(__fadd_rn(__fadd_rn(g[e], p[e]), pos)) : 0.f;
    }
    *reinterpret_cast<float4*>(H + r * G::LD + 4 * c4) = make_float4(h[0], h[1], h[2], h[3]);
    if (dirs != nullptr && c4 == 0) dirs[r] = make_float4(dx, dy, dz, 0.f);
  }
}

// The same h0 rows as three bf16 planes (the forward's MFMA A operand, mfma_x6): row r's
// 8-channel chunk g at r * (D / 8) + (g ^ (r & 15)) (the 32 lanes of an operand read hit 16
// distinct chunk positions); this thread's 4 channels are half a chunk (8 bytes per plane).
template <int D>
__device__ __forceinline__ void wide_build_planes(const WideLoads<D>& L, int k, int rg, int c4,
                                                  const float4* wposT, bf16x8 (*Hp)[32 * D / 8]) {
  using G = WideGeo<D>;
  float wp[4][3], bp[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float4 v = wposT[4 * c4 + e];
    wp[e][0] = v.x;
    wp[e][1] = v.y;
    wp[e][2] = v.z;
    bp[e] = v.w;
  }
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int i = 0; i < G::RPT; ++i) {
    const int r = rg + G::RG * i;
    const float dx = L.x2[i][0] - L.x1[0], dy = L.x2[i][1] - L.x1[1], dz = L.x2[i][2] - L.x1[2];
    const float g[4] = {L.p2[i].x, L.p2[i].y, L.p2[i].z, L.p2[i].w};
    const float p[4] = {L.p1.x, L.p1.y, L.p1.z, L.p1.w};
    bf16x4 hh, hm, hl;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float pos = __fadd_rn(
          __builtin_fmaf(wp[e][2], dz, __builtin_fmaf(wp[e][1], dy, __fmul_rn(wp[e][0], dx))), bp[e]);
      const float h = r < k ? lrelu(__fadd_rn(__fadd_rn(g[e], p[e]), pos)) : 0.f;
      __bf16 a, b2, c2;
      split3(h, a, b2, c2);
      hh[e] = a;
      hm[e] = b2;
      hl[e] = c2;
    }
    const int cix = r * (D / 8) + ((c4 >> 1) ^ (r & 15));
    const int sub = c4 & 1;  // which half of the chunk
    reinterpret_cast<bf16x4*>(&Hp[0][cix])[sub] = hh;
    reinterpret_cast<bf16x4*>(&Hp[1][cix])[sub] = hm;
    reinterpret_cast<bf16x4*>(&Hp[2][cix])[sub] = hl;
  }
}

// (Wpos row, bpos) per channel into an LDS table: wposT[c] = (wx, wy, wz, b)
template <int D>
__device__ __forceinline__ void wide_consts(const float* __restrict__ wpos,
                                            const float* __restrict__ bpos, float4* wposT) {
  for (int c = threadIdx.x; c < D; c += blockDim.x)
    wposT[c] = make_float4(wpos[c * 3 + 0], wpos[c * 3 + 1], wpos[c * 3 + 2], bpos[c]);
}

template <int D>
__device__ __forceinline__ WideSrc wide_src(int b, int n1, int n2, int k, const float* x1,
                                            const float* x2, const int* idx, const float* p1,
                                            const float* p2) {
  WideSrc s;
  const long long nq = (long long)b * n1;
  s.x1 = rsrc_of(x1, nq * 12);
  s.x2 = rsrc_of(x2, (long long)b * n2 * 12);
  s.idx = rsrc_of(idx, nq * k * 4);
  s.p1 = rsrc_of(p1, nq * D * 4);
  s.p2 = rsrc_of(p2, (long long)b * n2 * D * 4);
  s.n1 = n1;
  s.n2 = n2;
  s.k = k;
  s.nq = (int)nq;
  return s;
}

// Forward.  grid.x workgroups, `qpw` consecutive queries each.
template <int D>
__global__ __launch_bounds__(2 * D) void cvw_fused_fwd_kernel(
    int b, int n1, int n2, int k, int qpw, const float* __restrict__ x1,
    const float* __restrict__ x2, const int* __restrict__ idx, const float* __restrict__ p1,
    const float* __restrict__ p2, const float* __restrict__ wpos, const float* __restrict__ bpos,
    const float* __restrict__ w1, const float* __restrict__ b1, float* __restrict__ out,
    unsigned char* __restrict__ amax) {
  using G = WideGeo<D>;
  constexpr int NKS = D / 16;  // 16-deep K-steps of the D x D MLP (mfma_x6)
  // h0 of a query as bf16 planes (wide_build_planes), double-buffered
  __shared__ __attribute__((aligned(16))) bf16x8 Hp[2][3][32 * D / 8];
  __shared__ __attribute__((aligned(16))) float4 wposT[D];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, half = lane >> 5, l32 = lane & 31;
  const int c4 = t % G::C4, rg = t / G::C4;
  const WideSrc s = wide_src<D>(b, n1, n2, k, x1, x2, idx, p1, p2);
  const int q0 = blockIdx.x * qpw;
  const int q1 = min(s.nq, q0 + qpw);
  if (q0 >= q1) return;  // workgroup-uniform
  wide_consts<D>(wpos, bpos, wposT);
  // B planes: lane supplies W1[32w + l32][16 ks + 8 half + 0..7] for K-step ks, split once
  Planes bw[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    // scalar loads: w1 may be a view at any 4-byte offset (the flat parameter buffer)
    const float* src = w1 + (long long)(32 * w + l32) * D + 16 * ks + 8 * half;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = src[j];
    bw[ks] = split8(v);
  }
  const float bias = b1[32 * w + l32];

  int jn[G::RPT], jn2[G::RPT];
  WideLoads<D> L;
  wide_load_idx<D>(s, q0, jn, rg);
  wide_load<D>(s, q0, jn, rg, c4, L);
  wide_load_idx<D>(s, q0 + 1, jn2, rg);
  __syncthreads();  // wposT
  wide_build_planes<D>(L, k, rg, c4, wposT, Hp[0]);
  __syncthreads();
  for (int q = q0; q < q1; ++q) {
    const int p = (q - q0) & 1;
    // next query's gathers (indices were loaded one iteration earlier), then q+2's indices
#pragma unroll
    for (int i = 0; i < G::RPT; ++i) jn[i] = jn2[i];
    wide_load<D>(s, q + 1 < q1 ? q + 1 : s.nq, jn, rg, c4, L);
    wide_load_idx<D>(s, q + 2 < q1 ? q + 2 : s.nq, jn2, rg);
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int cix = l32 * (D / 8) + ((2 * ks + half) ^ (l32 & 15));
      acc = mfma_x6(Hp[p][0][cix], Hp[p][1][cix], Hp[p][2][cix], bw[ks].h, bw[ks].m, bw[ks].l, acc);
    }
    // max over the query's rows (< k) in LeakyReLU space, first maximal row
    float m = -INFINITY;
    int mr = 0;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = (e & 3) + 8 * (e >> 2) + 4 * half;
      const float v = lrelu(__fadd_rn(acc[e], bias));
      if (row < k && v > m) {
        m = v;
        mr = row;
      }
    }
    const float pm = __shfl_xor(m, 32, kWave);
    const int pr = __shfl_xor(mr, 32, kWave);
    if (pm > m || (pm == m && pr < mr)) {
      m = pm;
      mr = pr;
    }
    if (half == 0) {
      out[(long long)q * D + 32 * w + l32] = m;
      amax[(long long)q * D + 32 * w + l32] = (unsigned char)mr;
    }
    if (q + 1 < q1) wide_build_planes<D>(L, k, rg, c4, wposT, Hp[p ^ 1]);
    __syncthreads();
  }
}

// Backward.  Per query: h0 rebuilt (LDS tile), g'[o] = dout * LReLU'(out) and the argmax
// rows am[o]; dh0 = M W1 on the bf16 matrix cores (mfma_x6; M[r][o] = g'[o] [am[o] == r]: one
// nonzero per column); dW1[o,:] += g'[o] h0[am[o],:] on the VALU (1/32 of a dense
// update); dz0 = dh0 * LReLU'(h0) in place; then per-row / per-channel passes write dP1,
// the dP2 / d(dir) rows (summed per reference point by the caller through the CSR) and dx1,
// and accumulate db1 / dWpos / dbpos.  Parameter gradients leave as one slab per workgroup
// (summed in a fixed order by colsum: no float atomics).
// B operand of dh0: W1's bf16 planes in fragment order (cvw_w1_planes_kernel, L2-resident),
// streamed per query two K-steps ahead.
template <int D>
struct WideBwd {
  static constexpr int OSPLIT = D <= 128 ? 1 : 2;  // dW1 o-halves (grid.y of the PART 2 kernel)
  static constexpr int NKS = D / 16;  // 16-deep K-steps of dh0 = M W1 (mfma_x6)
  // the next query's gathers issued at the top of the iteration (held in registers across
  // the MFMA phase) for D = 128; at D = 256 the dW1 accumulators need those registers
  static constexpr bool PREFETCH = D <= 128;
  static constexpr int OG = WideGeo<D>::NT / WideGeo<D>::C4;  // dW1 o-groups (8)
  static constexpr int OPT = D / OG / OSPLIT;                   // o rows per thread
  static constexpr int SLAB = D * D + D + 4 * D;                // dW1 | db1 | dWpos^T | dbpos
};

// PART: 0 = everything (D = 128), 1 = all but dW1 / db1, 2 = dW1 / db1 only (the D = 256
// pair: the dW1 accumulators and the rest do not fit one wave's 256 registers together).
// OVR: slope0 (B*N1, K, D) u8 overrides the first LeakyReLU's derivative (test seam; see
// cost_volume_bwd_kernel in cost_volume.hip)
template <int D, int PART, bool OVR>
__global__ __launch_bounds__(2 * D) __attribute__((amdgpu_waves_per_eu(D == 128 ? 1 : 2))) void cvw_fused_bwd_kernel(
    int b, int n1, int n2, int k, int qpw, const float* __restrict__ x1,
    const float* __restrict__ x2, const int* __restrict__ idx, const float* __restrict__ p1,
    const float* __restrict__ p2, const float* __restrict__ wpos, const float* __restrict__ bpos,
    const float* __restrict__ w1, const bf16x8* __restrict__ w1p, const float* __restrict__ out,
    const unsigned char* __restrict__ amax, const unsigned char* __restrict__ slope0,
    const float* __restrict__ dout,
    float* __restrict__ dp1, float* __restrict__ dp2_rows, float* __restrict__ dx1,
    float* __restrict__ ddir_rows, const int* __restrict__ rank, float* __restrict__ rows,
    float* __restrict__ slab) {
  using G = WideGeo<D>;
  // ranked rows: dP2 rows (P, D), then d(dir) rows (P, 4) (cost_volume.hip)
  using W = WideBwd<D>;
  constexpr int NG2 = G::NT / 32;  // channel groups of the direction pass
  constexpr int CPG = D / NG2;     // channels per group
  constexpr bool MAIN = PART != 2, DW1 = PART != 1;
  __shared__ __attribute__((aligned(16))) float Hs[2][32 * G::LD];
  __shared__ __attribute__((aligned(16))) float4 dirs[2][32];
  __shared__ __attribute__((aligned(16))) float2 gam[2][D];   // (g', argmax row) per output
  // the same per output as the bf16 planes of g' and the argmax row as u16: the A operand of
  // dh0 = M W1 (M[r][o] = g'[o] [am[o] == r]) is 8 outputs' planes masked per 16-bit half
  __shared__ __attribute__((aligned(16))) __bf16 gpl[2][3][D];
  __shared__ __attribute__((aligned(16))) unsigned short gam16[2][D];
  __shared__ __attribute__((aligned(16))) float4 red[G::RG][G::C4];  // dP1 partials
  __shared__ __attribute__((aligned(16))) float4 red2[NG2][32];      // d(dir) partials
  __shared__ __attribute__((aligned(16))) float4 wposT[D];           // Wpos rows (x, y, z, 0)
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, half = lane >> 5, l32 = lane & 31;
  const int c4 = t % G::C4, rg = t / G::C4;
  const WideSrc s = wide_src<D>(b, n1, n2, k, x1, x2, idx, p1, p2);
  const int q0 = blockIdx.x * qpw;
  const int q1 = min(s.nq, q0 + qpw);
  float* sb = slab + (long long)blockIdx.x * W::SLAB;
  const int obase = DW1 ? (int)blockIdx.y * (D / W::OSPLIT) : 0;  // this launch's dW1 rows
  if (q0 >= q1) {  // every slab row is written (this PART's entries)
    for (int e = t; e < W::SLAB; e += G::NT) {
      const bool dw = e < D * D ? (e / D - obase >= 0 && e / D - obase < D / W::OSPLIT)
                                : (e < D * D + D && blockIdx.y == 0);
      if (dw ? DW1 : (MAIN && e >= D * D + D)) sb[e] = 0.f;
    }
    return;
  }
  const __amdgpu_buffer_rsrc_t outr = rsrc_of(out, (long long)s.nq * D * 4);
  const __amdgpu_buffer_rsrc_t dor = rsrc_of(dout, (long long)s.nq * D * 4);
  const __amdgpu_buffer_rsrc_t amr = rsrc_of(amax, (long long)s.nq * D);
  const __amdgpu_buffer_rsrc_t s0r = rsrc_of(OVR ? slope0 : amax, OVR ? (long long)s.nq * k * D : 0);
  // ranked rows: row (q, r) -> slot rank[q*k + r]; a query's slots are loaded as it starts
  // and used by its column / direction passes after the MFMAs
  const bool ranked = rank != nullptr;
  const __amdgpu_buffer_rsrc_t rkr = rsrc_of(ranked ? rank : idx, ranked ? (long long)s.nq * k * 4 : 0);
  wide_consts<D>(wpos, bpos, wposT);
  // B planes of dh0 (cvw_w1_planes_kernel): this wave's column block, K-step ks, plane pl at
  // [(3 ks + pl) * 64], streamed from L2 PF K-steps ahead
  const bf16x8* w1row = w1p + (long long)(w * W::NKS * 3) * 64 + lane;
  // accumulators: dW1 rows o = og*OPT + i at channels 4 c4 .. +3 (og = rg), db1 (t < D),
  // dWpos / dbpos at (rg rows, channels 4 c4 .. +3)
  float4 gw[DW1 ? W::OPT : 1];
#pragma unroll
  for (int i = 0; i < (DW1 ? W::OPT : 1); ++i) gw[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  float gb1 = 0.f;
  float4 gwp[3], gbp = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < 3; ++j) gwp[j] = make_float4(0.f, 0.f, 0.f, 0.f);

  // per-output loads of a query: g' and argmax for outputs o = t (t < D)
  float ov = 0.f, dv = 0.f;
  unsigned av = 0;
  auto load_out = [&](int q) {
    const bool ok = q < s.nq && t < D;
    const unsigned oo = (unsigned)q * D + t;
    ov = bld(outr, ok ? oo * 4u : kOOB);
    dv = bld(dor, ok ? oo * 4u : kOOB);
    av = __builtin_amdgcn_raw_buffer_load_b8(amr, (int)(ok ? oo : kOOB), 0, 0);
  };
  int rk[G::RPT], rkd = -1;  // slots: column-pass rows, row-per-lane (direction pass)
  auto load_rank = [&](int q) {
#pragma unroll
    for (int i = 0; i < G::RPT; ++i) {
      const int r = rg + G::RG * i;
      rk[i] = (int)__builtin_amdgcn_raw_buffer_load_b32(
          rkr, (int)(r < k ? ((unsigned)q * (unsigned)k + r) * 4u : kOOB), 0, 0);
    }
    rkd = (int)__builtin_amdgcn_raw_buffer_load_b32(
        rkr, (int)(l32 < k ? ((unsigned)q * (unsigned)k + l32) * 4u : kOOB), 0, 0);
  };
  auto stage_out = [&](int p) {
    if (t < D) {
      const float g = ov > 0.f ? dv : dv * kSlope;
      gam[p][t] = make_float2(g, __int_as_float((int)av));
      __bf16 gh, gm, gl;
      split3(g, gh, gm, gl);
      gpl[p][0][t] = gh;
      gpl[p][1][t] = gm;
      gpl[p][2][t] = gl;
      gam16[p][t] = (unsigned short)av;
    }
  };

  int jn[G::RPT], jn2[G::RPT];
  WideLoads<D> L;
  wide_load_idx<D>(s, q0, jn, rg);
  wide_load<D>(s, q0, jn, rg, c4, L);
  load_out(q0);
  wide_load_idx<D>(s, q0 + 1, jn2, rg);
  __syncthreads();  // wposT
  wide_build<D>(L, k, rg, c4, wposT, Hs[0], dirs[0]);
  stage_out(0);
  __syncthreads();
  for (int q = q0; q < q1; ++q) {
    const int p = (q - q0) & 1;
    const bool more = q + 1 < q1;
    if (MAIN && ranked) load_rank(q);
    auto next_loads = [&]() {
#pragma unroll
      for (int i = 0; i < G::RPT; ++i) jn[i] = jn2[i];
      wide_load<D>(s, more ? q + 1 : s.nq, jn, rg, c4, L);
      load_out(more ? q + 1 : s.nq);
      wide_load_idx<D>(s, q + 2 < q1 ? q + 2 : s.nq, jn2, rg);
    };
    if constexpr (W::PREFETCH) next_loads();  // in flight under this query's MFMAs
    float* H = Hs[p];
    const float2* ga = gam[p];
    // ---- dh0 = M W1 (rows = neighbours, columns 32w .. +31 of Din) on mfma_x6: K-step ks,
    // lane half h: outputs o = 16 ks + 8 h + j; A[l32][o] = planes of g'[o] where am[o] == l32
    // (a 16-bit mask per output from the packed u16 rows: (am ^ l32) - 1 < 0 <=> am == l32)
    f32x16 dacc;
    if constexpr (MAIN) {
#pragma unroll
    for (int e = 0; e < 16; ++e) dacc[e] = 0.f;
    constexpr int PF = 2;  // K-steps of B planes in flight
    Planes bq[PF];
    auto bload = [&](int ks, Planes& bb) {
      bb.h = w1row[(3 * ks + 0) * 64];
      bb.m = w1row[(3 * ks + 1) * 64];
      bb.l = w1row[(3 * ks + 2) * 64];
    };
#pragma unroll
    for (int i = 0; i < PF; ++i) bload(i, bq[i]);
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    const unsigned tgt = (unsigned)l32 * 0x00010001u;
#pragma unroll 2
    for (int ks = 0; ks < W::NKS; ++ks) {
      const int o0 = 16 * ks + 8 * half;
      const uint4 av4 = *reinterpret_cast<const uint4*>(&gam16[p][o0]);
      const uint4 ph = *reinterpret_cast<const uint4*>(&gpl[p][0][o0]);
      const uint4 pm = *reinterpret_cast<const uint4*>(&gpl[p][1][o0]);
      const uint4 pl = *reinterpret_cast<const uint4*>(&gpl[p][2][o0]);
      const unsigned aw[4] = {av4.x, av4.y, av4.z, av4.w};
      unsigned mk[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const s16x2 d = __builtin_bit_cast(s16x2, aw[i] ^ tgt) - (s16x2){1, 1};
        mk[i] = __builtin_bit_cast(unsigned, d >> (s16x2){15, 15});
      }
      const uint4 mh = make_uint4(ph.x & mk[0], ph.y & mk[1], ph.z & mk[2], ph.w & mk[3]);
      const uint4 mm = make_uint4(pm.x & mk[0], pm.y & mk[1], pm.z & mk[2], pm.w & mk[3]);
      const uint4 ml = make_uint4(pl.x & mk[0], pl.y & mk[1], pl.z & mk[2], pl.w & mk[3]);
      dacc = mfma_x6(__builtin_bit_cast(bf16x8, mh), __builtin_bit_cast(bf16x8, mm),
                     __builtin_bit_cast(bf16x8, ml), bq[ks % PF].h, bq[ks % PF].m, bq[ks % PF].l,
                     dacc);
      if (ks + PF < W::NKS) bload(ks + PF, bq[ks % PF]);
      // one K-step's LDS reads ahead at most
      __builtin_amdgcn_sched_barrier(0);
    }
    }  // MAIN
    // ---- dW1[o, 4c4..] += g'[o] h0[am[o], 4c4..] for this thread's o rows; db1
    if constexpr (DW1) {
#pragma unroll
    for (int i = 0; i < W::OPT; ++i) {
      const float2 g = ga[obase + rg * W::OPT + i];
      const float4 hv = *reinterpret_cast<const float4*>(H + __float_as_int(g.y) * G::LD + 4 * c4);
      gw[i].x = __builtin_fmaf(g.x, hv.x, gw[i].x);
      gw[i].y = __builtin_fmaf(g.x, hv.y, gw[i].y);
      gw[i].z = __builtin_fmaf(g.x, hv.z, gw[i].z);
      gw[i].w = __builtin_fmaf(g.x, hv.w, gw[i].w);
      if (i % 4 == 3) __builtin_amdgcn_sched_barrier(0);  // bound the hoisted LDS reads
    }
    if (t < D && blockIdx.y == 0) gb1 = __fadd_rn(gb1, ga[t].x);
    }  // DW1
    __syncthreads();  // every read of h0 done
    if constexpr (MAIN) {
    // ---- dz0 = dh0 * LeakyReLU'(h0), in place (accumulator layout)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = (e & 3) + 8 * (e >> 2) + 4 * half;
      const int a = row * G::LD + 32 * w + l32;
      const float hv = H[a];
      float sl = hv > 0.f ? 1.f : kSlope;
      if constexpr (OVR) {  // rows >= k: dacc is 0 there
        const unsigned o = __builtin_amdgcn_raw_buffer_load_b8(
            s0r, (int)(((unsigned)q * (unsigned)k + row) * D + 32 * w + l32), 0, 0);
        sl = o == 1u ? 1.f : (o == 2u ? kSlope : sl);
      }
      H[a] = dacc[e] * sl;
    }
    __syncthreads();
    // ---- column pass: dP2 rows out, dP1 partials, dWpos / dbpos
    {
      float4 sp = make_float4(0.f, 0.f, 0.f, 0.f);
      float* d2 = dp2_rows + (long long)q * k * D + 4 * c4;
#pragma unroll
      for (int i = 0; i < G::RPT; ++i) {
        const int r = rg + G::RG * i;
        const float4 v = *reinterpret_cast<const float4*>(H + r * G::LD + 4 * c4);
        const float4 dr = dirs[p][r];
        if (ranked) {
          if (r < k && rk[i] >= 0) *reinterpret_cast<float4*>(rows + (long long)rk[i] * D + 4 * c4) = v;
        } else if (r < k && dp2_rows) {  // null: the pull-form caller sums per point itself
          *reinterpret_cast<float4*>(d2 + (long long)r * D) = v;
        }
        sp.x = __fadd_rn(sp.x, v.x);
        sp.y = __fadd_rn(sp.y, v.y);
        sp.z = __fadd_rn(sp.z, v.z);
        sp.w = __fadd_rn(sp.w, v.w);
        const float dd[3] = {dr.x, dr.y, dr.z};
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          gwp[j].x = __builtin_fmaf(v.x, dd[j], gwp[j].x);
          gwp[j].y = __builtin_fmaf(v.y, dd[j], gwp[j].y);
          gwp[j].z = __builtin_fmaf(v.z, dd[j], gwp[j].z);
          gwp[j].w = __builtin_fmaf(v.w, dd[j], gwp[j].w);
        }
      }
      red[rg][c4] = sp;
    }
    // ---- direction pass: d(dir_r) = Wpos^T dz0[r], partial over channel group g2
    {
      const int r = t & 31, g2 = t >> 5;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll 4
      for (int i = 0; i < CPG / 4; ++i) {
        const int c = g2 * CPG + 4 * i;
        const float4 v = *reinterpret_cast<const float4*>(H + r * G::LD + c);
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float4 wq = wposT[c + e];
          a0 = __builtin_fmaf(wq.x, vv[e], a0);
          a1 = __builtin_fmaf(wq.y, vv[e], a1);
          a2 = __builtin_fmaf(wq.z, vv[e], a2);
        }
      }
      red2[g2][r] = make_float4(a0, a1, a2, 0.f);
    }
    // ---- the next query's tile (other buffer) from the loads issued at the top
    }  // MAIN
    if constexpr (!W::PREFETCH) next_loads();
    if (more) {
      wide_build<D>(L, k, rg, c4, wposT, Hs[p ^ 1], dirs[p ^ 1]);
      stage_out(p ^ 1);
    }
    __syncthreads();
    // ---- per-query sums in a fixed order: dP1 (threads of row group 0), d(dir) rows + dx1
    if (MAIN && rg == 0) {
      float4 v = red[0][c4];
#pragma unroll
      for (int g = 1; g < G::RG; ++g) {
        const float4 x = red[g][c4];
        v.x = __fadd_rn(v.x, x.x);
        v.y = __fadd_rn(v.y, x.y);
        v.z = __fadd_rn(v.z, x.z);
        v.w = __fadd_rn(v.w, x.w);
      }
      *reinterpret_cast<float4*>(dp1 + (long long)q * D + 4 * c4) = v;
      gbp.x = __fadd_rn(gbp.x, v.x);
      gbp.y = __fadd_rn(gbp.y, v.y);
      gbp.z = __fadd_rn(gbp.z, v.z);
      gbp.w = __fadd_rn(gbp.w, v.w);
    }
    if (MAIN && w == G::NW - 1 && half == 0) {  // one half-wave: lane l32 = neighbour row
      float4 v = red2[0][l32];
#pragma unroll
      for (int g = 1; g < NG2; ++g) {
        const float4 x = red2[g][l32];
        v.x = __fadd_rn(v.x, x.x);
        v.y = __fadd_rn(v.y, x.y);
        v.z = __fadd_rn(v.z, x.z);
      }
      const bool row = l32 < k;
      if (row && ranked) {
        if (rkd >= 0)
          *reinterpret_cast<float4*>(rows + (long long)b * n1 * k * D + (long long)rkd * 4) =
              make_float4(v.x, v.y, v.z, 0.f);
      } else if (row && ddir_rows) {
        float* dd = ddir_rows + ((long long)q * k + l32) * 3;
        dd[0] = v.x;
        dd[1] = v.y;
        dd[2] = v.z;
      }
      float s0 = row ? v.x : 0.f, s1 = row ? v.y : 0.f, s2 = row ? v.z : 0.f;
#pragma unroll
      for (int m = 16; m >= 1; m >>= 1) {
        s0 = __fadd_rn(s0, __shfl_xor(s0, m, kWave));
        s1 = __fadd_rn(s1, __shfl_xor(s1, m, kWave));
        s2 = __fadd_rn(s2, __shfl_xor(s2, m, kWave));
      }
      if (l32 == 0) {
        float* o = dx1 + (long long)q * 3;
        o[0] = -s0;
        o[1] = -s1;
        o[2] = -s2;
      }
    }
  }
  // ---- workgroup slab: dW1 (o, c) | db1 | dWpos^T (x, y, z rows) | dbpos; the dWpos partials
  // of the row groups are folded in row-group order through LDS
  if constexpr (DW1) {
#pragma unroll
    for (int i = 0; i < W::OPT; ++i)
      *reinterpret_cast<float4*>(sb + (long long)(obase + rg * W::OPT + i) * D + 4 * c4) = gw[i];
    if (t < D && blockIdx.y == 0) sb[D * D + t] = gb1;
  }
  if constexpr (!MAIN) return;
  __syncthreads();
  float4* fold = reinterpret_cast<float4*>(&Hs[0][0]);  // [RG][3][C4]
#pragma unroll
  for (int j = 0; j < 3; ++j) fold[(rg * 3 + j) * G::C4 + c4] = gwp[j];
  __syncthreads();
  if (rg == 0) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float4 v = fold[j * G::C4 + c4];
      for (int g = 1; g < G::RG; ++g) {
        const float4 x = fold[(g * 3 + j) * G::C4 + c4];
        v.x = __fadd_rn(v.x, x.x);
        v.y = __fadd_rn(v.y, x.y);
        v.z = __fadd_rn(v.z, x.z);
        v.w = __fadd_rn(v.w, x.w);
      }
      *reinterpret_cast<float4*>(sb + D * D + D + j * D + 4 * c4) = v;
    }
    *reinterpret_cast<float4*>(sb + D * D + 4 * D + 4 * c4) = gbp;
  }
}

// w1 (D, D) -> the backward's streamed B planes of dh0 = M W1 (mfma_x6): bf16x8 (wave w, ks,
// plane, lane) = plane of W1[16 ks + 8 (lane >> 5) + 0..7][32 w + (lane & 31)]
__global__ __launch_bounds__(256) void cvw_w1_planes_kernel(int d, const float* __restrict__ w1,
                                                            bf16x8* __restrict__ w1p) {
  const int e = blockIdx.x * 256 + threadIdx.x;  // (w, ks, lane)
  const int nks = d / 16;
  if (e >= (d / 32) * nks * 64) return;
  const int lane = e & 63, q = e >> 6, ks = q % nks, w = q / nks;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = w1[(16 * ks + 8 * (lane >> 5) + j) * d + 32 * w + (lane & 31)];
  const Planes pl = split8(v);
  bf16x8* dst = w1p + (long long)q * 3 * 64 + lane;
  dst[0] = pl.h;
  dst[64] = pl.m;
  dst[128] = pl.l;
}

// queries per workgroup: A/B at the model's calls (round 4, B=16 pair batch, K=32): forward
// D=128 512 workgroups (108.5 us; 256: 140), D=256 256 (173.6 vs 180.7 at 512); backward 256
// for both (cross2 251 vs 256 us, cross3 394 vs 428 us).  The backward's parameter-gradient
// slab count follows it, so the dW1 / dWpos sums are grouped by it.
inline int fused_qpw(long long nq, int d, bool bwd) {
  const int target = bwd || d == 256 ? 256 : 512;
  return (int)std::max<long long>(2, divupll(nq, target));
}

}  // namespace

namespace kdpc {

bool cost_volume_wide_fused_supported(int din, int dout, int k) {
  return din == dout && (din == 128 || din == 256) && k >= 1 && k <= 32;
}

hipError_t cost_volume_wide_fused_fwd(int b, int n1, int n2, int k, int d, const float* x1,
                                      const float* x2, const int* idx, const float* p1,
                                      const float* p2, const float* wpos, const float* bpos,
                                      const float* w1, const float* b1, float* out,
                                      unsigned char* amax, hipStream_t st) {
  const long long nq = (long long)b * n1;
  const int qpw = fused_qpw(nq, d, false);
  const dim3 grid((unsigned)divupll(nq, qpw));
  if (d == 128)
    hipLaunchKernelGGL(cvw_fused_fwd_kernel<128>, grid, dim3(256), 0, st, b, n1, n2, k, qpw, x1,
                       x2, idx, p1, p2, wpos, bpos, w1, b1, out, amax);
  else
    hipLaunchKernelGGL(cvw_fused_fwd_kernel<256>, grid, dim3(512), 0, st, b, n1, n2, k, qpw, x1,
                       x2, idx, p1, p2, wpos, bpos, w1, b1, out, amax);
  return hipGetLastError();
}

size_t cost_volume_wide_fused_bwd_workspace_floats(int b, int n1, int d) {
  const long long nq = (long long)b * n1;
  const long long nwg = divupll(nq, fused_qpw(nq, d, true));
  const long long len = (long long)d * d + 5 * d;
  // + the B planes of W1 (6 bytes per element)
  return (size_t)(nwg * len + colsum_scratch_floats((int)nwg, len) + (long long)d * d * 3 / 2 + 4);
}

hipError_t cost_volume_wide_fused_bwd(int b, int n1, int n2, int k, int d, const float* x1,
                                      const float* x2, const int* idx, const float* p1,
                                      const float* p2, const float* wpos, const float* bpos,
                                      const float* w1, const float* out,
                                      const unsigned char* amax, const unsigned char* slope0,
                                      const float* dout, float* dp1, float* dp2_rows, float* dx1,
                                      float* ddir_rows, const int* rank, float* rows, float* ws,
                                      float* dparams, hipStream_t st) {
  const long long nq = (long long)b * n1;
  const int qpw = fused_qpw(nq, d, true);
  const int nwg = (int)divupll(nq, qpw);
  const long long len = (long long)d * d + 5 * d;
  float* slab = ws;
  float* scratch = ws + (long long)nwg * len;
  // 16-byte aligned (the float count before it is a multiple of 4 only by luck: round up)
  bf16x8* w1p = reinterpret_cast<bf16x8*>(
      (reinterpret_cast<uintptr_t>(scratch + colsum_scratch_floats(nwg, len)) + 15) & ~(uintptr_t)15);
#define KDPC_CVW_BWD(DD, PART, OV, GRID)                                                          \
  hipLaunchKernelGGL((cvw_fused_bwd_kernel<DD, PART, OV>), GRID, dim3(2 * DD), 0, st, b, n1, n2, k, \
                     qpw, x1, x2, idx, p1, p2, wpos, bpos, w1, w1p, out, amax, slope0, dout, dp1,    \
                     dp2_rows, dx1, ddir_rows, rank, rows, slab)
  hipLaunchKernelGGL(cvw_w1_planes_kernel, dim3(divup((d / 32) * (d / 16) * 64, 256)), dim3(256),
                     0, st, d, w1, w1p);
  {
    const hipError_t e0 = hipGetLastError();
    if (e0 != hipSuccess) return e0;
  }
  if (d == 128) {
    if (slope0)
      KDPC_CVW_BWD(128, 0, true, dim3(nwg));
    else
      KDPC_CVW_BWD(128, 0, false, dim3(nwg));
  } else {
    hipError_t e;
    if (slope0)
      KDPC_CVW_BWD(256, 1, true, dim3(nwg));
    else
      KDPC_CVW_BWD(256, 1, false, dim3(nwg));
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // dW1 / db1 read g', argmax and h0 only: no slope0 there
    KDPC_CVW_BWD(256, 2, false, dim3(nwg, WideBwd<256>::OSPLIT));
  }
#undef KDPC_CVW_BWD
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return colsum(nwg, len, slab, dparams, scratch, st);
}

}  // namespace kdpc

namespace {
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
