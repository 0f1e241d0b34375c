// Shared device helpers of the PointConv kernels (pointconv_fused.hip, pointconv_ws.hip):
// the tile geometry, the MFMA step, the neighbour gathers through buffer loads and the
// packed-f32 row build.  Internal linkage: each translation unit gets its own copy.
#pragma once

#include "kdpc_common.h"
#include "split_bf16.h"

using namespace kdpc;

namespace kdpc_pc {

using namespace kdpc_x6;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kW = 16;              // WeightNet width (weightnet=16 in every model layer)
constexpr int kCC = 8;              // channels per chunk
constexpr int kNC = kCC * kW;       // A columns per chunk (128)
constexpr int kKMax = 16;           // neighbours per row supported
constexpr int kBlk = 32 * 4 + 16;   // floats per 4-column block of a 32-row MFMA-A tile
constexpr int kTS = 32 + 4;         // row stride of transposed (inner = row) 32-row tiles
constexpr int kDaS = kNC + 4;       // row stride of the dA chunk
constexpr int kTargetWG = 512;      // grid size the split heuristics aim for
constexpr int kCUs = 256;           // MI355X compute units

struct Geo {
  int n, s, k, d, c, r, nch, c8;  // c = 3 + d, r = B*S rows, nch = ceil(c/8), c8 = 8*nch
  int bn;                         // B*N points
  const float* xyz;               // (B,N,3)
  const float* center;            // (B,S,3)
  const float* feats;             // (B,N,D)
  const int* idx;                 // (B,S,K)
  const int* rank;                // (B*S*K) CSR slot of each (row, neighbour) (backward only)
  // tiled backward (tile_plan.hip; null otherwise): per 32-row tile its global rows
  // (trow, -1 = none), its pairs sorted by (destination, pair) (tpair), each destination's
  // first sorted position (tsoff, stride 32K+1) and partial-row slot (tdst, stride 32K)
  const int* trow;
  const int* tpair;
  const int* tsoff;
  const int* tdst;
  int ntrow;  // entries of trow (tiles * 32)
};

__device__ __forceinline__ f32x16 mfma4(float4 a, float4 b, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// global row of neighbour kk of row `row` (b*N + idx), -1 past the last row
__device__ __forceinline__ int nbr_of(const Geo& g, int row, int kk) {
  if (row >= g.r) return -1;
  return (row / g.s) * g.n + g.idx[(long long)row * g.k + kk];
}

// Gathers go through buffer loads: 32-bit byte offsets (one VGPR per in-flight slot instead
// of a 64-bit address) and hardware bounds checks (an offset past the buffer reads 0).
constexpr unsigned kOOB = 0x80000000u;  // byte offset that is always out of range

// CSR slot of neighbour kk of row `row` (the dG row it writes), -1 for none / out of range
__device__ __forceinline__ int slot_of(const Geo& g, int row, int kk) {
  return g.rank[(long long)row * g.k + kk];
}

// float offset of dG row `slot`'s 8 values of chunk ch: rows of C8 floats in CSR order (the
// pair's slot, slot_of), each row's 32 bytes of a chunk sit C8*4 bytes apart; pc_csr_sum
// reads every point's rows as one contiguous run (chunk-major rows -- full-line stores --
// measured round 2: data kernel 576 -> 514 us but pc_csr_sum 86 -> 173 us from its 32-byte
// gathers, a net loss).
__device__ __forceinline__ long long dg_off(long long pos, int ch, long long /*rk*/, int c8) {
  return pos * c8 + (long long)ch * kCC;
}

struct Srcs {
  __amdgpu_buffer_rsrc_t xyz, center, feats;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p, long long nfloats) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)(nfloats * 4),
                                           0x00020000);
}

__device__ __forceinline__ Srcs srcs_of(const Geo& g) {
  Srcs s;
  s.xyz = rsrc(g.xyz, (long long)g.bn * 3);
  s.center = rsrc(g.center, (long long)g.r * 3);
  s.feats = rsrc(g.feats, (long long)g.bn * g.d);
  return s;
}

__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)byte_off, 0, 0));
}

// byte offset of neighbour nb's feature row (kOOB for none)
__device__ __forceinline__ unsigned feat_off(const Geo& g, int nb) {
  return nb < 0 ? kOOB : (unsigned)nb * (unsigned)g.d * 4u;
}

// G value of channel cg for neighbour row nb of row `row`
__device__ __forceinline__ float g_fetch(const Geo& g, const Srcs& s, int nb, int row, int cg) {
  if (nb < 0) return 0.f;
  if (cg < 3)
    return bload(s.xyz, ((unsigned)nb * 3u + cg) * 4u) - bload(s.center, ((unsigned)row * 3u + cg) * 4u);
  if (cg < g.c) return bload(s.feats, (unsigned)nb * (unsigned)g.d * 4u + (unsigned)(cg - 3) * 4u);
  return 0.f;
}

// acc[c] = sum_k G[r,k,c] wk[k] over the tile's LDS gather (ascending k, one fma each;
// scalar fmas: kdpc_common.h, no packed f32).
template <int KM>
__device__ __forceinline__ void build_row(const float* gl, int r, int k_n, const float* wk,
                                          float (&a)[kCC]) {
#pragma unroll
  for (int c = 0; c < kCC; ++c) a[c] = 0.f;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (k < k_n) {
      const float4 lo = *reinterpret_cast<const float4*>(gl + (r * k_n + k) * kCC);
      const float4 hi = *reinterpret_cast<const float4*>(gl + (r * k_n + k) * kCC + 4);
      const float w = wk[k];
      a[0] = __builtin_fmaf(lo.x, w, a[0]);
      a[1] = __builtin_fmaf(lo.y, w, a[1]);
      a[2] = __builtin_fmaf(lo.z, w, a[2]);
      a[3] = __builtin_fmaf(lo.w, w, a[3]);
      a[4] = __builtin_fmaf(hi.x, w, a[4]);
      a[5] = __builtin_fmaf(hi.y, w, a[5]);
      a[6] = __builtin_fmaf(hi.z, w, a[6]);
      a[7] = __builtin_fmaf(hi.w, w, a[7]);
    }
    if (k % 4 == 3) __builtin_amdgcn_sched_barrier(0);  // bound the hoisted LDS reads
  }
}

}  // namespace kdpc_pc
