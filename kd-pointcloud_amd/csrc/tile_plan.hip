// Row tiles with shared neighbours for the PointConv backward's dG reduction.
//
// The data kernel (pointconv_fused.hip) produces one dG row per (row, neighbour) pair, and
// every point's gradient is the sum of the dG rows naming it.  Written per pair and summed
// through the kNN's CSR, that is R*K*C8*4 bytes out and back (321 MB for the level-0
// estimator's second layer at B=8) -- the "2.8x" of the round-3 traffic figure.  With the
// rows of a tile chosen close in space, the 32*K pairs of a 32-row tile name far fewer
// distinct points (self-kNN, K=9, FlyingThings-shaped clouds: 69 of 288 at N=8192 in Morton
// order, 284 of 288 in input order), so the kernel sums the pairs of one destination inside
// the tile in LDS and writes one partial row per (tile, destination); the CSR then runs over
// those partial rows.  Every sum keeps a fixed order: pairs of a destination in ascending
// pair order inside a tile, tiles in ascending tile order.
//
//   kdpc_morton_order: per batch element, the rows in Morton order of their centers
//     (6 bits per axis over the element's bounding box; ties by index) -- one 1024-thread
//     workgroup per element, a bitonic sort of (code << 13 | index) keys in LDS.
//   kdpc_pc_tile_plan: per 32-row tile, its rows, its pairs sorted by (destination, pair),
//     each destination's first sorted position, and the destination keys that the CSR of
//     the partial rows is built over (kdpc_csr_build / kdpc_csr_rank).
#include "kdpc_common.h"

using namespace kdpc;

namespace {

constexpr int kMortonMax = 8192;  // rows per batch element the LDS sort holds
constexpr int kTileRows = 32;     // = the data kernel's row tile

__device__ __forceinline__ unsigned spread3(unsigned v) {  // 6 bits -> every third bit
  unsigned r = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) r |= ((v >> i) & 1u) << (3 * i);
  return r;
}

__device__ __forceinline__ float wave_min_f(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// ascending bitonic sort of key[0..p) (p a power of two) by the whole workgroup
template <int NT>
__device__ void bitonic_sort(unsigned* key, int p) {
  for (int kk = 2; kk <= p; kk <<= 1) {
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < p; i += NT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned a = key[i], c = key[ixj];
          if ((a > c) == ((i & kk) == 0)) {
            key[i] = c;
            key[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(1024) void morton_order_kernel(int s, const float* __restrict__ xyz,
                                                            int* __restrict__ order) {
  __shared__ unsigned key[kMortonMax];
  __shared__ float box[6][16];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const float* x = xyz + (long long)b * s * 3;
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = t; i < s; i += 1024)
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const float v = x[i * 3 + d];
      lo[d] = fminf(lo[d], v);
      hi[d] = fmaxf(hi[d], v);
    }
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    lo[d] = wave_min_f(lo[d]);
    hi[d] = wave_max_f(hi[d]);
  }
  if (lane == 0)
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      box[d][wv] = lo[d];
      box[3 + d][wv] = hi[d];
    }
  __syncthreads();
  float scale[3];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    float l = box[d][0], h = box[3 + d][0];
    for (int w = 1; w < 16; ++w) {
      l = fminf(l, box[d][w]);
      h = fmaxf(h, box[3 + d][w]);
    }
    lo[d] = l;
    const float ext = h - l;
    scale[d] = ext > 0.f ? 64.f / ext : 0.f;
  }
  int p = 1;
  while (p < s) p <<= 1;
  for (int i = t; i < p; i += 1024) {
    unsigned k = 0xFFFFFFFFu;
    if (i < s) {
      unsigned code = 0;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const float q = (x[i * 3 + d] - lo[d]) * scale[d];
        const unsigned c = q >= 63.f ? 63u : (q > 0.f ? (unsigned)q : 0u);  // NaN -> 0
        code |= spread3(c) << d;
      }
      k = (code << 13) | (unsigned)i;
    }
    key[i] = k;
  }
  __syncthreads();
  bitonic_sort<1024>(key, p);
  for (int i = t; i < s; i += 1024) order[(long long)b * s + i] = (int)(key[i] & 8191u);
}

// block-wide exclusive scan of one value per thread (256 threads); returns the total
__device__ int block_scan_excl(int v, int* excl, int* wsum) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  int base = 0, total = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    base += w < wv ? wsum[w] : 0;
    total += wsum[w];
  }
  *excl = base + x - v;
  __syncthreads();  // wsum reusable
  return total;
}

// one 256-thread workgroup per 32-row tile; tiles do not span batch elements (tb per element)
__global__ __launch_bounds__(256) void pc_tile_plan_kernel(int s, int n, int k, int tb,
                                                           const int* __restrict__ idx,
                                                           const int* __restrict__ order,
                                                           int* __restrict__ trow,
                                                           int* __restrict__ tpair,
                                                           int* __restrict__ tsoff,
                                                           int* __restrict__ tkey) {
  __shared__ unsigned key[512];
  __shared__ int rl[kTileRows];
  __shared__ int wsum[4];
  const int tile = blockIdx.x, b = tile / tb, t0 = (tile - b * tb) * kTileRows;
  const int t = threadIdx.x;
  const int trk = kTileRows * k;
  if (t < kTileRows) {
    const int local = t0 + t;
    const int r = local < s ? (order ? order[(long long)b * s + local] : local) : -1;
    rl[t] = r;
    trow[(long long)tile * kTileRows + t] = r < 0 ? -1 : b * s + r;
  }
  __syncthreads();
  for (int p = t; p < 512; p += 256) {
    unsigned kv = 0xFFFFFFFFu;
    if (p < trk) {
      const int r = rl[p / k];
      if (r >= 0) {
        const int j = idx[((long long)b * s + r) * k + (p % k)];
        if (j >= 0 && j < n) kv = ((unsigned)j << 9) | (unsigned)p;
      }
    }
    key[p] = kv;
  }
  __syncthreads();
  bitonic_sort<256>(key, 512);
  // thread t owns sorted positions 2t, 2t+1: a position starts a destination group when it
  // is valid and its destination differs from the previous position's
  unsigned kk[2];
  int f[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int i = 2 * t + e;
    kk[e] = key[i];
    f[e] = kk[e] != 0xFFFFFFFFu && (i == 0 || (key[i - 1] >> 9) != (kk[e] >> 9));
  }
  int nvalid_part = (kk[0] != 0xFFFFFFFFu) + (kk[1] != 0xFFFFFFFFu);
  int excl;
  const int ngroups = block_scan_excl(f[0] + f[1], &excl, wsum);
  int vexcl;
  const int nvalid = block_scan_excl(nvalid_part, &vexcl, wsum);
  (void)vexcl;
  int* sp = tpair + (long long)tile * trk;
  int* so = tsoff + (long long)tile * (trk + 1);
  int* sk = tkey + (long long)tile * trk;
  int slot = excl;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int i = 2 * t + e;
    if (i < trk) sp[i] = kk[e] != 0xFFFFFFFFu ? (int)(kk[e] & 511u) : -1;
    if (f[e]) {
      so[slot] = i;
      sk[slot] = (int)(kk[e] >> 9);
      ++slot;
    }
  }
  for (int g = ngroups + t; g <= trk; g += 256) {
    so[g] = nvalid;
    if (g < trk) sk[g] = -1;
  }
}

}  // namespace

KDPC_API int kdpc_morton_order(int b, int s, const float* xyz, int* order, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && s >= 0 && s <= kMortonMax && b <= 65535);
  if (b == 0 || s == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(xyz && order);
  hipLaunchKernelGGL(morton_order_kernel, dim3(b), dim3(1024), 0, (hipStream_t)stream, s, xyz,
                     order);
  KDPC_RETURN_LAUNCH();
}

KDPC_API int kdpc_pc_tile_plan(int b, int s, int n, int k, const int* idx, const int* order,
                               int* trow, int* tpair, int* tsoff, int* tkey, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && s >= 0 && n > 0 && n < (1 << 22) && k >= 1 && k <= 16);
  const long long tiles = (long long)b * divup(s, kTileRows);
  KDPC_CHECK_ARG(tiles < (1ll << 31) / 512);
  if (tiles == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(idx && trow && tpair && tsoff && tkey);
  hipLaunchKernelGGL(pc_tile_plan_kernel, dim3((unsigned)tiles), dim3(256), 0,
                     (hipStream_t)stream, s, n, k, divup(s, kTileRows), idx, order, trow, tpair,
                     tsoff, tkey);
  KDPC_RETURN_LAUNCH();
}
