// Streaming k-nearest-neighbour selection: the MI355X replacement for the reference's
// knn_point (pointconv_util.py:96-107) = square_distance (:73-94, a materialised (B,S,N)
// matrix) + torch.topk(largest=False, sorted=False).
//
// Semantics: for each query, the K refs with the smallest expanded-form squared distance
//   d = (-2 * fma(z,z',fma(y,y',x*x')) + |q|^2) + |r|^2
// (bit-identical to torch's square_distance, see kdpc_common.h), ordered ascending by
// (d, index).  topk(sorted=False) leaves order and exact-tie choice unspecified; we fix
// them (ascending, lower index wins a tie), which the oracle (oracle_knn) restates.
//
// Design (no S x N matrix is ever written):
//   * a workgroup = 4 waves; each wave owns QW queries; the workgroup streams the refs of
//     its cloud through LDS in tiles of float4 {x, y, z, |r|^2} (|r|^2 computed once at
//     staging), read by ds_read_b128 lane-contiguous (conflict-free);
//   * each query's current best-64 list lives in the wave's registers, rank r in lane r
//     ({d, idx} = 2 VGPRs per query); the K-th entry is the rejection threshold;
//   * per 64-ref chunk a query costs 4 VALU + one compare whose VCC mask is the ballot;
//     a chunk with no candidate (the common case once the list is warm) is skipped by
//     a scalar branch;
//   * few candidates: serial insertion with a DPP wave_shr:1 shift (~10 instr each);
//     many candidates (the first chunks): 64-lane bitonic sort of the chunk + bitonic
//     merge with the list.
#include "kdpc_common.h"

using namespace kdpc;

namespace {

// torch's expanded form ((-2*dot + |q|^2) + |r|^2), one rounding fewer to issue: -2*dot is
// exact, so fma(-2, dot, |q|^2) == round(round(-2*dot) + |q|^2) bit for bit.
__device__ __forceinline__ float sqdist_fast(float qx, float qy, float qz, float sq, float rx,
                                             float ry, float rz, float sr) {
  const float dot = __builtin_fmaf(qz, rz, __builtin_fmaf(qy, ry, __fmul_rn(qx, rx)));
  return __fadd_rn(__builtin_fmaf(-2.0f, dot, sq), sr);
}

constexpr int kTile = 2048;      // refs per LDS tile (32 KiB of float4)
constexpr int kSerialMax = 8;    // candidates per chunk inserted one by one

__device__ __forceinline__ bool kv_less(float ad, int ai, float bd, int bi) {
  return ad < bd || (ad == bd && ai < bi);
}

// bitonic compare-exchange step across lanes l and l^jj
__device__ __forceinline__ void bitonic_step(float& d, int& i, int jj, bool up) {
  const float od = __shfl_xor(d, jj, kWave);
  const int oi = __shfl_xor(i, jj, kWave);
  const bool lower = (lane_id() & jj) == 0;
  const bool o_less = kv_less(od, oi, d, i);
  const bool take = (lower == up) ? o_less : !o_less && !(od == d && oi == i);
  d = take ? od : d;
  i = take ? oi : i;
}

__device__ __forceinline__ void bitonic_sort64(float& d, int& i) {
#pragma unroll
  for (int kk = 2; kk <= 64; kk <<= 1) {
    const bool up = (lane_id() & kk) == 0 || kk == 64;
#pragma unroll
    for (int jj = kk >> 1; jj > 0; jj >>= 1) bitonic_step(d, i, jj, up);
  }
}

__device__ __forceinline__ void bitonic_merge64(float& d, int& i) {
#pragma unroll
  for (int jj = 32; jj > 0; jj >>= 1) bitonic_step(d, i, jj, true);
}

// Merge the chunk's candidates (cand lanes carry {d, gi}) into the sorted list {ld, li}.
__device__ __forceinline__ void insert_candidates(unsigned long long mask, bool cand, float d,
                                                  int gi, float& ld, int& li) {
  if (__popcll(mask) > kSerialMax) {
    float cd = cand ? d : INFINITY;
    int ci = cand ? gi : 0x7fffffff;
    bitonic_sort64(cd, ci);
    const int src = 63 - lane_id();
    const float rd = __shfl(cd, src, kWave);
    const int ri = __shfl(ci, src, kWave);
    const bool take = kv_less(rd, ri, ld, li);
    ld = take ? rd : ld;
    li = take ? ri : li;
    bitonic_merge64(ld, li);
  } else {
    // candidates arrive in ascending index order and every list entry has a smaller
    // index, so an equal distance keeps the existing entry first (strict >).
    while (mask) {
      const int j = __ffsll((long long)mask) - 1;
      mask &= mask - 1;
      const float cd = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d), j));
      const int ci = __builtin_amdgcn_readlane(gi, j);
      const float pd = wave_shr1(ld, -INFINITY);
      const int pi = wave_shr1(li, 0);
      const bool gt = ld > cd;
      const bool pgt = pd > cd;
      const float nd = gt ? (pgt ? pd : cd) : ld;
      const int ni = gt ? (pgt ? pi : ci) : li;
      ld = nd;
      li = ni;
    }
  }
}

// ------------------------------------------------------------ seeded threshold
// The plain scan starts every query with an empty list, so the threshold only tightens as
// the list fills: about K ln(N/K) insertions per query (~110 serial + several bitonic
// merges for K=32, N=8192, random point order), several times the cost of the distances.
// Visiting nearby refs first does not fix that (a near-first order inserts MORE: every
// closer ref improves the list); a tight threshold from the start does:
//   1. the refs are counting-sorted into a 16^3 Morton-ordered cell grid over their
//      bounding box (one workgroup per cloud: LDS histogram, scan, scatter);
//   2. each query takes the kWin sorted refs around its own cell and selects the K-th
//      smallest of their distances exactly (32-step radix select on the order-preserving
//      key, one ballot popcount per step, no LDS): T >= its true K-th distance, and tight
//      because those refs are its spatial neighbours;
//   3. the unchanged index-order scan then starts with threshold "d <= T" (strict
//      d < nextafter(T)) instead of +inf: ~K candidates per query, spread over the chunks
//      so they go in one by one, and nearly every chunk is skipped by the scalar branch.
// Every ref is still scanned in index order and at least K refs satisfy d <= T, so the
// result is identical to the unseeded scan.
constexpr int kG = 16;                   // cells per axis
constexpr int kCells = kG * kG * kG;     // 4096
constexpr int kSortThreads = 1024;

__device__ __forceinline__ int spread4(int v) {  // bits b3..b0 -> b9,b6,b3,b0
  return (v & 1) | ((v & 2) << 2) | ((v & 4) << 4) | ((v & 8) << 6);
}

// bb = {min x, min y, min z, scale x, scale y, scale z}
__device__ __forceinline__ int cell_of(float x, float y, float z, const float* bb) {
  const float fx = fminf(fmaxf((x - bb[0]) * bb[3], 0.f), (float)(kG - 1));
  const float fy = fminf(fmaxf((y - bb[1]) * bb[4], 0.f), (float)(kG - 1));
  const float fz = fminf(fmaxf((z - bb[2]) * bb[5], 0.f), (float)(kG - 1));
  return spread4((int)fx) | (spread4((int)fy) << 1) | (spread4((int)fz) << 2);
}

// in-place exclusive scan of cnt[kCells] by kSortThreads threads (4 cells each)
__device__ void block_exclusive_scan(int* cnt, int* wsum) {
  const int t = threadIdx.x, lane = lane_id(), wv = t >> 6;
  int v[4], tot = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = cnt[4 * t + i];
    tot += v[i];
  }
  int inc = tot;  // inclusive wave scan
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int u = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += u;
  }
  if (lane == kWave - 1) wsum[wv] = inc;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wv; ++w) base += wsum[w];
  int run = base + inc - tot;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    cnt[4 * t + i] = run;
    run += v[i];
  }
  __syncthreads();
}

// One workgroup per cloud: bounding box, cell histogram, offsets, scatter.
// rs (B,N) float4 {x, y, z, |r|^2} in cell order, roff (B, kCells+1) first sorted position of
// each cell, bbox (B,8) = {min xyz, scale xyz}.
__global__ __launch_bounds__(kSortThreads) void ref_sort_kernel(int n,
                                                                const float* __restrict__ xyz,
                                                                float* __restrict__ bbox,
                                                                int* __restrict__ roff,
                                                                float4* __restrict__ rs) {
  __shared__ int cnt[kCells];
  __shared__ int wsum[kSortThreads / kWave];
  __shared__ float red[6][kSortThreads / kWave];
  __shared__ float bb[6];
  const int b = blockIdx.x, t = threadIdx.x, lane = lane_id(), wv = t >> 6;
  const float* p = xyz + (long long)b * n * 3;
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = t; i < n; i += kSortThreads) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = p[i * 3 + c];
      mn[c] = fminf(mn[c], v);
      mx[c] = fmaxf(mx[c], v);
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      mn[c] = fminf(mn[c], __shfl_xor(mn[c], o, kWave));
      mx[c] = fmaxf(mx[c], __shfl_xor(mx[c], o, kWave));
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      red[c][wv] = mn[c];
      red[3 + c][wv] = mx[c];
    }
  }
  for (int c = t; c < kCells; c += kSortThreads) cnt[c] = 0;
  __syncthreads();
  if (t < 3) {
    float a = INFINITY, z = -INFINITY;
    for (int w = 0; w < kSortThreads / kWave; ++w) {
      a = fminf(a, red[t][w]);
      z = fmaxf(z, red[3 + t][w]);
    }
    const float ext = z - a;
    bb[t] = a;
    bb[3 + t] = ext > 0.f ? (float)kG / ext : 0.f;
    bbox[b * 8 + t] = bb[t];
    bbox[b * 8 + 3 + t] = bb[3 + t];
  }
  __syncthreads();
  for (int i = t; i < n; i += kSortThreads)
    atomicAdd(&cnt[cell_of(p[i * 3], p[i * 3 + 1], p[i * 3 + 2], bb)], 1);
  __syncthreads();
  block_exclusive_scan(cnt, wsum);
  int* ro = roff + (long long)b * (kCells + 1);
  for (int c = t; c < kCells; c += kSortThreads) ro[c] = cnt[c];
  if (t == 0) ro[kCells] = n;
  __syncthreads();
  float4* rso = rs + (long long)b * n;
  for (int i = t; i < n; i += kSortThreads) {
    const float x = p[i * 3], y = p[i * 3 + 1], z = p[i * 3 + 2];
    const int pos = atomicAdd(&cnt[cell_of(x, y, z, bb)], 1);  // order within a cell: any
    rso[pos] = make_float4(x, y, z, sqnorm3(x, y, z));
  }
}

constexpr int kWin = 256;  // refs around a query's cell that seed its threshold

// order-preserving float -> unsigned key (total order of non-NaN floats)
__device__ __forceinline__ unsigned ord_key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float from_ord_key(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// Seed thr[q] (valid queries) with nextafter(T), T = the K-th smallest distance from the
// query to the kWin sorted refs around its cell.
template <int QW>
__device__ __forceinline__ void seed_thresholds(int n, int k, int b, int qbase, int s,
                                                const float* qx, const float* qy,
                                                const float* qz, const float* qs,
                                                const float4* __restrict__ rs,
                                                const float* __restrict__ bbox,
                                                const int* __restrict__ roff, float* thr) {
  const float4* rb = rs + (long long)b * n;
  float bb[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) bb[i] = bbox[b * 8 + i];
#pragma unroll
  for (int q = 0; q < QW; ++q) {  // one query at a time: 4 key VGPRs live, not 4 * QW
    unsigned key[kWin / kWave];
    int w0 = roff[(long long)b * (kCells + 1) + cell_of(qx[q], qy[q], qz[q], bb)] - kWin / 2;
    w0 = w0 < 0 ? w0 + n : w0;  // n >= kWin: one wrap at most
#pragma unroll
    for (int i = 0; i < kWin / kWave; ++i) {
      int pz = w0 + lane_id() + kWave * i;
      pz = pz >= n ? pz - n : pz;
      const float4 r = rb[pz];
      key[i] = ord_key(sqdist_fast(qx[q], qy[q], qz[q], qs[q], r.x, r.y, r.z, r.w));
    }
    unsigned ans = 0u;  // largest key with fewer than k window keys below it = k-th smallest
    for (int bit = 31; bit >= 0; --bit) {
      const unsigned t = ans | (1u << bit);
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < kWin / kWave; ++i) cnt += __popcll(__ballot(key[i] < t));
      ans = cnt < k ? t : ans;
    }
    // d < nextafter(T) <=> d <= T; a K-th at +inf or NaN (NaN coordinates) leaves no bound
    if (qbase + q < s && ans < ord_key(INFINITY)) thr[q] = from_ord_key(ans + 1u);
  }
}

template <int QW, bool SEED>
__global__ __launch_bounds__(256) void knn_kernel(int n, int s, int k,
                                                  const float* __restrict__ xyz,
                                                  const float* __restrict__ new_xyz,
                                                  int* __restrict__ idx,
                                                  float* __restrict__ dist,
                                                  const float4* __restrict__ rs,
                                                  const float* __restrict__ bbox,
                                                  const int* __restrict__ roff) {
  __shared__ float4 tile[kTile];
  const int b = blockIdx.y;
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int qbase = (blockIdx.x * 4 + wave) * QW;
  const float* xb = xyz + (long long)b * n * 3;

  float qx[QW], qy[QW], qz[QW], qs[QW], thr[QW], ld[QW];
  int li[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) {
    const int qi = min(qbase + q, s - 1);
    const float* qp = new_xyz + ((long long)b * s + qi) * 3;
    qx[q] = qp[0];
    qy[q] = qp[1];
    qz[q] = qp[2];
    qs[q] = sqnorm3(qx[q], qy[q], qz[q]);
    thr[q] = qbase + q < s ? INFINITY : -INFINITY;  // padding queries never take candidates
    ld[q] = INFINITY;
    li[q] = 0x7fffffff;
  }
  if constexpr (SEED) seed_thresholds<QW>(n, k, b, qbase, s, qx, qy, qz, qs, rs, bbox, roff, thr);

  for (int t0 = 0; t0 < n; t0 += kTile) {
    const int tn = min(kTile, n - t0);
    __syncthreads();
    for (int e = threadIdx.x; e < tn; e += blockDim.x) {
      const float* r = xb + (long long)(t0 + e) * 3;
      const float x = r[0], y = r[1], z = r[2];
      tile[e] = make_float4(x, y, z, sqnorm3(x, y, z));
    }
    __syncthreads();
    for (int c0 = 0; c0 < tn; c0 += kWave) {
      const int j = c0 + lane;
      const bool valid = j < tn;
      const float4 r = tile[valid ? j : 0];
      const int gi = t0 + j;
      // every query's candidate mask first, then ONE scalar branch for the common case of
      // no candidate in the chunk for any of the wave's queries
      float d[QW];
      unsigned long long m[QW];
      unsigned long long any = 0ull;
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        d[q] = sqdist_fast(qx[q], qy[q], qz[q], qs[q], r.x, r.y, r.z, r.w);
        m[q] = __ballot(valid && d[q] < thr[q]);
        any |= m[q];
      }
      if (any == 0ull) continue;
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        if (m[q] == 0ull) continue;  // wave-uniform
        insert_candidates(m[q], valid && d[q] < thr[q], d[q], gi, ld[q], li[q]);
        // seeded: the list's K-th is <= T once K entries are in, +inf before
        thr[q] = fminf(thr[q],
                       __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ld[q]), k - 1)));
      }
    }
  }

#pragma unroll
  for (int q = 0; q < QW; ++q) {
    const int qi = qbase + q;
    if (qi < s && lane < k) {
      const long long o = ((long long)b * s + qi) * k + lane;
      idx[o] = li[q];
      if (dist) dist[o] = ld[q];
    }
  }
}

struct SeedWs {
  float* bbox;
  int* roff;
  float4* rs;
  size_t bytes;
};

inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

SeedWs seed_ws(int b, int n, void* base) {
  SeedWs w{};
  char* p = reinterpret_cast<char*>(base);
  size_t o = 0;
  auto take = [&](size_t bytes) {
    char* q = p ? p + o : nullptr;
    o += align256(bytes);
    return q;
  };
  w.bbox = reinterpret_cast<float*>(take(sizeof(float) * 8 * b));
  w.roff = reinterpret_cast<int*>(take(sizeof(int) * (size_t)b * (kCells + 1)));
  w.rs = reinterpret_cast<float4*>(take(sizeof(float4) * (size_t)b * n));
  w.bytes = o;
  return w;
}

// The seed costs one sort launch (~10-20 us) and a 256-ref window per query; it pays once
// the plain scan's insertion work dominates, i.e. thousands of refs.
inline bool use_seed(int b, int n, int s) { return n >= 2048 && (long long)b * s >= 8192; }

template <bool SEED>
void launch_knn(int b, int n, int s, int k, const float* xyz, const float* new_xyz, int* idx,
                float* dist, const SeedWs& w, hipStream_t st) {
  // Large reference sets amortise the per-chunk scalar branch over 8 queries per wave; at
  // the model's sizes (N <= 8192) 4 per wave measured faster.
  if (n >= 32768)
    hipLaunchKernelGGL((knn_kernel<8, SEED>), dim3(divup(s, 32), b), dim3(256), 0, st, n, s, k,
                       xyz, new_xyz, idx, dist, w.rs, w.bbox, w.roff);
  else
    hipLaunchKernelGGL((knn_kernel<4, SEED>), dim3(divup(s, 16), b), dim3(256), 0, st, n, s, k,
                       xyz, new_xyz, idx, dist, w.rs, w.bbox, w.roff);
}

}  // namespace

// knn_point(nsample=k, xyz (B,N,3) refs, new_xyz (B,S,3) queries) -> idx (B,S,K) int32,
// optional dist (B,S,K) f32 (expanded-form squared distances).  Requires 1 <= K <= min(N,64).
// Replaces pointconv_util.py:96-107 (which returns int64 from topk).
KDPC_API int kdpc_knn_point(int b, int n, int s, int k, const float* xyz, const float* new_xyz,
                            int* idx, float* dist, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n > 0 && s >= 0 && k >= 1 && k <= 64 && k <= n && b <= 65535);
  if ((long long)b * s == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(xyz && new_xyz && idx);
  launch_knn<false>(b, n, s, k, xyz, new_xyz, idx, dist, SeedWs{}, (hipStream_t)stream);
  KDPC_RETURN_LAUNCH();
}

// Scratch bytes for kdpc_knn_point_ws; 0 when the problem is small enough that the plain
// scan is used (then pass workspace = NULL).
KDPC_API size_t kdpc_knn_workspace_bytes(int b, int n, int s) {
  if (b <= 0 || n <= 0 || s <= 0 || !use_seed(b, n, s)) return 0;
  return seed_ws(b, n, nullptr).bytes;
}

// kdpc_knn_point with scratch for the seeded threshold (identical results).
KDPC_API int kdpc_knn_point_ws(int b, int n, int s, int k, const float* xyz,
                               const float* new_xyz, int* idx, float* dist, void* workspace,
                               size_t workspace_bytes, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n > 0 && s >= 0 && k >= 1 && k <= 64 && k <= n && b <= 65535);
  if ((long long)b * s == 0) return (int)hipSuccess;
  const size_t need = kdpc_knn_workspace_bytes(b, n, s);
  if (need == 0 || workspace == nullptr)
    return kdpc_knn_point(b, n, s, k, xyz, new_xyz, idx, dist, stream);
  KDPC_CHECK_ARG(xyz && new_xyz && idx && workspace_bytes >= need);
  hipStream_t st = (hipStream_t)stream;
  const SeedWs w = seed_ws(b, n, workspace);
  hipLaunchKernelGGL(ref_sort_kernel, dim3(b), dim3(kSortThreads), 0, st, n, xyz, w.bbox, w.roff,
                     w.rs);
  launch_knn<true>(b, n, s, k, xyz, new_xyz, idx, dist, w, st);
  KDPC_RETURN_LAUNCH();
}
