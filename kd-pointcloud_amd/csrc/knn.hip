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
  // non-short-circuit: lane masks combined with s_and / s_or, no exec-mask branches
  return (ad < bd) | ((ad == bd) & (ai < bi));
}

// bitonic compare-exchange step across lanes l and l^jj
__device__ __forceinline__ void bitonic_step(float& d, int& i, int jj, bool up) {
  const float od = __shfl_xor(d, jj, kWave);
  const int oi = __shfl_xor(i, jj, kWave);
  const bool lower = (lane_id() & jj) == 0;
  const bool o_less = kv_less(od, oi, d, i);
  const bool same = (od == d) & (oi == i);
  const bool take = (lower == up) ? o_less : (!o_less & !same);
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
// ASC: candidates arrive in ascending index order, after every list entry (index-order
// scan); otherwise any order, compared by (d, index).  SERIAL: most candidates inserted
// one by one (each ~a dozen instructions; a bitonic merge is a chain of 27 cross-lane
// steps).
template <bool ASC = true, int SERIAL = kSerialMax>
__device__ __forceinline__ void insert_candidates(unsigned long long mask, bool cand, float d,
                                                  int gi, float& ld, int& li) {
  if (__popcll(mask) > SERIAL) {
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
      const bool gt = ASC ? ld > cd : kv_less(cd, ci, ld, li);
      const bool pgt = ASC ? pd > cd : kv_less(cd, ci, pd, pi);
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
                                                                float4* __restrict__ rs,
                                                                int* __restrict__ ri) {
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
    if (ri) ri[(long long)b * n + pos] = i;
  }
}

// Boxes of the sorted 64-ref chunks, one wave per chunk: cbox (B, nch, 2) =
// {lo xyz, max |r|^2}, {hi xyz, 0}.
__global__ __launch_bounds__(256) void chunk_box_kernel(int n, const float4* __restrict__ rs,
                                                        float4* __restrict__ cbox) {
  const int b = blockIdx.y, lane = lane_id();
  const int nch = divup(n, kWave);
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nch) return;
  const int j = c * kWave + lane;
  const float4 r = rs[(long long)b * n + (j < n ? j : c * kWave)];
  float lo[4] = {r.x, r.y, r.z, -r.w}, hi[3] = {r.x, r.y, r.z};
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
#pragma unroll
    for (int a = 0; a < 4; ++a) lo[a] = fminf(lo[a], __shfl_xor(lo[a], o, kWave));
#pragma unroll
    for (int a = 0; a < 3; ++a) hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], o, kWave));
  }
  if (lane == 0) {
    float4* cb = cbox + ((long long)b * nch + c) * 2;
    cb[0] = make_float4(lo[0], lo[1], lo[2], -lo[3]);
    cb[1] = make_float4(hi[0], hi[1], hi[2], 0.f);
  }
}

constexpr int kWin = 256;  // refs around a query's cell that seed its threshold

// Queries of each cloud in the refs' cell order (so a wave's queries are spatial
// neighbours): qrec (B,S) = {x, y, z, original index} and qwin (B,S) = first of the kWin
// sorted refs around the query's cell, at each sorted position.  One dependent load per
// query in the kNN kernel instead of index -> coordinates -> cell offset.
__global__ __launch_bounds__(kSortThreads) void query_sort_kernel(int s, int n,
                                                                  const float* __restrict__ new_xyz,
                                                                  const float* __restrict__ bbox,
                                                                  const int* __restrict__ roff,
                                                                  float4* __restrict__ qrec,
                                                                  int* __restrict__ qwin) {
  __shared__ int cnt[kCells];
  __shared__ int wsum[kSortThreads / kWave];
  __shared__ float bb[6];
  const int b = blockIdx.x, t = threadIdx.x;
  const float* p = new_xyz + (long long)b * s * 3;
  if (t < 6) bb[t] = bbox[b * 8 + t];
  for (int c = t; c < kCells; c += kSortThreads) cnt[c] = 0;
  __syncthreads();
  for (int i = t; i < s; i += kSortThreads)
    atomicAdd(&cnt[cell_of(p[i * 3], p[i * 3 + 1], p[i * 3 + 2], bb)], 1);
  __syncthreads();
  block_exclusive_scan(cnt, wsum);
  const int* ro = roff + (long long)b * (kCells + 1);
  for (int i = t; i < s; i += kSortThreads) {
    const float x = p[i * 3], y = p[i * 3 + 1], z = p[i * 3 + 2];
    const int cell = cell_of(x, y, z, bb);
    const int pos = atomicAdd(&cnt[cell], 1);
    int w0 = ro[cell] - kWin / 2;
    w0 = w0 < 0 ? w0 + n : w0;  // n >= kWin: one wrap at most
    qrec[(long long)b * s + pos] = make_float4(x, y, z, __int_as_float(i));
    qwin[(long long)b * s + pos] = w0;
  }
}


// order-preserving float -> unsigned key (total order of non-NaN floats)
__device__ __forceinline__ unsigned ord_key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float from_ord_key(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// Seed thr[q] (valid queries) with nextafter(T): T >= the K-th smallest distance from the
// query to the kWin sorted refs around its cell.  The radix select fixes the top 16 bits of
// that K-th key (sign, exponent, 7 mantissa bits) and T sets the 16 low bits, so T is within
// 2^-7 of the K-th, an upper bound of it and of the query's true K-th distance.  The QW
// selects run interleaved (independent chains of ballot / popcount / select).
template <int QW>
__device__ __forceinline__ void seed_thresholds(int n, int k, int b, int qbase, int s,
                                                const float* qx, const float* qy,
                                                const float* qz, const float* qs,
                                                const int* w0, const float4* __restrict__ rs,
                                                float* thr) {
  const float4* rb = rs + (long long)b * n;
  unsigned key[QW][kWin / kWave];
#pragma unroll
  for (int q = 0; q < QW; ++q) {
#pragma unroll
    for (int i = 0; i < kWin / kWave; ++i) {
      int pz = w0[q] + lane_id() + kWave * i;
      pz = pz >= n ? pz - n : pz;
      const float4 r = rb[pz];
      key[q][i] = ord_key(sqdist_fast(qx[q], qy[q], qz[q], qs[q], r.x, r.y, r.z, r.w));
    }
  }
  unsigned ans[QW];  // largest prefix with fewer than k window keys below it
#pragma unroll
  for (int q = 0; q < QW; ++q) ans[q] = 0u;
  for (int bit = 31; bit >= 16; --bit) {
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const unsigned t = ans[q] | (1u << bit);
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < kWin / kWave; ++i) cnt += __popcll(__ballot(key[q][i] < t));
      ans[q] = cnt < k ? t : ans[q];
    }
  }
#pragma unroll
  for (int q = 0; q < QW; ++q) {
    const unsigned tk = ans[q] | 0xffffu;  // >= the window's K-th key
    // d < nextafter(T) <=> d <= T; a bound at +inf or NaN (NaN coordinates) is no bound
    if (qbase + q < s && tk < ord_key(INFINITY)) thr[q] = from_ord_key(tk + 1u);
  }
}

// A query's K results (lane r holds rank r) written at row offset o: for K % 4 == 0 (every
// K of the models) lane t < K/4 collects ranks 4t..4t+3 by shuffles and writes them as one
// 16-byte store, so a row is K/4 full-width stores instead of K 4-byte ones.
__device__ __forceinline__ void store_row(int* __restrict__ idx, float* __restrict__ dist,
                                          long long o, int k, int li, float ld) {
  const int lane = lane_id();
  const bool aligned = ((reinterpret_cast<unsigned long long>(idx) |
                         reinterpret_cast<unsigned long long>(dist)) & 15ull) == 0ull;
  if ((k & 3) == 0 && aligned) {
    int iv[4];
    float dv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      iv[e] = __shfl(li, 4 * (lane & 15) + e, kWave);
      dv[e] = __shfl(ld, 4 * (lane & 15) + e, kWave);
    }
    if (lane < (k >> 2)) {
      *reinterpret_cast<int4*>(idx + o + 4 * lane) = make_int4(iv[0], iv[1], iv[2], iv[3]);
      if (dist)
        *reinterpret_cast<float4*>(dist + o + 4 * lane) = make_float4(dv[0], dv[1], dv[2], dv[3]);
    }
  } else if (lane < k) {
    idx[o + lane] = li;
    if (dist) dist[o + lane] = ld;
  }
}

template <int QW>
__global__ __launch_bounds__(256) void knn_kernel(int n, int s, int k,
                                                  const float* __restrict__ xyz,
                                                  const float* __restrict__ new_xyz,
                                                  int* __restrict__ idx,
                                                  float* __restrict__ dist) {
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
        thr[q] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ld[q]), k - 1));
      }
    }
  }

#pragma unroll
  for (int q = 0; q < QW; ++q)
    if (qbase + q < s) store_row(idx, dist, ((long long)b * s + qbase + q) * k, k, li[q], ld[q]);
}

constexpr int kBuf = 128;  // candidate slots per query (LDS)

// Sort QW wave-wide lists (lane l holds entry l of each) ascending by (d, index); the QW
// bitonic networks run interleaved.
template <int QW>
__device__ __forceinline__ void sort64_multi(float (&d)[QW], int (&i)[QW]) {
#pragma unroll
  for (int kk = 2; kk <= 64; kk <<= 1) {
    const bool up = (lane_id() & kk) == 0 || kk == 64;
#pragma unroll
    for (int jj = kk >> 1; jj > 0; jj >>= 1) {
#pragma unroll
      for (int q = 0; q < QW; ++q) bitonic_step(d[q], i[q], jj, up);
    }
  }
}

// Reduce a query's candidate buffer (cnt > 64 entries) to its 64 smallest, sorted, in
// slots 0..63; tighten thr to the K-th of them.  (This and shrink_buffer are inlined: as
// called functions (__noinline__ until round 6) their by-reference cnt / thr lived in
// scratch and every call saved registers there -- 48 B per lane; inlined the kernel needs
// no scratch and configs[4] runs 1222 -> 838 us.)
__device__ __forceinline__ void compact_buffer(float2* buf, int& cnt, float& thr, int k) {
  const int lane = lane_id();
  const float2 a = lane < cnt ? buf[lane] : make_float2(INFINITY, __int_as_float(0x7fffffff));
  const float2 c = lane + kWave < cnt ? buf[kWave + lane]
                                      : make_float2(INFINITY, __int_as_float(0x7fffffff));
  float ad = a.x, cd = c.x;
  int ai = __float_as_int(a.y), ci = __float_as_int(c.y);
  bitonic_sort64(ad, ai);
  bitonic_sort64(cd, ci);
  const float rd = __shfl(cd, 63 - lane, kWave);
  const int ri = __shfl(ci, 63 - lane, kWave);
  if (kv_less(rd, ri, ad, ai)) {
    ad = rd;
    ai = ri;
  }
  bitonic_merge64(ad, ai);
  wave_lds_sync();
  buf[lane] = make_float2(ad, __int_as_float(ai));
  wave_lds_sync();
  cnt = kWave;
  const float kth = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ad), k - 1));
  if (kth < INFINITY) thr = fminf(thr, from_ord_key(ord_key(kth) + 1u));
}

// Box-culled scan over the cell-sorted refs.  With the seeded threshold (d <= T, T an upper
// bound of the query's true K-th distance, tight), a 64-ref chunk whose bounding box lies
// farther than T from every query of the wave cannot hold a candidate and is skipped
// without computing its distances.  A wave's queries are spatial neighbours (queries in
// cell order), so a wave visits the few chunks around them: the scan is sub-linear in N.
// Culling is exact: a chunk is skipped only if its box bound exceeds the threshold by more
// than the rounding error of the expanded-form distance (|d - D| <= 12 eps (|q|^2+|r|^2)
// for the fma chain; the margin allows 32 eps plus 16 eps |thr| for the bound's own
// rounding).  Because T is tight, a query collects only ~K..1.5K candidates: they are
// appended to an LDS buffer (no list maintenance during the scan) and sorted once by
// (d, index) at the end; a buffer that would overflow is first compacted to its 64
// smallest (K <= 64), which also tightens the threshold.
// Keep only the buffer entries whose key is <= T, an upper bound of the K-th smallest
// among them (16-bit radix select over the <= 128 entries, two per lane: ballot popcounts,
// no cross-lane data movement), compacted in place; tighten thr to d <= T.  Everything
// dropped is farther than K buffered candidates, so it is not among the K nearest.
__device__ __forceinline__ void shrink_buffer(float2* buf, int& cnt, float& thr, int k) {
  const int lane = lane_id();
  const bool v0 = lane < cnt, v1 = lane + kWave < cnt;
  const float2 e0 = v0 ? buf[lane] : make_float2(INFINITY, 0.f);
  const float2 e1 = v1 ? buf[kWave + lane] : make_float2(INFINITY, 0.f);
  const unsigned k0 = v0 ? ord_key(e0.x) : 0xffffffffu;
  const unsigned k1 = v1 ? ord_key(e1.x) : 0xffffffffu;
  unsigned ans = 0u;
  for (int bit = 31; bit >= 16; --bit) {
    const unsigned t = ans | (1u << bit);
    const int c = __popcll(__ballot(k0 < t)) + __popcll(__ballot(k1 < t));
    ans = c < k ? t : ans;
  }
  const unsigned tk = ans | 0xffffu;
  const unsigned long long m0 = __ballot(v0 && k0 <= tk), m1 = __ballot(v1 && k1 <= tk);
  const int p0 = __builtin_amdgcn_mbcnt_hi((unsigned)(m0 >> 32),
                                           __builtin_amdgcn_mbcnt_lo((unsigned)m0, 0u));
  const int p1 = __popcll(m0) + __builtin_amdgcn_mbcnt_hi((unsigned)(m1 >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((unsigned)m1, 0u));
  wave_lds_sync();
  if (v0 && k0 <= tk) buf[p0] = e0;
  if (v1 && k1 <= tk) buf[p1] = e1;
  wave_lds_sync();
  cnt = __popcll(m0) + __popcll(m1);
  if (tk < ord_key(INFINITY)) thr = fminf(thr, from_ord_key(tk + 1u));
}

// STATS: also count the distance evaluations the wave issues (visited 64-ref chunks x 64
// lanes x QW queries, plus the kWin-ref seed window per query) into *evals -- the work the
// culled scan really performs, for the roofline (kdpc_knn_point_evals; never on the
// product path).
//
// (Measured and rejected, round 4: an XCD-aware block order giving each XCD one contiguous
// run of cell-sorted query blocks -- configs[4] 1270 -> 1527 us: contiguous regions carry
// unequal work (point density varies), while the default round-robin deal gives every XCD a
// uniform sample of the cloud.)
template <int QW, bool STATS>
__global__ __launch_bounds__(256) void knn_cull_kernel(
    int n, int s, int k, int* __restrict__ idx, float* __restrict__ dist,
    const float4* __restrict__ rs, const int* __restrict__ ri, const float4* __restrict__ cbox,
    const float4* __restrict__ qrec, const int* __restrict__ qwin,
    unsigned long long* __restrict__ evals) {
  __shared__ float2 cand_buf[4][QW][kBuf];
  const int b = blockIdx.y, bx = blockIdx.x;
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int qbase = (bx * 4 + wave) * QW;  // sorted query positions
  unsigned visits = 0;
  const int nch = divup(n, kWave);
  const float4* rb = rs + (long long)b * n;
  const int* ib = ri + (long long)b * n;
  const float4* cb = cbox + (long long)b * nch * 2;

  float qx[QW], qy[QW], qz[QW], qs[QW], thr[QW];
  int qid[QW], cnt[QW], w0[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) {
    const long long pos = (long long)b * s + min(qbase + q, s - 1);
    const float4 r = qrec[pos];
    w0[q] = qwin[pos];
    qx[q] = r.x;
    qy[q] = r.y;
    qz[q] = r.z;
    qid[q] = __float_as_int(r.w);
    qs[q] = sqnorm3(qx[q], qy[q], qz[q]);
    thr[q] = qbase + q < s ? INFINITY : -INFINITY;  // padding queries never take candidates
    cnt[q] = 0;
  }
  // the first block of chunk boxes is independent of the seed: in flight during it
  float4 lo = lane < nch ? cb[2 * lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 hi = lane < nch ? cb[2 * lane + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
  seed_thresholds<QW>(n, k, b, qbase, s, qx, qy, qz, qs, w0, rs, thr);

  // visit every chunk of `todo` (chunk cbase + bit), the next chunk's refs loaded while
  // this one is used; candidates (d < thr) are appended to the query's buffer
  auto run = [&](unsigned long long todo, int cbase) {
    if (todo == 0ull) return;
    int cc = cbase + __ffsll((long long)todo) - 1;
    todo &= todo - 1;
    int j = cc * kWave + lane;
    float4 r = rb[j < n ? j : cc * kWave];
    int gi = ib[j < n ? j : cc * kWave];
    while (true) {
      if (STATS) ++visits;
      const bool valid = j < n;
      const bool more = todo != 0ull;
      const int cn = more ? cbase + __ffsll((long long)todo) - 1 : cc;
      todo &= todo - 1;
      const int jn = cn * kWave + lane;
      const float4 rn = rb[jn < n ? jn : cn * kWave];
      const int gn = ib[jn < n ? jn : cn * kWave];
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        const float d = sqdist_fast(qx[q], qy[q], qz[q], qs[q], r.x, r.y, r.z, r.w);
        bool cand = valid && d < thr[q];
        unsigned long long m = __ballot(cand);
        if (m == 0ull) continue;  // wave-uniform
        if (cnt[q] + __popcll(m) > kBuf) {
          shrink_buffer(cand_buf[wave][q], cnt[q], thr[q], k);
          if (cnt[q] + __popcll(m) > kBuf)  // exact ties keep > 64: sort-based fallback
            compact_buffer(cand_buf[wave][q], cnt[q], thr[q], k);
          cand = cand && d < thr[q];
          m = __ballot(cand);
        }
        const int pos = cnt[q] + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        if (cand) cand_buf[wave][q][pos] = make_float2(d, __int_as_float(gi));
        cnt[q] += __popcll(m);
      }
      if (!more) break;
      cc = cn;
      j = jn;
      r = rn;
      gi = gn;
    }
  };
  // per 64-chunk block: the chunks whose box contains a query first, then a tightened
  // threshold from what they gave, then the remaining chunks re-tested against it
  for (int cbase = 0; cbase < nch; cbase += kWave) {
    const int c = cbase + lane;
    if (cbase > 0 && c < nch) {
      lo = cb[2 * c];
      hi = cb[2 * c + 1];
    }
    float lbq[QW];
    bool need = false, inside = false;
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const float dx = fmaxf(fmaxf(lo.x - qx[q], qx[q] - hi.x), 0.f);
      const float dy = fmaxf(fmaxf(lo.y - qy[q], qy[q] - hi.y), 0.f);
      const float dz = fmaxf(fmaxf(lo.z - qz[q], qz[q] - hi.z), 0.f);
      lbq[q] = dx * dx + dy * dy + dz * dz;
      const float marg = (qs[q] + lo.w) * 0x1p-19f + fabsf(thr[q]) * 0x1p-20f;
      const bool ok = c < nch && qbase + q < s;
      need |= ok && !(lbq[q] > thr[q] + marg);
      inside |= ok && lbq[q] == 0.f;
    }
    const unsigned long long near_m = __ballot(inside && need);
    const unsigned long long need_m = __ballot(need);
    if (need_m == 0ull) continue;
    run(near_m, cbase);
    if (need_m == near_m) continue;
#pragma unroll
    for (int q = 0; q < QW; ++q)
      if (near_m != 0ull && cnt[q] >= k) shrink_buffer(cand_buf[wave][q], cnt[q], thr[q], k);
    bool need2 = false;
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const float marg = (qs[q] + lo.w) * 0x1p-19f + fabsf(thr[q]) * 0x1p-20f;
      need2 |= c < nch && qbase + q < s && !(lbq[q] > thr[q] + marg);
    }
    run(__ballot(need2) & need_m & ~near_m, cbase);
  }

  if (STATS && lane == 0) {
    int live = 0;
#pragma unroll
    for (int q = 0; q < QW; ++q) live += qbase + q < s ? 1 : 0;
    if (live > 0)
      atomicAdd(evals, (unsigned long long)visits * kWave * QW + (unsigned long long)kWin * live);
  }
  wave_lds_sync();
#pragma unroll
  for (int q = 0; q < QW; ++q) {
    if (cnt[q] > kWave) shrink_buffer(cand_buf[wave][q], cnt[q], thr[q], k);
    if (cnt[q] > kWave) compact_buffer(cand_buf[wave][q], cnt[q], thr[q], k);
  }
  float ld[QW];
  int li[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) {
    const float2 v = lane < cnt[q] ? cand_buf[wave][q][lane]
                                   : make_float2(INFINITY, __int_as_float(0x7fffffff));
    ld[q] = v.x;
    li[q] = __float_as_int(v.y);
  }
  sort64_multi<QW>(ld, li);
#pragma unroll
  for (int q = 0; q < QW; ++q)
    if (qbase + q < s) store_row(idx, dist, ((long long)b * s + qid[q]) * k, k, li[q], ld[q]);
}

struct SeedWs {
  float* bbox;
  int* roff;
  float4* rs;
  int* ri;
  float4* cbox;
  float4* qrec;
  int* qwin;
  size_t bytes;
};

inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

SeedWs seed_ws(int b, int n, int s, void* base) {
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
  w.ri = reinterpret_cast<int*>(take(sizeof(int) * (size_t)b * n));
  w.cbox = reinterpret_cast<float4*>(take(sizeof(float4) * 2 * (size_t)b * divup(n, kWave)));
  w.qrec = reinterpret_cast<float4*>(take(sizeof(float4) * (size_t)b * s));
  w.qwin = reinterpret_cast<int*>(take(sizeof(int) * (size_t)b * s));
  w.bytes = o;
  return w;
}

// The seed costs one sort launch (~10-20 us) and a 256-ref window per query; it pays once
// the plain scan's insertion work dominates, i.e. thousands of refs.
#ifndef KNN_QW
#define KNN_QW 4
#endif
// smallest reference set the culled scan is used for (round 2, whole-step A/B: 1024 beats
// 2048 by 0.5 %, 512 loses -- below that the sort / box setup launches outweigh the culling)
#ifndef KDPC_KNN_CULL_MIN_N
#define KDPC_KNN_CULL_MIN_N 1024
#endif
inline bool use_seed(int b, int n, int s) {
  return n >= KDPC_KNN_CULL_MIN_N && (long long)b * s >= 8192;
}

void launch_knn(int b, int n, int s, int k, const float* xyz, const float* new_xyz, int* idx,
                float* dist, hipStream_t st) {
  // Large reference sets amortise the per-chunk scalar branch over 8 queries per wave; at
  // the model's sizes (N <= 8192) 4 per wave measured faster.
  if (n >= 32768)
    hipLaunchKernelGGL(knn_kernel<8>, dim3(divup(s, 32), b), dim3(256), 0, st, n, s, k, xyz,
                       new_xyz, idx, dist);
  else
    hipLaunchKernelGGL(knn_kernel<4>, dim3(divup(s, 16), b), dim3(256), 0, st, n, s, k, xyz,
                       new_xyz, idx, dist);
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
  launch_knn(b, n, s, k, xyz, new_xyz, idx, dist, (hipStream_t)stream);
  KDPC_RETURN_LAUNCH();
}

// Scratch bytes for kdpc_knn_point_ws; 0 when the problem is small enough that the plain
// scan is used (then pass workspace = NULL).
KDPC_API size_t kdpc_knn_workspace_bytes(int b, int n, int s) {
  if (b <= 0 || n <= 0 || s <= 0 || !use_seed(b, n, s)) return 0;
  return seed_ws(b, n, s, nullptr).bytes;
}

namespace {
int knn_culled(int b, int n, int s, int k, const float* xyz, const float* new_xyz, int* idx,
               float* dist, void* workspace, unsigned long long* evals, hipStream_t st) {
  const SeedWs w = seed_ws(b, n, s, workspace);
  hipLaunchKernelGGL(ref_sort_kernel, dim3(b), dim3(kSortThreads), 0, st, n, xyz, w.bbox, w.roff,
                     w.rs, w.ri);
  hipLaunchKernelGGL(chunk_box_kernel, dim3(divup(divup(n, kWave), 4), b), dim3(256), 0, st, n,
                     w.rs, w.cbox);
  hipLaunchKernelGGL(query_sort_kernel, dim3(b), dim3(kSortThreads), 0, st, s, n, new_xyz,
                     w.bbox, w.roff, w.qrec, w.qwin);
  static_assert(KNN_QW == 4 || KNN_QW == 8, "KNN_QW");
  constexpr int QW = KNN_QW;
  const dim3 grid(divup(s, 4 * QW), b);
  if (evals)
    hipLaunchKernelGGL((knn_cull_kernel<QW, true>), grid, dim3(256), 0, st, n, s, k, idx, dist,
                       w.rs, w.ri, w.cbox, w.qrec, w.qwin, evals);
  else
    hipLaunchKernelGGL((knn_cull_kernel<QW, false>), grid, dim3(256), 0, st, n, s, k, idx, dist,
                       w.rs, w.ri, w.cbox, w.qrec, w.qwin, evals);
  KDPC_RETURN_LAUNCH();
}
}  // namespace

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
  return knn_culled(b, n, s, k, xyz, new_xyz, idx, dist, workspace, nullptr,
                    (hipStream_t)stream);
}

// kdpc_knn_point_ws (culled scan only) that also adds the number of distance evaluations it
// issues to *evals (a device u64): the roofline's work count.  Same results.
KDPC_API int kdpc_knn_point_evals(int b, int n, int s, int k, const float* xyz,
                                  const float* new_xyz, int* idx, void* workspace,
                                  size_t workspace_bytes, unsigned long long* evals,
                                  void* stream) {
  KDPC_CHECK_ARG(b >= 1 && n > 0 && s >= 1 && k >= 1 && k <= 64 && k <= n && b <= 65535);
  const size_t need = kdpc_knn_workspace_bytes(b, n, s);
  KDPC_CHECK_ARG(need > 0 && xyz && new_xyz && idx && evals && workspace &&
                 workspace_bytes >= need);
  return knn_culled(b, n, s, k, xyz, new_xyz, idx, nullptr, workspace, evals,
                    (hipStream_t)stream);
}
