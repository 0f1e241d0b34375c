// Furthest point sampling for gfx950.
//
// Semantics (bit-exact with the reference, pointnet2/src/sampling_gpu.cu:93-209):
//   T = opt_n_threads(N) (cuda_utils.h:10-14).  Reference thread t scans k = t, t+T, ...
//   keeping the first k with the strictly greatest d2 = min(dist(k, old), temp[k]); the
//   shared-memory tree (__update, :86-91) then keeps the lower slot unless the upper one is
//   strictly greater.  Net effect: argmax d2, ties resolved by the smallest bit-reversed
//   thread id (log2 T bits), then by the smallest k inside that thread.
//
// MI355X design:
//   * one workgroup per cloud, the reference's point->thread mapping (so the in-thread
//     tie rule is literally the same); a thread keeps its <= PPT points' xyz and running
//     min-distance in VGPRs for all M steps (no temp[] round trip per step);
//   * the cloud's xyz is staged once in LDS so the winner's coordinates are an LDS
//     broadcast read, not a dependent global load;
//   * per step: a DPP/readlane 32-bit max over the wave (tie -> bit-reversed-tid rule only
//     on the rare exact tie), one u64 {d2 bits, tie-key|k} per wave into a
//     double-buffered LDS slot, ONE barrier, then every wave reduces the <=16 slots
//     itself.  (The reference's read of dists_i[0] without a trailing barrier, :205 vs
//     :139-140, is a latent race; the double buffer removes it.)
#include "kdpc_common.h"

using namespace kdpc;

namespace {

constexpr int kMaxSlots = 16;  // 1024 threads / 64

// max over the wave of a u32, every lane gets it.  DPP within each 16-lane row, then
// readlane of the four row results.
__device__ __forceinline__ unsigned wave_max_dpp(unsigned v) {
  unsigned w;
  w = __builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  v = w > v ? w : v;
  w = __builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
  v = w > v ? w : v;
  w = __builtin_amdgcn_mov_dpp((int)v, 0x141, 0xf, 0xf, false);  // row_half_mirror
  v = w > v ? w : v;
  w = __builtin_amdgcn_mov_dpp((int)v, 0x140, 0xf, 0xf, false);  // row_mirror
  v = w > v ? w : v;
  unsigned r0 = __builtin_amdgcn_readlane((int)v, 0);
  unsigned r1 = __builtin_amdgcn_readlane((int)v, 16);
  unsigned r2 = __builtin_amdgcn_readlane((int)v, 32);
  unsigned r3 = __builtin_amdgcn_readlane((int)v, 48);
  r0 = r0 > r1 ? r0 : r1;
  r2 = r2 > r3 ? r2 : r3;
  return r0 > r2 ? r0 : r2;
}

// Resolve a wave's candidates {hi = d2 bits, lo = tie-key|k}: the max hi, then the max lo
// among lanes holding that hi (lo encodes the preferred thread in its top bits).
__device__ __forceinline__ unsigned long long wave_argmax_key(unsigned hi, unsigned lo) {
  const unsigned vmax = wave_max_dpp(hi);
  const unsigned long long mask = __ballot(hi == vmax);
  unsigned lbest;
  if (__popcll(mask) == 1) {
    lbest = __builtin_amdgcn_readlane((int)lo, __ffsll((long long)mask) - 1);
  } else {
    lbest = wave_max_dpp(hi == vmax ? lo : 0u);
  }
  return ((unsigned long long)vmax << 32) | lbest;
}

// FULL: every thread owns exactly PPT points (N = T * PPT, T = BLOCK; the model's 8192 ->
// 2048 case): no ownership selects.  Scalar f32 only (kdpc_common.h: no packed f32).
template <int BLOCK, int PPT, bool LDS_XYZ, bool FULL>
__global__ __launch_bounds__(BLOCK) void fps_kernel(int n, int m, int T, int log2T,
                                                    const float* __restrict__ xyz,
                                                    float* __restrict__ temp,
                                                    int* __restrict__ idx) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  unsigned long long* slots = reinterpret_cast<unsigned long long*>(smem);  // [2][16]
  float* sxyz = reinterpret_cast<float*>(smem + 2 * kMaxSlots * sizeof(unsigned long long));

  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int nwaves = BLOCK / kWave;
  const float* ds = xyz + (size_t)b * n * 3;
  float* tp = temp + (size_t)b * n;
  int* ix = idx + (size_t)b * m;

  if (LDS_XYZ) {
    for (int e = tid; e < n * 3; e += BLOCK) sxyz[e] = ds[e];
  }

  // this thread's points (reference mapping: k = tid + p*T), only tid < T own points
  float px[PPT], py[PPT], pz[PPT], pt[PPT];
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    const int k = tid + p * T;
    const bool ok = tid < T && k < n;
    px[p] = ok ? ds[k * 3 + 0] : 0.f;
    py[p] = ok ? ds[k * 3 + 1] : 0.f;
    pz[p] = ok ? ds[k * 3 + 2] : 0.f;
    pt[p] = ok ? tp[k] : 0.f;
  }
  // tie key: the preferred thread has the smallest bit-reversed id -> largest (T-1-rt)
  const unsigned rt = log2T == 0 ? 0u : (__brev((unsigned)tid) >> (32 - log2T));
  const unsigned tiekey = tid < T ? ((unsigned)(T - 1) - rt) << 22 : 0u;

  if (tid == 0 && m > 0) ix[0] = 0;
  __syncthreads();
  float x1, y1, z1;
  if (LDS_XYZ) {
    x1 = sxyz[0]; y1 = sxyz[1]; z1 = sxyz[2];
  } else {
    x1 = ds[0]; y1 = ds[1]; z1 = ds[2];
  }

  for (int j = 1; j < m; ++j) {
    float best = -1.f;
    int bestk = 0;
    if constexpr (FULL) {
#pragma unroll
      for (int p = 0; p < PPT; ++p) {  // points in the reference's scan order
        const float d2 = fminf(dist3(x1, y1, z1, px[p], py[p], pz[p]), pt[p]);
        pt[p] = d2;
        const bool better = d2 > best;
        bestk = better ? tid + p * T : bestk;
        best = better ? d2 : best;
      }
    } else {
#pragma unroll
      for (int p = 0; p < PPT; ++p) {
        const float d = dist3(x1, y1, z1, px[p], py[p], pz[p]);
        const float d2 = fminf(d, pt[p]);
        const bool own = tid < T && tid + p * T < n;
        pt[p] = own ? d2 : pt[p];
        const bool better = own && d2 > best;
        bestk = better ? tid + p * T : bestk;
        best = better ? d2 : best;
      }
    }
    const unsigned hi = best >= 0.f ? __float_as_uint(best) : 0u;
    const unsigned lo = best >= 0.f ? (tiekey | (unsigned)bestk) : 0u;
    const unsigned long long wkey = wave_argmax_key(hi, lo);
    unsigned long long* sl = slots + (j & 1) * kMaxSlots;
    if (lane_id() == 0) sl[wave] = wkey;
    __syncthreads();
    const unsigned long long c = lane_id() < nwaves ? sl[lane_id()] : 0ull;
    const unsigned long long gkey = wave_argmax_key((unsigned)(c >> 32), (unsigned)c);
    const int old = (int)(gkey & 0x3FFFFFu);
    if (tid == 0) ix[j] = old;
    if (LDS_XYZ) {
      x1 = sxyz[old * 3 + 0]; y1 = sxyz[old * 3 + 1]; z1 = sxyz[old * 3 + 2];
    } else {
      x1 = ds[old * 3 + 0]; y1 = ds[old * 3 + 1]; z1 = ds[old * 3 + 2];
    }
  }
  // write back the running min distances (the reference leaves them in temp)
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    const int k = tid + p * T;
    if (tid < T && k < n) tp[k] = pt[p];
  }
}

// Fallback for N > 32768: points and temp streamed from global memory every step
// (the reference's own structure), same reductions.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void fps_kernel_global(int n, int m, int T, int log2T,
                                                           const float* __restrict__ xyz,
                                                           float* __restrict__ temp,
                                                           int* __restrict__ idx) {
  __shared__ unsigned long long slots[2 * kMaxSlots];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int nwaves = BLOCK / kWave;
  const float* ds = xyz + (size_t)b * n * 3;
  float* tp = temp + (size_t)b * n;
  int* ix = idx + (size_t)b * m;
  const unsigned rt = log2T == 0 ? 0u : (__brev((unsigned)tid) >> (32 - log2T));
  const unsigned tiekey = tid < T ? ((unsigned)(T - 1) - rt) << 22 : 0u;
  if (tid == 0 && m > 0) ix[0] = 0;
  float x1 = ds[0], y1 = ds[1], z1 = ds[2];
  for (int j = 1; j < m; ++j) {
    float best = -1.f;
    int bestk = 0;
    if (tid < T) {
      for (int k = tid; k < n; k += T) {
        const float d = dist3(x1, y1, z1, ds[k * 3 + 0], ds[k * 3 + 1], ds[k * 3 + 2]);
        const float d2 = fminf(d, tp[k]);
        tp[k] = d2;
        bestk = d2 > best ? k : bestk;
        best = d2 > best ? d2 : best;
      }
    }
    const unsigned hi = best >= 0.f ? __float_as_uint(best) : 0u;
    const unsigned lo = best >= 0.f ? (tiekey | (unsigned)bestk) : 0u;
    const unsigned long long wkey = wave_argmax_key(hi, lo);
    unsigned long long* sl = slots + (j & 1) * kMaxSlots;
    if (lane_id() == 0) sl[wave] = wkey;
    __syncthreads();
    const unsigned long long c = lane_id() < nwaves ? sl[lane_id()] : 0ull;
    const unsigned long long gkey = wave_argmax_key((unsigned)(c >> 32), (unsigned)c);
    const int old = (int)(gkey & 0x3FFFFFu);
    if (tid == 0) ix[j] = old;
    x1 = ds[old * 3 + 0]; y1 = ds[old * 3 + 1]; z1 = ds[old * 3 + 2];
  }
}

int host_opt_n_threads(int work_size) {
  int pow_2 = 0;
  // reference: (int)(log(n)/log(2.0)); computed exactly for powers of two as well
  double l = __builtin_log((double)work_size) / __builtin_log(2.0);
  pow_2 = (int)l;
  int v = 1 << pow_2;
  if (v > 1024) v = 1024;
  if (v < 1) v = 1;
  return v;
}

template <int BLOCK, int PPT>
hipError_t launch_reg(int b, int n, int m, int T, int log2T, const float* xyz, float* temp,
                      int* idx, hipStream_t st) {
  const size_t slot_bytes = 2 * kMaxSlots * sizeof(unsigned long long);
  const size_t lds = slot_bytes + (size_t)n * 3 * sizeof(float);
  const bool full = PPT % 2 == 0 && T == BLOCK && n == T * PPT;
  if (lds <= 160 * 1024) {
    // once per process and instantiation (thread-safe static initialisation)
    static const hipError_t attr = [] {
      hipError_t e = hipFuncSetAttribute((const void*)fps_kernel<BLOCK, PPT, true, false>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      if (e == hipSuccess && PPT % 2 == 0)
        e = hipFuncSetAttribute((const void*)fps_kernel<BLOCK, PPT, true, PPT % 2 == 0>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      return e;
    }();
    if (attr != hipSuccess) return attr;
    if (full)
      hipLaunchKernelGGL((fps_kernel<BLOCK, PPT, true, PPT % 2 == 0>), dim3(b), dim3(BLOCK), lds,
                         st, n, m, T, log2T, xyz, temp, idx);
    else
      hipLaunchKernelGGL((fps_kernel<BLOCK, PPT, true, false>), dim3(b), dim3(BLOCK), lds, st, n,
                         m, T, log2T, xyz, temp, idx);
  } else {
    hipLaunchKernelGGL((fps_kernel<BLOCK, PPT, false, false>), dim3(b), dim3(BLOCK), slot_bytes,
                       st, n, m, T, log2T, xyz, temp, idx);
  }
  return hipGetLastError();
}

template <int BLOCK>
hipError_t launch_block(int b, int n, int m, int T, int log2T, const float* xyz, float* temp,
                        int* idx, hipStream_t st) {
  // T < 1024 implies N < 2T, so only the 1024-thread block holds more than 2 points/thread;
  // beyond 16 points/thread (N > 16384) the register file is exhausted: stream instead.
  const int ppt = divup(n, T);
  if (ppt <= 1) return launch_reg<BLOCK, 1>(b, n, m, T, log2T, xyz, temp, idx, st);
  if (ppt <= 2) return launch_reg<BLOCK, 2>(b, n, m, T, log2T, xyz, temp, idx, st);
  if constexpr (BLOCK == 1024) {
    if (ppt <= 4) return launch_reg<BLOCK, 4>(b, n, m, T, log2T, xyz, temp, idx, st);
    if (ppt <= 8) return launch_reg<BLOCK, 8>(b, n, m, T, log2T, xyz, temp, idx, st);
    if (ppt <= 16) return launch_reg<BLOCK, 16>(b, n, m, T, log2T, xyz, temp, idx, st);
  }
  hipLaunchKernelGGL((fps_kernel_global<BLOCK>), dim3(b), dim3(BLOCK), 0, st, n, m, T, log2T,
                     xyz, temp, idx);
  return hipGetLastError();
}

}  // namespace

// Reference: furthest_point_sampling_wrapper(b, n, m, points, temp, idx)
// (sampling.cpp:38-49).  points (B,N,3) f32, temp (B,N) f32 pre-filled by the caller
// (reference: 1e10), idx (B,M) i32 output.
KDPC_API int kdpc_furthest_point_sampling(int b, int n, int m, const float* points, float* temp,
                                          int* idx, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n > 0 && m >= 0 && points && temp && idx);
  KDPC_CHECK_ARG(n < (1 << 22));
  if (b == 0 || m == 0) return (int)hipSuccess;
  hipStream_t st = (hipStream_t)stream;
  const int T = host_opt_n_threads(n);
  int log2T = 0;
  while ((1 << log2T) < T) ++log2T;
  const int block = T < 64 ? 64 : T;
  switch (block) {
    case 64: return (int)launch_block<64>(b, n, m, T, log2T, points, temp, idx, st);
    case 128: return (int)launch_block<128>(b, n, m, T, log2T, points, temp, idx, st);
    case 256: return (int)launch_block<256>(b, n, m, T, log2T, points, temp, idx, st);
    case 512: return (int)launch_block<512>(b, n, m, T, log2T, points, temp, idx, st);
    default: return (int)launch_block<1024>(b, n, m, T, log2T, points, temp, idx, st);
  }
}

KDPC_API int kdpc_opt_n_threads(int n) { return host_opt_n_threads(n); }
