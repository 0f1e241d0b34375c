// Fused cost volume: CrossLayerLight.cross / FlowEmbeddingLayer
// (reference pointconv_util.py:1826-1850, :1497-1517), forward and backward.
//
//   per query n of cloud 1 and its K neighbours j_k = idx[n,k] in cloud 2:
//     dir_k   = x2[j_k] - x1[n]
//     z0[k,:] = (P2[j_k,:] + P1[n,:]) + (Wpos dir_k + bpos)      h0 = LeakyReLU(z0, 0.1)
//     z1[k,:] = W1 h0[k,:] + b1                                    h1 = LeakyReLU(z1, 0.1)
//     out[n,:] = max_k h1[k,:]
//
// The reference materialises every (B, D, K, N) intermediate (gather, +, pos conv, +,
// LeakyReLU, conv, LeakyReLU, max): ~0.5 GB per tensor at level 0.  Here one wave owns one
// query: the K<=32 neighbour rows of h0 are built in LDS straight from the gathered P2 rows,
// the D_IN -> D_OUT MLP runs on the f32 matrix cores (v_mfma_f32_32x32x2_f32: the 32 rows of
// the MFMA tile ARE the query's 32 neighbours), and the max over K is a column reduction of
// the accumulator tile.  Only (N, D_OUT) outputs and a uint8 argmax leave the chip.
//
// Backward (same one-wave-per-query structure): the max routes each output channel's
// gradient to one neighbour row, so dz1 has one nonzero per column; dh0 = dz1 W1 is a
// sparse row update in LDS; dz0 = dh0 * LeakyReLU'(h0); then
//   dP1[n] = sum_k dz0[k]              (written directly)
//   dP2 rows, d(dir) rows              (per (n,k) rows; summed per reference point through the
//                                       kNN index's CSR: deterministic, no float atomics)
//   dx1[n] = -sum_k d(dir_k)
//   dW1, db1, dWpos, dbpos             (per-workgroup partial slabs in registers -> summed in a
//                                       fixed order by a second kernel)
// Supported: D_IN, D_OUT in {32, 64}, K <= 32 (the K=32 levels 0-1 of the models; the
// small levels 2-3 with D >= 128 keep the unfused path).
#include "kdpc_common.h"

using namespace kdpc;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr float kSlope = 0.1f;
constexpr int kRows = 32;        // MFMA M-tile = neighbour rows of one query
constexpr int kWaves = 4;        // per workgroup

__device__ __forceinline__ float lrelu(float x) { return x > 0.f ? x : x * kSlope; }

// Build h0 (and keep nothing else) for query n into lds_h[kRows][D_IN+1].
// Lane roles: per pass, lanes cover (rows, channels): RPP = 64 / D_IN rows per pass.
template <int D_IN>
__device__ __forceinline__ void build_h0(int n, int k, const float* __restrict__ x1b,
                                         const float* __restrict__ x2b,
                                         const int* __restrict__ idxb,
                                         const float* __restrict__ p1b,
                                         const float* __restrict__ p2b,
                                         const float* __restrict__ wpos,
                                         const float* __restrict__ bpos, float* lds_h,
                                         int& my_j, float& my_dx, float& my_dy, float& my_dz) {
  constexpr int LD = D_IN + 1;
  constexpr int RPP = 64 / D_IN;  // 2 for D_IN=32, 1 for 64
  const int lane = lane_id();
  // lane r (< k) owns neighbour row r: index and direction
  const float qx = x1b[n * 3 + 0], qy = x1b[n * 3 + 1], qz = x1b[n * 3 + 2];
  my_j = 0;
  my_dx = my_dy = my_dz = 0.f;
  if (lane < k) {
    my_j = idxb[(long long)n * k + lane];
    my_dx = x2b[my_j * 3 + 0] - qx;
    my_dy = x2b[my_j * 3 + 1] - qy;
    my_dz = x2b[my_j * 3 + 2] - qz;
  }
  const int c = lane % D_IN;
  const int sub = lane / D_IN;  // row offset inside a pass
  const float p1 = p1b[(long long)n * D_IN + c];
  const float w0 = wpos[c * 3 + 0], w1 = wpos[c * 3 + 1], w2 = wpos[c * 3 + 2];
  const float bp = bpos[c];
  // row broadcasts by readlane (uniform lane index: SGPR, no LDS round trip); the loop is
  // unrolled so all of the query's neighbour gathers are in flight together
#pragma unroll
  for (int r0 = 0; r0 < kRows; r0 += RPP) {
    const int r = r0 + sub;
    const int ja = __builtin_amdgcn_readlane(my_j, r0);
    const float dxa = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_dx), r0));
    const float dya = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_dy), r0));
    const float dza = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_dz), r0));
    int j = ja;
    float dx = dxa, dy = dya, dz = dza;
    if (RPP == 2) {
      const int jb = __builtin_amdgcn_readlane(my_j, r0 + 1);
      const float dxb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_dx), r0 + 1));
      const float dyb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_dy), r0 + 1));
      const float dzb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_dz), r0 + 1));
      j = sub ? jb : ja;
      dx = sub ? dxb : dxa;
      dy = sub ? dyb : dya;
      dz = sub ? dzb : dza;
    }
    float h = 0.f;
    if (r < k) {
      const float g2 = p2b[(long long)j * D_IN + c];
      const float pos = __fadd_rn(__builtin_fmaf(w2, dz, __builtin_fmaf(w1, dy, __fmul_rn(w0, dx))), bp);
      h = lrelu(__fadd_rn(__fadd_rn(g2, p1), pos));
    }
    lds_h[r * LD + c] = h;
  }
}

template <int D_IN, int D_OUT>
__global__ __launch_bounds__(256) void cost_volume_fwd_kernel(
    int n1, int n2, int k, int queries_per_wave, const float* __restrict__ x1,
    const float* __restrict__ x2, const int* __restrict__ idx, const float* __restrict__ p1,
    const float* __restrict__ p2, const float* __restrict__ wpos, const float* __restrict__ bpos,
    const float* __restrict__ w1, const float* __restrict__ b1, float* __restrict__ out,
    unsigned char* __restrict__ amax) {
  constexpr int LD = D_IN + 1;
  constexpr int TILES = D_OUT / 32;
  __shared__ float lds[kWaves][kRows * LD];
  const int b = blockIdx.y;
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  float* lds_h = lds[wave];
  const float* x1b = x1 + (long long)b * n1 * 3;
  const float* x2b = x2 + (long long)b * n2 * 3;
  const int* idxb = idx + (long long)b * n1 * k;
  const float* p1b = p1 + (long long)b * n1 * D_IN;
  const float* p2b = p2 + (long long)b * n2 * D_IN;
  float* outb = out + (long long)b * n1 * D_OUT;
  unsigned char* amb = amax + (long long)b * n1 * D_OUT;
  const int q0 = (blockIdx.x * kWaves + wave) * queries_per_wave;
  // B fragments of W1 (lane l: W1[t*32 + (l&31)][2s + (l>>5)]), reused for every query
  float bw[TILES][D_IN / 2];
#pragma unroll
  for (int t = 0; t < TILES; ++t)
#pragma unroll
    for (int s = 0; s < D_IN / 2; ++s)
      bw[t][s] = w1[(t * 32 + (lane & 31)) * D_IN + 2 * s + (lane >> 5)];
  float bias[TILES];
#pragma unroll
  for (int t = 0; t < TILES; ++t) bias[t] = b1[t * 32 + (lane & 31)];

  for (int qi = 0; qi < queries_per_wave; ++qi) {
    const int n = q0 + qi;
    if (n >= n1) break;  // wave-uniform
    int j;
    float dx, dy, dz;
    build_h0<D_IN>(n, k, x1b, x2b, idxb, p1b, p2b, wpos, bpos, lds_h, j, dx, dy, dz);
    __builtin_amdgcn_wave_barrier();
    f32x16 acc[TILES];
#pragma unroll
    for (int t = 0; t < TILES; ++t) acc[t] = f32x16{0};
#pragma unroll
    for (int s = 0; s < D_IN / 2; ++s) {
      const float a = lds_h[(lane & 31) * LD + 2 * s + (lane >> 5)];
#pragma unroll
      for (int t = 0; t < TILES; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bw[t][s], acc[t], 0, 0, 0);
    }
    const int h = lane >> 5;
#pragma unroll
    for (int t = 0; t < TILES; ++t) {
      float m = -INFINITY;
      int mr = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        const float v = lrelu(__fadd_rn(acc[t][r], bias[t]));
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
      if (h == 0) {
        outb[(long long)n * D_OUT + t * 32 + lane] = m;
        amb[(long long)n * D_OUT + t * 32 + lane] = (unsigned char)mr;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------------------ backward
template <int D_IN, int D_OUT>
__global__ __launch_bounds__(256) void cost_volume_bwd_kernel(
    int n1, int n2, int k, int queries_per_wave, const float* __restrict__ x1,
    const float* __restrict__ x2, const int* __restrict__ idx, const float* __restrict__ p1,
    const float* __restrict__ p2, const float* __restrict__ wpos, const float* __restrict__ bpos,
    const float* __restrict__ w1, const float* __restrict__ out,
    const unsigned char* __restrict__ amax, const float* __restrict__ dout,
    float* __restrict__ dp1, float* __restrict__ dp2_rows, float* __restrict__ dx1,
    float* __restrict__ ddir_rows, float* __restrict__ slab) {
  constexpr int LD = D_IN + 1;
  constexpr int RPP = 64 / D_IN;
  constexpr int TI = D_IN / 32;  // 32-column tiles of dh0
  constexpr int SLAB = D_OUT * D_IN + D_OUT + 4 * D_IN;
  constexpr int PER_WAVE = 2 * kRows * LD;
  // the per-wave h0 / dh0 tiles and, after the query loop, the workgroup's partial-sum
  // buffer share one LDS block (2 workgroups per CU instead of 1)
  constexpr int LDS_FLOATS = kWaves * (PER_WAVE > SLAB ? PER_WAVE : SLAB);
  __shared__ float lds_all[LDS_FLOATS];
  const int b = blockIdx.y;
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int half = lane >> 5, l32 = lane & 31;
  float* lds_h = lds_all + wave * PER_WAVE;
  float* lds_d = lds_h + kRows * LD;
  // B fragments of W1 for dh0 = M W1 (inner index d = output channel): lane l supplies
  // W1[2s + half][32t + l32]
  float bwt[TI][D_OUT / 2];
#pragma unroll
  for (int t = 0; t < TI; ++t)
#pragma unroll
    for (int s2 = 0; s2 < D_OUT / 2; ++s2) bwt[t][s2] = w1[(2 * s2 + half) * D_IN + 32 * t + l32];
  const float* x1b = x1 + (long long)b * n1 * 3;
  const float* x2b = x2 + (long long)b * n2 * 3;
  const int* idxb = idx + (long long)b * n1 * k;
  const float* p1b = p1 + (long long)b * n1 * D_IN;
  const float* p2b = p2 + (long long)b * n2 * D_IN;
  const int c = lane % D_IN;
  const int sub = lane / D_IN;
  // per-lane parameter-gradient accumulators (lane c < D_IN; lanes >= D_IN of the D_IN=32
  // case duplicate and are ignored at the end)
  float gw1[D_OUT];
#pragma unroll
  for (int d = 0; d < D_OUT; ++d) gw1[d] = 0.f;
  float gb1 = 0.f, gwp0 = 0.f, gwp1 = 0.f, gwp2 = 0.f, gbp = 0.f;

  const int q0 = (blockIdx.x * kWaves + wave) * queries_per_wave;
  for (int qi = 0; qi < queries_per_wave; ++qi) {
    const int n = q0 + qi;
    if (n >= n1) break;
    int j;
    float dx, dy, dz;
    build_h0<D_IN>(n, k, x1b, x2b, idxb, p1b, p2b, wpos, bpos, lds_h, j, dx, dy, dz);
    // g'[d] = dout[d] * LeakyReLU'(z1[am[d], d]); sign(z1) at the argmax == sign(out[d])
    const long long ob = ((long long)b * n1 + n) * D_OUT;
    const int dl = lane % D_OUT;
    const float od = out[ob + dl];
    const float gd_l = dout[ob + dl] * (od > 0.f ? 1.f : kSlope);
    const int am_l = amax[ob + dl];
    // dh0 = M W1 on the matrix cores, M[r][d] = g'[d] [am[d] == r] (one nonzero per column):
    // the MFMA's f32 accumulation is the fma chain over ascending d, i.e. the same sums as
    // scattering g'[d] W1[d, :] into row am[d] in ascending d
    f32x16 dacc[TI];
#pragma unroll
    for (int t = 0; t < TI; ++t) dacc[t] = f32x16{0};
#pragma unroll
    for (int s2 = 0; s2 < D_OUT / 2; ++s2) {
      const float g_lo = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gd_l), 2 * s2));
      const float g_hi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gd_l), 2 * s2 + 1));
      const int r_lo = __builtin_amdgcn_readlane(am_l, 2 * s2);
      const int r_hi = __builtin_amdgcn_readlane(am_l, 2 * s2 + 1);
      const float a = half ? (r_hi == l32 ? g_hi : 0.f) : (r_lo == l32 ? g_lo : 0.f);
#pragma unroll
      for (int t = 0; t < TI; ++t)
        dacc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bwt[t][s2], dacc[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < TI; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        lds_d[((e & 3) + 8 * (e >> 2) + 4 * half) * LD + 32 * t + l32] = dacc[t][e];
    // dW1[d, :] += g'[d] * h0[am[d], :]
#pragma unroll
    for (int d = 0; d < D_OUT; ++d) {
      const float gd = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gd_l), d));
      const int r = __builtin_amdgcn_readlane(am_l, d);
      gw1[d] = __builtin_fmaf(gd, lds_h[r * LD + c], gw1[d]);
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < D_OUT) gb1 += gd_l;
    __builtin_amdgcn_wave_barrier();
    // dz0 = dh0 * LeakyReLU'(h0) in place; rows written out; per-lane channel sums
    float dp1_acc = 0.f;
    for (int r0 = 0; r0 < kRows; r0 += RPP) {
      const int r = r0 + sub;
      if (r < k) {
        const float hv = lds_h[r * LD + c];
        const float dz0 = lds_d[r * LD + c] * (hv > 0.f ? 1.f : kSlope);
        lds_d[r * LD + c] = dz0;
        dp2_rows[(((long long)b * n1 + n) * k + r) * D_IN + c] = dz0;
      }
    }
    __builtin_amdgcn_wave_barrier();
    // channel sums over rows in ascending order (every lane runs the loop so the row
    // broadcasts are wave-uniform; only sub==0 lanes own a channel)
    for (int r = 0; r < k; ++r) {
      const float rdx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dx), r));
      const float rdy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dy), r));
      const float rdz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dz), r));
      const float dzv = lds_d[r * LD + c];
      dp1_acc = __fadd_rn(dp1_acc, dzv);
      gwp0 = __builtin_fmaf(dzv, rdx, gwp0);
      gwp1 = __builtin_fmaf(dzv, rdy, gwp1);
      gwp2 = __builtin_fmaf(dzv, rdz, gwp2);
      gbp = __fadd_rn(gbp, dzv);
    }
    if (sub == 0) dp1[((long long)b * n1 + n) * D_IN + c] = dp1_acc;
    // d(dir_r) = Wpos^T dz0[r]   (lane r owns row r; ascending channel order)
    float g0 = 0.f, g1 = 0.f, g2 = 0.f;
    if (lane < k) {
      for (int cc = 0; cc < D_IN; ++cc) {
        const float dzv = lds_d[lane * LD + cc];
        g0 = __builtin_fmaf(wpos[cc * 3 + 0], dzv, g0);
        g1 = __builtin_fmaf(wpos[cc * 3 + 1], dzv, g1);
        g2 = __builtin_fmaf(wpos[cc * 3 + 2], dzv, g2);
      }
      float* dd = ddir_rows + (((long long)b * n1 + n) * k + lane) * 3;
      dd[0] = g0;
      dd[1] = g1;
      dd[2] = g2;
    }
    // dx1[n] = -sum_r d(dir_r), ascending r (uniform broadcasts, lane 0 stores)
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int r = 0; r < k; ++r) {
      s0 = __fadd_rn(s0, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g0), r)));
      s1 = __fadd_rn(s1, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g1), r)));
      s2 = __fadd_rn(s2, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g2), r)));
    }
    if (lane == 0) {
      float* o = dx1 + ((long long)b * n1 + n) * 3;
      o[0] = -s0;
      o[1] = -s1;
      o[2] = -s2;
    }
    __builtin_amdgcn_wave_barrier();
  }
  // workgroup partials: waves write their accumulators, wave 0 sums them in wave order
  __syncthreads();  // every wave is done with its h0/dh0 tiles (the buffer is reused)
  float* rw = lds_all + wave * SLAB;
  if (sub == 0) {
#pragma unroll
    for (int d = 0; d < D_OUT; ++d) rw[d * D_IN + c] = gw1[d];
    rw[D_OUT * D_IN + D_OUT + 0 * D_IN + c] = gwp0;
    rw[D_OUT * D_IN + D_OUT + 1 * D_IN + c] = gwp1;
    rw[D_OUT * D_IN + D_OUT + 2 * D_IN + c] = gwp2;
    rw[D_OUT * D_IN + D_OUT + 3 * D_IN + c] = gbp;
  }
  if (lane < D_OUT) rw[D_OUT * D_IN + lane] = gb1;
  __syncthreads();
  float* sb = slab + ((long long)blockIdx.y * gridDim.x + blockIdx.x) * SLAB;
  for (int e = threadIdx.x; e < SLAB; e += blockDim.x) {
    float v = lds_all[e];
    for (int w = 1; w < kWaves; ++w) v = __fadd_rn(v, lds_all[w * SLAB + e]);
    sb[e] = v;
  }
}

constexpr int kFwdQPW = 8;
constexpr int kBwdQPW = 32;

inline int slab_len(int din, int dout) { return dout * din + dout + 4 * din; }

template <int DI, int DO>
hipError_t fwd_launch(int b, int n1, int n2, int k, const float* x1, const float* x2,
                      const int* idx, const float* p1, const float* p2, const float* wpos,
                      const float* bpos, const float* w1, const float* b1, float* out,
                      unsigned char* amax, hipStream_t st) {
  dim3 grid(divup(n1, kWaves * kFwdQPW), b);
  hipLaunchKernelGGL((cost_volume_fwd_kernel<DI, DO>), grid, dim3(256), 0, st, n1, n2, k,
                     kFwdQPW, x1, x2, idx, p1, p2, wpos, bpos, w1, b1, out, amax);
  return hipGetLastError();
}

template <int DI, int DO>
hipError_t bwd_launch(int b, int n1, int n2, int k, const float* x1, const float* x2,
                      const int* idx, const float* p1, const float* p2, const float* wpos,
                      const float* bpos, const float* w1, const float* out,
                      const unsigned char* amax, const float* dout, float* dp1, float* dp2_rows,
                      float* dx1, float* ddir_rows, float* slab, float* dparams,
                      hipStream_t st) {
  dim3 grid(divup(n1, kWaves * kBwdQPW), b);
  hipLaunchKernelGGL((cost_volume_bwd_kernel<DI, DO>), grid, dim3(256), 0, st, n1, n2, k,
                     kBwdQPW, x1, x2, idx, p1, p2, wpos, bpos, w1, out, amax, dout, dp1,
                     dp2_rows, dx1, ddir_rows, slab);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int len = slab_len(DI, DO);
  const int nslab = (int)(grid.x * grid.y);
  return colsum(nslab, len, slab, dparams, slab + (size_t)nslab * len, st);
}

bool supported(int din, int dout, int k) {
  return (din == 32 || din == 64) && (dout == 32 || dout == 64) && k >= 1 && k <= 32;
}

}  // namespace

// Forward.  x1 (B,N1,3), x2 (B,N2,3), idx (B,N1,K) int32 in [0,N2), p1 (B,N1,Din),
// p2 (B,N2,Din), wpos (Din,3), bpos (Din), w1 (Dout,Din), b1 (Dout) ->
// out (B,N1,Dout) channel-last, amax (B,N1,Dout) uint8 (argmax neighbour row).
KDPC_API int kdpc_cost_volume_fwd(int b, int n1, int n2, int k, int din, int dout, const float* x1,
                                  const float* x2, const int* idx, const float* p1,
                                  const float* p2, const float* wpos, const float* bpos,
                                  const float* w1, const float* b1, float* out,
                                  unsigned char* amax, void* stream) {
  KDPC_CHECK_ARG(b >= 0 && n1 >= 0 && n2 > 0 && supported(din, dout, k) && b <= 65535);
  if ((long long)b * n1 == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(x1 && x2 && idx && p1 && p2 && wpos && bpos && w1 && b1 && out && amax);
  hipStream_t st = (hipStream_t)stream;
#define KDPC_CV_FWD(DI, DO)                                                                  \
  if (din == DI && dout == DO)                                                               \
    return (int)fwd_launch<DI, DO>(b, n1, n2, k, x1, x2, idx, p1, p2, wpos, bpos, w1, b1, out, \
                                   amax, st);
  KDPC_CV_FWD(32, 32)
  KDPC_CV_FWD(32, 64)
  KDPC_CV_FWD(64, 32)
  KDPC_CV_FWD(64, 64)
#undef KDPC_CV_FWD
  return (int)hipErrorInvalidValue;
}

// Scratch for the backward's per-workgroup parameter-gradient slabs.
KDPC_API size_t kdpc_cost_volume_bwd_workspace_bytes(int b, int n1, int din, int dout) {
  if (b <= 0 || n1 <= 0 || !supported(din, dout, 1)) return 0;
  const long long nslabs = (long long)divup(n1, kWaves * kBwdQPW) * b;
  const int len = slab_len(din, dout);
  return (size_t)(nslabs * len + colsum_scratch_floats((int)nslabs, len)) * sizeof(float);
}

// Backward.  dout (B,N1,Dout) channel-last gradient of out.  Writes
//   dp1 (B,N1,Din), dp2_rows (B,N1,K,Din), dx1 (B,N1,3), ddir_rows (B,N1,K,3)
//   dparams = [dW1 (Dout*Din) | db1 (Dout) | dWpos^T (3*Din: x,y,z rows) | dbpos (Din)]
// dp2_rows / ddir_rows are summed per reference point by the caller through the CSR of idx
// (kdpc_group_rows_grad_csr); dx2 = that sum of ddir_rows.
KDPC_API int kdpc_cost_volume_bwd(int b, int n1, int n2, int k, int din, int dout,
                                  const float* x1, const float* x2, const int* idx,
                                  const float* p1, const float* p2, const float* wpos,
                                  const float* bpos, const float* w1, const float* out,
                                  const unsigned char* amax, const float* dout_grad, float* dp1,
                                  float* dp2_rows, float* dx1, float* ddir_rows, void* workspace,
                                  size_t workspace_bytes, float* dparams, void* stream) {
  KDPC_CHECK_ARG(b > 0 && n1 > 0 && n2 > 0 && supported(din, dout, k) && b <= 65535);
  KDPC_CHECK_ARG(x1 && x2 && idx && p1 && p2 && wpos && bpos && w1 && out && amax && dout_grad &&
                 dp1 && dp2_rows && dx1 && ddir_rows && workspace && dparams);
  KDPC_CHECK_ARG(workspace_bytes >= kdpc_cost_volume_bwd_workspace_bytes(b, n1, din, dout));
  hipStream_t st = (hipStream_t)stream;
  float* slab = (float*)workspace;
#define KDPC_CV_BWD(DI, DO)                                                                    \
  if (din == DI && dout == DO)                                                                 \
    return (int)bwd_launch<DI, DO>(b, n1, n2, k, x1, x2, idx, p1, p2, wpos, bpos, w1, out, amax, \
                                   dout_grad, dp1, dp2_rows, dx1, ddir_rows, slab, dparams, st);
  KDPC_CV_BWD(32, 32)
  KDPC_CV_BWD(32, 64)
  KDPC_CV_BWD(64, 32)
  KDPC_CV_BWD(64, 64)
#undef KDPC_CV_BWD
  return (int)hipErrorInvalidValue;
}
