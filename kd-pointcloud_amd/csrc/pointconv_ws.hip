// Warp-specialised PointConv data-gradient kernel (reference pointconv_util.py:217-258
// backward; the math is pointconv_fused.hip's "data" pass).  A translation unit of its own
// because it is built without SLP vectorisation (build_native.py EXTRA_FLAGS): the SLP pass
// paired the producer's per-channel dot products across channels (packed fmas fed by
// duplicated WeightNet registers) and the kernel spilled 177 VGPRs; the packed fmas that do
// pay (dwt += dA G, broadcast G) are written out explicitly below.
#include "pointconv_tile.h"

namespace kdpc_pc {
namespace {

// acc[0:2] += a[0:2] * s as one v_pk_fma_f32 (the same IEEE fma per element)
__device__ __forceinline__ void pk_fma_to(float* acc, const float* a, float s) {
  const f32x2 r = __builtin_elementwise_fma(f32x2{a[0], a[1]}, f32x2{s, s}, f32x2{acc[0], acc[1]});
  acc[0] = r.x;
  acc[1] = r.y;
}

// Warp-specialised data kernel (K <= 9): the pipelined kernel's two halves on separate
// waves of one 512-thread workgroup.  Waves 0-3 (one per SIMD) only run the chunk MFMAs,
// dA(ch) = dy wl_ch, into a double-buffered LDS tile; waves 4-7 (one per SIMD) run the pair
// phase of the previous chunk from the other tile -- dG = dA wt per (row, neighbour) stored
// as 32-byte rows, dwt += dA G, dcenter -- and gather the next chunk's neighbour channels.
// One barrier per chunk; each SIMD's matrix core is fed by its consumer wave while its
// producer wave issues the VALU / LDS / memory work beside it.  Same pair mapping, same fma
// chains and the same chunk order as pc_bwd_data_pipe_kernel: bit-identical dG / dwt / dcenter.
template <int O, int KM>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
void pc_bwd_data_ws_kernel(Geo g, const float* __restrict__ wt, const float4* __restrict__ wsw,
                           const float* __restrict__ dy, float* __restrict__ dgr,
                           float* __restrict__ dwt, float* __restrict__ dcenter,
                           int chunks_per_split) {
  constexpr int TR = 32;
  constexpr int NT = 256;  // producer threads
  constexpr int PP = (TR * KM) / NT;
  constexpr int XP = TR * KM - PP * NT;
  constexpr bool XI = XP > 0;
  static_assert(PP >= 1 && (!XI || XP * kCC == NT), "left-over pairs must fill one item/thread");
  constexpr int NOG = O / 8;
  constexpr int PF = NOG < 8 ? NOG : 8;
  __shared__ __attribute__((aligned(16))) float dyl[(O / 4) * kBlk];
  __shared__ __attribute__((aligned(16))) float dal[2][32 * kDaS];
  __shared__ float dcl[TR * KM * 3];
  const int row0 = blockIdx.x * TR;
  const int split = blockIdx.y;
  const int ch0 = split * chunks_per_split;
  const int ch1 = min(g.nch, ch0 + chunks_per_split);
  const int t = threadIdx.x, lane = t & 63, half = lane >> 5, l32 = lane & 31;
  // the wave index through readfirstlane: the role branch is then uniform to the compiler
  // (a threadIdx-derived condition is divergent to it: both roles' code got structurised
  // into one exec-masked sequence, their registers live together)
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool consumer = wv < 4;
  const long long rk_total = (long long)g.r * g.k;

  for (int e = t; e < 32 * O; e += 512) {
    const int r = e / O, o = e % O;
    const int row = row0 + r;
    dyl[(o >> 2) * kBlk + r * 4 + (o & 3)] = row < g.r ? dy[(long long)row * O + o] : 0.f;
  }
  __syncthreads();
  const int nch = ch1 - ch0;
  if (consumer) {
    // ---- dA(ch) for ch = ch0 .. ch1-1 into dal[(ch - ch0) & 1]; iteration i computes chunk
    // ch0 + i while the producers consume chunk ch0 + i - 1
    auto brow = [&](int ch) { return wsw + (long long)((ch * 4 + wv) * NOG) * 64 + lane; };
    float4 bq[PF];
    if (nch > 0) {
      const float4* w0 = brow(ch0);
#pragma unroll
      for (int p2 = 0; p2 < PF; ++p2) bq[p2] = w0[p2 * 64];
    }
#pragma unroll 1
    for (int i = 0; i <= nch; ++i) {
      if (i < nch) {
        const int ch = ch0 + i;
        const float4* wrow = brow(ch);
        f32x16 acc = zero16();
#pragma unroll
        for (int og = 0; og < NOG; ++og) {
          const float4 av = *reinterpret_cast<const float4*>(dyl + (2 * og + half) * kBlk + l32 * 4);
          acc = mfma4(av, bq[og % PF], acc);
          if (og + PF < NOG) bq[og % PF] = wrow[(og + PF) * 64];
        }
        if (i + 1 < nch) {  // the next chunk's first B blocks, in flight over the barrier
          const float4* w1 = brow(ch + 1);
#pragma unroll
          for (int p2 = 0; p2 < PF; ++p2) bq[p2] = w1[p2 * 64];
        }
        float* da = dal[i & 1];
#pragma unroll
        for (int e = 0; e < 16; ++e)
          da[((e & 3) + 8 * (e >> 2) + 4 * half) * kDaS + wv * 32 + l32] = acc[e];
      }
      __syncthreads();
    }
    return;
  }

  // ---- producers: pt = the thread index of pc_bwd_data_pipe_kernel
  const int pt = t - 256;
  const Srcs src = srcs_of(g);
  float wp[PP][kW], dw[PP][kW];
  int pr[PP], pk[PP], pn[PP], ps[PP], prc[PP];
#pragma unroll
  for (int q = 0; q < PP; ++q) {
    const int p = pt + NT * q;
    pr[q] = p / g.k;
    pk[q] = p - pr[q] * g.k;
    prc[q] = min(pr[q], TR - 1);
    const bool ok = p < TR * g.k && row0 + pr[q] < g.r;
    pn[q] = ok ? nbr_of(g, row0 + pr[q], pk[q]) : -1;
    ps[q] = ok ? slot_of(g, row0 + pr[q], pk[q]) : -1;
    const long long pos = (long long)(row0 + pr[q]) * g.k + pk[q];
#pragma unroll
    for (int v = 0; v < kW / 4; ++v) {
      const float4 x = ok ? reinterpret_cast<const float4*>(wt + pos * kW)[v]
                          : make_float4(0.f, 0.f, 0.f, 0.f);
      wp[q][4 * v + 0] = x.x;
      wp[q][4 * v + 1] = x.y;
      wp[q][4 * v + 2] = x.z;
      wp[q][4 * v + 3] = x.w;
    }
#pragma unroll
    for (int w = 0; w < kW; ++w) dw[q][w] = 0.f;
  }
  const int xp = PP * NT + pt / kCC, xc = pt % kCC;
  const int xr = XI ? xp / g.k : 0;
  const int xrc = min(xr, TR - 1);
  const bool xok = XI && xp < TR * g.k && row0 + xr < g.r;
  const int xn = xok ? nbr_of(g, row0 + xr, xp - xr * g.k) : -1;
  const int xsl = xok ? slot_of(g, row0 + xr, xp - xr * g.k) : -1;
  const long long xpos = (long long)(row0 + xr) * g.k + (xp - xr * g.k);
  float xw[kW], xd[kW], xg = 0.f, xgn = 0.f;
  if constexpr (XI) {
#pragma unroll
    for (int v = 0; v < kW / 4; ++v) {
      const float4 x = xok ? reinterpret_cast<const float4*>(wt + xpos * kW)[v]
                           : make_float4(0.f, 0.f, 0.f, 0.f);
      xw[4 * v + 0] = x.x;
      xw[4 * v + 1] = x.y;
      xw[4 * v + 2] = x.z;
      xw[4 * v + 3] = x.w;
    }
#pragma unroll
    for (int w = 0; w < kW; ++w) xd[w] = 0.f;
  }
  auto gather_x = [&](int ch) {
    const int cg = ch * kCC + xc;
    const bool live = xn >= 0;
    const unsigned fo = (live && cg >= 3 && cg < g.c) ? ((unsigned)xn * (unsigned)g.d + (unsigned)(cg - 3)) * 4u : kOOB;
    const unsigned xo = (live && cg < 3) ? ((unsigned)xn * 3u + (unsigned)cg) * 4u : kOOB;
    const unsigned co = (live && cg < 3) ? ((unsigned)(row0 + xr) * 3u + (unsigned)cg) * 4u : kOOB;
    return bload(src.feats, fo) + (bload(src.xyz, xo) - bload(src.center, co));
  };
  auto gather = [&](int ch, float (&dst)[PP][kCC]) {
    const bool c0 = ch == 0;
    const unsigned lo_ch = c0 ? 0u : (unsigned)(ch * kCC - 3) * 4u;
    const unsigned hi_ch = c0 ? 4u : lo_ch + 16u;
#pragma unroll
    for (int q = 0; q < PP; ++q) {
      const int nb = pn[q];
      const bool live = nb >= 0;
      const unsigned fo = live ? (unsigned)nb * (unsigned)g.d * 4u : kOOB;
      const f32x4 lo = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     src.feats, (int)(fo + lo_ch), 0, 0));
      const f32x4 hi = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     src.feats, (int)(fo + hi_ch), 0, 0));
      const unsigned xo = (c0 && live) ? (unsigned)nb * 12u : kOOB;
      const unsigned co = (c0 && live) ? (unsigned)(row0 + pr[q]) * 12u : kOOB;
      const f32x4 x = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                    src.xyz, (int)xo, 0, 0));
      const f32x4 cc = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     src.center, (int)co, 0, 0));
      float v[kCC];
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = (c0 ? 0.f : lo[c]) + (x[c] - cc[c]);
      v[3] = c0 ? lo[0] : lo[3];
#pragma unroll
      for (int c = 4; c < kCC; ++c) v[c] = hi[c - 4];
#pragma unroll
      for (int c = 0; c < kCC; ++c) dst[q][c] = ch * kCC + c < g.c ? v[c] : 0.f;
    }
  };
  const __amdgpu_buffer_rsrc_t dg_rs = __builtin_amdgcn_make_buffer_rsrc(
      dgr, (short)0, (int)((long long)g.r * g.k * g.c8 * 4), 0x00020000);
  float gv[PP][kCC], gn[PP][kCC];
  if (nch > 0) {
    gather(ch0, gv);
    if constexpr (XI) xg = gather_x(ch0);
  }
  __syncthreads();  // iteration 0: the consumers compute chunk ch0
#pragma unroll 1
  for (int i = 1; i <= nch; ++i) {
    const int ch = ch0 + i - 1;  // the chunk this iteration consumes
    const float* dab = dal[(i - 1) & 1];
    const bool more = i < nch;
    if (more) {  // uniform: the next chunk's gathers, in flight during this chunk's VALU work
      gather(ch + 1, gn);
      if constexpr (XI) xgn = gather_x(ch + 1);
    }
    // the pair items of the pipelined kernel's step (pair q channel cl, then the left-over
    // item), one channel's dA row in registers at a time
    constexpr int NIT = PP * kCC + (XI ? 1 : 0);
    float sv[PP][kCC];
    float xs = 0.f;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      if (XI && it == NIT - 1) {
        const float4* drow = reinterpret_cast<const float4*>(dab + xrc * kDaS) + xc * (kW / 4);
        float da[kW];
#pragma unroll
        for (int v = 0; v < kW / 4; ++v) {
          const float4 x = drow[v];
          da[4 * v + 0] = x.x;
          da[4 * v + 1] = x.y;
          da[4 * v + 2] = x.z;
          da[4 * v + 3] = x.w;
        }
        float sacc = 0.f;
#pragma unroll
        for (int w = 0; w < kW; ++w) sacc = __builtin_fmaf(da[w], xw[w], sacc);
        xs = sacc;
#pragma unroll
        for (int w = 0; w < kW; w += 2) pk_fma_to(xd + w, da + w, xg);
      } else {
        const int q = it / kCC, cl = it % kCC;
        const float4* drow = reinterpret_cast<const float4*>(dab + prc[q] * kDaS) + cl * (kW / 4);
        float da[kW];
#pragma unroll
        for (int v = 0; v < kW / 4; ++v) {
          const float4 x = drow[v];
          da[4 * v + 0] = x.x;
          da[4 * v + 1] = x.y;
          da[4 * v + 2] = x.z;
          da[4 * v + 3] = x.w;
        }
        float sacc = 0.f;
#pragma unroll
        for (int w = 0; w < kW; ++w) sacc = __builtin_fmaf(da[w], wp[q][w], sacc);
        sv[q][cl] = sacc;
        const float gc = gv[q][cl];
#pragma unroll
        for (int w = 0; w < kW; w += 2) pk_fma_to(dw[q] + w, da + w, gc);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // dG rows of this chunk (branch-free buffer stores; nothing to store -> out of range)
#pragma unroll
    for (int q = 0; q < PP; ++q) {
      const unsigned off = ps[q] >= 0 ? (unsigned)dg_off(ps[q], ch, rk_total, g.c8) * 4u : kOOB;
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(f32x4, make_float4(sv[q][0], sv[q][1], sv[q][2], sv[q][3])), dg_rs,
          (int)off, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(f32x4, make_float4(sv[q][4], sv[q][5], sv[q][6], sv[q][7])), dg_rs,
          (int)(off == kOOB ? kOOB : off + 16u), 0, 0);
      if (ch == 0) {
#pragma unroll
        for (int cl = 0; cl < 3; ++cl) dcl[(pt + NT * q) * 3 + cl] = sv[q][cl];
      }
    }
    if constexpr (XI) {
      const unsigned off = xsl >= 0 ? (unsigned)(dg_off(xsl, ch, rk_total, g.c8) + xc) * 4u : kOOB;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, xs), dg_rs, (int)off, 0, 0);
      if (xn >= 0 && ch == 0 && xc < 3) dcl[xp * 3 + xc] = xs;
    }
    if (more) {
#pragma unroll
      for (int q = 0; q < PP; ++q)
#pragma unroll
        for (int c = 0; c < kCC; ++c) gv[q][c] = gn[q][c];
      xg = xgn;
    }
    __syncthreads();
  }
  // dcenter (chunk 0 lives in split 0): the producers' dcl (written before the barrier that
  // closed the chunk-0 iteration), summed in neighbour order
  if (ch0 == 0 && pt < TR * 3) {
    const int r = pt / 3, i = pt - (pt / 3) * 3;
    const int row = row0 + r;
    if (row < g.r) {
      float sum = 0.f;
      for (int k = 0; k < g.k; ++k) sum = __fadd_rn(sum, dcl[(r * g.k + k) * 3 + i]);
      dcenter[(long long)row * 3 + i] = -sum;
    }
  }
  float* dwt_dst = dwt + (long long)split * rk_total * kW;
#pragma unroll
  for (int q = 0; q < PP; ++q) {
    if (pn[q] < 0) continue;
    const long long pos = (long long)(row0 + pr[q]) * g.k + pk[q];
    float4* dst = reinterpret_cast<float4*>(dwt_dst + pos * kW);
#pragma unroll
    for (int v = 0; v < kW / 4; ++v)
      dst[v] = make_float4(dw[q][4 * v], dw[q][4 * v + 1], dw[q][4 * v + 2], dw[q][4 * v + 3]);
  }
  if constexpr (XI) {
#pragma unroll
    for (int w = 0; w < kW; ++w) {
      float v = xd[w];
      v += __shfl_xor(v, 4);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 1);
      xd[w] = v;
    }
    float2 out = make_float2(xd[0], xd[1]);
#pragma unroll
    for (int c = 1; c < kCC; ++c)
      if (xc == c) out = make_float2(xd[2 * c], xd[2 * c + 1]);
    if (xn >= 0) reinterpret_cast<float2*>(dwt_dst + xpos * kW)[xc] = out;
  }
}

}  // namespace

hipError_t pc_bwd_data_ws(int o, const Geo& g, dim3 grid, const float* wt, const float4* wsw,
                          const float* dy, float* dgr, float* dwt, float* dcenter,
                          int chunks_per_split, hipStream_t st) {
  switch (o) {
    case 64:
      hipLaunchKernelGGL((pc_bwd_data_ws_kernel<64, 9>), grid, dim3(512), 0, st, g, wt, wsw, dy,
                         dgr, dwt, dcenter, chunks_per_split);
      break;
    case 128:
      hipLaunchKernelGGL((pc_bwd_data_ws_kernel<128, 9>), grid, dim3(512), 0, st, g, wt, wsw, dy,
                         dgr, dwt, dcenter, chunks_per_split);
      break;
    case 256:
      hipLaunchKernelGGL((pc_bwd_data_ws_kernel<256, 9>), grid, dim3(512), 0, st, g, wt, wsw, dy,
                         dgr, dwt, dcenter, chunks_per_split);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace kdpc_pc
