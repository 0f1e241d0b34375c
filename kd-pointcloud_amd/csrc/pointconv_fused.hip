// Fused PointConv layer on the f32 matrix cores (reference pointconv_util.py:217-258 and
// 401-446: group -> cat -> (C x K)(K x 16) matmul per point -> Linear(16C -> O)).
//
//   G[r,k,c] = cat(xyz[idx[r,k]] - center[r], feats[idx[r,k]])         c < C = 3 + D
//   A[r, c*16+w] = sum_k G[r,k,c] * wt[r,k,w]                           (never stored)
//   y[r, o]  = sum_j A[r,j] * wl[o,j] + bias[o]
//
// The reference materialises A (R x 16C: 549 MB for the level-0 scene-flow estimator at
// batch 8) and runs the Linear as a separate GEMM.  Here a workgroup owns a tile of 32 or
// 64 rows and walks the channels in chunks of 8 (128 columns of A): the chunk's neighbour
// channels are gathered into LDS (software-pipelined: the next chunk's gather is in flight
// in registers while this chunk computes), the tile's block of A is formed on the VALU (K
// fmas per element, WeightNet weights held in registers), and multiplied into the output
// tile with v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulation; the Linear
// weight streams from L2, one block ahead).  A never touches HBM.
//
// Backward (no float atomics; every sum in a fixed order):
//   data:   dA = dy wl per chunk (MFMA), then per (row, neighbour) on the VALU
//             dG[r,k,c]  = sum_w dA[r,c*16+w] wt[r,k,w]   -> rows [R*K][C8], summed per point
//                                                          through the kNN CSR
//             dwt[r,k,w] = sum_c dA[r,c*16+w] G[r,k,c]
//             dcenter[r] = -sum_k dG[r,k,0:3]
//   weight: dwl[o, j] = sum_r dy[r,o] A[r,j] with A recomputed per (chunk, row split) and
//           the splits' partial tiles summed in split order.  Splits are placed so that
//           every chunk of one split runs on the same XCD (they share its dy / wt rows in L2).
//
// MFMA operand mapping (v_mfma_f32_32x32x2_f32, wave64): lane l supplies A[l&31][l>>5] and
// B[l>>5][l&31]; the result register i of lane l is D[(i&3) + 8*(i>>2) + 4*(l>>5)][l&31].
// The GEMM's inner index is walked in blocks of 8: MFMA step j of block b uses inner
// indices 8b+j (lanes 0-31) and 8b+4+j (lanes 32-63), so every lane's operands for four
// steps are one float4 (LDS: ds_read_b128; global: one 16-byte load).
#include <algorithm>
#include <type_traits>

#include "pointconv_tile.h"

using namespace kdpc_pc;

namespace {

// ------------------------------------------------------------------------------ forward
// grid (row tiles, channel splits); a split > 1 writes a partial tile to slab[split].
// 256 threads.  Tile = 32*MT rows; output tiles 32x32 spread over the 4 waves.
// TP: the tile's rows come from the backward's tile plan (g.trow: Morton-ordered 32-row
// tiles, two per 64-row forward tile), so a tile's neighbour gathers hit few distinct points;
// every row's arithmetic is unchanged (bit-identical outputs).
// The Linear runs on the bf16 matrix cores (mfma_x6, f32 accuracy): each builder thread's
// 8 values of A (row r, WeightNet column w, the chunk's 8 channels) are one 16-byte chunk of
// each bf16 plane, so the MFMA inner index of K-step ks / lane half h is (channel j, column
// w = 2 ks + h) -- any inner order gives the same product -- and wl's B planes come
// pre-split in that order (pc_swizzle_fwd3_kernel).
template <int O, int KM, bool EX, bool TP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void pc_fwd_kernel(Geo g, const float* __restrict__ wt, const bf16x8* __restrict__ wsf,
                   const float* __restrict__ bias, float* __restrict__ y,
                   float* __restrict__ slab, int chunks_per_split) {
  constexpr int MT = KM <= 9 ? 2 : 1;
  constexpr int TM = 32 * MT;
  constexpr int NT = O / 32;
  constexpr bool SPLIT_M = (MT == 2 && NT < 4);   // O = 64: waves split the two row tiles
  constexpr int KG = (MT * NT < 4) ? 4 / (MT * NT) : 1;  // O = 64, 32 rows: waves split the
                                                           // chunk's K-steps in KG groups
  constexpr int MPW = (MT == 2 && !SPLIT_M) ? 2 : 1;
  constexpr int NPW = KG > 1 ? 1 : (MT * NT / 4) / MPW;
  constexpr int RPT = TM / 16;                    // builder rows per thread
  constexpr int GS = (TM * KM + 127) / 128;       // gather slots (float4) per thread
  constexpr int NKS = 8 / KG;                     // 16-deep K-steps per wave and chunk
  constexpr int PF = NKS < 2 ? NKS : 2;           // K-steps of B planes issued ahead
  __shared__ __attribute__((aligned(16))) float gl[TM * KM * kCC];
  // A planes: per 32-row tile, row r's chunk w at r * 16 + (w ^ (r & 15))
  __shared__ __attribute__((aligned(16))) bf16x8 alp[MT][3][32 * kW];

  const int row0 = blockIdx.x * TM;
  // global row of tile row r, -1 for none
  auto grow = [&](int r) -> int {
    if constexpr (TP) {
      return row0 + r < g.ntrow ? g.trow[row0 + r] : -1;
    } else {
      return row0 + r < g.r ? row0 + r : -1;
    }
  };
  const int kk = EX ? KM : g.k;  // exact-K instantiation: constant trip counts
  const int split = blockIdx.y;
  const int ch0 = split * chunks_per_split;
  const int ch1 = min(g.nch, ch0 + chunks_per_split);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, half = lane >> 5, l32 = lane & 31;
  const int w = t & (kW - 1), rr = t >> 4;
  const int m0 = SPLIT_M ? (wv >> 1) : 0;
  const int n0 = SPLIT_M ? (wv & 1) : (KG > 1 ? wv % (4 / KG) : wv * NPW);
  const int kgrp = KG > 1 ? wv / (4 / KG) : 0;
  const int tk = TM * kk;

  float wr[RPT][KM];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int row = grow(rr + 16 * q);
#pragma unroll
    for (int k = 0; k < KM; ++k)
      wr[q][k] = (row >= 0 && k < kk) ? wt[((long long)row * kk + k) * kW + w] : 0.f;
  }
  const Srcs src = srcs_of(g);
  // gather slots: (row, neighbour) rk = (t >> 1) + 128 i, channels 4*h4 .. 4*h4+3 of the
  // chunk -- one 16-byte buffer load per slot (two lanes cover a neighbour's 8 channels)
  const int h4 = t & 1;
  unsigned nbf[GS];  // byte offsets of the slots' neighbour feature rows
  float4 gr[GS];
#pragma unroll
  for (int i = 0; i < GS; ++i) {
    const int rk = (t >> 1) + 128 * i;
    const int r = rk / kk;
    const int row = rk < tk ? grow(r) : -1;
    const int nb = row >= 0 ? nbr_of(g, row, rk - r * kk) : -1;
    nbf[i] = feat_off(g, nb);
    float v[4];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) v[e2] = g_fetch(g, src, nb, row, ch0 * kCC + 4 * h4 + e2);
    gr[i] = make_float4(v[0], v[1], v[2], v[3]);
  }
  f32x16 acc[MPW][NPW];
#pragma unroll
  for (int i = 0; i < MPW; ++i)
#pragma unroll
    for (int j = 0; j < NPW; ++j) acc[i][j] = zero16();

  for (int ch = ch0; ch < ch1; ++ch) {
    const int c0 = ch * kCC;
    __syncthreads();  // previous chunk's MFMAs are done with alp; gl is free
#pragma unroll
    for (int i = 0; i < GS; ++i) {
      const int rk = (t >> 1) + 128 * i;
      if (rk < tk) *reinterpret_cast<float4*>(gl + rk * kCC + 4 * h4) = gr[i];
    }
    __syncthreads();
    // The chunk's B planes (served from L2): the first PF K-steps are issued now and land
    // while the A block is built; each later one PF K-steps ahead of its MFMAs.
    const bf16x8* brow[NPW];
#pragma unroll
    for (int j = 0; j < NPW; ++j)
      brow[j] = wsf + ((long long)(ch * NT + n0 + j) * 8 * 3) * 64 + lane;
    const int kbeg = kgrp * NKS;
    auto bload = [&](int ks, int j, Planes& b) {
      b.h = brow[j][(3 * ks + 0) * 64];
      b.m = brow[j][(3 * ks + 1) * 64];
      b.l = brow[j][(3 * ks + 2) * 64];
    };
    Planes bq[PF][NPW];
#pragma unroll
    for (int p2 = 0; p2 < PF; ++p2)
#pragma unroll
      for (int j = 0; j < NPW; ++j) bload(kbeg + p2, j, bq[p2][j]);
    // next chunk's gather (feature channels only), in flight during build + MFMA.  Issued
    // AFTER the B planes: vmcnt retires loads in issue order, so an MFMA waiting on a
    // B plane issued after the gathers would wait for the gathers too.
    // (issued on the last chunk too -- the values are unused there -- so the loop body is
    // straight-line code and the compiler's load counting stays exact)
    {
      const int cg = c0 + kCC + 4 * h4;  // first of the slot's 4 channels (>= 8: features)
      const unsigned co = (unsigned)(cg - 3) * 4u;
#pragma unroll
      for (int i = 0; i < GS; ++i) {
        // out-of-range offsets read 0; channels past the row are masked
        const f32x4 v = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(src.feats, (int)(nbf[i] + co), 0, 0));
        gr[i] = make_float4(cg < g.c ? v[0] : 0.f, cg + 1 < g.c ? v[1] : 0.f,
                            cg + 2 < g.c ? v[2] : 0.f, cg + 3 < g.c ? v[3] : 0.f);
      }
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int r = rr + 16 * q;
      float a[kCC];
      build_row<KM>(gl, r, kk, wr[q], a);
      const Planes pl = split8(a);
      const int rt = r & 31, cix = rt * kW + (w ^ (rt & 15));
      alp[r >> 5][0][cix] = pl.h;
      alp[r >> 5][1][cix] = pl.m;
      alp[r >> 5][2][cix] = pl.l;
      __builtin_amdgcn_sched_barrier(0);  // keep the rows' LDS reads from piling up
    }
    __syncthreads();
#pragma unroll
    for (int s2 = 0; s2 < NKS; ++s2) {
      const int ks = kbeg + s2;
      const int cw = 2 * ks + half;  // WeightNet column of this K-step's lane half
#pragma unroll
      for (int i = 0; i < MPW; ++i) {
        const int cix = l32 * kW + (cw ^ (l32 & 15));
        const bf16x8 ah = alp[m0 + i][0][cix], am = alp[m0 + i][1][cix], al = alp[m0 + i][2][cix];
#pragma unroll
        for (int j = 0; j < NPW; ++j)
          acc[i][j] = mfma_x6(ah, am, al, bq[s2 % PF][j].h, bq[s2 % PF][j].m, bq[s2 % PF][j].l,
                              acc[i][j]);
      }
      if (s2 + PF < NKS) {
#pragma unroll
        for (int j = 0; j < NPW; ++j) bload(ks + PF, j, bq[s2 % PF][j]);
      }
    }
  }

  if (KG > 1) {  // fold the inner-index groups in group order
    __syncthreads();
    float* red = gl;  // (KG-1) * (4/KG) waves x 16 registers x 64 lanes
    if (kgrp > 0) {
#pragma unroll
      for (int e = 0; e < 16; ++e)
        red[(((kgrp - 1) * (4 / KG) + n0) * 16 + e) * 64 + lane] = acc[0][0][e];
    }
    __syncthreads();
    if (kgrp > 0) return;
    for (int k2 = 1; k2 < KG; ++k2)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        acc[0][0][e] = __fadd_rn(acc[0][0][e], red[(((k2 - 1) * (4 / KG) + n0) * 16 + e) * 64 + lane]);
  }

#pragma unroll
  for (int j = 0; j < NPW; ++j) {
    const int n = (n0 + j) * 32 + l32;
    const float bn = slab ? 0.f : bias[n];
#pragma unroll
    for (int i = 0; i < MPW; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = grow((m0 + i) * 32 + (e & 3) + 8 * (e >> 2) + 4 * half);
        if (row >= 0) {
          if (slab)
            slab[((long long)split * g.r + row) * O + n] = acc[i][j][e];
          else
            y[(long long)row * O + n] = __fadd_rn(acc[i][j][e], bn);
        }
      }
  }
}

// wl (O, 16C) -> the forward's B planes (mfma_x6): bf16x8 (ch, n tile nb, ks, plane, lane) =
// plane {h, m, l} of wl[nb * 32 + (lane & 31)][ch * 128 + 16 j + 2 ks + (lane >> 5)], j = 0..7,
// zero past column 16C.  One thread per (ch, nb, ks, lane).
__global__ __launch_bounds__(256) void pc_swizzle_fwd3_kernel(int o, int c16, int nch,
                                                              const float* __restrict__ wl,
                                                              bf16x8* __restrict__ wsf) {
  const long long total = (long long)nch * (o / 32) * 8 * 64;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int lane = (int)(e & 63);
    const long long q = e >> 6;  // (ch * NT + nb) * 8 + ks
    const int ks = (int)(q & 7);
    const long long cn = q >> 3;
    const int nt = o / 32;
    const int nb = (int)(cn % nt), ch = (int)(cn / nt);
    const float* src = wl + (long long)(nb * 32 + (lane & 31)) * c16;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = ch * 128 + 16 * j + 2 * ks + (lane >> 5);
      v[j] = col < c16 ? src[col] : 0.f;
    }
    const Planes p = split8(v);
    bf16x8* dst = wsf + (q * 3) * 64 + lane;
    dst[0] = p.h;
    dst[64] = p.m;
    dst[128] = p.l;
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
    int s = 0;
    for (; s + 4 <= nslabs; s += 4) {  // four slabs' loads in flight, adds in slab order
      const float x0 = slab[(long long)s * len + e], x1 = slab[(long long)(s + 1) * len + e];
      const float x2 = slab[(long long)(s + 2) * len + e], x3 = slab[(long long)(s + 3) * len + e];
      v = __fadd_rn(__fadd_rn(__fadd_rn(__fadd_rn(v, x0), x1), x2), x3);
    }
    for (; s < nslabs; ++s) v = __fadd_rn(v, slab[(long long)s * len + e]);
    if (bias) v = __fadd_rn(v, bias[e % o]);
    dst[e] = v;
  }
}

// -------------------------------------------------------------------- backward: data
// grid (TR-row tiles, channel splits), 256 threads; each thread owns (row, neighbour)
// pairs t and t+256.  dgr: dG rows [R*K][C8].  Measured alternatives for K = 9 (flow0):
// 28-row tiles, one pair per thread (934 vs 854 us, round 1); 320 threads, one pair each,
// a fifth wave with no MFMA tile (931 us at 3 waves/SIMD with spills, 761 us at 2, vs 622):
// the second pair pass of wave 0 is cheaper than the lost occupancy.
template <int KM>
constexpr int bwd_tile_rows() { return 32; }
template <int KM>
constexpr int bwd_threads() { return 256; }

template <int O, int KM>
__global__ __launch_bounds__(bwd_threads<KM>()) __attribute__((amdgpu_waves_per_eu(2)))
void pc_bwd_data_kernel(Geo g, const float* __restrict__ wt, const bf16x8* __restrict__ wsw,
                        const float* __restrict__ dy, float* __restrict__ dgr,
                        float* __restrict__ dwt, float* __restrict__ dcenter,
                        int chunks_per_split) {
  constexpr int TR = bwd_tile_rows<KM>();
  constexpr int NT = bwd_threads<KM>();
  // (row, neighbour) pairs: PP whole pairs per thread, then the XP left over (K = 9: 288 =
  // 256 + 32) as (pair, chunk channel) items, one per thread -- so every wave carries the
  // same VALU work (round 2 stamps: with a second whole pair on wave 0 its pair phase took
  // 1.8x the other waves', which waited for it at the barrier)
  constexpr int PP = (TR * KM) / NT;
  constexpr int XP = TR * KM - PP * NT;
  constexpr bool XI = XP > 0;
  static_assert(PP >= 1 && (!XI || XP * kCC == NT), "left-over pairs must fill one item/thread");
  // dy as three bf16 planes (dA on the bf16 matrix cores, mfma_x6; layout as
  // pc_bwd_data_pipe_kernel's)
  constexpr int DCH = O / 8;
  constexpr int SW = (DCH < 16 ? DCH : 16) - 1;
  __shared__ __attribute__((aligned(16))) bf16x8 dyp[3][32 * DCH];
  __shared__ __attribute__((aligned(16))) float dal[32 * kDaS];
  __shared__ float dcl[TR * KM * 3];
  const int row0 = blockIdx.x * TR;
  const int split = blockIdx.y;
  const int ch0 = split * chunks_per_split;
  const int ch1 = min(g.nch, ch0 + chunks_per_split);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, half = lane >> 5, l32 = lane & 31;
  const long long c16 = (long long)g.c * kW;
  const long long rk_total = (long long)g.r * g.k;
  const Srcs src = srcs_of(g);

  for (int e = t; e < 32 * DCH; e += NT) {
    const int r = e / DCH, c = e % DCH;
    const int row = row0 + r;
    float v[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 x = (r < TR && row < g.r)
                           ? reinterpret_cast<const float4*>(dy + (long long)row * O)[2 * c + h]
                           : make_float4(0.f, 0.f, 0.f, 0.f);
      v[4 * h + 0] = x.x;
      v[4 * h + 1] = x.y;
      v[4 * h + 2] = x.z;
      v[4 * h + 3] = x.w;
    }
    const Planes pl = split8(v);
    const int cix = r * DCH + (c ^ (r & SW));
    dyp[0][cix] = pl.h;
    dyp[1][cix] = pl.m;
    dyp[2][cix] = pl.l;
  }
  float wp[PP][kW], dw[PP][kW];
  int pr[PP], pk[PP], pn[PP], ps[PP];
#pragma unroll
  for (int q = 0; q < PP; ++q) {
    const int p = t + NT * q;
    pr[q] = p / g.k;
    pk[q] = p - pr[q] * g.k;
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
  // left-over item: pair xp, channel xc of every chunk (8 consecutive lanes share the pair)
  const int xp = PP * NT + t / kCC, xc = t % kCC;
  const int xr = XI ? xp / g.k : 0;
  const int xrc = min(xr, TR - 1);  // dA row read (any row when the item is dead)
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
  // the item's G value of a chunk: branch-free loads, out-of-range offsets read 0
  auto gather_x = [&](int ch) {
    const int cg = ch * kCC + xc;
    const bool live = xn >= 0;
    const unsigned fo = (live && cg >= 3 && cg < g.c) ? ((unsigned)xn * (unsigned)g.d + (unsigned)(cg - 3)) * 4u : kOOB;
    const unsigned xo = (live && cg < 3) ? ((unsigned)xn * 3u + (unsigned)cg) * 4u : kOOB;
    const unsigned co = (live && cg < 3) ? ((unsigned)(row0 + xr) * 3u + (unsigned)cg) * 4u : kOOB;
    return bload(src.feats, fo) + (bload(src.xyz, xo) - bload(src.center, co));
  };
  __syncthreads();

  const bool mw = wv < 4;            // the MFMA waves (wave 4 of a 320-thread group: none)
  const int n0 = (mw ? wv : 3) * 32;  // this wave's 32 dA columns of the chunk
  // Load order matters: loads and stores retire in issue order (vmcnt), so an MFMA waiting
  // on a B fragment also waits for every older gather and dG store.  Per chunk: the first
  // PF B blocks and the neighbour gathers of chunk ch+1 are issued right after chunk ch's
  // MFMAs -- before ch's dG stores -- so ch+1's first MFMAs wait only on those, and the
  // gathers land during ch's VALU phase (they are used in ch+1's VALU phase).
  // B operand = the Linear weight columns of the chunk over the O outputs as bf16 planes,
  // pre-split by pc_swizzle_bwd3_kernel into the order the waves read them (one wave's
  // plane of one K-step is 1 KiB contiguous); zero past the last column.
  constexpr int NKS = O / 16;
  constexpr int PF = NKS < 2 ? NKS : 2;
  auto brow = [&](int ch) {
    return wsw + (long long)((ch * 4 + n0 / 32) * NKS * 3) * 64 + lane;
  };
  auto bload = [&](const bf16x8* wr, int ks, Planes& b) {
    b.h = wr[(3 * ks + 0) * 64];
    b.m = wr[(3 * ks + 1) * 64];
    b.l = wr[(3 * ks + 2) * 64];
  };
  Planes bq[PF];
  float gv[PP][kCC], gn[PP][kCC];
  // a pair's 8 channels of a chunk: two 16-byte buffer loads of its neighbour's feature row
  // (dword-aligned; past-the-row lanes masked, past-the-buffer reads 0), plus, for chunk 0,
  // xyz - center.  Branch-free: every chunk issues the same four loads (the xyz / center
  // ones out of range except in chunk 0) and adds the xyz terms unconditionally, so no load
  // sits under a branch (which would drain the load queue right behind it).
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
  if (ch0 < ch1) {
    const bf16x8* wr0 = brow(ch0);
#pragma unroll
    for (int p2 = 0; p2 < PF; ++p2) bload(wr0, p2, bq[p2]);
    gather(ch0, gv);
    if constexpr (XI) xg = gather_x(ch0);
  }
  // dG of chunk ch is stored after chunk ch+1's MFMA loop has issued its B loads: loads and
  // stores retire in issue order (vmcnt), so a B block issued behind a chunk's dG stores waits
  // for them; held here meanwhile
  float svh[PP][kCC], xsh = 0.f;
  auto store_dg = [&](int ch) {
    const int c0 = ch * kCC;
#pragma unroll
    for (int q = 0; q < PP; ++q) {
      if (ps[q] < 0) continue;
      float4* dgo = reinterpret_cast<float4*>(dgr + dg_off(ps[q], ch, rk_total, g.c8));
      dgo[0] = make_float4(svh[q][0], svh[q][1], svh[q][2], svh[q][3]);
      dgo[1] = make_float4(svh[q][4], svh[q][5], svh[q][6], svh[q][7]);
    }
    if (XI && xsl >= 0) dgr[dg_off(xsl, ch, rk_total, g.c8) + xc] = xsh;
  };
  for (int ch = ch0; ch < ch1; ++ch) {
    const int c0 = ch * kCC;
    const bf16x8* wrow = brow(ch);
    f32x16 acc = zero16();
    if (mw) {  // wave-uniform
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const int cix = l32 * DCH + ((2 * ks + half) ^ (l32 & SW));
        acc = mfma_x6(dyp[0][cix], dyp[1][cix], dyp[2][cix], bq[ks % PF].h, bq[ks % PF].m,
                      bq[ks % PF].l, acc);
        if (ks + PF < NKS) bload(wrow, ks + PF, bq[ks % PF]);
      }
    }
    if (ch > ch0) store_dg(ch - 1);
    if (ch + 1 < ch1) {
      const bf16x8* wr1 = brow(ch + 1);
#pragma unroll
      for (int p2 = 0; p2 < PF; ++p2) bload(wr1, p2, bq[p2]);
      gather(ch + 1, gn);
      if constexpr (XI) xgn = gather_x(ch + 1);
    }
    if (mw) {
#pragma unroll
      for (int e = 0; e < 16; ++e)
        dal[((e & 3) + 8 * (e >> 2) + 4 * half) * kDaS + n0 + l32] = acc[e];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PP; ++q) {
      if (pn[q] < 0) continue;
      const int r = pr[q];
      const long long pos = (long long)(row0 + r) * g.k + pk[q];
      // the pair's 8 dG values are 32 contiguous (32-byte aligned) bytes: two 16-byte stores.
      // Channel cl + 1's dA row is read from LDS while channel cl computes (the scheduling
      // barrier keeps the compiler from hoisting further reads, which spilled).
      const float4* drow = reinterpret_cast<const float4*>(dal + r * kDaS);
      float4 cur[kW / 4], nxt[kW / 4];
#pragma unroll
      for (int v = 0; v < kW / 4; ++v) cur[v] = drow[v];
      float sv[kCC];
#pragma unroll
      for (int cl = 0; cl < kCC; ++cl) {
        if (cl + 1 < kCC) {
#pragma unroll
          for (int v = 0; v < kW / 4; ++v) nxt[v] = drow[(cl + 1) * (kW / 4) + v];
        }
        float da[kW];
#pragma unroll
        for (int v = 0; v < kW / 4; ++v) {
          da[4 * v + 0] = cur[v].x;
          da[4 * v + 1] = cur[v].y;
          da[4 * v + 2] = cur[v].z;
          da[4 * v + 3] = cur[v].w;
        }
        float sacc = 0.f;
#pragma unroll
        for (int w = 0; w < kW; ++w) sacc = __builtin_fmaf(da[w], wp[q][w], sacc);
        sv[cl] = sacc;
        if (c0 == 0 && cl < 3) dcl[(r * g.k + pk[q]) * 3 + cl] = sacc;
        const float gc = gv[q][cl];
#pragma unroll
        for (int w = 0; w < kW; ++w) dw[q][w] = __builtin_fmaf(da[w], gc, dw[q][w]);
#pragma unroll
        for (int v = 0; v < kW / 4; ++v) cur[v] = nxt[v];
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int c = 0; c < kCC; ++c) svh[q][c] = sv[c];
      (void)pos;
    }
    if constexpr (XI) {  // the left-over item: same fma order as a whole pair's channel
      const float4* drow = reinterpret_cast<const float4*>(dal + xrc * kDaS) + xc * (kW / 4);
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
#pragma unroll
      for (int w = 0; w < kW; ++w) xd[w] = __builtin_fmaf(da[w], xg, xd[w]);
      xsh = sacc;
      if (xn >= 0 && c0 == 0 && xc < 3) dcl[xp * 3 + xc] = sacc;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PP; ++q)
#pragma unroll
      for (int c = 0; c < kCC; ++c) gv[q][c] = gn[q][c];
    xg = xgn;
  }
  if (ch0 < ch1) store_dg(ch1 - 1);
  if (ch0 == 0 && t < TR * 3) {
    const int r = t / 3, i = t - (t / 3) * 3;
    const int row = row0 + r;
    if (row < g.r) {
      float s = 0.f;
      for (int k = 0; k < g.k; ++k) s = __fadd_rn(s, dcl[(r * g.k + k) * 3 + i]);
      dcenter[(long long)row * 3 + i] = -s;
    }
  }
  float* dwt_dst = dwt + (long long)split * rk_total * kW;  // slab index when split
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
    // the item's dwt partials (channels xc, xc + 8, ...) summed over the pair's 8 lanes in a
    // fixed butterfly (every lane ends with the same value); lane xc stores w = 2xc, 2xc + 1
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

// Software-pipelined variant of the data kernel.  The kernel above runs each chunk as an
// MFMA phase (dA = dy wl for the chunk) then, after a barrier, a VALU phase (dG / dwt from
// that dA): inside one workgroup the two never overlap, and the matrix cores idle through
// the VALU phase unless the CU's other workgroup happens to be in its MFMA phase.  Here dA is
// double-buffered in LDS and iteration ch issues chunk ch+1's MFMAs and chunk ch's VALU work
// in one loop body (step i: one K-step of ch+1 -- 6 bf16 MFMAs --, then pair-channel item i of ch), so the VALU
// and LDS work fills the MFMAs' 64-cycle issue shadows of the same wave.  One barrier per
// chunk.  Identical arithmetic to pc_bwd_data_kernel (same fma order in every sum), so the
// two produce bit-identical dG / dwt / dcenter.
// TP (tiled plan, tile_plan.hip): the tile's rows come from g.trow, and instead of one dG
// row per pair the kernel writes one partial row per (tile, destination point): each chunk's
// pair values go to LDS (red), and the next step sums every destination's pairs in
// ascending pair order (g.tpair / g.tsoff) into registers, stored at the step's store slot
// (partial row g.tdst).  The forward arithmetic per pair is unchanged.
template <int O, int KM, bool TP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void pc_bwd_data_pipe_kernel(Geo g, const float* __restrict__ wt, const bf16x8* __restrict__ wsw,
                             const float* __restrict__ dy, float* __restrict__ dgr,
                             float* __restrict__ dwt, float* __restrict__ dcenter,
                             int chunks_per_split) {
  constexpr int TR = 32;
  constexpr int NT = 256;
  // whole pairs per thread + the left-over pairs as one (pair, channel) item per thread, as
  // in pc_bwd_data_kernel (every wave the same VALU work)
  constexpr int PP = (TR * KM) / NT;
  constexpr int XP = TR * KM - PP * NT;
  constexpr bool XI = XP > 0;
  static_assert(PP >= 1 && (!XI || XP * kCC == NT), "left-over pairs must fill one item/thread");
  // dA = dy wl on the bf16 matrix cores (mfma_x6): NKS 16-deep K-steps per chunk, 6 MFMAs each
  constexpr int NKS = O / 16;
  // B planes in flight: the first PF K-steps of the next chunk are issued before its gathers,
  // the rest inside the step, PF steps ahead of their MFMAs (behind the gathers in vmcnt order)
  constexpr int PF = NKS < 2 ? NKS : 2;
  constexpr int NIT = PP * kCC + (XI ? 1 : 0);  // VALU items per chunk per thread
  constexpr int STEPS = NKS > NIT ? NKS : NIT;
  // dy of the tile as three bf16 planes (A operands), rows of O/8 16-byte chunks, chunk c of
  // row r at c ^ (r & SW) (the 32 lanes of a half read one chunk column of 32 rows)
  constexpr int DCH = O / 8;
  constexpr int SW = (DCH < 16 ? DCH : 16) - 1;
  __shared__ __attribute__((aligned(16))) bf16x8 dyp[3][32 * DCH];
  __shared__ __attribute__((aligned(16))) float dal[2][32 * kDaS];
  // dcenter partials of every pair slot (chunk 0's first three channels): held in registers
  // through the chunk loop, then written over dal (free after the last step) and summed
  float* dcl = dal[0];
  static_assert(TR * KM * 3 <= 2 * 32 * kDaS, "dcenter partials fit over dA");
  // TP: the chunk's per-pair dG values (double-buffered by chunk parity) and the tile's
  // pairs in (destination, pair) order
  constexpr int TRK = TR * KM;
  constexpr int NJ = TP ? (2 * TRK + NT - 1) / NT : 1;  // (destination, half) items/thread
  __shared__ __attribute__((aligned(16))) float red[TP ? 2 : 1][TP ? TRK * kCC : 4];
  __shared__ int tpl[TP ? TRK : 1], tsl[TP ? TRK + 1 : 1], tdl[TP ? TRK : 1];
  const int row0 = blockIdx.x * TR;
  // global row of tile row r (< TR), -1 for none
  auto grow = [&](int r) -> int {
    if constexpr (TP) {
      return g.trow[(long long)blockIdx.x * TR + r];
    } else {
      return row0 + r < g.r ? row0 + r : -1;
    }
  };
  const int split = blockIdx.y;
  const int ch0 = split * chunks_per_split;
  const int ch1 = min(g.nch, ch0 + chunks_per_split);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, half = lane >> 5, l32 = lane & 31;
  const long long rk_total = (long long)g.r * g.k;
  const Srcs src = srcs_of(g);

  for (int e = t; e < 32 * DCH; e += NT) {
    const int r = e / DCH, c = e % DCH;
    const int row = grow(r);
    float v[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 x = row >= 0 ? reinterpret_cast<const float4*>(dy + (long long)row * O)[2 * c + h]
                                : make_float4(0.f, 0.f, 0.f, 0.f);
      v[4 * h + 0] = x.x;
      v[4 * h + 1] = x.y;
      v[4 * h + 2] = x.z;
      v[4 * h + 3] = x.w;
    }
    const Planes pl = split8(v);
    const int cix = r * DCH + (c ^ (r & SW));
    dyp[0][cix] = pl.h;
    dyp[1][cix] = pl.m;
    dyp[2][cix] = pl.l;
  }
  float wp[PP][kW], dw[PP][kW];
  int pr[PP], pk[PP], pn[PP], ps[PP], prc[PP], prow[PP];
#pragma unroll
  for (int q = 0; q < PP; ++q) {
    const int p = t + NT * q;
    pr[q] = p / g.k;
    pk[q] = p - pr[q] * g.k;
    prc[q] = min(pr[q], TR - 1);  // dA row read by this slot (any row when the pair is dead)
    prow[q] = p < TR * g.k ? grow(pr[q]) : -1;
    const bool ok = prow[q] >= 0;
    pn[q] = ok ? nbr_of(g, prow[q], pk[q]) : -1;
    ps[q] = (ok && !TP) ? slot_of(g, prow[q], pk[q]) : -1;
    const long long pos = (long long)prow[q] * g.k + pk[q];
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
  const int xp = PP * NT + t / kCC, xc = t % kCC;
  const int xr = XI ? xp / g.k : 0;
  const int xrc = min(xr, TR - 1);
  const int xrow = (XI && xp < TR * g.k) ? grow(xrc) : -1;
  const bool xok = xrow >= 0;
  const int xn = xok ? nbr_of(g, xrow, xp - xr * g.k) : -1;
  const int xsl = (xok && !TP) ? slot_of(g, xrow, xp - xr * g.k) : -1;
  const long long xpos = (long long)xrow * g.k + (xp - xr * g.k);
  // TP: the tile's plan in LDS (sorted pairs tpl, destination starts tsl, partial rows tdl);
  // thread t owns the (destination, half) items t + NT j.  Registers are the constraint here
  // (the untiled kernel holds 232 VGPRs), so nothing of it lives in registers across steps.
  if constexpr (TP) {
    const long long tb = (long long)blockIdx.x;
    const int trk = TR * g.k;
    for (int i = t; i < TRK; i += NT) {
      tpl[i] = i < trk ? g.tpair[tb * trk + i] : -1;
      tdl[i] = i < trk ? g.tdst[tb * trk + i] : -1;
    }
    for (int i = t; i <= TRK; i += NT) tsl[i] = i <= trk ? g.tsoff[tb * (trk + 1) + i] : 0;
  }
  float xw[kW], xd[kW], xg = 0.f, xgn = 0.f, xs = 0.f;
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
    const unsigned co = (live && cg < 3) ? ((unsigned)xrow * 3u + (unsigned)cg) * 4u : kOOB;
    return bload(src.feats, fo) + (bload(src.xyz, xo) - bload(src.center, co));
  };

  // this wave's B planes of chunk ch: K-step ks, plane p at [(3 ks + p) * 64]
  auto brow = [&](int ch) { return wsw + (long long)((ch * 4 + wv) * NKS * 3) * 64 + lane; };
  // one K-step of dA: A planes from dyp (row l32, 16-byte chunk 2 ks + half), B planes in b
  auto kstep = [&](int ks, const Planes& b, f32x16 acc) {
    const int cix = l32 * DCH + ((2 * ks + half) ^ (l32 & SW));
    return mfma_x6(dyp[0][cix], dyp[1][cix], dyp[2][cix], b.h, b.m, b.l, acc);
  };
  auto bload = [&](const bf16x8* wr, int ks, Planes& b) {
    b.h = wr[(3 * ks + 0) * 64];
    b.m = wr[(3 * ks + 1) * 64];
    b.l = wr[(3 * ks + 2) * 64];
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
      const unsigned co = (c0 && live) ? (unsigned)prow[q] * 12u : kOOB;
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
  auto store_da = [&](const f32x16& acc, int buf) {
#pragma unroll
    for (int e = 0; e < 16; ++e)
      dal[buf][((e & 3) + 8 * (e >> 2) + 4 * half) * kDaS + wv * 32 + l32] = acc[e];
  };

  Planes bq[PF];
  float gv[PP][kCC], gn[PP][kCC];
  if (ch0 < ch1) {
    const bf16x8* wr0 = brow(ch0);
#pragma unroll
    for (int p2 = 0; p2 < PF; ++p2) bload(wr0, p2, bq[p2]);
    gather(ch0, gv);
    if constexpr (XI) xg = gather_x(ch0);
  }
  __syncthreads();  // dyp
  if (ch0 < ch1) {  // prologue: chunk ch0's dA
    const bf16x8* wrow = brow(ch0);
    f32x16 acc = zero16();
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      acc = kstep(ks, bq[ks % PF], acc);
      if (ks + PF < NKS) bload(wrow, ks + PF, bq[ks % PF]);
    }
    store_da(acc, 0);
    if (ch0 + 1 < ch1) {
      const bf16x8* wr1 = brow(ch0 + 1);
#pragma unroll
      for (int p2 = 0; p2 < PF; ++p2) bload(wr1, p2, bq[p2]);
    }
  }
  __syncthreads();
  // one chunk step: chunk ch+1's MFMAs (when MF) interleaved with chunk ch's VALU items.
  // Branch-free body (dead pair slots compute zeros from zero weights / gathers on a clamped
  // dA row) so the MFMAs and the VALU work share one basic block for the scheduler.
  // dG of chunk ch-1 is held in registers and stored inside chunk ch's step, right after its
  // last B load is issued: a B wait then never waits behind dG stores (vmcnt retires in order)
  float svh[PP][kCC], xsh = 0.f;
  // branch-free buffer stores (a store under a uniform branch would split the step's block):
  // nothing to store -> an out-of-range offset, which the hardware drops
  const __amdgpu_buffer_rsrc_t dg_rs = __builtin_amdgcn_make_buffer_rsrc(
      dgr, (short)0, (int)((long long)g.r * g.k * g.c8 * 4), 0x00020000);
  auto store_dg = [&](int ch) {
    const bool on = ch >= 0;
    const int chs = on ? ch : 0;
    if constexpr (TP) {
      // every destination's sum, left by reduce() at its first pair's LDS slot
      const float* rb = red[(chs - ch0) & 1];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int it = t + NT * j, sl = min(it >> 1, TR * g.k - 1);
        const int b0 = tsl[sl], e0 = tsl[sl + 1], d = tdl[sl];
        const bool ok = on && (it >> 1) < TR * g.k && e0 > b0 && d >= 0;
        const int p0 = tpl[min(b0, TRK - 1)];
        const float4 v =
            *reinterpret_cast<const float4*>(rb + max(p0, 0) * kCC + 4 * (it & 1));
        const unsigned off = ok ? (unsigned)(d * g.c8 + chs * kCC + 4 * (it & 1)) * 4u : kOOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4, v), dg_rs, (int)off,
                                               0, 0);
      }
    } else {
#pragma unroll
    for (int q = 0; q < PP; ++q) {
      const unsigned off = (on && ps[q] >= 0) ? (unsigned)dg_off(ps[q], chs, rk_total, g.c8) * 4u : kOOB;
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(f32x4, make_float4(svh[q][0], svh[q][1], svh[q][2], svh[q][3])),
          dg_rs, (int)off, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(f32x4, make_float4(svh[q][4], svh[q][5], svh[q][6], svh[q][7])),
          dg_rs, (int)(off == kOOB ? kOOB : off + 16u), 0, 0);
    }
    if constexpr (XI) {
      const unsigned off = (on && xsl >= 0) ? (unsigned)(dg_off(xsl, chs, rk_total, g.c8) + xc) * 4u : kOOB;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, xsh), dg_rs, (int)off, 0, 0);
    }
    }
  };
  // TP: every destination's pairs of one chunk summed in ascending pair order (LDS only: no
  // memory operation inside the data-dependent loop, so the load counting stays exact)
  // (each sum overwrites its first pair's values: no other item reads them)
  auto reduce = [&](float* rb) {
    for (int j = 0; j < NJ; ++j) {
      const int it = t + NT * j;
      if ((it >> 1) >= TR * g.k) break;
      const int h4 = (it & 1) * 4;
      const int b0 = tsl[it >> 1], e0 = tsl[(it >> 1) + 1];
      if (e0 - b0 <= 1) continue;  // none, or a single pair: its value is its sum
      auto add = [](float4& a, const float4& x) {
        a.x = __fadd_rn(a.x, x.x);
        a.y = __fadd_rn(a.y, x.y);
        a.z = __fadd_rn(a.z, x.z);
        a.w = __fadd_rn(a.w, x.w);
      };
      float4 v = *reinterpret_cast<const float4*>(rb + tpl[b0] * kCC + h4);
      int i = b0 + 1;
      // four pairs' reads in flight per round (the adds stay in pair order): a group is up
      // to ~K+ pairs and a wave waits for its largest group
      for (; i + 4 <= e0; i += 4) {
        const int q0 = tpl[i], q1 = tpl[i + 1], q2 = tpl[i + 2], q3 = tpl[i + 3];
        const float4 x0 = *reinterpret_cast<const float4*>(rb + q0 * kCC + h4);
        const float4 x1 = *reinterpret_cast<const float4*>(rb + q1 * kCC + h4);
        const float4 x2 = *reinterpret_cast<const float4*>(rb + q2 * kCC + h4);
        const float4 x3 = *reinterpret_cast<const float4*>(rb + q3 * kCC + h4);
        add(v, x0);
        add(v, x1);
        add(v, x2);
        add(v, x3);
      }
      for (; i < e0; ++i) add(v, *reinterpret_cast<const float4*>(rb + tpl[i] * kCC + h4));
      *reinterpret_cast<float4*>(rb + tpl[b0] * kCC + h4) = v;
    }
  };
  constexpr int SI = NKS - PF > 0 ? NKS - PF - 1 : 0;  // step issuing the last B load
  auto step = [&](auto mf, const float* dab, const bf16x8* wr1, f32x16& acc,
                  float (&sv)[PP][kCC], int prev) {
#pragma unroll
    for (int i = 0; i < STEPS; ++i) {
      if constexpr (decltype(mf)::value) {
        if (i < NKS) {
          acc = kstep(i, bq[i % PF], acc);
          if (i + PF < NKS) bload(wr1, i + PF, bq[i % PF]);
        }
      }
      if (XI && i == NIT - 1) {  // the left-over item
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
        for (int w = 0; w < kW; ++w) xd[w] = __builtin_fmaf(da[w], xg, xd[w]);
      } else if (i < NIT) {
        const int q = i / kCC, cl = i % kCC;
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
        for (int w = 0; w < kW; ++w) dw[q][w] = __builtin_fmaf(da[w], gc, dw[q][w]);
      }
      if (i == SI) store_dg(prev);  // prev < 0: nothing stored (branch-free)
      // keep each step's loads with its own math (hoisting every step's dA reads spilled)
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  float dcr[PP][3], dcx = 0.f;  // chunk 0's dcenter partials (dcl after the loop)
  for (int ch = ch0; ch < ch1; ++ch) {
    const int buf = (ch - ch0) & 1;
    const bool more = ch + 1 < ch1;  // uniform
    const int c0 = ch * kCC;
    if (more) {
      gather(ch + 1, gn);
      if constexpr (XI) xgn = gather_x(ch + 1);
    }
    if constexpr (TP) {
      if (ch > ch0) reduce(red[(ch - 1 - ch0) & 1]);
    }
    f32x16 acc = zero16();
    float sv[PP][kCC];
    const int prev = ch > ch0 ? ch - 1 : -1;
    if (more)
      step(std::true_type{}, dal[buf], brow(ch + 1), acc, sv, prev);
    else
      step(std::false_type{}, dal[buf], brow(ch + 1), acc, sv, prev);
#pragma unroll
    for (int q = 0; q < PP; ++q) {
      if (c0 == 0) {
#pragma unroll
        for (int cl = 0; cl < 3; ++cl) dcr[q][cl] = sv[q][cl];
      }
      if constexpr (TP) {
        float4* rp = reinterpret_cast<float4*>(red[buf] + (t + NT * q) * kCC);
        rp[0] = make_float4(sv[q][0], sv[q][1], sv[q][2], sv[q][3]);
        rp[1] = make_float4(sv[q][4], sv[q][5], sv[q][6], sv[q][7]);
      } else {
#pragma unroll
        for (int c = 0; c < kCC; ++c) svh[q][c] = sv[q][c];
      }
    }
    if constexpr (XI) {
      xsh = xs;
      if constexpr (TP) red[buf][xp * kCC + xc] = xs;
      if (c0 == 0) dcx = xs;
    }
    if (more) {
      store_da(acc, buf ^ 1);
      if (ch + 2 < ch1) {
        const bf16x8* wr2 = brow(ch + 2);
#pragma unroll
        for (int p2 = 0; p2 < PF; ++p2) bload(wr2, p2, bq[p2]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PP; ++q)
#pragma unroll
      for (int c = 0; c < kCC; ++c) gv[q][c] = gn[q][c];
    xg = xgn;
  }
  if (ch0 < ch1) {
    if constexpr (TP) reduce(red[(ch1 - 1 - ch0) & 1]);
    store_dg(ch1 - 1);
  }
  if (ch0 == 0) {  // uniform: the loop's last barrier has retired every dA read
#pragma unroll
    for (int q = 0; q < PP; ++q)
#pragma unroll
      for (int cl = 0; cl < 3; ++cl) dcl[(t + NT * q) * 3 + cl] = dcr[q][cl];
    if constexpr (XI) {
      if (xn >= 0 && xc < 3) dcl[xp * 3 + xc] = dcx;
    }
    __syncthreads();
    if (t < TR * 3) {
      const int r = t / 3, i = t - (t / 3) * 3;
      const int row = grow(r);
      if (row >= 0) {
        float s = 0.f;
        for (int k = 0; k < g.k; ++k) s = __fadd_rn(s, dcl[(r * g.k + k) * 3 + i]);  // slot p
        dcenter[(long long)row * 3 + i] = -s;
      }
    }
  }
  float* dwt_dst = dwt + (long long)split * rk_total * kW;
#pragma unroll
  for (int q = 0; q < PP; ++q) {
    if (pn[q] < 0) continue;
    const long long pos = (long long)prow[q] * g.k + pk[q];
    float4* dst = reinterpret_cast<float4*>(dwt_dst + pos * kW);
#pragma unroll
    for (int v = 0; v < kW / 4; ++v)
      dst[v] = make_float4(dw[q][4 * v], dw[q][4 * v + 1], dw[q][4 * v + 2], dw[q][4 * v + 3]);
  }
  if constexpr (XI) {  // as in pc_bwd_data_kernel
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

// wl (O, 16C) -> the data kernels' B operand planes (split-bf16 MFMA, mfma_x6):
// bf16x8 (ch, wave, ks, plane, lane) = plane {h, m, l} of wl[16 ks + 8 (lane >> 5) + 0..7]
// [ch * 128 + 32 wave + (lane & 31)], zero past column 16C.  One thread per (ch, wave, ks,
// lane); a wave reads 32 consecutive columns of 8 rows.
__global__ __launch_bounds__(256) void pc_swizzle_bwd3_kernel(int o, int c16, int nch,
                                                              const float* __restrict__ wl,
                                                              bf16x8* __restrict__ wsw) {
  const int nks = o / 16;
  const long long total = (long long)nch * 4 * nks * 64;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int lane = (int)(e & 63);
    const long long q = e >> 6;
    const int ks = (int)(q % nks);
    const long long cw = q / nks;  // ch * 4 + wave
    const int col = (int)(cw * 32) + (lane & 31);
    const int o0 = 16 * ks + 8 * (lane >> 5);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = col < c16 ? wl[(long long)(o0 + j) * c16 + col] : 0.f;
    const Planes p = split8(v);
    bf16x8* dst = wsw + (q * 3) * 64 + lane;
    dst[0] = p.h;
    dst[64] = p.m;
    dst[128] = p.l;
  }
}

// d_xyz / d_feats of every point = sum of its dG rows, which the data kernels wrote in CSR
// order (slot = rank of the pair): point key's rows are the contiguous slots
// [offsets[key], offsets[key+1]), ascending position.  One thread per (point, 4 channels).
__global__ __launch_bounds__(256) void pc_csr_sum_kernel(long long npts, long long rk, int c, int c8, int d,
                                                         const float* __restrict__ dgr,
                                                         const int* __restrict__ offsets,
                                                         float* __restrict__ dxyz,
                                                         float* __restrict__ dfeats) {
  const int nv = c8 / 4;
  const long long total = npts * nv;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long key = e / nv;
    const int v = (int)(e - key * nv);
    const int j0 = offsets[key], j1 = offsets[key + 1];
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    auto add = [&](const float4 x) {
      s.x = __fadd_rn(s.x, x.x);
      s.y = __fadd_rn(s.y, x.y);
      s.z = __fadd_rn(s.z, x.z);
      s.w = __fadd_rn(s.w, x.w);
    };
    // unrolled 8 wide: the rows are in flight before the (ordered) adds
    int j = j0;
    for (; j + 8 <= j1; j += 8) {
      float4 x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        x[u] = *reinterpret_cast<const float4*>(dgr + dg_off(j + u, v >> 1, rk, c8) + 4 * (v & 1));
#pragma unroll
      for (int u = 0; u < 8; ++u) add(x[u]);
    }
    for (; j < j1; ++j)
      add(*reinterpret_cast<const float4*>(dgr + dg_off(j, v >> 1, rk, c8) + 4 * (v & 1)));
    const float sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ch = 4 * v + i;
      if (ch < 3) {
        if (dxyz) dxyz[key * 3 + ch] = sv[i];
      } else if (ch < c) {
        dfeats[key * d + (ch - 3)] = sv[i];
      }
    }
  }
}

// ------------------------------------------------------------------ backward: weight
// 1-D grid of nch x splits workgroups (512 threads); each owns the O x 128 tile of dwl for
// one chunk over one split's rows, walked in tiles of TR rows (the MFMA inner dimension).
// With >= 8 splits, the chunks of split s all run on XCD s % 8 (workgroups are dealt
// round-robin by id): they share that split's dy / wt rows in one L2.
//
// Software pipeline over the row tiles, two LDS buffers for the MFMA operands: while the
// matrix cores run tile t's MFMAs (dy^T from dyt[t&1], A from at[t&1]), the same waves build
// tile t+1's block of A on the VALU (gathered G in gl, WeightNet weights in registers) into
// at[(t+1)&1]; tile t+2's loads, issued at the top of the step, land meanwhile (staged to LDS
// after the barrier, so no load latency sits between barriers).  The phases are independent
// within one basic block, so the MFMAs' 64-cycle shadows carry the build (the unpipelined
// kernel serialised them behind barriers: ~27 % MFMA busy, profiles/round02).
//
// O <= 128 runs 256-thread workgroups on 32-row tiles with ONE dy^T buffer (dy of tile t+1 is
// staged after tile t's MFMAs): 62-71 KB of LDS, so two workgroups share a CU and one's
// barriers / build phases overlap the other's MFMAs.  O = 256 (acc registers for 8 output
// tiles per wave do not fit) keeps one 512-thread workgroup per CU with two dy^T buffers.
constexpr int wgt_threads(int o) { return o <= 128 ? 256 : 512; }

template <int O, int KM>
constexpr int wgt_tile_rows() {
  return wgt_threads(O) == 256 ? 32 : (O == 256 || (O == 128 && KM > 9) ? 32 : 64);
}

template <int O, int KM, bool EX>
__global__ __launch_bounds__(wgt_threads(O)) __attribute__((amdgpu_waves_per_eu(2)))
void pc_bwd_weight_kernel(Geo g, const float* __restrict__ wt, const float* __restrict__ dy,
                          float* __restrict__ dwl, int rows_per_split, int nsplit, int xcd_map,
                          float* __restrict__ dbias) {
  constexpr int TR = wgt_tile_rows<O, KM>();
  constexpr int TS = TR + 4;               // row stride of the transposed tiles
  constexpr int NT = wgt_threads(O);       // threads
  constexpr bool SDY = NT == 256;          // single dy^T buffer (dy fetched one tile ahead)
  constexpr int RS = NT / 16;              // rows per build pass (16 threads per row)
  constexpr int RP = TR / RS;              // build passes (rows rb, rb + RS, ...)
  constexpr int MT = O / 32;
  constexpr int RG = NT / 256;             // row-tile groups (waves = 4 column tiles x RG)
  constexpr int MPW = MT / RG > 0 ? MT / RG : 1;
  constexpr int GS = (TR * KM + NT / 2 - 1) / (NT / 2);  // gather slots (float4) per thread
  constexpr int DV = TR * O / (NT * 4);    // dy float4 slots per thread
  static_assert(RP >= 1 && TR % RS == 0, "tile rows must split into build passes");
  static_assert(DV >= 1 && TR * O % (NT * 4) == 0, "dy tile must split into float4 slots");
  static_assert(MT >= 2, "O >= 64");
  __shared__ __attribute__((aligned(16))) float gl[TR * KM * kCC];
  __shared__ __attribute__((aligned(16))) float dyt[SDY ? 1 : 2][O * TS];
  __shared__ __attribute__((aligned(16))) float at[2][kNC * TS];

  // XCD fill: workgroups are dealt to the 8 XCDs round-robin by id, so block L runs on XCD
  // L % 8; give each XCD a contiguous run of (split, chunk) pairs (split-major), so the
  // chunks of one split -- which all read that split's dy / wt rows -- share at most two
  // L2s (a plain split-major order spreads them over all eight).  Speed only: any
  // placement computes the same result.
  const int L = blockIdx.x;
  int ch, split;
  if (xcd_map) {
    const int per_xcd = (int)gridDim.x >> 3;
    const int pidx = (L & 7) * per_xcd + (L >> 3);
    split = pidx / g.nch;
    ch = pidx % g.nch;
  } else {
    ch = L % g.nch;
    split = L / g.nch;
  }
  if (split >= nsplit) return;
  const int c0 = ch * kCC;
  const int kk = EX ? KM : g.k;  // exact-K instantiation: constant trip counts
  const int rbeg = split * rows_per_split;
  const int rend = min(g.r, rbeg + rows_per_split);
  const int ntiles = (rend - rbeg + TR - 1) / TR;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, half = lane >> 5, l32 = lane & 31;
  const int w = t & (kW - 1), rb = t >> 4;
  const int nt = wv & 3;
  const int m0 = (wv >> 2) * MPW;
  const long long c16 = (long long)g.c * kW;
  const int tk = TR * kk;
  const Srcs src = srcs_of(g);

  // tile registers: WeightNet weights (row rb + 32 p2, all K, column w), gathered G
  // (row-neighbour rk = (t >> 1) + 256 i, channels 4*h4 .. +3), dy (float4 slots).  The
  // gathers' neighbour indices are loaded one fetch AHEAD (nbi): a gather issued right
  // behind its own index load would stall the wave on that load (vmcnt retires in order).
  const int h4 = t & 1;
  float wr[RP][KM], wc[RP][KM];
  float4 gr[GS], dr[DV];
  int nbi[GS];  // global neighbour row (b*N + idx) of each gather slot, >= b*n for none
  // Every load of the tile is unconditional (a load under a branch -- or under a select the
  // compiler turns into one -- makes it drain the whole load queue right behind it): rows past
  // the split read through an out-of-range buffer offset, which returns 0 without touching
  // memory.  Neighbour slots past the tile get the index kNoNbr (>= b*n: gathers read 0).
  constexpr int kNoNbr = 1 << 30;
  const __amdgpu_buffer_rsrc_t idx_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int*>(g.idx), (short)0, (int)((long long)g.r * g.k * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t wt_rs = rsrc(wt, (long long)g.r * kk * kW);
  const __amdgpu_buffer_rsrc_t dy_rs = rsrc(dy, (long long)g.r * O);
  // batch base (b * n) of a row: one integer division per tile; a row x = rr + r rows past
  // the tile's first cloud start (x < s + TR) lies in cloud b0 + x / s, taken from a float
  // quotient corrected by one step either way (its error is below 1) -- branch-free, so the
  // loads stay in one scheduling region with the MFMAs
  const float inv_s = 1.f / (float)g.s;
  auto fetch_idx = [&](int tile) {
    const int row0 = rbeg + tile * TR;
    const int b0 = row0 / g.s;
    const int rr = row0 - b0 * g.s;
#pragma unroll
    for (int i = 0; i < GS; ++i) {
      const int rk = (t >> 1) + (NT / 2) * i;
      const int r = rk / kk;
      const int rw = row0 + r;
      const bool ok = rk < tk && rw < rend;
      const int x = rr + r;
      int q = (int)((float)x * inv_s);
      q += ((q + 1) * g.s <= x ? 1 : 0) - (q * g.s > x ? 1 : 0);
      const int bb = b0 + q;
      const int base = ok ? bb * g.n : kNoNbr;
      const unsigned off = ok ? ((unsigned)rw * (unsigned)g.k + (unsigned)(rk - r * kk)) * 4u : kOOB;
      nbi[i] = base + (int)__builtin_amdgcn_raw_buffer_load_b32(idx_rs, (int)off, 0, 0);
    }
  };
  auto fetch_g = [&](int tile) {
    const int row0 = rbeg + tile * TR;
#pragma unroll
    for (int p2 = 0; p2 < RP; ++p2) {
      const int row = row0 + rb + RS * p2;
      const unsigned base = row < rend ? ((unsigned)row * (unsigned)kk * kW + w) * 4u : kOOB;
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const unsigned off = k < kk ? base + (unsigned)(k * kW * 4) : kOOB;
        wr[p2][k] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(wt_rs, (int)off, 0, 0));
      }
    }
    // Branch-free gathers (a load under a branch makes the compiler drain the whole load
    // queue right behind it): every slot issues the same three 16-byte buffer loads, with
    // out-of-range offsets (which read 0 without touching memory) for what it does not need.
    // Slot channels 4*h4 .. +3 of the chunk: for chunk 0, lane half 0 holds xyz - center and
    // feature 0, lane half 1 features 1..4; otherwise 4 consecutive features.
#pragma unroll
    for (int i = 0; i < GS; ++i) {
      const int rk = (t >> 1) + (NT / 2) * i;
      const int rw = row0 + rk / kk;
      const int nb = nbi[i];
      const bool live = (unsigned)nb < (unsigned)g.bn;
      const bool xyz = c0 == 0 && h4 == 0;
      const int vch = c0 == 0 ? (h4 ? 1 : 0) : c0 - 3 + 4 * h4;  // first feature of the load
      const unsigned voff = live ? (unsigned)nb * (unsigned)g.d * 4u + (unsigned)vch * 4u : kOOB;
      const unsigned xoff = (xyz && live) ? (unsigned)nb * 12u : kOOB;
      const unsigned coff = (xyz && live) ? (unsigned)rw * 12u : kOOB;
      const f32x4 v =
          __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(src.feats, (int)voff, 0, 0));
      const f32x4 x = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(src.xyz, (int)xoff, 0, 0));
      const f32x4 cc = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(src.center, (int)coff, 0, 0));
      // The xyz - center terms are added unconditionally (they are 0 - 0 outside the xyz
      // slots): a select on them would let the compiler sink their loads under a branch.
      const int cg = c0 + 4 * h4;  // first chunk channel of the slot
      const float a0 = xyz ? 0.f : (cg < g.c ? v[0] : 0.f);
      const float a1 = xyz ? 0.f : (cg + 1 < g.c ? v[1] : 0.f);
      const float a2 = xyz ? 0.f : (cg + 2 < g.c ? v[2] : 0.f);
      const float a3 = xyz ? (3 < g.c ? v[0] : 0.f) : (cg + 3 < g.c ? v[3] : 0.f);
      gr[i] = make_float4(a0 + (x[0] - cc[0]), a1 + (x[1] - cc[1]), a2 + (x[2] - cc[2]), a3);
    }
    fetch_idx(tile + 1);
  };
  // dy slot q = t + NT i: row q % TR (consecutive lanes: consecutive rows, so the
  // transposed LDS writes below hit consecutive banks), columns 4 (q / TR) .. +3
  auto fetch_dy = [&](int tile) {
    const int row0 = rbeg + tile * TR;
#pragma unroll
    for (int i = 0; i < DV; ++i) {
      const int q = t + NT * i;
      const int rw = row0 + q % TR;
      const unsigned off = rw < rend ? ((unsigned)rw * O + 4u * (unsigned)(q / TR)) * 4u : kOOB;
      dr[i] = __builtin_bit_cast(
          float4, __builtin_amdgcn_raw_buffer_load_b128(dy_rs, (int)off, 0, 0));
    }
  };
  // registers -> LDS: gathered G into gl, weights into wc; dy transposed into dyt[buf]
  auto stage_g = [&]() {
#pragma unroll
    for (int i = 0; i < GS; ++i) {
      const int rk = (t >> 1) + (NT / 2) * i;
      if (rk < tk) *reinterpret_cast<float4*>(gl + rk * kCC + 4 * h4) = gr[i];
    }
#pragma unroll
    for (int p2 = 0; p2 < RP; ++p2)
#pragma unroll
      for (int k = 0; k < KM; ++k) wc[p2][k] = wr[p2][k];
  };
  auto stage_dy = [&](int buf) {
    float* dt = dyt[buf];
#pragma unroll
    for (int i = 0; i < DV; ++i) {
      const int q = t + NT * i;
      const int r = q % TR, o = 4 * (q / TR);
      dt[(o + 0) * TS + r] = dr[i].x;
      dt[(o + 1) * TS + r] = dr[i].y;
      dt[(o + 2) * TS + r] = dr[i].z;
      dt[(o + 3) * TS + r] = dr[i].w;
    }
  };
  // A block of the tile staged in gl / wc -> at[buf] (transposed: column-major rows)
  // bias gradient for free (dbias != null): the first padding channel's w = 0 column of A
  // (always 0 otherwise: C % 8 != 0 puts it in the last chunk) is set to 1, so that column
  // of the MFMA output is sum_r dy[r, o] -- the rows past the split read dy = 0
  const int ones_col = (dbias != nullptr && ch == g.nch - 1 && g.c % kCC != 0)
                           ? (g.c % kCC) * kW : -1;
  auto build = [&](int buf) {
    float* ab = at[buf];
#pragma unroll
    for (int p2 = 0; p2 < RP; ++p2) {
      float a[kCC];
      build_row<KM>(gl, rb + RS * p2, kk, wc[p2], a);
#pragma unroll
      for (int c = 0; c < kCC; ++c)
        ab[(c * kW + w) * TS + rb + RS * p2] = c * kW + w == ones_col ? 1.f : a[c];
    }
  };

  f32x16 acc[MPW];
#pragma unroll
  for (int i = 0; i < MPW; ++i) acc[i] = zero16();
  if (ntiles <= 0) return;
  // prologue: tile 0 staged and built, tile 1's G / weights (and dy with two buffers) staged
  fetch_idx(0);
  fetch_g(0);
  fetch_dy(0);
  stage_g();
  stage_dy(0);
  __syncthreads();
  build(0);
  fetch_g(1);
  if (!SDY) fetch_dy(1);
  __syncthreads();
  stage_g();
  if (!SDY) stage_dy(1);
  __syncthreads();
  for (int tile = 0; tile < ntiles; ++tile) {
    const int cur = tile & 1;
    // tile+2's loads (tile+1's dy with one buffer) are issued first and land under this
    // tile's MFMAs; tile's MFMAs || tile+1's build (independent: at[cur] / dyt vs gl, wc ->
    // at[!cur])
    fetch_g(tile + 2);
    fetch_dy(SDY ? tile + 1 : tile + 2);
    const float* dt = dyt[SDY ? 0 : cur];
    const float* ab = at[cur];
#pragma unroll
    for (int gb = 0; gb < TR / 8; ++gb) {
      const float4 bv = *reinterpret_cast<const float4*>(ab + (nt * 32 + l32) * TS + 8 * gb + 4 * half);
#pragma unroll
      for (int i = 0; i < MPW; ++i) {
        const float4 av =
            *reinterpret_cast<const float4*>(dt + ((m0 + i) * 32 + l32) * TS + 8 * gb + 4 * half);
        acc[i] = mfma4(av, bv, acc[i]);
      }
    }
    build(cur ^ 1);
    __syncthreads();  // at[cur] / dyt / gl consumed; at[cur ^ 1] complete
    stage_g();        // tile + 2
    stage_dy(SDY ? 0 : cur);  // tile + 1 (one buffer) or tile + 2
    __syncthreads();
  }
  const long long col = (long long)c0 * kW + nt * 32 + l32;
  if (ones_col >= 0 && col == (long long)c0 * kW + ones_col) {
    float* bd = dbias + (long long)split * O;  // slab index when the rows are split
#pragma unroll
    for (int i = 0; i < MPW; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) bd[(m0 + i) * 32 + (e & 3) + 8 * (e >> 2) + 4 * half] = acc[i][e];
  }
  if (col >= c16) return;
  float* dst = dwl + (long long)split * O * c16;  // slab index when the rows are split
#pragma unroll
  for (int i = 0; i < MPW; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int o = (m0 + i) * 32 + (e & 3) + 8 * (e >> 2) + 4 * half;
      dst[o * c16 + col] = acc[i][e];
    }
}

// Split-bf16 weight kernel (O <= 128; mfma_x6): the same (chunk, split) workgroups and row
// tiles as pc_bwd_weight_kernel, with the MFMA operands as bf16 planes in LDS: dy^T planes
// (o, 8-row group) and A planes (column, 8-row group), 16-byte chunks, the group index
// XOR-swizzled by (index >> 2) & 3 so that the 32 lanes of an MFMA operand read hit 16
// distinct chunk positions.  Each thread builds two adjacent rows of one WeightNet column for
// the 8 channels of the chunk (one packed 32-bit plane word per channel) and splits two
// adjacent rows of 8 dy columns.  One A buffer: per 32-row tile, [MFMAs of tile t] barrier
// [build + split of tile t+1, dy of t+1 and G of t+2 to LDS] barrier -- 62-68 KB of LDS, two
// workgroups per CU, whose phases overlap each other (a bf16 MFMA leaves 24 of its 32 cycles
// of vector issue to other waves).  G is double-buffered (tile t+2's gathers land while tile
// t+1 is built from the other buffer).
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void split_pair(float a, float b, unsigned& h, unsigned& m,
                                           unsigned& l) {
  __bf16 h0, m0, l0, h1, m1, l1;
  split3(a, h0, m0, l0);
  split3(b, h1, m1, l1);
  h = __builtin_bit_cast(unsigned, bf16x2{h0, h1});
  m = __builtin_bit_cast(unsigned, bf16x2{m0, m1});
  l = __builtin_bit_cast(unsigned, bf16x2{l0, l1});
}

template <int O, int KM, bool EX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void pc_bwd_weight_x6_kernel(Geo g, const float* __restrict__ wt, const float* __restrict__ dy,
                             float* __restrict__ dwl, int rows_per_split, int nsplit,
                             int xcd_map, float* __restrict__ dbias) {
  constexpr int TR = 32;                   // tile rows: two 16-deep K-steps
  constexpr int NT = 256;
  constexpr int NG = TR / 8;               // 8-row groups (16-byte plane chunks) per column
  constexpr int MT = O / 32;               // output tiles per wave (o blocks)
  constexpr int GS = (TR * KM + NT / 2 - 1) / (NT / 2);  // gather slots (float4) per thread
  constexpr int DI = (TR / 2) * (O / 8);   // dy items: (row pair, 8 columns)
  constexpr int DVI = (DI + NT - 1) / NT;  // dy items per thread
  static_assert(O == 64 || O == 128, "x6 weight kernel: O in {64, 128}");
  __shared__ __attribute__((aligned(16))) float gl[2][TR * KM * kCC];
  __shared__ __attribute__((aligned(16))) bf16x8 dyp[3][O * NG];
  __shared__ __attribute__((aligned(16))) bf16x8 atp[3][kNC * NG];
  auto cidx = [](int x, int grp) { return x * NG + (grp ^ ((x >> 2) & (NG - 1))); };

  const int L = blockIdx.x;
  int ch, split;
  if (xcd_map) {  // as pc_bwd_weight_kernel: a split's chunks share an XCD's L2
    const int per_xcd = (int)gridDim.x >> 3;
    const int pidx = (L & 7) * per_xcd + (L >> 3);
    split = pidx / g.nch;
    ch = pidx % g.nch;
  } else {
    ch = L % g.nch;
    split = L / g.nch;
  }
  if (split >= nsplit) return;
  const int c0 = ch * kCC;
  const int kk = EX ? KM : g.k;
  const int rbeg = split * rows_per_split;
  const int rend = min(g.r, rbeg + rows_per_split);
  const int ntiles = (rend - rbeg + TR - 1) / TR;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, half = lane >> 5, l32 = lane & 31;
  const int w = t & (kW - 1), rp = t >> 4;  // build: WeightNet column w, rows 2 rp, 2 rp + 1
  const long long c16 = (long long)g.c * kW;
  const int tk = TR * kk;
  const Srcs src = srcs_of(g);

  const int h4 = t & 1;
  float wc[2][KM];  // WeightNet weights of the row pair being built
  float4 gr[GS];
  float dr[DVI][2][8];
  int nbi[GS];
  constexpr int kNoNbr = 1 << 30;
  const __amdgpu_buffer_rsrc_t idx_rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int*>(g.idx), (short)0, (int)((long long)g.r * g.k * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t wt_rs = rsrc(wt, (long long)g.r * kk * kW);
  const __amdgpu_buffer_rsrc_t dy_rs = rsrc(dy, (long long)g.r * O);
  const float inv_s = 1.f / (float)g.s;
  // neighbour indices one fetch ahead (as pc_bwd_weight_kernel)
  auto fetch_idx = [&](int tile) {
    const int row0 = rbeg + tile * TR;
    const int b0 = row0 / g.s;
    const int rr = row0 - b0 * g.s;
#pragma unroll
    for (int i = 0; i < GS; ++i) {
      const int rk = (t >> 1) + (NT / 2) * i;
      const int r = rk / kk;
      const int rw = row0 + r;
      const bool ok = rk < tk && rw < rend;
      const int x = rr + r;
      int q = (int)((float)x * inv_s);
      q += ((q + 1) * g.s <= x ? 1 : 0) - (q * g.s > x ? 1 : 0);
      const int base = ok ? (b0 + q) * g.n : kNoNbr;
      const unsigned off = ok ? ((unsigned)rw * (unsigned)g.k + (unsigned)(rk - r * kk)) * 4u : kOOB;
      nbi[i] = base + (int)__builtin_amdgcn_raw_buffer_load_b32(idx_rs, (int)off, 0, 0);
    }
  };
  // WeightNet weights of rows 2 rp, 2 rp + 1 of a tile, straight into wc: issued right after
  // the build that last read wc, they land under the next MFMA phase (no second register set)
  auto fetch_w = [&](int tile) {
    const int row0 = rbeg + tile * TR;
#pragma unroll
    for (int p2 = 0; p2 < 2; ++p2) {
      const int row = row0 + 2 * rp + p2;
      const unsigned base = row < rend ? ((unsigned)row * (unsigned)kk * kW + w) * 4u : kOOB;
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const unsigned off = k < kk ? base + (unsigned)(k * kW * 4) : kOOB;
        wc[p2][k] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(wt_rs, (int)off, 0, 0));
      }
    }
  };
  // the tile's gathered G (branch-free loads)
  auto fetch_g = [&](int tile) {
    const int row0 = rbeg + tile * TR;
#pragma unroll
    for (int i = 0; i < GS; ++i) {
      const int rk = (t >> 1) + (NT / 2) * i;
      const int rw = row0 + rk / kk;
      const int nb = nbi[i];
      const bool live = (unsigned)nb < (unsigned)g.bn;
      const bool xyz = c0 == 0 && h4 == 0;
      const int vch = c0 == 0 ? (h4 ? 1 : 0) : c0 - 3 + 4 * h4;
      const unsigned voff = live ? (unsigned)nb * (unsigned)g.d * 4u + (unsigned)vch * 4u : kOOB;
      const unsigned xoff = (xyz && live) ? (unsigned)nb * 12u : kOOB;
      const unsigned coff = (xyz && live) ? (unsigned)rw * 12u : kOOB;
      const f32x4 v =
          __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(src.feats, (int)voff, 0, 0));
      const f32x4 x = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(src.xyz, (int)xoff, 0, 0));
      const f32x4 cc = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(src.center, (int)coff, 0, 0));
      const int cg = c0 + 4 * h4;
      const float a0 = xyz ? 0.f : (cg < g.c ? v[0] : 0.f);
      const float a1 = xyz ? 0.f : (cg + 1 < g.c ? v[1] : 0.f);
      const float a2 = xyz ? 0.f : (cg + 2 < g.c ? v[2] : 0.f);
      const float a3 = xyz ? (3 < g.c ? v[0] : 0.f) : (cg + 3 < g.c ? v[3] : 0.f);
      gr[i] = make_float4(a0 + (x[0] - cc[0]), a1 + (x[1] - cc[1]), a2 + (x[2] - cc[2]), a3);
    }
    fetch_idx(tile + 1);
  };
  // dy item q = t + NT i: row pair q % (TR / 2) (consecutive threads: consecutive pairs, so
  // the plane-word writes below fill consecutive banks), columns 8 (q / (TR / 2)) .. +7
  auto fetch_dy = [&](int tile) {
    const int row0 = rbeg + tile * TR;
#pragma unroll
    for (int i = 0; i < DVI; ++i) {
      const int q = t + NT * i;
      const int pr = q % (TR / 2), oc = q / (TR / 2);
#pragma unroll
      for (int p2 = 0; p2 < 2; ++p2) {
        const int rw = row0 + 2 * pr + p2;
        const unsigned off = (q < DI && rw < rend) ? ((unsigned)rw * O + 8u * (unsigned)oc) * 4u : kOOB;
        const f32x4 lo = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(dy_rs, (int)off, 0, 0));
        const f32x4 hi = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(dy_rs, (int)(off == kOOB ? kOOB : off + 16u), 0, 0));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          dr[i][p2][j] = lo[j];
          dr[i][p2][4 + j] = hi[j];
        }
      }
    }
  };
  auto stage_g = [&](float* gb) {
#pragma unroll
    for (int i = 0; i < GS; ++i) {
      const int rk = (t >> 1) + (NT / 2) * i;
      if (rk < tk) *reinterpret_cast<float4*>(gb + rk * kCC + 4 * h4) = gr[i];
    }
  };
  auto stage_dy = [&]() {
#pragma unroll
    for (int i = 0; i < DVI; ++i) {
      const int q = t + NT * i;
      if (q < DI) {
        const int pr = q % (TR / 2), oc = q / (TR / 2);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          unsigned h, m, l;
          split_pair(dr[i][0][j], dr[i][1][j], h, m, l);
          const int o = 8 * oc + j;
          unsigned* base = reinterpret_cast<unsigned*>(dyp[0]);
          const int word = cidx(o, pr >> 2) * 4 + (pr & 3);
          base[word] = h;
          reinterpret_cast<unsigned*>(dyp[1])[word] = m;
          reinterpret_cast<unsigned*>(dyp[2])[word] = l;
        }
      }
    }
  };
  // bias gradient for free (as pc_bwd_weight_kernel): the first padding column of the last
  // chunk is set to 1 (planes 1, 0, 0: exact)
  const int ones_col = (dbias != nullptr && ch == g.nch - 1 && g.c % kCC != 0)
                           ? (g.c % kCC) * kW : -1;
  auto build = [&](const float* gb) {
    float a[2][kCC];
    build_row<KM>(gb, 2 * rp, kk, wc[0], a[0]);
    build_row<KM>(gb, 2 * rp + 1, kk, wc[1], a[1]);
#pragma unroll
    for (int c = 0; c < kCC; ++c) {
      const int col = c * kW + w;
      unsigned h, m, l;
      split_pair(a[0][c], a[1][c], h, m, l);
      if (col == ones_col) {  // 1.0 in both rows: planes (1, 0, 0)
        h = 0x3F803F80u;
        m = 0u;
        l = 0u;
      }
      const int word = cidx(col, rp >> 2) * 4 + (rp & 3);
      reinterpret_cast<unsigned*>(atp[0])[word] = h;
      reinterpret_cast<unsigned*>(atp[1])[word] = m;
      reinterpret_cast<unsigned*>(atp[2])[word] = l;
    }
  };

  f32x16 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = zero16();
  if (ntiles <= 0) return;
  // prologue: tile 0 built (A planes), dy of tile 0 split, G of tile 1 in gl[1]
  fetch_idx(0);
  fetch_g(0);
  fetch_w(0);
  fetch_dy(0);
  stage_g(gl[0]);
  stage_dy();
  fetch_g(1);
  __syncthreads();
  build(gl[0]);
  fetch_w(1);
  stage_g(gl[1]);
  __syncthreads();
  const int col = wv * 32 + l32;  // this lane's A column (B operand) of the chunk
  for (int tile = 0; tile < ntiles; ++tile) {
    // loads of tile+2's G / weights and tile+1's dy land under this tile's MFMAs
    fetch_g(tile + 2);
    fetch_dy(tile + 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int bi = cidx(col, 2 * ks + half);
      const bf16x8 bh = atp[0][bi], bm = atp[1][bi], bl = atp[2][bi];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int ai = cidx(m * 32 + l32, 2 * ks + half);
        acc[m] = mfma_x6(dyp[0][ai], dyp[1][ai], dyp[2][ai], bh, bm, bl, acc[m]);
      }
    }
    __syncthreads();  // atp / dyp consumed
    // the prefetched dy (tile + 1) and G (tile + 2) go to LDS before the build, so their
    // registers are free while it runs (no packed f32: the scalar build needs the room)
    stage_dy();                 // tile + 1
    stage_g(gl[tile & 1]);      // tile + 2 (G of tile: built last iteration)
    build(gl[(tile + 1) & 1]);  // tile + 1 (G staged one iteration ago, weights in wc)
    fetch_w(tile + 2);          // into wc, consumed by the next iteration's build
    __syncthreads();
  }
  const long long cc16 = (long long)c0 * kW + col;
  if (ones_col >= 0 && col == ones_col) {
    float* bd = dbias + (long long)split * O;  // slab index when the rows are split
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) bd[i * 32 + (e & 3) + 8 * (e >> 2) + 4 * half] = acc[i][e];
  }
  if (cc16 >= c16) return;
  float* dst = dwl + (long long)split * O * c16;  // slab index when the rows are split
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int o = i * 32 + (e & 3) + 8 * (e >> 2) + 4 * half;
      dst[o * c16 + cc16] = acc[i][e];
    }
}

// ------------------------------------------------------------------------------- host
struct Plan {
  int r, c, nch, c8, tm, rt;  // tm: forward tile rows
  int ks, cps;                 // fwd channel splits / chunks per split
  int bks, bcps;               // bwd-data channel splits (32-row tiles)
  int rs, rps, xcd, wgs;       // bwd-weight row splits, rows per split, XCD map, grid
  size_t fwd_slab, fwd_wsf, dgr, dwt_slab, dwl_slab, wlt;  // bytes
};

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

inline int km_of(int k) { return k <= 9 ? 9 : 16; }

// CUs the weight half fills when it runs on its own stream (kdpc_pointconv_bwd_weight): all of
// them.  Its workgroups hold 90-158 KB of LDS each, one per CU, so it shuts the main stream's
// kernels out until it ends, but capping its grid measured slower (round 4 A/B: 256 CUs
// 16.26 ms per train step, 192 16.77, 128 17.36, 64 20.8): the side work is the long pole.
inline int side_weight_cus() { return kCUs; }

// workgroups the backward data kernel's channel splits aim for (round-4 A/B, tiled data half:
// 512 beats 256 / 1024 / 2048 at flow2, 112 vs 125-135 us, and ties at flow0 / flow1)
inline int bwd_target_wg() { return kTargetWG; }

// every gathered table must be addressable by a 31-bit byte offset (buffer loads)

inline bool fits_buffers(long long b, long long n, long long s, int d) {
  const long long lim = 1ll << 31;
  return b * n * 4 * std::max(d, 3) < lim && b * s * 12 < lim;
}

void channel_split(int nch, int tiles, int* ks, int* cps, int target = kTargetWG) {
  int s = tiles > 0 ? std::min(nch, std::max(1, divup(target, tiles))) : 1;
  *cps = divup(nch, s);
  *ks = divup(nch, *cps);
}

bool plan_of(int b, int s, int k, int d, int o, Plan* p, int wcus = kCUs) {
  if (b < 0 || s < 0 || k < 1 || k > kKMax || d < 0 || !(o == 64 || o == 128 || o == 256))
    return false;
  const long long r = (long long)b * s;
  if (r > (1ll << 26) || (long long)(3 + d) * kW * o > (1ll << 30)) return false;
  p->r = (int)r;
  p->c = 3 + d;
  p->nch = divup(p->c, kCC);
  p->c8 = p->nch * kCC;
  p->tm = km_of(k) <= 9 ? 64 : 32;
  p->rt = divup(p->r, p->tm);
  channel_split(p->nch, p->rt, &p->ks, &p->cps);
  channel_split(p->nch, divup(p->r, 32), &p->bks, &p->bcps, bwd_target_wg());
  // bwd-weight row splits: every (chunk, split) workgroup carries the same MFMA work and
  // all of them are resident at once (one 512-thread workgroup per CU: the pipelined kernel
  // double-buffers its operands in 90-158 KB of LDS), so the kernel takes (workgroups on the
  // busiest CU) x (tiles per split); pick the split count minimising that.  Multiples of 8
  // keep the XCD mapping (a split's chunks share its dy / wt rows in one L2) unless >6%
  // slower.  (round 1, unpipelined: 2-3 co-resident workgroups per CU ran slower than one.)
  // (O <= 128: 256-thread workgroups, two per CU -- wgt_threads)
  const int trw = wgt_threads(o) == 256 ? 32 : (km_of(k) <= 9 ? (o == 256 ? 32 : 64) : 32);
  wcus *= wgt_threads(o) == 256 ? 2 : 1;
  const int t32 = std::max(1, divup(p->r, trw));
  const int cap = std::max(1, std::min(t32, wcus / p->nch));
  auto cost = [&](int rs) {
    const int rps = divup(t32, rs);
    const int per = divup(p->nch * divup(t32, rps), wcus);
    return (double)per * (rps + 2);  // + the pipeline's prologue
  };
  int best = 1, best8 = 0;
  for (int rs = 1; rs <= cap; ++rs) {
    if (cost(rs) < cost(best)) best = rs;
    if (rs % 8 == 0 && (best8 == 0 || cost(rs) < cost(best8))) best8 = rs;
  }
  const int rs = (best8 > 0 && cost(best8) <= 1.06 * cost(best)) ? best8 : best;
  p->rps = divup(t32, rs) * trw;
  p->rs = std::max(1, divup(p->r, p->rps));
  p->xcd = 1;
  p->wgs = divup(p->nch * p->rs, 8) * 8;  // XCD fill: a multiple of 8 workgroups
  const size_t c16 = (size_t)p->c * kW;
  p->fwd_slab = p->ks > 1 ? align256((size_t)p->ks * p->r * o * 4) : 0;
  // the forward's B planes (pc_swizzle_fwd3_kernel): (nch, O/32, 8 K-steps, 3 planes) x 1 KB
  p->fwd_wsf = align256((size_t)p->nch * (o / 32) * 8 * 3 * 64 * 16);
  // dG rows: one per pair, or (tiled) one per (32-row tile, destination): at most 32K per
  // tile, tiles per batch element
  p->dgr = align256((size_t)b * divup(s, 32) * 32 * k * p->c8 * 4);
  p->dwt_slab = p->bks > 1 ? align256((size_t)p->bks * p->r * k * kW * 4) : 0;
  p->dwl_slab = p->rs > 1 ? align256((size_t)p->rs * o * c16 * 4) : 0;
  // swizzled B (three bf16 planes, 6 B per element), padded to whole chunks
  p->wlt = align256((size_t)p->nch * kNC * o * 6);
  return true;
}

hipError_t slab_sum(int nslabs, long long len, const float* slab, const float* bias, int o,
                    float* dst, hipStream_t st) {
  const int grid = (int)std::min<long long>(divupll(len, 256), 4096);
  hipLaunchKernelGGL(pc_slab_sum_kernel, dim3(grid), dim3(256), 0, st, nslabs, len, slab, bias, o,
                     dst);
  return hipGetLastError();
}

// workspace: [B planes of wl (p.fwd_wsf) | channel-split slabs (p.fwd_slab)]
template <int O, int KM>
hipError_t fwd_launch(const Geo& g, const Plan& p, const float* wt, const float* wl,
                      const float* bias, float* y, char* ws, hipStream_t st) {
  bf16x8* wsf = reinterpret_cast<bf16x8*>(ws);
  float* slab = reinterpret_cast<float*>(ws + p.fwd_wsf);
  float* sl = p.ks > 1 ? slab : nullptr;
  const long long nsw = (long long)g.nch * (O / 32) * 8 * 64;
  hipLaunchKernelGGL(pc_swizzle_fwd3_kernel, dim3((unsigned)divupll(nsw, 256)), dim3(256), 0, st,
                     O, g.c * kW, g.nch, wl, wsf);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (g.trow) {  // tiled plan: exact-K only (the estimators' K = 9)
    const unsigned rt = (unsigned)divup(g.ntrow, p.tm);
    hipLaunchKernelGGL((pc_fwd_kernel<O, KM, true, true>), dim3(rt, p.ks), dim3(256), 0, st, g,
                       wt, wsf, bias, y, sl, p.cps);
  } else if (g.k == KM) {
    hipLaunchKernelGGL((pc_fwd_kernel<O, KM, true, false>), dim3(p.rt, p.ks), dim3(256), 0, st, g,
                       wt, wsf, bias, y, sl, p.cps);
  } else {
    hipLaunchKernelGGL((pc_fwd_kernel<O, KM, false, false>), dim3(p.rt, p.ks), dim3(256), 0, st,
                       g, wt, wsf, bias, y, sl, p.cps);
  }
  e = hipGetLastError();
  if (e != hipSuccess || p.ks == 1) return e;
  return slab_sum(p.ks, (long long)p.r * O, slab, bias, O, y, st);
}

// Data kernel choice.  The pipelined kernel (chunk ch+1's MFMAs interleaved with chunk ch's
// pair work) for K <= 9: with every wave carrying the same pair work (one whole pair + one
// left-over item) it is faster there (flow0, B=8, N=8192: 534 vs 584 us per launch, round 2);
// for K = 16 (two whole pairs per thread) the two are within 2 % and the unpipelined kernel
// stays.  Round-1 note: the pipelined kernel without the balanced pair mapping made every
// wave run two pairs and did not pay (1199 vs 1191 us).
template <int KM>
constexpr bool bwd_pipe_enabled() { return KM <= 9; }

// Data half of the backward: dxyz, dfeats, dcenter, dwt (workspace: dG rows | dwt slabs | -
// | swizzled wl).
template <int O, int KM>
hipError_t bwd_data_launch(const Geo& g, const Plan& p, int b, const float* wt, const float* wl,
                           const float* dy, const int* offsets, float* dxyz, float* dfeats,
                           float* dcenter, float* dwt, char* ws, hipStream_t st) {
  float* dgr = reinterpret_cast<float*>(ws);
  float* dwt_slab = reinterpret_cast<float*>(ws + p.dgr);
  char* wsb = ws + p.dgr + p.dwt_slab + p.dwl_slab;  // swizzled wl (p.wlt bytes)
  const int c16 = g.c * kW;
  // the pipelined kernels store dG through a buffer resource (31-bit byte offsets)
  const bool dg31 = (long long)p.r * g.k * p.c8 * 4 < (1ll << 31);
  const long long rk = (long long)p.r * g.k;
  // wl as bf16 B planes (every data kernel multiplies dA = dy wl with mfma_x6)
  bf16x8* wsw = reinterpret_cast<bf16x8*>(wsb);
  const long long nsw = (long long)g.nch * 4 * (O / 16) * 64;
  hipLaunchKernelGGL(pc_swizzle_bwd3_kernel, dim3((unsigned)divupll(nsw, 256)), dim3(256), 0, st,
                     O, c16, g.nch, wl, wsw);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (g.trow)  // tiled plan (checked by the entry point: dG partial rows fit 31 bits)
    hipLaunchKernelGGL((pc_bwd_data_pipe_kernel<O, KM, true>),
                       dim3((unsigned)((long long)b * divup(g.s, 32)), p.bks), dim3(256), 0, st,
                       g, wt, wsw, dy, dgr, p.bks > 1 ? dwt_slab : dwt, dcenter, p.bcps);
  else if (bwd_pipe_enabled<KM>() && dg31)
    hipLaunchKernelGGL((pc_bwd_data_pipe_kernel<O, KM, false>), dim3(divup(p.r, 32), p.bks),
                       dim3(256), 0, st, g, wt, wsw, dy, dgr, p.bks > 1 ? dwt_slab : dwt, dcenter,
                       p.bcps);
  else
    hipLaunchKernelGGL((pc_bwd_data_kernel<O, KM>), dim3(divup(p.r, bwd_tile_rows<KM>()), p.bks),
                       dim3(bwd_threads<KM>()), 0, st,
                       g, wt, wsw, dy, dgr, p.bks > 1 ? dwt_slab : dwt, dcenter, p.bcps);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (p.bks > 1 && (e = slab_sum(p.bks, rk * kW, dwt_slab, nullptr, 1, dwt, st)) != hipSuccess)
    return e;
  const long long npts = (long long)b * g.n;
  const long long work = npts * (p.c8 / 4);
  hipLaunchKernelGGL(pc_csr_sum_kernel,
                     dim3((unsigned)std::min<long long>(divupll(work, 256), 1 << 20)), dim3(256),
                     0, st, npts, rk, g.c, p.c8, g.d, dgr, offsets, dxyz, dfeats);
  return hipGetLastError();
}

// Weight half: dwl (workspace: its row-split slabs only, dwl_slab bytes).  Reads the same
// G / wt / dy as the data half and nothing it writes, so it may run on another stream.
template <int O, int KM>
hipError_t bwd_weight_launch(const Geo& g, const Plan& p, const float* wt, const float* dy,
                             float* dwl, char* ws, hipStream_t st, float* dbias = nullptr) {
  float* dwl_slab = reinterpret_cast<float*>(ws);
  float* wdst = p.rs > 1 ? dwl_slab : dwl;
  // bias slab after the dwl slabs (kdpc_pointconv_bwd_weight_workspace_bytes)
  float* bias_slab = reinterpret_cast<float*>(ws + p.dwl_slab);
  float* bdst = dbias == nullptr ? nullptr : (p.rs > 1 ? bias_slab : dbias);
  if constexpr (O <= 128) {  // split-bf16 MFMAs, 256 threads (wgt_threads)
    if (g.k == KM)
      hipLaunchKernelGGL((pc_bwd_weight_x6_kernel<O, KM, true>), dim3(p.wgs), dim3(256), 0, st, g,
                         wt, dy, wdst, p.rps, p.rs, p.xcd, bdst);
    else
      hipLaunchKernelGGL((pc_bwd_weight_x6_kernel<O, KM, false>), dim3(p.wgs), dim3(256), 0, st, g,
                         wt, dy, wdst, p.rps, p.rs, p.xcd, bdst);
  } else {
    if (g.k == KM)
      hipLaunchKernelGGL((pc_bwd_weight_kernel<O, KM, true>), dim3(p.wgs), dim3(wgt_threads(O)), 0,
                         st, g, wt, dy, wdst, p.rps, p.rs, p.xcd, bdst);
    else
      hipLaunchKernelGGL((pc_bwd_weight_kernel<O, KM, false>), dim3(p.wgs), dim3(wgt_threads(O)), 0,
                         st, g, wt, dy, wdst, p.rps, p.rs, p.xcd, bdst);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || p.rs == 1) return e;
  if ((e = slab_sum(p.rs, (long long)O * g.c * kW, dwl_slab, nullptr, 1, dwl, st)) != hipSuccess)
    return e;
  return dbias == nullptr ? hipSuccess : slab_sum(p.rs, O, bias_slab, nullptr, 1, dbias, st);
}

template <int O, int KM>
hipError_t bwd_launch(const Geo& g, const Plan& p, int b, const float* wt, const float* wl,
                      const float* dy, const int* offsets, float* dxyz,
                      float* dfeats, float* dcenter, float* dwt, float* dwl, char* ws,
                      hipStream_t st) {
  hipError_t e = bwd_data_launch<O, KM>(g, p, b, wt, wl, dy, offsets, dxyz, dfeats, dcenter, dwt,
                                        ws, st);
  if (e != hipSuccess) return e;
  return bwd_weight_launch<O, KM>(g, p, wt, dy, dwl, ws + p.dgr + p.dwt_slab, st);
}

Geo geo_of(int b, int n, int s, int k, int d, const Plan& p, const float* xyz, const float* center,
           const float* feats, const int* idx) {
  Geo g;
  g.n = n;
  g.s = s;
  g.k = k;
  g.d = d;
  g.c = p.c;
  g.r = p.r;
  g.nch = p.nch;
  g.c8 = p.c8;
  g.bn = b * n;
  g.xyz = xyz;
  g.center = center;
  g.feats = feats;
  g.idx = idx;
  g.rank = nullptr;
  g.trow = g.tpair = g.tsoff = g.tdst = nullptr;
  g.ntrow = 0;
  return g;
}

// instantiate FN<O, KM> for the runtime (o, k)
#define KDPC_PC_DISPATCH(FN, ...)                                                         \
  (km_of(k) == 9                                                                          \
       ? (o == 64 ? FN<64, 9>(__VA_ARGS__)                                                \
                  : (o == 128 ? FN<128, 9>(__VA_ARGS__) : FN<256, 9>(__VA_ARGS__)))       \
       : (o == 64 ? FN<64, 16>(__VA_ARGS__)                                               \
                  : (o == 128 ? FN<128, 16>(__VA_ARGS__) : FN<256, 16>(__VA_ARGS__))))

}  // namespace


KDPC_API int kdpc_pointconv_supported(int k, int d, int o) {
  Plan p;
  return plan_of(1, 1, k, d, o, &p) ? 1 : 0;
}

KDPC_API size_t kdpc_pointconv_fwd_workspace_bytes(int b, int s, int k, int d, int o) {
  Plan p;
  return plan_of(b, s, k, d, o, &p) ? p.fwd_wsf + p.fwd_slab : 0;
}

KDPC_API int kdpc_pointconv_fwd(int b, int n, int s, int k, int d, int o, const float* xyz,
                                const float* center, const float* feats, const int* idx,
                                const float* wt, const float* wl, const float* bias, float* y,
                                void* workspace, size_t workspace_bytes, void* stream) {
  Plan p;
  KDPC_CHECK_ARG(n > 0 && b <= 65535 && plan_of(b, s, k, d, o, &p) && fits_buffers(b, n, s, d));
  if (p.r == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(xyz && center && idx && wt && wl && bias && y && (d == 0 || feats));
  KDPC_CHECK_ARG(workspace && workspace_bytes >= p.fwd_wsf + p.fwd_slab);
  const Geo g = geo_of(b, n, s, k, d, p, xyz, center, feats, idx);
  char* ws = reinterpret_cast<char*>(workspace);
  hipStream_t st = (hipStream_t)stream;
  return (int)KDPC_PC_DISPATCH(fwd_launch, g, p, wt, wl, bias, y, ws, st);
}

KDPC_API size_t kdpc_pointconv_bwd_workspace_bytes(int b, int s, int k, int d, int o) {
  Plan p;
  return plan_of(b, s, k, d, o, &p) ? p.dgr + p.dwt_slab + p.dwl_slab + p.wlt : 0;
}

KDPC_API int kdpc_pointconv_bwd(int b, int n, int s, int k, int d, int o, const float* xyz,
                                const float* center, const float* feats, const int* idx,
                                const float* wt, const float* wl, const float* dy,
                                const int* offsets, const int* rank, float* dxyz, float* dfeats,
                                float* dcenter, float* dwt, float* dwl, void* workspace,
                                size_t workspace_bytes, void* stream) {
  Plan p;
  KDPC_CHECK_ARG(n > 0 && b <= 65535 && plan_of(b, s, k, d, o, &p) && fits_buffers(b, n, s, d));
  hipStream_t st = (hipStream_t)stream;
  if (p.r == 0) {
    hipError_t e = hipSuccess;
    if (dxyz) e = hipMemsetAsync(dxyz, 0, sizeof(float) * b * n * 3, st);
    if (e == hipSuccess && d > 0) e = hipMemsetAsync(dfeats, 0, sizeof(float) * b * n * d, st);
    if (e == hipSuccess) e = hipMemsetAsync(dwl, 0, sizeof(float) * o * p.c * kW, st);
    return (int)e;
  }
  KDPC_CHECK_ARG(xyz && center && idx && wt && wl && dy && offsets && rank && dcenter && dwt &&
                 dwl && (d == 0 || (feats && dfeats)));
  KDPC_CHECK_ARG(workspace && workspace_bytes >= p.dgr + p.dwt_slab + p.dwl_slab + p.wlt);
  Geo g = geo_of(b, n, s, k, d, p, xyz, center, feats, idx);
  g.rank = rank;
  char* ws = reinterpret_cast<char*>(workspace);
  return (int)KDPC_PC_DISPATCH(bwd_launch, g, p, b, wt, wl, dy, offsets, dxyz, dfeats,
                               dcenter, dwt, dwl, ws, st);
}

KDPC_API size_t kdpc_pointconv_bwd_weight_workspace_bytes(int b, int s, int k, int d, int o) {
  Plan p;
  return plan_of(b, s, k, d, o, &p, side_weight_cus())
             ? std::max<size_t>(p.dwl_slab + (p.rs > 1 ? align256((size_t)p.rs * o * 4) : 0), 256)
             : 0;
}

KDPC_API int kdpc_pointconv_bwd_data(int b, int n, int s, int k, int d, int o, const float* xyz,
                                     const float* center, const float* feats, const int* idx,
                                     const float* wt, const float* wl, const float* dy,
                                     const int* offsets, const int* rank, float* dxyz,
                                     float* dfeats, float* dcenter, float* dwt, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  Plan p;
  KDPC_CHECK_ARG(n > 0 && b <= 65535 && plan_of(b, s, k, d, o, &p) && fits_buffers(b, n, s, d));
  hipStream_t st = (hipStream_t)stream;
  if (p.r == 0) {
    hipError_t e = hipSuccess;
    if (dxyz) e = hipMemsetAsync(dxyz, 0, sizeof(float) * b * n * 3, st);
    if (e == hipSuccess && d > 0) e = hipMemsetAsync(dfeats, 0, sizeof(float) * b * n * d, st);
    return (int)e;
  }
  KDPC_CHECK_ARG(xyz && center && idx && wt && wl && dy && offsets && rank && dcenter && dwt &&
                 (d == 0 || (feats && dfeats)));
  KDPC_CHECK_ARG(workspace && workspace_bytes >= p.dgr + p.dwt_slab + p.dwl_slab + p.wlt);
  Geo g = geo_of(b, n, s, k, d, p, xyz, center, feats, idx);
  g.rank = rank;
  char* ws = reinterpret_cast<char*>(workspace);
  return (int)KDPC_PC_DISPATCH(bwd_data_launch, g, p, b, wt, wl, dy, offsets, dxyz, dfeats,
                               dcenter, dwt, ws, st);
}

KDPC_API int kdpc_pointconv_bwd_weight(int b, int n, int s, int k, int d, int o, const float* xyz,
                                       const float* center, const float* feats, const int* idx,
                                       const float* wt, const float* dy, float* dwl,
                                       void* workspace, size_t workspace_bytes, void* stream) {
  Plan p;
  KDPC_CHECK_ARG(n > 0 && b <= 65535 && plan_of(b, s, k, d, o, &p, side_weight_cus()) && fits_buffers(b, n, s, d));
  hipStream_t st = (hipStream_t)stream;
  if (p.r == 0) return (int)hipMemsetAsync(dwl, 0, sizeof(float) * o * p.c * kW, st);
  KDPC_CHECK_ARG(xyz && center && idx && wt && dy && dwl && (d == 0 || feats));
  KDPC_CHECK_ARG(workspace && workspace_bytes >= kdpc_pointconv_bwd_weight_workspace_bytes(b, s, k, d, o));
  const Geo g = geo_of(b, n, s, k, d, p, xyz, center, feats, idx);
  char* ws = reinterpret_cast<char*>(workspace);
  return (int)KDPC_PC_DISPATCH(bwd_weight_launch, g, p, wt, dy, dwl, ws, st);
}

// Tiled backward (tile_plan.hip): offsets = the CSR of the plan's partial-row keys over the
// B*N points (kdpc_csr_build of tkey viewed as (B, ceil(S/32)*32K)), tdst its kdpc_csr_rank.
namespace {
bool tiled_ok(int b, int s, int k, const Plan& p) {
  return (long long)b * divup(s, 32) * 32 * k * p.c8 * 4 < (1ll << 31);
}
}  // namespace

KDPC_API int kdpc_pointconv_bwd_data_tiled(int b, int n, int s, int k, int d, int o,
                                           const float* xyz, const float* center,
                                           const float* feats, const int* idx, const float* wt,
                                           const float* wl, const float* dy, const int* offsets,
                                           const int* trow, const int* tpair, const int* tsoff,
                                           const int* tdst, float* dxyz, float* dfeats,
                                           float* dcenter, float* dwt, void* workspace,
                                           size_t workspace_bytes, void* stream) {
  Plan p;
  KDPC_CHECK_ARG(n > 0 && b <= 65535 && plan_of(b, s, k, d, o, &p) && fits_buffers(b, n, s, d) &&
                 tiled_ok(b, s, k, p));
  if (p.r == 0)
    return kdpc_pointconv_bwd_data(b, n, s, k, d, o, xyz, center, feats, idx, wt, wl, dy, offsets,
                                   nullptr, dxyz, dfeats, dcenter, dwt, workspace,
                                   workspace_bytes, stream);
  KDPC_CHECK_ARG(xyz && center && idx && wt && wl && dy && offsets && trow && tpair && tsoff &&
                 tdst && dcenter && dwt && (d == 0 || (feats && dfeats)));
  KDPC_CHECK_ARG(workspace && workspace_bytes >= p.dgr + p.dwt_slab + p.dwl_slab + p.wlt);
  Geo g = geo_of(b, n, s, k, d, p, xyz, center, feats, idx);
  g.trow = trow, g.tpair = tpair, g.tsoff = tsoff, g.tdst = tdst;
  char* ws = reinterpret_cast<char*>(workspace);
  hipStream_t st = (hipStream_t)stream;
  return (int)KDPC_PC_DISPATCH(bwd_data_launch, g, p, b, wt, wl, dy, offsets, dxyz, dfeats,
                               dcenter, dwt, ws, st);
}

KDPC_API int kdpc_pointconv_bwd_tiled(int b, int n, int s, int k, int d, int o, const float* xyz,
                                      const float* center, const float* feats, const int* idx,
                                      const float* wt, const float* wl, const float* dy,
                                      const int* offsets, const int* trow, const int* tpair,
                                      const int* tsoff, const int* tdst, float* dxyz,
                                      float* dfeats, float* dcenter, float* dwt, float* dwl,
                                      void* workspace, size_t workspace_bytes, void* stream) {
  Plan p;
  KDPC_CHECK_ARG(n > 0 && b <= 65535 && plan_of(b, s, k, d, o, &p) && fits_buffers(b, n, s, d) &&
                 tiled_ok(b, s, k, p));
  KDPC_CHECK_ARG(dwl);
  const int e = kdpc_pointconv_bwd_data_tiled(b, n, s, k, d, o, xyz, center, feats, idx, wt, wl,
                                              dy, offsets, trow, tpair, tsoff, tdst, dxyz, dfeats,
                                              dcenter, dwt, workspace, workspace_bytes, stream);
  if (e != (int)hipSuccess) return e;
  hipStream_t st = (hipStream_t)stream;
  if (p.r == 0) return (int)hipMemsetAsync(dwl, 0, sizeof(float) * o * p.c * kW, st);
  const Geo g = geo_of(b, n, s, k, d, p, xyz, center, feats, idx);
  char* ws = reinterpret_cast<char*>(workspace) + p.dgr + p.dwt_slab;
  return (int)KDPC_PC_DISPATCH(bwd_weight_launch, g, p, wt, dy, dwl, ws, st);
}

// Forward through the backward's tile plan (rows of each 64-row tile = two consecutive
// 32-row plan tiles): same outputs as kdpc_pointconv_fwd, bit for bit.  K must be 9 or 16
// (the exact-K kernels); trow (ntrow = tiles * 32 entries) from kdpc_pc_tile_plan.
KDPC_API int kdpc_pointconv_fwd_tiled(int b, int n, int s, int k, int d, int o, const float* xyz,
                                      const float* center, const float* feats, const int* idx,
                                      const float* wt, const float* wl, const float* bias,
                                      const int* trow, int ntrow, float* y, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  Plan p;
  KDPC_CHECK_ARG(n > 0 && b <= 65535 && plan_of(b, s, k, d, o, &p) && fits_buffers(b, n, s, d));
  KDPC_CHECK_ARG(k == km_of(k) && ntrow >= 0 && ntrow == b * divup(s, 32) * 32);
  if (p.r == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(xyz && center && idx && wt && wl && bias && y && trow && (d == 0 || feats));
  KDPC_CHECK_ARG(workspace && workspace_bytes >= p.fwd_wsf + p.fwd_slab);
  Geo g = geo_of(b, n, s, k, d, p, xyz, center, feats, idx);
  g.trow = trow;
  g.ntrow = ntrow;
  char* ws = reinterpret_cast<char*>(workspace);
  hipStream_t st = (hipStream_t)stream;
  return (int)KDPC_PC_DISPATCH(fwd_launch, g, p, wt, wl, bias, y, ws, st);
}

// Weight half plus the bias gradient (column sums of dy) from the same MFMAs: a padding
// column of A set to 1 (needs C % 8 != 0, i.e. a padding channel in the last chunk).
KDPC_API int kdpc_pointconv_bwd_weight_bias(int b, int n, int s, int k, int d, int o,
                                            const float* xyz, const float* center,
                                            const float* feats, const int* idx, const float* wt,
                                            const float* dy, float* dwl, float* dbias,
                                            void* workspace, size_t workspace_bytes,
                                            void* stream) {
  Plan p;
  KDPC_CHECK_ARG(n > 0 && b <= 65535 && plan_of(b, s, k, d, o, &p, side_weight_cus()) &&
                 fits_buffers(b, n, s, d) && (3 + d) % kCC != 0);
  hipStream_t st = (hipStream_t)stream;
  if (p.r == 0) {
    hipError_t e = hipMemsetAsync(dwl, 0, sizeof(float) * o * p.c * kW, st);
    if (e == hipSuccess) e = hipMemsetAsync(dbias, 0, sizeof(float) * o, st);
    return (int)e;
  }
  KDPC_CHECK_ARG(xyz && center && idx && wt && dy && dwl && dbias && (d == 0 || feats));
  KDPC_CHECK_ARG(workspace &&
                 workspace_bytes >= kdpc_pointconv_bwd_weight_workspace_bytes(b, s, k, d, o));
  const Geo g = geo_of(b, n, s, k, d, p, xyz, center, feats, idx);
  char* ws = reinterpret_cast<char*>(workspace);
  return (int)KDPC_PC_DISPATCH(bwd_weight_launch, g, p, wt, dy, dwl, ws, st, dbias);
}
