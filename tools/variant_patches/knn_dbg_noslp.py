# Diagnostic variant of csrc/knn.hip (never product): knn_cull_kernel<QW,false> checks, as it
# runs, that what it reads is consistent with the inputs (sorted queries vs new_xyz, visited
# refs vs xyz, refs inside their chunk's box) and, for every query that ends with fewer than K
# candidates, counts by brute force how many refs lie under its final threshold and how many
# chunk boxes of its cloud do not contain their refs.  Findings go to a device array read by
# kdpc_knn_dbg_read (tools/knn_race.py dbg=1).
DBG_GLOBALS = r'''
constexpr int kDbgRec = 64;
__device__ unsigned long long g_knn_dbg[8 + kDbgRec * 8];
// counters: [0] query record mismatch, [1] ref vs xyz mismatch, [2] ref outside its chunk box,
// [3] query short of K, [4] chunk boxes not containing their refs (failing clouds), [5] launches
__device__ void dbg_rec(int type, unsigned long long a, unsigned long long b2,
                        unsigned long long c, unsigned long long d, unsigned long long e) {
  const unsigned long long slot = atomicAdd(&g_knn_dbg[type], 1ull);
  const unsigned long long r = atomicAdd(&g_knn_dbg[7], 1ull);
  if (r < kDbgRec && slot < 16) {
    unsigned long long* p = g_knn_dbg + 8 + r * 8;
    p[0] = type; p[1] = a; p[2] = b2; p[3] = c; p[4] = d; p[5] = e;
  }
}
__global__ void dbg_hdr_kernel(unsigned long long* hdr, const float* xyz, const float* nx) {
  if (threadIdx.x == 0) {
    hdr[0] = (unsigned long long)xyz;
    hdr[1] = (unsigned long long)nx;
    atomicAdd(&g_knn_dbg[5], 1ull);
  }
}
constexpr int kBuf = 128;  // candidate slots per query (LDS)
'''

REPL = [
    ("csrc/knn.hip", "constexpr int kBuf = 128;  // candidate slots per query (LDS)\n", DBG_GLOBALS),
    # after the query records are loaded: check them against new_xyz
    ("csrc/knn.hip", """  // the first block of chunk boxes is independent of the seed: in flight during it
""", """  const unsigned long long* dbg_hdr = STATS ? nullptr : evals;
  const float* dbg_x = dbg_hdr ? (const float*)dbg_hdr[0] : nullptr;
  const float* dbg_q = dbg_hdr ? (const float*)dbg_hdr[1] : nullptr;
  if (dbg_hdr) {
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      if (qbase + q >= s) continue;
      bool bad = qid[q] < 0 || qid[q] >= s || w0[q] < 0 || w0[q] >= n;
      if (!bad) {
        const float* p = dbg_q + ((long long)b * s + qid[q]) * 3;
        bad = p[0] != qx[q] || p[1] != qy[q] || p[2] != qz[q];
      }
      if (bad && lane == 0) dbg_rec(0, b, qbase + q, (unsigned)qid[q], (unsigned)w0[q], 0);
    }
  }
  // the first block of chunk boxes is independent of the seed: in flight during it
"""),
    ("csrc/knn.hip", """  seed_thresholds<QW>(n, k, b, qbase, s, qx, qy, qz, qs, w0, rs, thr);
""", """  seed_thresholds<QW>(n, k, b, qbase, s, qx, qy, qz, qs, w0, rs, thr);
  float seed[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) seed[q] = thr[q];
"""),
    # every visited chunk: refs vs xyz, refs inside the chunk's box
    ("csrc/knn.hip", """    while (true) {
      if (STATS) ++visits;
      const bool valid = j < n;
""", """    while (true) {
      if (STATS) ++visits;
      const bool valid = j < n;
      if (dbg_hdr) {
        bool bad = false;
        if (valid) {
          bad = gi < 0 || gi >= n;
          if (!bad) {
            const float* p = dbg_x + ((long long)b * n + gi) * 3;
            bad = p[0] != r.x || p[1] != r.y || p[2] != r.z || r.w != sqnorm3(r.x, r.y, r.z);
          }
        }
        const unsigned long long bm = __ballot(bad);
        if (bm && lane == __ffsll((long long)bm) - 1) dbg_rec(1, b, cc, j, (unsigned)gi, 0);
        const int src = cc - cbase;
        const float blx = __shfl(lo.x, src), bly = __shfl(lo.y, src), blz = __shfl(lo.z, src);
        const float bhx = __shfl(hi.x, src), bhy = __shfl(hi.y, src), bhz = __shfl(hi.z, src);
        const float bw = __shfl(lo.w, src);
        const bool out = valid && (r.x < blx || r.x > bhx || r.y < bly || r.y > bhy ||
                                   r.z < blz || r.z > bhz || r.w > bw);
        const unsigned long long om = __ballot(out);
        if (om && lane == __ffsll((long long)om) - 1) dbg_rec(2, b, cc, j, (unsigned)gi, 0);
      }
"""),
    # queries short of K: brute force under the final threshold + box audit of the cloud
    ("csrc/knn.hip", """  float ld[QW];
  int li[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) {
    const float2 v = lane < cnt[q] ? cand_buf[wave][q][lane]""", """  if (dbg_hdr) {
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      if (qbase + q >= s || cnt[q] >= k) continue;
      int under = 0, under_seed = 0;
      for (int j0 = 0; j0 < n; j0 += kWave) {
        const int jj = j0 + lane;
        const float4 r = rb[jj < n ? jj : 0];
        const float d = sqdist_fast(qx[q], qy[q], qz[q], qs[q], r.x, r.y, r.z, r.w);
        under += __popcll(__ballot(jj < n && d < thr[q]));
        under_seed += __popcll(__ballot(jj < n && d < seed[q]));
      }
      int badbox = 0;
      for (int c0 = 0; c0 < nch; ++c0) {
        const int jj = c0 * kWave + lane;
        const float4 r = rb[jj < n ? jj : c0 * kWave];
        const float4 blo = cb[2 * c0], bhi = cb[2 * c0 + 1];
        const bool out = jj < n && (r.x < blo.x || r.x > bhi.x || r.y < blo.y || r.y > bhi.y ||
                                    r.z < blo.z || r.z > bhi.z || r.w > blo.w);
        badbox += __ballot(out) ? 1 : 0;
      }
      if (lane == 0) {
        dbg_rec(3, ((unsigned long long)b << 32) | (unsigned)(qbase + q), (unsigned)cnt[q],
                ((unsigned long long)(unsigned)under << 32) | (unsigned)under_seed,
                ((unsigned long long)__float_as_uint(seed[q]) << 32) | __float_as_uint(thr[q]),
                (unsigned)badbox);
        if (badbox) atomicAdd(&g_knn_dbg[4], (unsigned long long)badbox);
      }
    }
  }
  float ld[QW];
  int li[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) {
    const float2 v = lane < cnt[q] ? cand_buf[wave][q][lane]"""),
    # workspace: a 256-byte header for the input pointers
    ("csrc/knn.hip", """  int* qwin;
  size_t bytes;
};""", """  int* qwin;
  unsigned long long* hdr;
  size_t bytes;
};"""),
    ("csrc/knn.hip", """  w.qwin = reinterpret_cast<int*>(take(sizeof(int) * (size_t)b * s));
""", """  w.qwin = reinterpret_cast<int*>(take(sizeof(int) * (size_t)b * s));
  w.hdr = reinterpret_cast<unsigned long long*>(take(256));
"""),
    ("csrc/knn.hip", """  else
    hipLaunchKernelGGL((knn_cull_kernel<QW, false>), grid, dim3(256), 0, st, n, s, k, idx, dist,
                       w.rs, w.ri, w.cbox, w.qrec, w.qwin, evals);""", """  else {
    hipLaunchKernelGGL(dbg_hdr_kernel, dim3(1), dim3(64), 0, st, w.hdr, xyz, new_xyz);
    hipLaunchKernelGGL((knn_cull_kernel<QW, false>), grid, dim3(256), 0, st, n, s, k, idx, dist,
                       w.rs, w.ri, w.cbox, w.qrec, w.qwin, w.hdr);
  }"""),
    ("csrc/knn.hip", """// Scratch bytes for kdpc_knn_point_ws;""", """KDPC_API int kdpc_knn_dbg_read(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_knn_dbg), sizeof(g_knn_dbg));
  if (e == hipSuccess && reset) {
    static unsigned long long zero[8 + kDbgRec * 8] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_knn_dbg), zero, sizeof(zero));
  }
  return (int)e;
}

// Scratch bytes for kdpc_knn_point_ws;"""),
]

REPL.append(("build_native.py", 'EXTRA_FLAGS = {"cost_volume.hip": ["-fno-slp-vectorize"]}',
             'EXTRA_FLAGS = {"cost_volume.hip": ["-fno-slp-vectorize"], "knn.hip": ["-fno-slp-vectorize"]}'))
