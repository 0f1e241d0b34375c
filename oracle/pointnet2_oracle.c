/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into or called by the product
 * path (kd-pointcloud_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / CPU baseline.
 *
 * Plain-C CPU restatement of the reference's pointnet2 CUDA extension
 * (yunminjin2/KD-PointCloud, pointnet2/src/{sampling,ball_query,group_points,interpolate}_gpu.cu) plus the torch-side kNN of
 * pointconv_util.py.  Each function cites the reference lines it follows.
 *
 * Parity status:
 *   - The reference CUDA extension cannot be built or run here (no nvcc, no GPU;
 *     the only binary is a Windows sm_75 .pyd).  There are no reference tests or
 *     golden vectors for these kernels.  The integer-index kernels (FPS,
 *     ball_query, three_nn) are therefore restated literally, including the
 *     thread-strided FPS scan and its shared-memory tree reduction.  The only
 *     unpinned detail is the FMA contraction of `dx*dx + dy*dy + dz*dz` chosen by
 *     nvcc -O2 (fmad=true); we use fmaf(dz,dz,fmaf(dy,dy,dx*dx)), which is what the
 *     LLVM contraction rule produces for the identical source (checked on hipcc).
 *   - square_distance/knn restate pointconv_util.py:73-107 and are pinned against
 *     the reference Python itself (tests/golden, made by oracle/make_fixtures.py).
 *
 * Build: oracle/Makefile  ->  oracle/lib/libpointnet2_oracle.so
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>


/* reference: pointnet2/src/cuda_utils.h:10-14 */
int oracle_opt_n_threads(int work_size) {
    const int pow_2 = (int)(log((double)work_size) / log(2.0));
    int v = 1 << pow_2;
    if (v > 1024) v = 1024;
    if (v < 1) v = 1;
    return v;
}

/* nvcc -O2 contraction of (x2-x1)^2 + (y2-y1)^2 + (z2-z1)^2 */
static inline float dist3(float x1, float y1, float z1, float x2, float y2, float z2) {
    float dx = x2 - x1, dy = y2 - y1, dz = z2 - z1;
    return fmaf(dz, dz, fmaf(dy, dy, dx * dx));
}

/* reference: sampling_gpu.cu:93-209 (kernel), :211-253 (launcher), sampling.cpp:38-49,
 * pointnet2_utils.py:10-36 (temp = 1e10).  Literal simulation of the block:
 * T threads scan k = t, t+T, ...; then the shared-memory tree (__update, :86-91). */
void oracle_furthest_point_sampling(int b, int n, int m, const float *dataset,
                                    float *temp, int *idxs) {
    if (m <= 0) return;
    const int T = oracle_opt_n_threads(n);
    float *dists = (float *)malloc(sizeof(float) * T);
    int *dists_i = (int *)malloc(sizeof(int) * T);
    for (int bi = 0; bi < b; ++bi) {
        const float *ds = dataset + (size_t)bi * n * 3;
        float *tp = temp + (size_t)bi * n;
        int *ix = idxs + (size_t)bi * m;
        int old = 0;
        ix[0] = old;
        for (int j = 1; j < m; ++j) {
            const float x1 = ds[old * 3 + 0], y1 = ds[old * 3 + 1], z1 = ds[old * 3 + 2];
            for (int tid = 0; tid < T; ++tid) {
                int besti = 0;
                float best = -1.f;
                for (int k = tid; k < n; k += T) {
                    float d = dist3(x1, y1, z1, ds[k * 3 + 0], ds[k * 3 + 1], ds[k * 3 + 2]);
                    float d2 = fminf(d, tp[k]);
                    tp[k] = d2;
                    besti = d2 > best ? k : besti;
                    best = d2 > best ? d2 : best;
                }
                dists[tid] = best;
                dists_i[tid] = besti;
            }
            for (int s = T / 2; s >= 1; s >>= 1) {
                for (int tid = 0; tid < s; ++tid) {
                    const float v1 = dists[tid], v2 = dists[tid + s];
                    const int i1 = dists_i[tid], i2 = dists_i[tid + s];
                    dists[tid] = fmaxf(v1, v2);
                    dists_i[tid] = v2 > v1 ? i2 : i1;
                }
            }
            old = dists_i[0];
            ix[j] = old;
        }
    }
    free(dists);
    free(dists_i);
}

/* reference: sampling_gpu.cu:8-24 */
void oracle_gather_points(int b, int c, int n, int m, const float *points, const int *idx,
                          float *out) {
    for (int bi = 0; bi < b; ++bi)
        for (int ci = 0; ci < c; ++ci)
            for (int p = 0; p < m; ++p)
                out[((size_t)bi * c + ci) * m + p] =
                    points[((size_t)bi * c + ci) * n + idx[(size_t)bi * m + p]];
}

/* reference: sampling_gpu.cu:46-63 (atomicAdd scatter).  Oracle accumulates in
 * ascending position order (the reference's atomic order is unspecified). */
void oracle_gather_points_grad(int b, int c, int n, int m, const float *grad_out,
                               const int *idx, float *grad_points) {
    for (int bi = 0; bi < b; ++bi)
        for (int ci = 0; ci < c; ++ci)
            for (int p = 0; p < m; ++p)
                grad_points[((size_t)bi * c + ci) * n + idx[(size_t)bi * m + p]] +=
                    grad_out[((size_t)bi * c + ci) * m + p];
}

/* reference: ball_query_gpu.cu:9-45; idx pre-zeroed by pointnet2_utils.py:218 */
void oracle_ball_query(int b, int n, int m, float radius, int nsample, const float *new_xyz,
                       const float *xyz, int *idx) {
    const float radius2 = radius * radius;
    for (int bi = 0; bi < b; ++bi)
        for (int p = 0; p < m; ++p) {
            const float *q = new_xyz + ((size_t)bi * m + p) * 3;
            const float *x = xyz + (size_t)bi * n * 3;
            int *o = idx + ((size_t)bi * m + p) * nsample;
            int cnt = 0;
            for (int k = 0; k < n; ++k) {
                float d2 = dist3(x[k * 3 + 0], x[k * 3 + 1], x[k * 3 + 2], q[0], q[1], q[2]);
                if (d2 < radius2) {
                    if (cnt == 0)
                        for (int l = 0; l < nsample; ++l) o[l] = k;
                    o[cnt] = k;
                    ++cnt;
                    if (cnt >= nsample) break;
                }
            }
        }
}

/* reference: group_points_gpu.cu:47-66 */
void oracle_group_points(int b, int c, int n, int npoints, int nsample, const float *points,
                         const int *idx, float *out) {
    const size_t sk = (size_t)npoints * nsample;
    for (int bi = 0; bi < b; ++bi)
        for (int ci = 0; ci < c; ++ci)
            for (size_t p = 0; p < sk; ++p)
                out[((size_t)bi * c + ci) * sk + p] =
                    points[((size_t)bi * c + ci) * n + idx[(size_t)bi * sk + p]];
}

/* reference: group_points_gpu.cu:8-25; sequential ascending (s,k) accumulation */
void oracle_group_points_grad(int b, int c, int n, int npoints, int nsample,
                              const float *grad_out, const int *idx, float *grad_points) {
    const size_t sk = (size_t)npoints * nsample;
    for (int bi = 0; bi < b; ++bi)
        for (int ci = 0; ci < c; ++ci)
            for (size_t p = 0; p < sk; ++p)
                grad_points[((size_t)bi * c + ci) * n + idx[(size_t)bi * sk + p]] +=
                    grad_out[((size_t)bi * c + ci) * sk + p];
}

/* reference: interpolate_gpu.cu:9-52 (double running bests, strict <) */
void oracle_three_nn(int b, int n, int m, const float *unknown, const float *known, float *dist2,
                     int *idx) {
    for (int bi = 0; bi < b; ++bi)
        for (int p = 0; p < n; ++p) {
            const float *u = unknown + ((size_t)bi * n + p) * 3;
            const float *kn = known + (size_t)bi * m * 3;
            double best1 = 1e40, best2 = 1e40, best3 = 1e40;
            int besti1 = 0, besti2 = 0, besti3 = 0;
            for (int k = 0; k < m; ++k) {
                float d = dist3(kn[k * 3 + 0], kn[k * 3 + 1], kn[k * 3 + 2], u[0], u[1], u[2]);
                if (d < best1) {
                    best3 = best2; besti3 = besti2;
                    best2 = best1; besti2 = besti1;
                    best1 = d; besti1 = k;
                } else if (d < best2) {
                    best3 = best2; besti3 = besti2;
                    best2 = d; besti2 = k;
                } else if (d < best3) {
                    best3 = d; besti3 = k;
                }
            }
            float *o = dist2 + ((size_t)bi * n + p) * 3;
            int *oi = idx + ((size_t)bi * n + p) * 3;
            o[0] = (float)best1; o[1] = (float)best2; o[2] = (float)best3;
            oi[0] = besti1; oi[1] = besti2; oi[2] = besti3;
        }
}

/* reference: interpolate_gpu.cu:77-97 */
void oracle_three_interpolate(int b, int c, int m, int n, const float *points, const int *idx,
                              const float *weight, float *out) {
    for (int bi = 0; bi < b; ++bi)
        for (int ci = 0; ci < c; ++ci)
            for (int p = 0; p < n; ++p) {
                const float *w = weight + ((size_t)bi * n + p) * 3;
                const int *ix = idx + ((size_t)bi * n + p) * 3;
                const float *pt = points + ((size_t)bi * c + ci) * m;
                out[((size_t)bi * c + ci) * n + p] =
                    fmaf(w[2], pt[ix[2]], fmaf(w[1], pt[ix[1]], w[0] * pt[ix[0]]));
            }
}

/* reference: interpolate_gpu.cu:120-142; sequential ascending (n, j) accumulation */
void oracle_three_interpolate_grad(int b, int c, int n, int m, const float *grad_out,
                                   const int *idx, const float *weight, float *grad_points) {
    for (int bi = 0; bi < b; ++bi)
        for (int ci = 0; ci < c; ++ci)
            for (int p = 0; p < n; ++p) {
                const float g = grad_out[((size_t)bi * c + ci) * n + p];
                const float *w = weight + ((size_t)bi * n + p) * 3;
                const int *ix = idx + ((size_t)bi * n + p) * 3;
                float *gp = grad_points + ((size_t)bi * c + ci) * m;
                for (int j = 0; j < 3; ++j) gp[ix[j]] += g * w[j];
            }
}

/* reference: pointconv_util.py:73-94 square_distance.
 *   dist  = -2 * (src @ dst^T)         (3-term dot as a k-ordered fma chain)
 *   dist += sum(src**2, -1)            ((x*x + y*y) + z*z, separately rounded)
 *   dist += sum(dst**2, -1)                                                         */
static inline float sqnorm3(const float *p) {
    float x2 = p[0] * p[0], y2 = p[1] * p[1], z2 = p[2] * p[2];
    return (x2 + y2) + z2;
}
static inline float sqdist_expanded(const float *q, float sq, const float *r, float sr) {
    float dot = fmaf(q[2], r[2], fmaf(q[1], r[1], q[0] * r[0]));
    float d = -2.f * dot;
    d = d + sq;
    d = d + sr;
    return d;
}

void oracle_square_distance(int b, int s, int n, const float *src, const float *dst, float *out) {
    for (int bi = 0; bi < b; ++bi)
        for (int i = 0; i < s; ++i) {
            const float *q = src + ((size_t)bi * s + i) * 3;
            const float sq = sqnorm3(q);
            for (int k = 0; k < n; ++k) {
                const float *r = dst + ((size_t)bi * n + k) * 3;
                out[((size_t)bi * s + i) * n + k] = sqdist_expanded(q, sq, r, sqnorm3(r));
            }
        }
}

/* reference: pointconv_util.py:96-107 knn_point(nsample, xyz, new_xyz): the nsample
 * smallest square_distance entries of each query.  torch.topk(sorted=False) leaves the
 * order and exact-tie choice unspecified; the oracle fixes both: ascending by
 * (distance, index).  idx is (B,S,K) int32; dist (optional) is (B,S,K) f32. */
typedef struct { float d; int i; } kv_t;
static int kv_cmp(const void *a, const void *b) {
    const kv_t *x = (const kv_t *)a, *y = (const kv_t *)b;
    if (x->d < y->d) return -1;
    if (x->d > y->d) return 1;
    return (x->i > y->i) - (x->i < y->i);
}
void oracle_knn(int b, int n, int s, int k, const float *xyz, const float *new_xyz, int *idx,
                float *dist) {
    kv_t *buf = (kv_t *)malloc(sizeof(kv_t) * (size_t)n);
    float *sr = (float *)malloc(sizeof(float) * (size_t)n);
    for (int bi = 0; bi < b; ++bi) {
        const float *x = xyz + (size_t)bi * n * 3;
        for (int j = 0; j < n; ++j) sr[j] = sqnorm3(x + j * 3);
        for (int i = 0; i < s; ++i) {
            const float *q = new_xyz + ((size_t)bi * s + i) * 3;
            const float sq = sqnorm3(q);
            for (int j = 0; j < n; ++j) {
                buf[j].d = sqdist_expanded(q, sq, x + j * 3, sr[j]);
                buf[j].i = j;
            }
            qsort(buf, (size_t)n, sizeof(kv_t), kv_cmp);
            for (int t = 0; t < k; ++t) {
                idx[((size_t)bi * s + i) * k + t] = t < n ? buf[t].i : 0;
                if (dist) dist[((size_t)bi * s + i) * k + t] = t < n ? buf[t].d : INFINITY;
            }
        }
    }
    free(buf);
    free(sr);
}
