/*
 * kdpc.h — C ABI of kd-pointcloud_amd's MI355X (gfx950) point-cloud kernels.
 *
 * Drop-in boundary for the reference's native extension `pointnet2_cuda`
 * (yunminjin2/KD-PointCloud pointnet2/src/pointnet2_api.cpp:10-24) and for the
 * torch-side kNN of pointconv_util.py.  Plain pointers and sizes only:
 *   - every pointer is DEVICE memory (hipMalloc / a torch-ROCm tensor's data_ptr());
 *   - float = f32, int = int32; layouts are the reference's (contiguous, row-major);
 *   - `stream` is a hipStream_t (NULL = default stream); every call is asynchronous on it,
 *     never synchronises the host, and allocates nothing (except the reference-shaped
 *     *_grad entry points, which take a stream-ordered temporary; their *_ws variants
 *     take a caller workspace instead);
 *   - return value is a hipError_t code (0 = hipSuccess).  Invalid sizes/pointers return
 *     hipErrorInvalidValue (1) without launching.  The reference instead printed and
 *     called exit(-1) on launch failure (e.g. sampling_gpu.cu:39-43).
 *
 * Outputs follow the reference's in-place contract (caller allocates), with these
 * documented strengthenings: ball_query writes every slot (the reference relied on the
 * caller's .zero_()), and every *_grad overwrites grad_points (the reference accumulated
 * into a caller-zeroed buffer with atomicAdd) with a deterministic sum.
 */
#ifndef KDPC_H_
#define KDPC_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* sha256 (hex) of the sources this library was built from (kd-pointcloud_amd/build_native.py
 * embeds it; the Python loader refuses a library whose id does not match its sources). */
const char *kdpc_build_id(void);

/* ---- sampling -------------------------------------------------------------------------- */

/* Replaces furthest_point_sampling_wrapper(b, n, m, points, temp, idx)
 * (pointnet2/src/sampling.cpp:38-49; kernel sampling_gpu.cu:93-209).
 * points (B,N,3), temp (B,N) scratch pre-filled by the caller (reference: 1e10) and left
 * holding the final min-distances, idx (B,M) out.  Bit-exact indices incl. tie-break.
 * Requires N < 2^22. */
int kdpc_furthest_point_sampling(int b, int n, int m, const float *points, float *temp, int *idx,
                                 void *stream);

/* The reference's block-size rule opt_n_threads (pointnet2/src/cuda_utils.h:10-14). */
int kdpc_opt_n_threads(int n);

/* Replaces gather_points_wrapper(b, c, n, npoints, points, idx, out)
 * (sampling.cpp:11-22; kernel sampling_gpu.cu:8-24).  points (B,C,N), idx (B,M), out (B,C,M). */
int kdpc_gather_points(int b, int c, int n, int npoints, const float *points, const int *idx,
                       float *out, void *stream);

/* Replaces gather_points_grad_wrapper(b, c, n, npoints, grad_out, idx, grad_points)
 * (sampling.cpp:25-35; kernel sampling_gpu.cu:46-63).  Overwrites grad_points (B,C,N) with a
 * deterministic sum.  Scratch: a stream-ordered temporary (hipMallocAsync on `stream`). */
int kdpc_gather_points_grad(int b, int c, int n, int npoints, const float *grad_out,
                            const int *idx, float *grad_points, void *stream);

/* Scratch bytes of the *_grad_ws entry points for an index of B x P values in [0, N)
 * (gather: P = npoints; group: P = npoints*nsample; three_interpolate: P = 3N, N -> M). */
size_t kdpc_grad_workspace_bytes(int b, int n, int p);

/* The three reference-shaped backward entry points with a caller-owned workspace (no
 * allocation at all: graph-capture safe). */
int kdpc_gather_points_grad_ws(int b, int c, int n, int npoints, const float *grad_out,
                               const int *idx, float *grad_points, void *workspace,
                               size_t workspace_bytes, void *stream);
int kdpc_group_points_grad_ws(int b, int c, int n, int npoints, int nsample,
                              const float *grad_out, const int *idx, float *grad_points,
                              void *workspace, size_t workspace_bytes, void *stream);
int kdpc_three_interpolate_grad_ws(int b, int c, int n, int m, const float *grad_out,
                                   const int *idx, const float *weight, float *grad_points,
                                   void *workspace, size_t workspace_bytes, void *stream);

/* ---- grouping -------------------------------------------------------------------------- */

/* Replaces ball_query_wrapper(b, n, m, radius, nsample, new_xyz, xyz, idx)
 * (ball_query.cpp:16-28; kernel ball_query_gpu.cu:9-45).  new_xyz (B,M,3), xyz (B,N,3),
 * idx (B,M,nsample) out.  Bit-exact. */
int kdpc_ball_query(int b, int n, int m, float radius, int nsample, const float *new_xyz,
                    const float *xyz, int *idx, void *stream);

/* Replaces group_points_wrapper(b, c, n, npoints, nsample, points, idx, out)
 * (group_points.cpp:27-38; kernel group_points_gpu.cu:47-66).
 * points (B,C,N), idx (B,npoints,nsample), out (B,C,npoints,nsample). */
int kdpc_group_points(int b, int c, int n, int npoints, int nsample, const float *points,
                      const int *idx, float *out, void *stream);

/* Replaces group_points_grad_wrapper(b, c, n, npoints, nsample, grad_out, idx, grad_points)
 * (group_points.cpp:11-24; kernel group_points_gpu.cu:8-25).  Overwrites grad_points (B,C,N).
 * Scratch: a stream-ordered temporary; kdpc_group_points_grad_ws takes a caller buffer. */
int kdpc_group_points_grad(int b, int c, int n, int npoints, int nsample, const float *grad_out,
                           const int *idx, float *grad_points, void *stream);

/* ---- interpolation --------------------------------------------------------------------- */

/* Replaces three_nn_wrapper(b, n, m, unknown, known, dist2, idx)
 * (interpolate.cpp:14-24; kernel interpolate_gpu.cu:9-52).  unknown (B,N,3), known (B,M,3),
 * dist2 (B,N,3) squared distances, idx (B,N,3). */
int kdpc_three_nn(int b, int n, int m, const float *unknown, const float *known, float *dist2,
                  int *idx, void *stream);

/* Replaces three_interpolate_wrapper(b, c, m, n, points, idx, weight, out)
 * (interpolate.cpp:27-41; kernel interpolate_gpu.cu:77-97).  points (B,C,M), idx/weight
 * (B,N,3), out (B,C,N). */
int kdpc_three_interpolate(int b, int c, int m, int n, const float *points, const int *idx,
                           const float *weight, float *out, void *stream);

/* Replaces three_interpolate_grad_wrapper(b, c, n, m, grad_out, idx, weight, grad_points)
 * (interpolate.cpp:43-57; kernel interpolate_gpu.cu:120-142).  Overwrites grad_points (B,C,M).
 * Scratch: a stream-ordered temporary; kdpc_three_interpolate_grad_ws takes a caller buffer. */
int kdpc_three_interpolate_grad(int b, int c, int n, int m, const float *grad_out,
                                const int *idx, const float *weight, float *grad_points,
                                void *stream);

/* ---- kNN (pointconv_util.py:73-107) ---------------------------------------------------- */

/* Replaces knn_point(nsample, xyz, new_xyz) = square_distance + topk(largest=False).
 * xyz (B,N,3) refs, new_xyz (B,S,3) queries, idx (B,S,K) int32 out ascending by
 * (distance, index), dist (B,S,K) optional (NULL to skip).  1 <= K <= min(N, 64). */
int kdpc_knn_point(int b, int n, int s, int k, const float *xyz, const float *new_xyz, int *idx,
                   float *dist, void *stream);

/* Scratch bytes for kdpc_knn_point_ws (0: the plain scan is used, pass workspace = NULL). */
size_t kdpc_knn_workspace_bytes(int b, int n, int s);

/* kdpc_knn_point with scratch: the refs are first counting-sorted into a Morton cell grid
 * and each query's threshold is seeded with the exact K-th distance to the 256 sorted refs
 * around its cell, so the scan inserts ~K candidates; results identical to kdpc_knn_point. */
int kdpc_knn_point_ws(int b, int n, int s, int k, const float *xyz, const float *new_xyz,
                      int *idx, float *dist, void *workspace, size_t workspace_bytes,
                      void *stream);

/* kdpc_knn_point_ws on the culled path (needs kdpc_knn_workspace_bytes(b, n, s) > 0) that
 * also adds the number of query-ref distance evaluations it issues to *evals (device u64):
 * the roofline's work count (bench.py configs[4]).  Same idx as kdpc_knn_point_ws. */
int kdpc_knn_point_evals(int b, int n, int s, int k, const float *xyz, const float *new_xyz,
                         int *idx, void *workspace, size_t workspace_bytes,
                         unsigned long long *evals, void *stream);

/* kNN in feature space (CrossLayerLightFG's knn_point over (B,N,D) features,
 * pointconv_util.py:1871-1957 with square_distance + topk :73-107): ref (B,N,D),
 * query (B,S,D) -> idx (B,S,K) int32 ascending by (dist, index), dist (B,S,K) if non-null,
 * dist = (-2 q.r + |q|^2) + |r|^2; the dot products run on the f32 matrix cores.
 * 1 <= D <= 128, 1 <= K <= min(32, N).  Workspace: the row norms. */
size_t kdpc_knn_feature_workspace_bytes(int b, int n, int s);
int kdpc_knn_feature(int b, int n, int s, int d, int k, const float *ref, const float *query,
                     int *idx, float *dist, void *workspace, size_t workspace_bytes,
                     void *stream);

/* ---- point-major grouping + deterministic scatter (no reference counterpart: these
 *      replace index_points_group's permute/grouping_operation/permute chain,
 *      pointconv_util.py:122-133, and its atomicAdd backward) ------------------------- */

/* out[b,p,:] = points[b, idx[b,p], :] ; points (B,N,C), idx (B,P), out (B,P,C). */
int kdpc_group_rows(int b, int n, int c, int p, const float *points, const int *idx, float *out,
                    void *stream);

/* Inverted index of idx (B,P) with values in [0,N): offsets (B*N+1) and perm (B*P) (flat
 * positions sorted by key b*N+idx, ascending position within a key).  workspace must hold
 * kdpc_csr_workspace_bytes(b, n, p) bytes (query returns 0 on invalid sizes). */
size_t kdpc_csr_workspace_bytes(int b, int n, int p);
int kdpc_csr_build(int b, int n, int p, const int *idx, void *workspace, size_t workspace_bytes,
                   int *offsets, int *perm, void *stream);

/* Inverse permutation of that CSR: rank (B*P), perm[rank[i]] == i (the slot of position i),
 * -1 where idx[i] is outside [0,N).  Lets a producer write per-position rows straight into
 * CSR order (kdpc_cost_volume_bwd_csr). */
int kdpc_csr_rank(int b, int n, int p, const int *idx, const int *offsets, const int *perm,
                  int *rank, void *stream);

/* grad_points[b,n,:] = sum of grad_out rows (B,P,C) that idx sent to n, ascending position. */
int kdpc_group_rows_grad_csr(int b, int n, int c, const float *grad_out, const int *offsets,
                             const int *perm, float *grad_points, void *stream);

/* dst[b,c,n] = sum of src[b,c,p] over the positions p that idx sent to n (src (B,C,P),
 * dst (B,C,N)): group_points_grad / gather_points_grad with a caller-built CSR. */
int kdpc_csr_sum_channels(int b, int c, int n, int p, const float *src, const int *offsets,
                          const int *perm, float *dst, void *stream);

/* three_interpolate_grad with a caller-built CSR over idx (B,N,3) (key space M). */
int kdpc_three_interpolate_grad_csr(int b, int c, int n, int m, const float *grad_out,
                                    const float *weight, const int *offsets, const int *perm,
                                    float *grad_points, void *stream);

/* ---- fused cost volume (CrossLayerLight.cross / FlowEmbeddingLayer,
 *      pointconv_util.py:1826-1850 / :1497-1517) ----------------------------------------- */

/* out[b,n,:] = max_k LeakyReLU(W1 LeakyReLU((P2[idx]+P1[n]) + Wpos(x2[idx]-x1[n]) + bpos) + b1)
 * x1 (B,N1,3), x2 (B,N2,3), idx (B,N1,K) int32, p1 (B,N1,Din), p2 (B,N2,Din), wpos (Din,3),
 * bpos (Din), w1 (Dout,Din), b1 (Dout) -> out (B,N1,Dout) channel-last, amax (B,N1,Dout) u8.
 * Din, Dout in {32,64}, or Din = Dout in {128,256} (fused wide kernels: the Din x Dout MLP on
 * the f32 matrix cores inside the same kernel); 1 <= K <= 32. */
int kdpc_cost_volume_fwd(int b, int n1, int n2, int k, int din, int dout, const float *x1,
                         const float *x2, const int *idx, const float *p1, const float *p2,
                         const float *wpos, const float *bpos, const float *w1, const float *b1,
                         float *out, unsigned char *amax, void *stream);

/* Backward: dout_grad (B,N1,Dout) -> dp1 (B,N1,Din), dp2_rows (B,N1,K,Din), dx1 (B,N1,3),
 * ddir_rows (B,N1,K,3), dparams = [dW1 (Dout*Din) | db1 (Dout) | dWpos^T (3*Din) | dbpos (Din)].
 * dp2_rows/ddir_rows are per-neighbour rows: sum them per reference point with
 * kdpc_group_rows_grad_csr over the CSR of idx.  workspace: see *_workspace_bytes.
 * The two LeakyReLUs' derivatives are the backward's only discrete inputs besides amax: the
 * second one's is read from the sign of `out`; slope0 (B,N1,K,Din) u8, nullable (null in
 * training) overrides the first one's per (query, neighbour, channel): 1 -> 1, 2 -> 0.1,
 * 0 -> the sign of the recomputed pre-activation.  The parity tests replay a float64
 * reference run's decisions at near-ties through slope0 and `out`. */
size_t kdpc_cost_volume_bwd_workspace_bytes(int b, int n1, int din, int dout);
int kdpc_cost_volume_bwd(int b, int n1, int n2, int k, int din, int dout, const float *x1,
                         const float *x2, const int *idx, const float *p1, const float *p2,
                         const float *wpos, const float *bpos, const float *w1, const float *out,
                         const unsigned char *amax, const unsigned char *slope0,
                         const float *dout_grad, float *dp1,
                         float *dp2_rows, float *dx1, float *ddir_rows, void *workspace,
                         size_t workspace_bytes, float *dparams, void *stream);

/* Backward with the per-reference-point sums done inside: offsets (B*N2+1) / rank (B*N1*K)
 * of the CSR of idx over the N2 points (kdpc_csr_build + kdpc_csr_rank).  The per-neighbour
 * rows are written in CSR order into the workspace and summed contiguously:
 * dp2 (B,N2,Din), dx2 (B,N2,3); dp1, dx1, dparams as kdpc_cost_volume_bwd.  Bit-identical to
 * kdpc_cost_volume_bwd followed by kdpc_group_rows_grad_csr of its rows (same sum order). */
size_t kdpc_cost_volume_bwd_csr_workspace_bytes(int b, int n1, int k, int din, int dout);
int kdpc_cost_volume_bwd_csr(int b, int n1, int n2, int k, int din, int dout, const float *x1,
                             const float *x2, const int *idx, const float *p1, const float *p2,
                             const float *wpos, const float *bpos, const float *w1,
                             const float *out, const unsigned char *amax,
                             const unsigned char *slope0, const float *dout_grad,
                             const int *offsets, const int *rank, float *dp1, float *dp2,
                             float *dx1, float *dx2, void *workspace, size_t workspace_bytes,
                             float *dparams, void *stream);

/* ---- unfused wide cost volume (same layers, the widths kdpc_cost_volume_fwd does not take,
 *      Din in {64,128,256,512}): the Din -> Dout MLP is the caller's BLAS GEMM between these
 *      fused pieces (csrc/cost_volume_wide.hip) --------------------------------------- */

int kdpc_cost_volume_wide_supported(int din, int dout, int k);

/* h0 (B,N1,K,Din) = LeakyReLU((P2[idx] + P1[n]) + (Wpos (x2[idx] - x1[n]) + bpos)) */
int kdpc_cost_volume_wide_h0(int b, int n1, int n2, int k, int din, const float *x1,
                             const float *x2, const int *idx, const float *p1, const float *p2,
                             const float *wpos, const float *bpos, float *h0, void *stream);

/* z1 (B,N1,K,Dout) pre-activation of the MLP -> out (B,N1,Dout) = LeakyReLU(max_k z1),
 * amax (B,N1,Dout) u8 = first maximal k. */
int kdpc_cost_volume_wide_max(int b, int n1, int k, int dout, const float *z1, float *out,
                              unsigned char *amax, void *stream);

/* gout (B,N1,Dout) -> dz1 (B,N1,K,Dout) dense (nonzero only at amax rows),
 * gsc (B,N1,Dout) = gout * LeakyReLU'(out) (its column sums are db1). */
int kdpc_cost_volume_wide_max_bwd(int b, int n1, int k, int dout, const float *gout,
                                  const float *out, const unsigned char *amax, float *dz1,
                                  float *gsc, void *stream);

/* Rows of the dWpos slab below (each Din*3 floats, summed with kdpc_colsum). */
int kdpc_cost_volume_wide_slab_rows(void);

/* dz (B,N1,K,Din): dh0 in, dz0 = dh0 * LeakyReLU'(h0) out (in place); dp1 (B,N1,Din) =
 * sum_k dz0; slab (slab_rows, Din*3) partial sums of dWpos[c][a] = sum dz0[.,c] dir[.,a]. */
int kdpc_cost_volume_wide_h0_bwd(int b, int n1, int n2, int k, int din, const float *x1,
                                 const float *x2, const int *idx, const float *h0, float *dz,
                                 float *dp1, float *slab, void *stream);

/* ---- fused PointConv neighbourhood contraction (pointconv_util.py:217-258, 401-446) ---- */

/* out[b,s, c*16+w] = sum_k G[b,s,k,c] * wt[b,s,k,w],  G = cat(xyz[idx]-center, feats[idx]).
 * xyz (B,N,3), center (B,S,3), feats (B,N,D), idx (B,S,K) int32, wt (B,S,K,16),
 * out (B,S,16*(3+D)). */
int kdpc_pointconv_contract_fwd(int b, int n, int s, int k, int d, const float *xyz,
                                const float *center, const float *feats, const int *idx,
                                const float *wt, float *out, void *stream);

/* dout (B,S,16*(3+D)) -> dg_rows (B,S,K,3+D) per-neighbour rows of dG (sum per point with
 * kdpc_group_rows_grad_csr), dwt (B,S,K,16), dcenter (B,S,3) = -sum_k dG[..., 0:3]. */
int kdpc_pointconv_contract_bwd(int b, int n, int s, int k, int d, const float *xyz,
                                const float *center, const float *feats, const int *idx,
                                const float *wt, const float *dout, float *dg_rows, float *dwt,
                                float *dcenter, void *stream);

/* ---- fused PointConv layer: gather + WeightNet contraction + Linear on the f32 matrix
 *      cores (pointconv_util.py:217-258 PointConv, :401-446 PointConvD, both without the
 *      BatchNorm/activation that follows the Linear) ------------------------------------ */

/* 1 if (K, D, O) is handled: 1 <= K <= 16, O in {64, 128, 256}, WeightNet width 16. */
int kdpc_pointconv_supported(int k, int d, int o);

/* y (B,S,O) = A wl^T + bias,  A[b,s, c*16+w] = sum_k G[b,s,k,c] wt[b,s,k,w],
 * G = cat(xyz[idx] - center, feats[idx]) (C = 3+D channels); A is never stored.
 * xyz (B,N,3), center (B,S,3), feats (B,N,D), idx (B,S,K) int32, wt (B,S,K,16),
 * wl (O, 16C) (nn.Linear weight), bias (O).  workspace: *_fwd_workspace_bytes (> 0: wl split
 * into the bf16 planes the kernel multiplies on the bf16 matrix cores, f32-accurate). */
size_t kdpc_pointconv_fwd_workspace_bytes(int b, int s, int k, int d, int o);
int kdpc_pointconv_fwd(int b, int n, int s, int k, int d, int o, const float *xyz,
                       const float *center, const float *feats, const int *idx, const float *wt,
                       const float *wl, const float *bias, float *y, void *workspace,
                       size_t workspace_bytes, void *stream);

/* Backward of kdpc_pointconv_fwd for dy (B,S,O): dxyz (B,N,3) (NULL to skip), dfeats (B,N,D),
 * dcenter (B,S,3), dwt (B,S,K,16), dwl (O,16C), all overwritten (bias grad = column sums of
 * dy, left to the caller).  offsets/rank: kdpc_csr_build + kdpc_csr_rank of idx with key
 * space N (the per-neighbour dG rows are written straight into CSR order and summed as
 * contiguous runs).  Deterministic: every sum runs in a fixed order. */
size_t kdpc_pointconv_bwd_workspace_bytes(int b, int s, int k, int d, int o);
int kdpc_pointconv_bwd(int b, int n, int s, int k, int d, int o, const float *xyz,
                       const float *center, const float *feats, const int *idx, const float *wt,
                       const float *wl, const float *dy, const int *offsets, const int *rank,
                       float *dxyz, float *dfeats, float *dcenter, float *dwt, float *dwl,
                       void *workspace, size_t workspace_bytes, void *stream);

/* The two halves of kdpc_pointconv_bwd (same kernels, same results bit for bit), so the weight
 * gradient -- needed only by the optimizer -- can run on a second stream beside the rest of
 * the backward: _bwd_data writes dxyz (NULL to skip), dfeats, dcenter, dwt (workspace:
 * kdpc_pointconv_bwd_workspace_bytes); _bwd_weight writes dwl (workspace:
 * kdpc_pointconv_bwd_weight_workspace_bytes) and reads only the inputs. */
int kdpc_pointconv_bwd_data(int b, int n, int s, int k, int d, int o, const float *xyz,
                            const float *center, const float *feats, const int *idx,
                            const float *wt, const float *wl, const float *dy, const int *offsets,
                            const int *rank, float *dxyz, float *dfeats, float *dcenter,
                            float *dwt, void *workspace, size_t workspace_bytes, void *stream);
size_t kdpc_pointconv_bwd_weight_workspace_bytes(int b, int s, int k, int d, int o);
int kdpc_pointconv_bwd_weight(int b, int n, int s, int k, int d, int o, const float *xyz,
                              const float *center, const float *feats, const int *idx,
                              const float *wt, const float *dy, float *dwl, void *workspace,
                              size_t workspace_bytes, void *stream);
/* The weight half plus the Linear's bias gradient dbias (O) = column sums of dy, from the
 * same MFMAs (a padding column of the contraction set to 1; requires (3 + d) % 8 != 0).
 * Same workspace as kdpc_pointconv_bwd_weight. */
int kdpc_pointconv_bwd_weight_bias(int b, int n, int s, int k, int d, int o, const float *xyz,
                                   const float *center, const float *feats, const int *idx,
                                   const float *wt, const float *dy, float *dwl, float *dbias,
                                   void *workspace, size_t workspace_bytes, void *stream);

/* Tiled PointConv backward: the same gradients with the dG rows summed per (32-row tile,
 * destination point) inside the data kernel (one partial row each instead of one row per
 * (row, neighbour) pair), then per point through the CSR of the partial rows.  The rows of
 * a tile come from a row order that keeps them close in space (kdpc_morton_order), so a
 * tile's 32K pairs name few distinct points.  Sums in a fixed order (pairs of a destination
 * in ascending pair order within a tile, tiles ascending): deterministic, rounding differs
 * from the untiled entry points.  Same as kdpc_pointconv_bwd(_data) (pointconv_util.py:
 * 217-258 backward) otherwise; same workspace.
 *
 * kdpc_morton_order: order (B,S) = each batch element's S <= 8192 centers (B,S,3) sorted by
 *   their Morton code (6 bits per axis over the element's bounding box), ties by index.
 * kdpc_pc_tile_plan: for idx (B,S,K) (K <= 16, values in [0,N)) and an optional order (NULL
 *   = identity), per tile t of T = B*ceil(S/32): trow (T*32) global rows or -1, tpair
 *   (T*32K) the tile's pairs (p = row_in_tile*K + k) sorted by (destination, p), -1 padded,
 *   tsoff (T*(32K+1)) each destination's first sorted position (then the pair count), tkey
 *   (T*32K) the destinations (-1 padded).  offsets / tdst = kdpc_csr_build / kdpc_csr_rank
 *   of tkey viewed as (B, ceil(S/32)*32K) over N keys. */
int kdpc_morton_order(int b, int s, const float *xyz, int *order, void *stream);
/* kdpc_pointconv_fwd with the rows of each 64-row tile taken from a tile plan's trow (two
 * consecutive 32-row tiles; ntrow = its entry count): the same outputs bit for bit, the
 * neighbour gathers of a tile spatially close.  K must be 9 or 16. */
int kdpc_pointconv_fwd_tiled(int b, int n, int s, int k, int d, int o, const float *xyz,
                             const float *center, const float *feats, const int *idx,
                             const float *wt, const float *wl, const float *bias,
                             const int *trow, int ntrow, float *y, void *workspace,
                             size_t workspace_bytes, void *stream);
int kdpc_pc_tile_plan(int b, int s, int n, int k, const int *idx, const int *order, int *trow,
                      int *tpair, int *tsoff, int *tkey, void *stream);
int kdpc_pointconv_bwd_data_tiled(int b, int n, int s, int k, int d, int o, const float *xyz,
                                  const float *center, const float *feats, const int *idx,
                                  const float *wt, const float *wl, const float *dy,
                                  const int *offsets, const int *trow, const int *tpair,
                                  const int *tsoff, const int *tdst, float *dxyz, float *dfeats,
                                  float *dcenter, float *dwt, void *workspace,
                                  size_t workspace_bytes, void *stream);
int kdpc_pointconv_bwd_tiled(int b, int n, int s, int k, int d, int o, const float *xyz,
                             const float *center, const float *feats, const int *idx,
                             const float *wt, const float *wl, const float *dy,
                             const int *offsets, const int *trow, const int *tpair,
                             const int *tsoff, const int *tdst, float *dxyz, float *dfeats,
                             float *dcenter, float *dwt, float *dwl, void *workspace,
                             size_t workspace_bytes, void *stream);

/* ---- fused WeightNet over grouped offsets (pointconv_util.py:184-215 as used by
 *      PointConv/PointConvD :217-258, :401-446: weightnet=16, hidden [8, 8], no BN) ------ */

/* Parameter-gradient layout of kdpc_weightnet_bwd (floats): dW0 (8,3) | db0 (8) | dW1 (8,8) |
 * db1 (8) | dW2 (16,8) | db2 (16); kdpc_weightnet_param_count() = 248. */
int kdpc_weightnet_param_count(void);

/* wt (B,S,K,16) = ReLU(W2 ReLU(W1 ReLU(W0 rel + b0) + b1) + b2) with
 * rel = xyz[b, idx[b,s,k]] - center[b,s].  xyz (B,N,3), center (B,S,3), idx (B,S,K);
 * W0 (8,3) b0 (8) W1 (8,8) b1 (8) W2 (16,8) b2 (16) (nn.Conv2d weights, row-major). */
int kdpc_weightnet_fwd(int b, int n, int s, int k, const float *xyz, const float *center,
                       const int *idx, const float *w0, const float *b0, const float *w1,
                       const float *b1, const float *w2, const float *b2, float *wt,
                       void *stream);

/* Scratch bytes kdpc_weightnet_bwd needs (independent of the problem size). */
size_t kdpc_weightnet_bwd_workspace_bytes(void);

/* Backward of kdpc_weightnet_fwd for dwt (B,S,K,16): overwrites dparams (248, layout above)
 * with deterministic fixed-order sums (no atomics) and, if drel != NULL, writes
 * drel (B,S,K,3). */
int kdpc_weightnet_bwd(int b, int n, int s, int k, const float *xyz, const float *center,
                       const int *idx, const float *w0, const float *b0, const float *w1,
                       const float *b1, const float *w2, const float *b2, const float *dwt,
                       float *drel, float *dparams, void *workspace, size_t workspace_bytes,
                       void *stream);

/* drel alone (the same rows, bit-identical to kdpc_weightnet_bwd's): with it the upstream
 * gradient does not wait for the parameter reduction, which can then run on another stream
 * (kdpc_weightnet_bwd with drel = NULL). */
int kdpc_weightnet_bwd_rel(int b, int n, int s, int k, const float *xyz, const float *center,
                           const int *idx, const float *w0, const float *b0, const float *w1,
                           const float *b1, const float *w2, const float *b2,
                           const float *dwt, float *drel, void *stream);

/* ---- WeightNet-weighted neighbour sums: PointConvFlow's point-to-patch and patch-to-patch
 *      cost sums (pointconv_util.py:2039-2112) ----------------------------------------- */

/* Floats of kdpc_wn_wsum_bwd's dparams for C output channels: dW0 (8,3) | db0 (8) |
 * dW1 (8,8) | db1 (8) | dW2 (C,8) | db2 (C) = 104 + 9C. */
int kdpc_wn_wsum_param_count(int c);

/* out[b,q,c] = sum_k w[b,q,k,c] * v(b,q,k,c), w = ReLU(W2 ReLU(W1 ReLU(W0 dir + b0) + b1) + b2)
 * of dir (B,N,K,3); v(b,q,k,c) = v[b,q,k,c] for idx == NULL (v (B,N,K,C)), else
 * v[b, idx[b,q,k], c] (v (B,M,C), idx (B,N,K) int32 in [0,M)).  W0 (8,3) b0 (8) W1 (8,8)
 * b1 (8) W2 (C,8) b2 (C) row-major (nn.Conv2d).  1 <= K <= 64, 1 <= C <= 256.
 * Replaces the reference's weightnet1/2(direction) + torch.sum(weights * points, dim=2)
 * (and index_points_group of the point-to-patch cost). */
int kdpc_wn_wsum_fwd(int b, int n, int m, int k, int c, const float *dir, const int *idx,
                     const float *v, const float *w0, const float *b0, const float *w1,
                     const float *b1, const float *w2, const float *b2, float *out, void *stream);

/* Scratch bytes of kdpc_wn_wsum_bwd. */
size_t kdpc_wn_wsum_bwd_workspace_bytes(int b, int n, int c);

/* Backward for dout (B,N,C): dv_rows (B,N,K,C) = w * dout (v's gradient when idx == NULL;
 * otherwise the per-(q,k) rows the caller sums per point through the CSR of idx),
 * ddir (B,N,K,3), dparams (layout above), deterministic fixed-order sums. */
int kdpc_wn_wsum_bwd(int b, int n, int m, int k, int c, const float *dir, const int *idx,
                     const float *v, const float *w0, const float *b0, const float *w1,
                     const float *b1, const float *w2, const float *b2, const float *dout,
                     float *dv_rows, float *ddir, float *dparams, void *workspace,
                     size_t workspace_bytes, void *stream);

/* ---- BatchNorm1d + LeakyReLU over point-major rows (pointconv_util.py:217-258, bn=True
 *      estimator PointConvs: Linear -> BatchNorm1d -> LeakyReLU(0.1)) ------------------- */

/* Scratch bytes for kdpc_batchnorm_lrelu_fwd / _bwd on an (R, C) tensor. */
size_t kdpc_batchnorm_workspace_bytes(int r, int c);

/* Train mode: per-column statistics of x (R, C) (biased variance for the normalisation,
 * unbiased for the running update, as torch.nn.BatchNorm1d), y = LeakyReLU_slope(
 * (x - mean) * invstd * weight + bias).  mean/invstd (C) are written for the backward;
 * run_mean/run_var updated with `momentum` (both NULL: not tracked).  C % 4 == 0,
 * C <= 1024.  Fixed-order reductions (deterministic). */
int kdpc_batchnorm_lrelu_fwd(int r, int c, const float *x, const float *weight, const float *bias,
                             float eps, float momentum, float slope, float *run_mean,
                             float *run_var, float *mean, float *invstd, float *y,
                             void *workspace, size_t workspace_bytes, void *stream);

/* y = LeakyReLU_slope((x - mean) * invstd * weight + bias) with given statistics (eval). */
int kdpc_batchnorm_lrelu_apply(int r, int c, const float *x, const float *mean,
                               const float *invstd, const float *weight, const float *bias,
                               float slope, float *y, void *stream);

/* Backward of kdpc_batchnorm_lrelu_fwd: dy_act and y_act (the forward output), x (its
 * input) -> dx (R, C), dweight, dbias (C). */
int kdpc_batchnorm_lrelu_bwd(int r, int c, const float *dy_act, const float *y_act,
                             const float *x, const float *weight, const float *mean,
                             const float *invstd, float slope, float *dx, float *dweight,
                             float *dbias, void *workspace, size_t workspace_bytes,
                             void *stream);

/* ---- 3-NN inverse-distance blend (UpsampleFlow / PointWarping, pointconv_util.py:2114-2172,
 *      replaces its torch norm/clamp/reciprocal/sum/div/mul/sum[/sub] chain) ------------- */

/* out[b,n,:] = sum_k w[b,n,k] vals[b, idx[b,n,k], :] (warp = 0) or qry[b,n,:] - that sum
 * (warp = 1, PointWarping, c must be 3), w_k = (1/d_k) / sum_j (1/d_j),
 * d_k = max(||ref[b,idx[b,n,k]] - qry[b,n]||, 1e-10); ref (B,S,3), qry (B,N,3), vals (B,S,C),
 * idx (B,N,3) int32, out (B,N,C); w (B,N,3) is written for the backward. */
int kdpc_idw_blend_fwd(int b, int n, int s, int c, const float *ref, const float *qry,
                       const float *vals, const int *idx, float *out, float *w, int warp,
                       void *stream);

/* dvals (B,S,C): the values' gradient, summed per reference point through the CSR of idx
 * (offsets B*S+1, perm B*3N from kdpc_csr_build over idx viewed as (B,3N)). */
int kdpc_idw_blend_bwd_vals(int b, int n, int s, int c, const float *dout, const float *w,
                            const int *offsets, const int *perm, float *dvals, int warp,
                            void *stream);

/* The coordinates' gradient: drow (B,N,3,3) per (query, neighbour) rows of d/d ref[idx]
 * (sum them per reference point with kdpc_group_rows_grad_csr over the same CSR), dqry
 * (B,N,3) (may be NULL). */
int kdpc_idw_blend_bwd_coords(int b, int n, int s, int c, const float *ref, const float *qry,
                              const float *vals, const int *idx, const float *dout,
                              float *drow, float *dqry, int warp, void *stream);

/* ---- skinny 1x1-layer weight gradients (dense_small.hip) ---------------------------- */

/* out (O x I) = A^T B for row-major A (R x O), B (R x I), min(O,I) <= 4, O + I <= 512: slab
 * partials + fixed-order column sum (replaces the BLAS split-K GEMM of dense.splitk_tn for
 * the 3-channel layers).  workspace: kdpc_dense_tn_small_workspace_bytes (0 = unsupported). */
size_t kdpc_dense_tn_small_workspace_bytes(int r, int o, int i);
int kdpc_dense_tn_small(int r, int o, int i, const float *a, const float *b, float *out,
                        void *workspace, size_t workspace_bytes, void *stream);

/* y (R x N) = x (R x K) m (K x N) [+ bias (N), may be NULL] for min(K, N) <= 4, K*N <= 4096:
 * the skinny forward / input-gradient GEMMs of the same layers. */
int kdpc_dense_small(int r, int k, int n, const float *x, const float *m, const float *bias,
                     float *y, void *stream);

/* ---- deterministic column sums (bias gradients, partial-slab reductions) -------------- */

/* Scratch bytes for kdpc_colsum over an (nrows, len) matrix (0 for nrows <= 64). */
size_t kdpc_colsum_workspace_bytes(int nrows, int len);

/* dst[i] = sum_r src[r][i] for a row-major (nrows, len) src, summed in fixed chunks (the
 * result depends only on the shape). */
int kdpc_colsum(int nrows, int len, const float *src, float *dst, void *workspace,
                size_t workspace_bytes, void *stream);

/* out (m, c) = -sum_{j<k} in (m, k, c) in ascending j: the center gradient -sum_k drel of the
 * grouped relative offsets (replaces the torch reduction of pointconv_util.py's WeightNet
 * backward: `-drel.sum(2)`). */
int kdpc_neg_sum_k(int m, int k, int c, const float *in, float *out, void *stream);

/* n byte copies dst[i] <- src[i] (bytes[i] a multiple of 4, 4-byte aligned pointers) in
 * ceil(n/128) launches.  Replaces torch._foreach_copy_ in the graphed training step (the
 * gradient pack into the flat buffer and the plan prefetch hand-over); no reference
 * counterpart: the reference steps its optimizer per parameter (train.py:150-160). */
int kdpc_copy_segments(int n, const void *const *src, void *const *dst, const long long *bytes,
                       void *stream);

/* One Adam step (L2 weight decay, no amsgrad) over flat float buffers of n elements (n a
 * multiple of 4, 16-byte aligned): param, exp_avg, exp_avg_sq updated in place from grad; lr and
 * step (already incremented) are device scalars, read by the kernel (graph replays see their
 * current values).  The same update as torch's fused Adam (ATen fused_adam_utils.cuh adam_math)
 * operation for operation; mode bit 0: the double expressions contracted as clang does by
 * default, bit 1: fast (not correctly rounded) f32 division and square root.  Replaces the multi-tensor fused Adam
 * in the graphed training step; the reference steps torch.optim.Adam (distilTrain.py:134-135). */
int kdpc_adam_step(long long n, float *param, const float *grad, float *exp_avg,
                   float *exp_avg_sq, const float *lr, const float *step, double beta1,
                   double beta2, double eps, double weight_decay, int maximize, int mode,
                   void *stream);

#ifdef __cplusplus
}
#endif

#endif /* KDPC_H_ */
