// PyTorch-ROCm custom-op surface of kd-pointcloud_amd: torch.ops.kdpc.*
//
// Registers (TORCH_LIBRARY(kdpc, m)) every entry point of the C ABI (include/kdpc.h) as a
// torch operator with a schema, implemented for the GPU dispatch key ("CUDA" -- ROCm torch
// masquerades HIP devices as CUDA) on the current torch stream of the inputs' device:
//
//   * the nine reference wrappers of pointnet2_cuda (reference pointnet2/src/
//     pointnet2_api.cpp:10-24) with their exact argument lists and in-place contract
//     (`*_wrapper(... , Tensor(a!) out) -> int`), so the reference's own
//     pointnet2_utils.py binds to torch.ops.kdpc unchanged;
//   * functional, allocating ops for everything the drop-in layers call (kNN, row
//     gathers, CSR scatter, fused PointConv / WeightNet / cost volume / BatchNorm).
//
// Host code only: every kernel lives in libkdpc_hip.so behind the C ABI.  Each op checks
// device, dtype and contiguity with TORCH_CHECK, allocates outputs and scratch from the
// torch caching allocator (so it is stream-ordered and graph-capture safe) and turns a
// non-zero hipError_t into a C++ exception (the reference printed and exit(-1)ed,
// e.g. sampling_gpu.cu:39-43).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime_api.h>
#include <torch/library.h>

#include <string>
#include <tuple>
#include <vector>

#include "kdpc.h"

namespace {

using at::Tensor;
using TT = std::tuple<Tensor, Tensor>;

void* stream_of(const Tensor& t) {
  return (void*)c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void check(int err, const char* fn) {
  TORCH_CHECK(err == 0, "kdpc: ", fn, " failed: ", hipGetErrorString((hipError_t)err), " (",
              err, ")");
}

void dev(const Tensor& t, at::ScalarType st, const char* name) {
  TORCH_CHECK(t.is_cuda(), "kdpc: ", name, " must be a GPU (HIP) tensor: there is no CPU path");
  TORCH_CHECK(t.scalar_type() == st, "kdpc: ", name, " must be ", c10::toString(st), ", got ",
              t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), "kdpc: ", name, " must be contiguous");
}

void same_device(const Tensor& a, const Tensor& b, const char* name) {
  TORCH_CHECK(a.device() == b.device(), "kdpc: ", name, " is on ", b.device(), ", expected ",
              a.device());
}

float* F(const Tensor& t) { return t.data_ptr<float>(); }
int* I(const Tensor& t) { return t.data_ptr<int>(); }
float* Fo(const c10::optional<Tensor>& t) { return t.has_value() ? F(*t) : nullptr; }

Tensor empty_f(at::IntArrayRef size, const Tensor& like) {
  return at::empty(size, like.options().dtype(at::kFloat));
}
Tensor empty_i(at::IntArrayRef size, const Tensor& like) {
  return at::empty(size, like.options().dtype(at::kInt));
}
Tensor workspace(size_t nbytes, const Tensor& like) {
  return at::empty({(int64_t)std::max<size_t>(nbytes, 1)}, like.options().dtype(at::kByte));
}

#define GUARD(t) c10::hip::HIPGuardMasqueradingAsCUDA guard_((t).device())
constexpr auto kF = at::kFloat;
constexpr auto kI = at::kInt;

// ------------------------------------------------ reference wrappers (pointnet2_api.cpp)
int64_t ball_query_wrapper(int64_t b, int64_t n, int64_t m, double radius, int64_t nsample,
                           Tensor new_xyz, Tensor xyz, Tensor idx) {
  dev(new_xyz, kF, "new_xyz"), dev(xyz, kF, "xyz"), dev(idx, kI, "idx");
  GUARD(xyz);
  check(kdpc_ball_query(b, n, m, (float)radius, nsample, F(new_xyz), F(xyz), I(idx),
                        stream_of(xyz)), "ball_query");
  return 1;
}

int64_t group_points_wrapper(int64_t b, int64_t c, int64_t n, int64_t npoints, int64_t nsample,
                             Tensor points, Tensor idx, Tensor out) {
  dev(points, kF, "points"), dev(idx, kI, "idx"), dev(out, kF, "out");
  GUARD(points);
  check(kdpc_group_points(b, c, n, npoints, nsample, F(points), I(idx), F(out),
                          stream_of(points)), "group_points");
  return 1;
}

int64_t group_points_grad_wrapper(int64_t b, int64_t c, int64_t n, int64_t npoints,
                                  int64_t nsample, Tensor grad_out, Tensor idx,
                                  Tensor grad_points) {
  dev(grad_out, kF, "grad_out"), dev(idx, kI, "idx"), dev(grad_points, kF, "grad_points");
  GUARD(grad_out);
  const size_t nb = kdpc_grad_workspace_bytes(b, n, npoints * nsample);
  Tensor ws = workspace(nb, grad_out);
  check(kdpc_group_points_grad_ws(b, c, n, npoints, nsample, F(grad_out), I(idx),
                                  F(grad_points), ws.data_ptr(), nb, stream_of(grad_out)),
        "group_points_grad");
  return 1;
}

int64_t gather_points_wrapper(int64_t b, int64_t c, int64_t n, int64_t npoints, Tensor points,
                              Tensor idx, Tensor out) {
  dev(points, kF, "points"), dev(idx, kI, "idx"), dev(out, kF, "out");
  GUARD(points);
  check(kdpc_gather_points(b, c, n, npoints, F(points), I(idx), F(out), stream_of(points)),
        "gather_points");
  return 1;
}

int64_t gather_points_grad_wrapper(int64_t b, int64_t c, int64_t n, int64_t npoints,
                                   Tensor grad_out, Tensor idx, Tensor grad_points) {
  dev(grad_out, kF, "grad_out"), dev(idx, kI, "idx"), dev(grad_points, kF, "grad_points");
  GUARD(grad_out);
  const size_t nb = kdpc_grad_workspace_bytes(b, n, npoints);
  Tensor ws = workspace(nb, grad_out);
  check(kdpc_gather_points_grad_ws(b, c, n, npoints, F(grad_out), I(idx), F(grad_points),
                                   ws.data_ptr(), nb, stream_of(grad_out)),
        "gather_points_grad");
  return 1;
}

int64_t furthest_point_sampling_wrapper(int64_t b, int64_t n, int64_t m, Tensor points,
                                        Tensor temp, Tensor idx) {
  dev(points, kF, "points"), dev(temp, kF, "temp"), dev(idx, kI, "idx");
  GUARD(points);
  check(kdpc_furthest_point_sampling(b, n, m, F(points), F(temp), I(idx), stream_of(points)),
        "furthest_point_sampling");
  return 1;
}

int64_t three_nn_wrapper(int64_t b, int64_t n, int64_t m, Tensor unknown, Tensor known,
                         Tensor dist2, Tensor idx) {
  dev(unknown, kF, "unknown"), dev(known, kF, "known"), dev(dist2, kF, "dist2");
  dev(idx, kI, "idx");
  GUARD(unknown);
  check(kdpc_three_nn(b, n, m, F(unknown), F(known), F(dist2), I(idx), stream_of(unknown)),
        "three_nn");
  return 1;
}

int64_t three_interpolate_wrapper(int64_t b, int64_t c, int64_t m, int64_t n, Tensor points,
                                  Tensor idx, Tensor weight, Tensor out) {
  dev(points, kF, "points"), dev(idx, kI, "idx"), dev(weight, kF, "weight");
  dev(out, kF, "out");
  GUARD(points);
  check(kdpc_three_interpolate(b, c, m, n, F(points), I(idx), F(weight), F(out),
                               stream_of(points)), "three_interpolate");
  return 1;
}

int64_t three_interpolate_grad_wrapper(int64_t b, int64_t c, int64_t n, int64_t m,
                                       Tensor grad_out, Tensor idx, Tensor weight,
                                       Tensor grad_points) {
  dev(grad_out, kF, "grad_out"), dev(idx, kI, "idx"), dev(weight, kF, "weight");
  dev(grad_points, kF, "grad_points");
  GUARD(grad_out);
  const size_t nb = kdpc_grad_workspace_bytes(b, m, 3 * n);
  Tensor ws = workspace(nb, grad_out);
  check(kdpc_three_interpolate_grad_ws(b, c, n, m, F(grad_out), I(idx), F(weight),
                                       F(grad_points), ws.data_ptr(), nb, stream_of(grad_out)),
        "three_interpolate_grad");
  return 1;
}

// ------------------------------------------------------------- functional pointnet2 ops
Tensor furthest_point_sample(Tensor xyz, int64_t npoint) {
  dev(xyz, kF, "xyz");
  TORCH_CHECK(xyz.dim() == 3 && xyz.size(2) == 3, "kdpc: xyz must be (B,N,3)");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1);
  Tensor idx = empty_i({b, npoint}, xyz);
  Tensor temp = at::full({b, n}, 1e10, xyz.options());  // reference pointnet2_utils.py:26
  check(kdpc_furthest_point_sampling(b, n, npoint, F(xyz), F(temp), I(idx), stream_of(xyz)),
        "furthest_point_sampling");
  return idx;
}

Tensor gather_points(Tensor points, Tensor idx) {
  dev(points, kF, "points"), dev(idx, kI, "idx"), same_device(points, idx, "idx");
  TORCH_CHECK(points.dim() == 3 && idx.dim() == 2 && idx.size(0) == points.size(0),
              "kdpc: gather_points expects points (B,C,N), idx (B,M)");
  GUARD(points);
  const int64_t b = points.size(0), c = points.size(1), n = points.size(2), m = idx.size(1);
  Tensor out = empty_f({b, c, m}, points);
  check(kdpc_gather_points(b, c, n, m, F(points), I(idx), F(out), stream_of(points)),
        "gather_points");
  return out;
}

Tensor ball_query(double radius, int64_t nsample, Tensor xyz, Tensor new_xyz) {
  dev(xyz, kF, "xyz"), dev(new_xyz, kF, "new_xyz"), same_device(xyz, new_xyz, "new_xyz");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1), m = new_xyz.size(1);
  Tensor idx = empty_i({b, m, nsample}, xyz);
  check(kdpc_ball_query(b, n, m, (float)radius, nsample, F(new_xyz), F(xyz), I(idx),
                        stream_of(xyz)), "ball_query");
  return idx;
}

Tensor group_points(Tensor points, Tensor idx) {
  dev(points, kF, "points"), dev(idx, kI, "idx"), same_device(points, idx, "idx");
  TORCH_CHECK(points.dim() == 3 && idx.dim() == 3 && idx.size(0) == points.size(0),
              "kdpc: group_points expects points (B,C,N), idx (B,S,K)");
  GUARD(points);
  const int64_t b = points.size(0), c = points.size(1), n = points.size(2);
  const int64_t s = idx.size(1), k = idx.size(2);
  Tensor out = empty_f({b, c, s, k}, points);
  check(kdpc_group_points(b, c, n, s, k, F(points), I(idx), F(out), stream_of(points)),
        "group_points");
  return out;
}

TT three_nn(Tensor unknown, Tensor known) {
  dev(unknown, kF, "unknown"), dev(known, kF, "known"), same_device(unknown, known, "known");
  GUARD(unknown);
  const int64_t b = unknown.size(0), n = unknown.size(1), m = known.size(1);
  Tensor dist2 = empty_f({b, n, 3}, unknown);
  Tensor idx = empty_i({b, n, 3}, unknown);
  check(kdpc_three_nn(b, n, m, F(unknown), F(known), F(dist2), I(idx), stream_of(unknown)),
        "three_nn");
  return {dist2, idx};
}

Tensor three_interpolate(Tensor points, Tensor idx, Tensor weight) {
  dev(points, kF, "points"), dev(idx, kI, "idx"), dev(weight, kF, "weight");
  GUARD(points);
  const int64_t b = points.size(0), c = points.size(1), m = points.size(2), n = idx.size(1);
  Tensor out = empty_f({b, c, n}, points);
  check(kdpc_three_interpolate(b, c, m, n, F(points), I(idx), F(weight), F(out),
                               stream_of(points)), "three_interpolate");
  return out;
}

// ------------------------------------------------------------------------------- kNN
TT knn_point_impl(int64_t nsample, const Tensor& xyz, const Tensor& new_xyz, bool with_dist,
                  bool seeded) {
  dev(xyz, kF, "xyz"), dev(new_xyz, kF, "new_xyz"), same_device(xyz, new_xyz, "new_xyz");
  TORCH_CHECK(xyz.dim() == 3 && new_xyz.dim() == 3 && xyz.size(0) == new_xyz.size(0),
              "kdpc: knn_point expects xyz (B,N,3), new_xyz (B,S,3)");
  const int64_t b = xyz.size(0), n = xyz.size(1), s = new_xyz.size(1);
  TORCH_CHECK(nsample <= n, "knn_point: nsample=", nsample, " > number of points ", n);
  GUARD(xyz);
  Tensor idx = empty_i({b, s, nsample}, xyz);
  Tensor dist = with_dist ? empty_f({b, s, nsample}, xyz) : Tensor();
  const size_t nb = seeded ? kdpc_knn_workspace_bytes(b, n, s) : 0;
  Tensor ws = nb ? workspace(nb, xyz) : Tensor();
  check(kdpc_knn_point_ws(b, n, s, nsample, F(xyz), F(new_xyz), I(idx),
                          with_dist ? F(dist) : nullptr, nb ? ws.data_ptr() : nullptr, nb,
                          stream_of(xyz)), "knn_point");
  return {idx, dist};
}

Tensor knn_point(int64_t nsample, Tensor xyz, Tensor new_xyz, bool seeded) {
  return std::get<0>(knn_point_impl(nsample, xyz, new_xyz, false, seeded));
}

TT knn_point_dist(int64_t nsample, Tensor xyz, Tensor new_xyz, bool seeded) {
  return knn_point_impl(nsample, xyz, new_xyz, true, seeded);
}

TT knn_feature_impl(int64_t nsample, Tensor ref, Tensor query, bool want_dist) {
  dev(ref, kF, "ref"), dev(query, kF, "query"), same_device(ref, query, "query");
  TORCH_CHECK(ref.dim() == 3 && query.dim() == 3 && ref.size(0) == query.size(0) &&
                  ref.size(2) == query.size(2),
              "kdpc: knn_feature expects ref (B,N,D), query (B,S,D)");
  GUARD(ref);
  const int64_t b = ref.size(0), n = ref.size(1), d = ref.size(2), s = query.size(1);
  Tensor idx = at::empty({b, s, nsample}, ref.options().dtype(at::kInt));
  Tensor dist = want_dist ? empty_f({b, s, nsample}, ref) : Tensor();
  const size_t nb = kdpc_knn_feature_workspace_bytes(b, n, s);
  Tensor ws = workspace(nb, ref);
  check(kdpc_knn_feature(b, n, s, d, nsample, F(ref), F(query), I(idx),
                         want_dist ? F(dist) : nullptr, ws.data_ptr(), nb, stream_of(ref)),
        "knn_feature");
  return {idx, dist};
}

Tensor knn_feature(int64_t nsample, Tensor ref, Tensor query) {
  return std::get<0>(knn_feature_impl(nsample, ref, query, false));
}

TT knn_feature_dist(int64_t nsample, Tensor ref, Tensor query) {
  return knn_feature_impl(nsample, ref, query, true);
}

// ------------------------------------------------------- point-major rows and the CSR
Tensor group_rows(Tensor points, Tensor idx) {
  dev(points, kF, "points"), dev(idx, kI, "idx"), same_device(points, idx, "idx");
  TORCH_CHECK(points.dim() == 3 && idx.dim() == 2 && idx.size(0) == points.size(0),
              "kdpc: group_rows expects points (B,N,C), idx (B,P)");
  GUARD(points);
  const int64_t b = points.size(0), n = points.size(1), c = points.size(2), p = idx.size(1);
  Tensor out = empty_f({b, p, c}, points);
  check(kdpc_group_rows(b, n, c, p, F(points), I(idx), F(out), stream_of(points)),
        "group_rows");
  return out;
}

TT csr_build(Tensor idx, int64_t n) {
  dev(idx, kI, "idx");
  TORCH_CHECK(idx.dim() == 2, "kdpc: csr_build expects idx (B,P)");
  GUARD(idx);
  const int64_t b = idx.size(0), p = idx.size(1);
  const size_t nb = kdpc_csr_workspace_bytes(b, n, p);
  TORCH_CHECK(nb > 0, "kdpc: csr_build: invalid sizes b=", b, " n=", n, " p=", p);
  Tensor ws = workspace(nb, idx);
  Tensor offsets = empty_i({b * n + 1}, idx);
  Tensor perm = empty_i({b * p}, idx);
  check(kdpc_csr_build(b, n, p, I(idx), ws.data_ptr(), nb, I(offsets), I(perm), stream_of(idx)),
        "csr_build");
  return {offsets, perm};
}

Tensor csr_rank(Tensor idx, Tensor offsets, Tensor perm, int64_t n) {
  dev(idx, kI, "idx"), dev(offsets, kI, "offsets"), dev(perm, kI, "perm");
  TORCH_CHECK(idx.dim() == 2, "kdpc: csr_rank expects idx (B,P)");
  GUARD(idx);
  const int64_t b = idx.size(0), p = idx.size(1);
  TORCH_CHECK(offsets.numel() >= b * n + 1 && perm.numel() >= b * p,
              "kdpc: csr_rank: offsets / perm do not match idx");
  Tensor rank = empty_i({b * p}, idx);
  check(kdpc_csr_rank(b, n, p, I(idx), I(offsets), I(perm), I(rank), stream_of(idx)),
        "csr_rank");
  return rank;
}

Tensor group_rows_grad(Tensor grad_out, Tensor offsets, Tensor perm, int64_t n) {
  dev(grad_out, kF, "grad_out"), dev(offsets, kI, "offsets"), dev(perm, kI, "perm");
  TORCH_CHECK(grad_out.dim() == 3, "kdpc: group_rows_grad expects grad_out (B,P,C)");
  GUARD(grad_out);
  const int64_t b = grad_out.size(0), c = grad_out.size(2);
  Tensor out = empty_f({b, n, c}, grad_out);
  check(kdpc_group_rows_grad_csr(b, n, c, F(grad_out), I(offsets), I(perm), F(out),
                                 stream_of(grad_out)), "group_rows_grad_csr");
  return out;
}

Tensor csr_sum_channels(Tensor src, Tensor offsets, Tensor perm, int64_t b, int64_t c,
                        int64_t n) {
  dev(src, kF, "src"), dev(offsets, kI, "offsets"), dev(perm, kI, "perm");
  GUARD(src);
  const int64_t p = b * c > 0 ? src.numel() / (b * c) : 0;
  Tensor out = empty_f({b, c, n}, src);
  check(kdpc_csr_sum_channels(b, c, n, p, F(src), I(offsets), I(perm), F(out), stream_of(src)),
        "csr_sum_channels");
  return out;
}

Tensor three_interpolate_grad_csr(Tensor grad_out, Tensor weight, Tensor offsets, Tensor perm,
                                  int64_t m) {
  dev(grad_out, kF, "grad_out"), dev(weight, kF, "weight"), dev(offsets, kI, "offsets");
  dev(perm, kI, "perm");
  GUARD(grad_out);
  const int64_t b = grad_out.size(0), c = grad_out.size(1), n = grad_out.size(2);
  Tensor out = empty_f({b, c, m}, grad_out);
  check(kdpc_three_interpolate_grad_csr(b, c, n, m, F(grad_out), F(weight), I(offsets), I(perm),
                                        F(out), stream_of(grad_out)),
        "three_interpolate_grad_csr");
  return out;
}

// ------------------------------------------------------------------ fused cost volume
TT cost_volume_fwd(Tensor x1, Tensor x2, Tensor idx, Tensor p1, Tensor p2, Tensor wpos,
                   Tensor bpos, Tensor w1, Tensor b1) {
  for (auto* t : {&x1, &x2, &p1, &p2, &wpos, &bpos, &w1, &b1}) dev(*t, kF, "cost volume input");
  dev(idx, kI, "idx");
  GUARD(x1);
  const int64_t b = x1.size(0), n1 = x1.size(1), n2 = x2.size(1), k = idx.size(2);
  const int64_t din = p1.size(2), dout = w1.size(0);
  Tensor out = empty_f({b, n1, dout}, x1);
  Tensor amax = at::empty({b, n1, dout}, x1.options().dtype(at::kByte));
  check(kdpc_cost_volume_fwd(b, n1, n2, k, din, dout, F(x1), F(x2), I(idx), F(p1), F(p2),
                             F(wpos), F(bpos), F(w1), F(b1), F(out), amax.data_ptr<uint8_t>(),
                             stream_of(x1)), "cost_volume_fwd");
  return {out, amax};
}

// slope0 (B,N1,K,Din) u8, optional: the first LeakyReLU's derivative per (query, neighbour,
// channel) for replaying a reference run's decisions (include/kdpc.h); None in training
static const uint8_t* slope0_of(const c10::optional<Tensor>& s0, int64_t b, int64_t n1,
                                int64_t k, int64_t din) {
  if (!s0.has_value()) return nullptr;
  dev(*s0, at::kByte, "slope0");
  TORCH_CHECK(s0->numel() == b * n1 * k * din, "kdpc: slope0 must be (B, N1, K, Din)");
  return s0->data_ptr<uint8_t>();
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> cost_volume_bwd(
    Tensor x1, Tensor x2, Tensor idx, Tensor p1, Tensor p2, Tensor wpos, Tensor bpos, Tensor w1,
    Tensor out, Tensor amax, Tensor gout, c10::optional<Tensor> slope0) {
  for (auto* t : {&x1, &x2, &p1, &p2, &wpos, &bpos, &w1, &out, &gout})
    dev(*t, kF, "cost volume input");
  dev(idx, kI, "idx"), dev(amax, at::kByte, "amax");
  GUARD(x1);
  const int64_t b = x1.size(0), n1 = x1.size(1), n2 = x2.size(1), k = idx.size(2);
  const int64_t din = p1.size(2), dout = w1.size(0);
  const uint8_t* s0 = slope0_of(slope0, b, n1, k, din);
  Tensor dp1 = empty_f({b, n1, din}, x1);
  Tensor dp2_rows = empty_f({b, n1, k, din}, x1);
  Tensor dx1 = empty_f({b, n1, 3}, x1);
  Tensor ddir_rows = empty_f({b, n1, k, 3}, x1);
  Tensor dparams = empty_f({dout * din + dout + 4 * din}, x1);
  const size_t nb = kdpc_cost_volume_bwd_workspace_bytes(b, n1, din, dout);
  Tensor ws = workspace(nb, x1);
  check(kdpc_cost_volume_bwd(b, n1, n2, k, din, dout, F(x1), F(x2), I(idx), F(p1), F(p2),
                             F(wpos), F(bpos), F(w1), F(out), amax.data_ptr<uint8_t>(), s0,
                             F(gout), F(dp1), F(dp2_rows), F(dx1), F(ddir_rows), ws.data_ptr(), nb,
                             F(dparams), stream_of(x1)), "cost_volume_bwd");
  return {dp1, dp2_rows, dx1, ddir_rows, dparams};
}

std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> cost_volume_bwd_csr(
    Tensor x1, Tensor x2, Tensor idx, Tensor p1, Tensor p2, Tensor wpos, Tensor bpos, Tensor w1,
    Tensor out, Tensor amax, Tensor gout, Tensor offsets, Tensor rank,
    c10::optional<Tensor> slope0) {
  for (auto* t : {&x1, &x2, &p1, &p2, &wpos, &bpos, &w1, &out, &gout})
    dev(*t, kF, "cost volume input");
  dev(idx, kI, "idx"), dev(amax, at::kByte, "amax"), dev(offsets, kI, "offsets");
  dev(rank, kI, "rank");
  GUARD(x1);
  const int64_t b = x1.size(0), n1 = x1.size(1), n2 = x2.size(1), k = idx.size(2);
  const int64_t din = p1.size(2), dout = w1.size(0);
  const uint8_t* s0 = slope0_of(slope0, b, n1, k, din);
  TORCH_CHECK(offsets.numel() >= b * n2 + 1 && rank.numel() >= b * n1 * k,
              "kdpc: cost_volume_bwd_csr: offsets / rank do not match idx");
  Tensor dp1 = empty_f({b, n1, din}, x1);
  Tensor dp2 = empty_f({b, n2, din}, x1);
  Tensor dx1 = empty_f({b, n1, 3}, x1);
  Tensor dx2 = empty_f({b, n2, 3}, x1);
  Tensor dparams = empty_f({dout * din + dout + 4 * din}, x1);
  const size_t nb = kdpc_cost_volume_bwd_csr_workspace_bytes(b, n1, k, din, dout);
  TORCH_CHECK(nb > 0, "kdpc: cost_volume_bwd_csr: unsupported shape");
  Tensor ws = workspace(nb, x1);
  check(kdpc_cost_volume_bwd_csr(b, n1, n2, k, din, dout, F(x1), F(x2), I(idx), F(p1), F(p2),
                                 F(wpos), F(bpos), F(w1), F(out), amax.data_ptr<uint8_t>(), s0,
                                 F(gout), I(offsets), I(rank), F(dp1), F(dp2), F(dx1), F(dx2),
                                 ws.data_ptr(), nb, F(dparams), stream_of(x1)),
        "cost_volume_bwd_csr");
  return {dp1, dp2, dx1, dx2, dparams};
}

Tensor cost_volume_wide_h0(Tensor x1, Tensor x2, Tensor idx, Tensor p1, Tensor p2, Tensor wpos,
                           Tensor bpos) {
  for (auto* t : {&x1, &x2, &p1, &p2, &wpos, &bpos}) dev(*t, kF, "cost volume input");
  dev(idx, kI, "idx");
  GUARD(x1);
  const int64_t b = x1.size(0), n1 = x1.size(1), n2 = x2.size(1), k = idx.size(2);
  const int64_t din = p1.size(2);
  Tensor h0 = empty_f({b, n1, k, din}, x1);
  check(kdpc_cost_volume_wide_h0(b, n1, n2, k, din, F(x1), F(x2), I(idx), F(p1), F(p2), F(wpos),
                                 F(bpos), F(h0), stream_of(x1)), "cost_volume_wide_h0");
  return h0;
}

TT cost_volume_wide_max(Tensor z1, int64_t b, int64_t n1, int64_t k, int64_t dout) {
  dev(z1, kF, "z1");
  GUARD(z1);
  Tensor out = empty_f({b, n1, dout}, z1);
  Tensor amax = at::empty({b, n1, dout}, z1.options().dtype(at::kByte));
  check(kdpc_cost_volume_wide_max(b, n1, k, dout, F(z1), F(out), amax.data_ptr<uint8_t>(),
                                  stream_of(z1)), "cost_volume_wide_max");
  return {out, amax};
}

TT cost_volume_wide_max_bwd(Tensor gout, Tensor out, Tensor amax, int64_t k) {
  dev(gout, kF, "gout"), dev(out, kF, "out"), dev(amax, at::kByte, "amax");
  GUARD(out);
  const int64_t b = out.size(0), n1 = out.size(1), dout = out.size(2);
  Tensor dz1 = empty_f({b * n1 * k, dout}, out);
  Tensor gsc = empty_f({b * n1, dout}, out);
  check(kdpc_cost_volume_wide_max_bwd(b, n1, k, dout, F(gout), F(out), amax.data_ptr<uint8_t>(),
                                      F(dz1), F(gsc), stream_of(out)),
        "cost_volume_wide_max_bwd");
  return {dz1, gsc};
}

TT cost_volume_wide_h0_bwd(Tensor x1, Tensor x2, Tensor idx, Tensor h0, Tensor dz) {
  dev(x1, kF, "x1"), dev(x2, kF, "x2"), dev(idx, kI, "idx"), dev(h0, kF, "h0");
  dev(dz, kF, "dz");
  GUARD(x1);
  const int64_t b = x1.size(0), n1 = x1.size(1), n2 = x2.size(1), k = idx.size(2);
  const int64_t din = h0.size(-1);
  Tensor slab = empty_f({kdpc_cost_volume_wide_slab_rows(), din * 3}, x1);
  Tensor dp1 = empty_f({b, n1, din}, x1);
  check(kdpc_cost_volume_wide_h0_bwd(b, n1, n2, k, din, F(x1), F(x2), I(idx), F(h0), F(dz),
                                     F(dp1), F(slab), stream_of(x1)), "cost_volume_wide_h0_bwd");
  return {dp1, slab};
}

// ------------------------------------------------------------------- fused PointConv
Tensor pointconv_fwd(Tensor xyz, Tensor center, Tensor feats, Tensor idx, Tensor wt, Tensor wl,
                     Tensor bias) {
  for (auto* t : {&xyz, &center, &feats, &wt, &wl, &bias}) dev(*t, kF, "pointconv input");
  dev(idx, kI, "idx");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1), s = idx.size(1), k = idx.size(2);
  const int64_t d = feats.size(2), o = wl.size(0);
  TORCH_CHECK(kdpc_pointconv_supported(k, d, o), "kdpc: pointconv shape (K=", k, ", D=", d,
              ", O=", o, ") not supported");
  const size_t nb = kdpc_pointconv_fwd_workspace_bytes(b, s, k, d, o);
  Tensor ws = workspace(nb, xyz);
  Tensor y = empty_f({b, s, o}, xyz);
  check(kdpc_pointconv_fwd(b, n, s, k, d, o, F(xyz), F(center), F(feats), I(idx), F(wt), F(wl),
                           F(bias), F(y), ws.data_ptr(), nb, stream_of(xyz)), "pointconv_fwd");
  return y;
}

Tensor pointconv_fwd_tiled(Tensor xyz, Tensor center, Tensor feats, Tensor idx, Tensor wt,
                           Tensor wl, Tensor bias, Tensor trow) {
  for (auto* t : {&xyz, &center, &feats, &wt, &wl, &bias}) dev(*t, kF, "pointconv input");
  dev(idx, kI, "idx"), dev(trow, kI, "trow");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1), s = idx.size(1), k = idx.size(2);
  const int64_t d = feats.size(2), o = wl.size(0);
  TORCH_CHECK(kdpc_pointconv_supported(k, d, o), "kdpc: pointconv shape (K=", k, ", D=", d,
              ", O=", o, ") not supported");
  TORCH_CHECK(trow.numel() == b * ((s + 31) / 32) * 32, "kdpc: pointconv_fwd_tiled: trow size");
  const size_t nb = kdpc_pointconv_fwd_workspace_bytes(b, s, k, d, o);
  Tensor ws = workspace(nb, xyz);
  Tensor y = empty_f({b, s, o}, xyz);
  check(kdpc_pointconv_fwd_tiled(b, n, s, k, d, o, F(xyz), F(center), F(feats), I(idx), F(wt),
                                 F(wl), F(bias), I(trow), (int)trow.numel(), F(y), ws.data_ptr(),
                                 nb, stream_of(xyz)),
        "pointconv_fwd_tiled");
  return y;
}

std::tuple<c10::optional<Tensor>, Tensor, Tensor, Tensor, Tensor> pointconv_bwd(
    Tensor xyz, Tensor center, Tensor feats, Tensor idx, Tensor wt, Tensor wl, Tensor dy,
    Tensor offsets, Tensor rank, bool need_xyz) {
  for (auto* t : {&xyz, &center, &feats, &wt, &wl, &dy}) dev(*t, kF, "pointconv input");
  dev(idx, kI, "idx"), dev(offsets, kI, "offsets"), dev(rank, kI, "rank");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1), s = idx.size(1), k = idx.size(2);
  const int64_t d = feats.size(2), o = wl.size(0), c = 3 + d;
  TORCH_CHECK(offsets.numel() >= b * n + 1 && rank.numel() >= b * s * k,
              "kdpc: pointconv_bwd: offsets / rank do not match idx");
  const size_t nb = kdpc_pointconv_bwd_workspace_bytes(b, s, k, d, o);
  TORCH_CHECK(nb > 0, "kdpc: pointconv_bwd: invalid sizes");
  Tensor ws = workspace(nb, xyz);
  Tensor dxyz = need_xyz ? empty_f({b, n, 3}, xyz) : Tensor();
  Tensor dfeats = empty_f({b, n, d}, xyz);
  Tensor dcenter = empty_f({b, s, 3}, xyz);
  Tensor dwt = empty_f({b, s, k, 16}, xyz);
  Tensor dwl = empty_f({o, 16 * c}, xyz);
  check(kdpc_pointconv_bwd(b, n, s, k, d, o, F(xyz), F(center), F(feats), I(idx), F(wt), F(wl),
                           F(dy), I(offsets), I(rank), need_xyz ? F(dxyz) : nullptr, F(dfeats),
                           F(dcenter), F(dwt), F(dwl), ws.data_ptr(), nb, stream_of(xyz)),
        "pointconv_bwd");
  return {need_xyz ? c10::optional<Tensor>(dxyz) : c10::nullopt, dfeats, dcenter, dwt, dwl};
}

std::tuple<c10::optional<Tensor>, Tensor, Tensor, Tensor> pointconv_bwd_data(
    Tensor xyz, Tensor center, Tensor feats, Tensor idx, Tensor wt, Tensor wl, Tensor dy,
    Tensor offsets, Tensor rank, bool need_xyz) {
  for (auto* t : {&xyz, &center, &feats, &wt, &wl, &dy}) dev(*t, kF, "pointconv input");
  dev(idx, kI, "idx"), dev(offsets, kI, "offsets"), dev(rank, kI, "rank");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1), s = idx.size(1), k = idx.size(2);
  const int64_t d = feats.size(2), o = wl.size(0);
  TORCH_CHECK(offsets.numel() >= b * n + 1 && rank.numel() >= b * s * k,
              "kdpc: pointconv_bwd_data: offsets / rank do not match idx");
  const size_t nb = kdpc_pointconv_bwd_workspace_bytes(b, s, k, d, o);
  TORCH_CHECK(nb > 0, "kdpc: pointconv_bwd_data: invalid sizes");
  Tensor ws = workspace(nb, xyz);
  Tensor dxyz = need_xyz ? empty_f({b, n, 3}, xyz) : Tensor();
  Tensor dfeats = empty_f({b, n, d}, xyz);
  Tensor dcenter = empty_f({b, s, 3}, xyz);
  Tensor dwt = empty_f({b, s, k, 16}, xyz);
  check(kdpc_pointconv_bwd_data(b, n, s, k, d, o, F(xyz), F(center), F(feats), I(idx), F(wt),
                                F(wl), F(dy), I(offsets), I(rank), need_xyz ? F(dxyz) : nullptr,
                                F(dfeats), F(dcenter), F(dwt), ws.data_ptr(), nb, stream_of(xyz)),
        "pointconv_bwd_data");
  return {need_xyz ? c10::optional<Tensor>(dxyz) : c10::nullopt, dfeats, dcenter, dwt};
}

// ---- tiled PointConv backward (tile_plan.hip)
Tensor morton_order(Tensor xyz) {
  dev(xyz, kF, "xyz");
  TORCH_CHECK(xyz.dim() == 3 && xyz.size(2) == 3 && xyz.size(1) <= 8192,
              "kdpc: morton_order expects (B,S<=8192,3)");
  GUARD(xyz);
  Tensor order = at::empty({xyz.size(0), xyz.size(1)}, xyz.options().dtype(at::kInt));
  check(kdpc_morton_order(xyz.size(0), xyz.size(1), F(xyz), I(order), stream_of(xyz)),
        "morton_order");
  return order;
}

std::tuple<Tensor, Tensor, Tensor, Tensor> pc_tile_plan(Tensor idx, c10::optional<Tensor> order,
                                                        int64_t n) {
  dev(idx, kI, "idx");
  TORCH_CHECK(idx.dim() == 3, "kdpc: pc_tile_plan expects idx (B,S,K)");
  const int64_t b = idx.size(0), s = idx.size(1), k = idx.size(2);
  const int* op = nullptr;
  if (order.has_value()) {
    dev(*order, kI, "order"), same_device(idx, *order, "order");
    TORCH_CHECK(order->numel() == b * s, "kdpc: pc_tile_plan: order must be (B,S)");
    op = I(*order);
  }
  GUARD(idx);
  const int64_t t = b * ((s + 31) / 32), trk = 32 * k;
  auto io = idx.options();
  Tensor trow = at::empty({t, 32}, io), tpair = at::empty({t, trk}, io);
  Tensor tsoff = at::empty({t, trk + 1}, io), tkey = at::empty({b, t / std::max<int64_t>(b, 1) * trk}, io);
  check(kdpc_pc_tile_plan(b, s, n, k, I(idx), op, I(trow), I(tpair), I(tsoff), I(tkey),
                          stream_of(idx)),
        "pc_tile_plan");
  return {trow, tpair, tsoff, tkey};
}

std::tuple<c10::optional<Tensor>, Tensor, Tensor, Tensor, c10::optional<Tensor>> pointconv_bwd_tiled(
    Tensor xyz, Tensor center, Tensor feats, Tensor idx, Tensor wt, Tensor wl, Tensor dy,
    Tensor offsets, Tensor trow, Tensor tpair, Tensor tsoff, Tensor tdst, bool need_xyz,
    bool weight) {
  for (auto* t : {&xyz, &center, &feats, &wt, &wl, &dy}) dev(*t, kF, "pointconv input");
  for (auto* t : {&idx, &offsets, &trow, &tpair, &tsoff, &tdst}) dev(*t, kI, "tile plan");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1), s = idx.size(1), k = idx.size(2);
  const int64_t d = feats.size(2), o = wl.size(0), c = 3 + d;
  const int64_t tiles = b * ((s + 31) / 32);
  TORCH_CHECK(offsets.numel() >= b * n + 1 && trow.numel() >= tiles * 32 &&
                  tpair.numel() >= tiles * 32 * k && tsoff.numel() >= tiles * (32 * k + 1) &&
                  tdst.numel() >= tiles * 32 * k,
              "kdpc: pointconv_bwd_tiled: the tile plan does not match idx");
  const size_t nb = kdpc_pointconv_bwd_workspace_bytes(b, s, k, d, o);
  TORCH_CHECK(nb > 0, "kdpc: pointconv_bwd_tiled: invalid sizes");
  Tensor ws = workspace(nb, xyz);
  Tensor dxyz = need_xyz ? empty_f({b, n, 3}, xyz) : Tensor();
  Tensor dfeats = empty_f({b, n, d}, xyz);
  Tensor dcenter = empty_f({b, s, 3}, xyz);
  Tensor dwt = empty_f({b, s, k, 16}, xyz);
  Tensor dwl = weight ? empty_f({o, 16 * c}, xyz) : Tensor();
  if (weight)
    check(kdpc_pointconv_bwd_tiled(b, n, s, k, d, o, F(xyz), F(center), F(feats), I(idx), F(wt),
                                   F(wl), F(dy), I(offsets), I(trow), I(tpair), I(tsoff),
                                   I(tdst), need_xyz ? F(dxyz) : nullptr, F(dfeats), F(dcenter),
                                   F(dwt), F(dwl), ws.data_ptr(), nb, stream_of(xyz)),
          "pointconv_bwd_tiled");
  else
    check(kdpc_pointconv_bwd_data_tiled(b, n, s, k, d, o, F(xyz), F(center), F(feats), I(idx),
                                        F(wt), F(wl), F(dy), I(offsets), I(trow), I(tpair),
                                        I(tsoff), I(tdst), need_xyz ? F(dxyz) : nullptr,
                                        F(dfeats), F(dcenter), F(dwt), ws.data_ptr(), nb,
                                        stream_of(xyz)),
          "pointconv_bwd_data_tiled");
  return {need_xyz ? c10::optional<Tensor>(dxyz) : c10::nullopt, dfeats, dcenter, dwt,
          weight ? c10::optional<Tensor>(dwl) : c10::nullopt};
}

Tensor pointconv_bwd_weight(Tensor xyz, Tensor center, Tensor feats, Tensor idx, Tensor wt,
                            Tensor dy, int64_t o) {
  for (auto* t : {&xyz, &center, &feats, &wt, &dy}) dev(*t, kF, "pointconv input");
  dev(idx, kI, "idx");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1), s = idx.size(1), k = idx.size(2);
  const int64_t d = feats.size(2), c = 3 + d;
  TORCH_CHECK(dy.numel() == b * s * o, "kdpc: pointconv_bwd_weight: dy does not match O");
  const size_t nb = kdpc_pointconv_bwd_weight_workspace_bytes(b, s, k, d, o);
  TORCH_CHECK(nb > 0, "kdpc: pointconv_bwd_weight: invalid sizes");
  Tensor ws = workspace(nb, xyz);
  Tensor dwl = empty_f({o, 16 * c}, xyz);
  check(kdpc_pointconv_bwd_weight(b, n, s, k, d, o, F(xyz), F(center), F(feats), I(idx), F(wt),
                                  F(dy), F(dwl), ws.data_ptr(), nb, stream_of(xyz)),
        "pointconv_bwd_weight");
  return dwl;
}

std::tuple<Tensor, Tensor> pointconv_bwd_weight_bias(Tensor xyz, Tensor center, Tensor feats,
                                                     Tensor idx, Tensor wt, Tensor dy,
                                                     int64_t o) {
  for (auto* t : {&xyz, &center, &feats, &wt, &dy}) dev(*t, kF, "pointconv input");
  dev(idx, kI, "idx");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1), s = idx.size(1), k = idx.size(2);
  const int64_t d = feats.size(2), c = 3 + d;
  TORCH_CHECK(dy.numel() == b * s * o, "kdpc: pointconv_bwd_weight_bias: dy does not match O");
  TORCH_CHECK(c % 8 != 0, "kdpc: pointconv_bwd_weight_bias needs C % 8 != 0");
  const size_t nb = kdpc_pointconv_bwd_weight_workspace_bytes(b, s, k, d, o);
  TORCH_CHECK(nb > 0, "kdpc: pointconv_bwd_weight_bias: invalid sizes");
  Tensor ws = workspace(nb, xyz);
  Tensor dwl = empty_f({o, 16 * c}, xyz);
  Tensor dbias = empty_f({o}, xyz);
  check(kdpc_pointconv_bwd_weight_bias(b, n, s, k, d, o, F(xyz), F(center), F(feats), I(idx),
                                       F(wt), F(dy), F(dwl), F(dbias), ws.data_ptr(), nb,
                                       stream_of(xyz)),
        "pointconv_bwd_weight_bias");
  return {dwl, dbias};
}

Tensor pointconv_contract_fwd(Tensor xyz, Tensor center, Tensor feats, Tensor idx, Tensor wt) {
  for (auto* t : {&xyz, &center, &feats, &wt}) dev(*t, kF, "pointconv input");
  dev(idx, kI, "idx");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1), s = idx.size(1), k = idx.size(2);
  const int64_t d = feats.size(2);
  Tensor out = empty_f({b, s, 16 * (3 + d)}, xyz);
  check(kdpc_pointconv_contract_fwd(b, n, s, k, d, F(xyz), F(center), F(feats), I(idx), F(wt),
                                    F(out), stream_of(xyz)), "pointconv_contract_fwd");
  return out;
}

std::tuple<Tensor, Tensor, Tensor> pointconv_contract_bwd(Tensor xyz, Tensor center,
                                                          Tensor feats, Tensor idx, Tensor wt,
                                                          Tensor dout) {
  for (auto* t : {&xyz, &center, &feats, &wt, &dout}) dev(*t, kF, "pointconv input");
  dev(idx, kI, "idx");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1), s = idx.size(1), k = idx.size(2);
  const int64_t d = feats.size(2);
  Tensor dg_rows = empty_f({b, s, k, 3 + d}, xyz);
  Tensor dwt = empty_f({b, s, k, 16}, xyz);
  Tensor dcenter = empty_f({b, s, 3}, xyz);
  check(kdpc_pointconv_contract_bwd(b, n, s, k, d, F(xyz), F(center), F(feats), I(idx), F(wt),
                                    F(dout), F(dg_rows), F(dwt), F(dcenter), stream_of(xyz)),
        "pointconv_contract_bwd");
  return {dg_rows, dwt, dcenter};
}

// ------------------------------------------------------------------- fused WeightNet
Tensor weightnet_fwd(Tensor xyz, Tensor center, Tensor idx, Tensor w0, Tensor b0, Tensor w1,
                     Tensor b1, Tensor w2, Tensor b2) {
  for (auto* t : {&xyz, &center, &w0, &b0, &w1, &b1, &w2, &b2}) dev(*t, kF, "weightnet input");
  dev(idx, kI, "idx");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1), s = idx.size(1), k = idx.size(2);
  Tensor wt = empty_f({b, s, k, 16}, xyz);
  check(kdpc_weightnet_fwd(b, n, s, k, F(xyz), F(center), I(idx), F(w0), F(b0), F(w1), F(b1),
                           F(w2), F(b2), F(wt), stream_of(xyz)), "weightnet_fwd");
  return wt;
}

std::tuple<c10::optional<Tensor>, Tensor> weightnet_bwd(Tensor xyz, Tensor center, Tensor idx, Tensor w0, Tensor b0, Tensor w1,
                 Tensor b1, Tensor w2, Tensor b2, Tensor dwt, bool need_rel) {
  for (auto* t : {&xyz, &center, &w0, &b0, &w1, &b1, &w2, &b2, &dwt})
    dev(*t, kF, "weightnet input");
  dev(idx, kI, "idx");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1), s = idx.size(1), k = idx.size(2);
  const size_t nb = kdpc_weightnet_bwd_workspace_bytes();
  Tensor ws = workspace(nb, xyz);
  Tensor dparams = empty_f({kdpc_weightnet_param_count()}, xyz);
  Tensor drel = need_rel ? empty_f({b, s, k, 3}, xyz) : Tensor();
  check(kdpc_weightnet_bwd(b, n, s, k, F(xyz), F(center), I(idx), F(w0), F(b0), F(w1), F(b1),
                           F(w2), F(b2), F(dwt), need_rel ? F(drel) : nullptr, F(dparams),
                           ws.data_ptr(), nb, stream_of(xyz)), "weightnet_bwd");
  return {need_rel ? c10::optional<Tensor>(drel) : c10::nullopt, dparams};
}

Tensor weightnet_bwd_rel(Tensor xyz, Tensor center, Tensor idx, Tensor w0, Tensor b0, Tensor w1,
                         Tensor b1, Tensor w2, Tensor b2, Tensor dwt) {
  for (auto* t : {&xyz, &center, &w0, &b0, &w1, &b1, &w2, &b2, &dwt})
    dev(*t, kF, "weightnet input");
  dev(idx, kI, "idx");
  GUARD(xyz);
  const int64_t b = xyz.size(0), n = xyz.size(1), s = idx.size(1), k = idx.size(2);
  Tensor drel = empty_f({b, s, k, 3}, xyz);
  check(kdpc_weightnet_bwd_rel(b, n, s, k, F(xyz), F(center), I(idx), F(w0), F(b0), F(w1),
                               F(b1), F(w2), F(b2), F(dwt), F(drel), stream_of(xyz)),
        "weightnet_bwd_rel");
  return drel;
}

// ---------------------------------------------------- WeightNet-weighted neighbour sums
Tensor wn_wsum_fwd(Tensor dir, c10::optional<Tensor> idx, Tensor v, Tensor w0, Tensor b0,
                   Tensor w1, Tensor b1, Tensor w2, Tensor b2) {
  for (auto* t : {&dir, &v, &w0, &b0, &w1, &b1, &w2, &b2}) dev(*t, kF, "wn_wsum input");
  if (idx) dev(*idx, kI, "idx");
  GUARD(dir);
  const int64_t b = dir.size(0), n = dir.size(1), k = dir.size(2), c = w2.size(0);
  const int64_t m = idx ? v.size(1) : 1;
  Tensor out = empty_f({b, n, c}, dir);
  check(kdpc_wn_wsum_fwd(b, n, m, k, c, F(dir), idx ? I(*idx) : nullptr, F(v), F(w0), F(b0),
                         F(w1), F(b1), F(w2), F(b2), F(out), stream_of(dir)), "wn_wsum_fwd");
  return out;
}

std::tuple<Tensor, Tensor, Tensor> wn_wsum_bwd(Tensor dir, c10::optional<Tensor> idx, Tensor v,
                                               Tensor w0, Tensor b0, Tensor w1, Tensor b1,
                                               Tensor w2, Tensor b2, Tensor dout) {
  for (auto* t : {&dir, &v, &w0, &b0, &w1, &b1, &w2, &b2, &dout}) dev(*t, kF, "wn_wsum input");
  if (idx) dev(*idx, kI, "idx");
  GUARD(dir);
  const int64_t b = dir.size(0), n = dir.size(1), k = dir.size(2), c = w2.size(0);
  const int64_t m = idx ? v.size(1) : 1;
  const size_t nb = kdpc_wn_wsum_bwd_workspace_bytes(b, n, c);
  Tensor ws = workspace(nb, dir);
  Tensor dv_rows = empty_f({b, n, k, c}, dir);
  Tensor ddir = empty_f({b, n, k, 3}, dir);
  Tensor dparams = empty_f({kdpc_wn_wsum_param_count(c)}, dir);
  check(kdpc_wn_wsum_bwd(b, n, m, k, c, F(dir), idx ? I(*idx) : nullptr, F(v), F(w0), F(b0),
                         F(w1), F(b1), F(w2), F(b2), F(dout), F(dv_rows), F(ddir), F(dparams),
                         ws.data_ptr(), nb, stream_of(dir)), "wn_wsum_bwd");
  return {dv_rows, ddir, dparams};
}

// ------------------------------------------------------- BatchNorm1d + LeakyReLU, colsum
std::tuple<Tensor, Tensor, Tensor> batchnorm_lrelu_fwd(Tensor x, Tensor weight, Tensor bias,
                                                       double eps, double momentum,
                                                       double slope,
                                                       c10::optional<Tensor> run_mean,
                                                       c10::optional<Tensor> run_var) {
  dev(x, kF, "x"), dev(weight, kF, "weight"), dev(bias, kF, "bias");
  if (run_mean) dev(*run_mean, kF, "running_mean");
  if (run_var) dev(*run_var, kF, "running_var");
  GUARD(x);
  const int64_t r = x.size(0), c = x.size(1);
  const size_t nb = kdpc_batchnorm_workspace_bytes(r, c);
  Tensor ws = workspace(nb, x);
  Tensor y = at::empty_like(x);
  Tensor mean = empty_f({c}, x), invstd = empty_f({c}, x);
  check(kdpc_batchnorm_lrelu_fwd(r, c, F(x), F(weight), F(bias), (float)eps, (float)momentum,
                                 (float)slope, Fo(run_mean), Fo(run_var), F(mean), F(invstd),
                                 F(y), ws.data_ptr(), nb, stream_of(x)), "batchnorm_lrelu_fwd");
  return {y, mean, invstd};
}

Tensor batchnorm_lrelu_apply(Tensor x, Tensor mean, Tensor invstd, Tensor weight, Tensor bias,
                             double slope) {
  for (auto* t : {&x, &mean, &invstd, &weight, &bias}) dev(*t, kF, "batchnorm input");
  GUARD(x);
  Tensor y = at::empty_like(x);
  check(kdpc_batchnorm_lrelu_apply(x.size(0), x.size(1), F(x), F(mean), F(invstd), F(weight),
                                   F(bias), (float)slope, F(y), stream_of(x)),
        "batchnorm_lrelu_apply");
  return y;
}

std::tuple<Tensor, Tensor, Tensor> batchnorm_lrelu_bwd(Tensor dy, Tensor y, Tensor x,
                                                       Tensor weight, Tensor mean,
                                                       Tensor invstd, double slope) {
  for (auto* t : {&dy, &y, &x, &weight, &mean, &invstd}) dev(*t, kF, "batchnorm input");
  GUARD(x);
  const int64_t r = x.size(0), c = x.size(1);
  const size_t nb = kdpc_batchnorm_workspace_bytes(r, c);
  Tensor ws = workspace(nb, x);
  Tensor dx = at::empty_like(x), dw = empty_f({c}, x), db = empty_f({c}, x);
  check(kdpc_batchnorm_lrelu_bwd(r, c, F(dy), F(y), F(x), F(weight), F(mean), F(invstd),
                                 (float)slope, F(dx), F(dw), F(db), ws.data_ptr(), nb,
                                 stream_of(x)), "batchnorm_lrelu_bwd");
  return {dx, dw, db};
}

Tensor neg_sum_k(Tensor x) {
  dev(x, kF, "x");
  TORCH_CHECK(x.dim() >= 2, "kdpc: neg_sum_k expects (..., K, C)");
  GUARD(x);
  const int64_t k = x.size(-2), c = x.size(-1);
  const int64_t m = k * c == 0 ? 0 : x.numel() / (k * c);
  std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end() - 2);
  shape.push_back(c);
  Tensor out = at::empty(shape, x.options());
  TORCH_CHECK(m < (int64_t(1) << 31), "kdpc: neg_sum_k: too many rows");
  check(kdpc_neg_sum_k((int)m, k, c, F(x), F(out), stream_of(x)), "neg_sum_k");
  return out;
}

// Adam over flat buffers (kdpc_adam_step): param / exp_avg / exp_avg_sq in place
void adam_step(Tensor param, Tensor grad, Tensor exp_avg, Tensor exp_avg_sq, Tensor lr,
               Tensor step, double beta1, double beta2, double eps, double weight_decay,
               bool maximize, int64_t mode) {
  dev(param, kF, "param");
  dev(grad, kF, "grad");
  dev(exp_avg, kF, "exp_avg");
  dev(exp_avg_sq, kF, "exp_avg_sq");
  dev(lr, kF, "lr");
  dev(step, kF, "step");
  const int64_t n = param.numel();
  TORCH_CHECK(grad.numel() == n && exp_avg.numel() == n && exp_avg_sq.numel() == n,
              "kdpc: adam_step: buffers of different sizes");
  TORCH_CHECK(lr.numel() == 1 && step.numel() == 1, "kdpc: adam_step: lr / step must be scalars");
  GUARD(param);
  check(kdpc_adam_step(n, F(param), F(grad), F(exp_avg), F(exp_avg_sq), F(lr), F(step), beta1,
                       beta2, eps, weight_decay, maximize ? 1 : 0, (int)mode,
                       stream_of(param)),
        "adam_step");
}

// dst[i] <- src[i] for same-size contiguous tensors on one device, one launch per 128 pairs
void copy_segments(at::TensorList dst, at::TensorList src) {
  TORCH_CHECK(dst.size() == src.size(), "kdpc: copy_segments: ", dst.size(), " destinations, ",
              src.size(), " sources");
  if (dst.empty()) return;
  std::vector<const void*> sp;
  std::vector<void*> dp;
  std::vector<long long> nb;
  for (size_t i = 0; i < dst.size(); ++i) {
    const Tensor &d = dst[i], &s = src[i];
    TORCH_CHECK(d.is_cuda() && s.is_cuda(), "kdpc: copy_segments: tensors must be on the GPU");
    same_device(dst[0], d, "dst"), same_device(dst[0], s, "src");
    TORCH_CHECK(d.is_contiguous() && s.is_contiguous() && d.dtype() == s.dtype() &&
                    d.numel() == s.numel(),
                "kdpc: copy_segments: pair ", i, " must be contiguous, same dtype and size");
    sp.push_back(s.data_ptr());
    dp.push_back(d.data_ptr());
    nb.push_back((long long)s.nbytes());
  }
  GUARD(dst[0]);
  check(kdpc_copy_segments((int)dst.size(), sp.data(), dp.data(), nb.data(), stream_of(dst[0])),
        "copy_segments");
}

Tensor colsum(Tensor x) {
  dev(x, kF, "src");
  TORCH_CHECK(x.dim() == 2, "kdpc: colsum expects a (rows, len) tensor");
  GUARD(x);
  const int64_t r = x.size(0), l = x.size(1);
  const size_t nb = kdpc_colsum_workspace_bytes(r, l);
  Tensor ws = workspace(nb, x);
  Tensor out = empty_f({l}, x);
  check(kdpc_colsum(r, l, F(x), F(out), ws.data_ptr(), nb, stream_of(x)), "colsum");
  return out;
}


}  // namespace

// ------------------------------------------- 3-NN inverse-distance blend (idw_blend.hip)
TT idw_blend_fwd(Tensor ref, Tensor qry, Tensor vals, Tensor idx, bool warp) {
  dev(ref, kF, "ref"), dev(qry, kF, "qry"), dev(vals, kF, "vals"), dev(idx, kI, "idx");
  same_device(ref, qry, "qry"), same_device(ref, vals, "vals"), same_device(ref, idx, "idx");
  TORCH_CHECK(ref.dim() == 3 && ref.size(2) == 3 && qry.dim() == 3 && qry.size(2) == 3 &&
                  vals.dim() == 3 && idx.dim() == 3 && idx.size(2) == 3 &&
                  vals.size(1) == ref.size(1) && idx.size(1) == qry.size(1) &&
                  ref.size(0) == qry.size(0) && vals.size(0) == ref.size(0) &&
                  idx.size(0) == ref.size(0),
              "kdpc: idw_blend expects ref (B,S,3), qry (B,N,3), vals (B,S,C), idx (B,N,3)");
  GUARD(ref);
  const int64_t b = ref.size(0), s = ref.size(1), n = qry.size(1), c = vals.size(2);
  Tensor out = empty_f({b, n, c}, ref);
  Tensor w = empty_f({b, n, 3}, ref);
  check(kdpc_idw_blend_fwd(b, n, s, c, F(ref), F(qry), F(vals), I(idx), F(out), F(w), warp,
                           stream_of(ref)), "idw_blend_fwd");
  return {out, w};
}

Tensor idw_blend_bwd_vals(Tensor dout, Tensor w, Tensor offsets, Tensor perm, int64_t s,
                          bool warp) {
  dev(dout, kF, "dout"), dev(w, kF, "w"), dev(offsets, kI, "offsets"), dev(perm, kI, "perm");
  same_device(dout, w, "w"), same_device(dout, offsets, "offsets");
  same_device(dout, perm, "perm");
  TORCH_CHECK(dout.dim() == 3 && w.dim() == 3 && w.size(2) == 3 && w.size(1) == dout.size(1) &&
                  w.size(0) == dout.size(0),
              "kdpc: idw_blend_bwd_vals expects dout (B,N,C), w (B,N,3)");
  const int64_t b = dout.size(0), n = dout.size(1), c = dout.size(2);
  TORCH_CHECK(s >= 0 && offsets.numel() == b * s + 1 && perm.numel() == b * n * 3,
              "kdpc: idw_blend_bwd_vals expects the CSR of idx (B,N,3) over S keys: offsets "
              "(B*S+1), perm (B*N*3); got ", offsets.numel(), " and ", perm.numel());
  GUARD(dout);
  Tensor dvals = empty_f({b, s, c}, dout);
  check(kdpc_idw_blend_bwd_vals(b, n, s, c, F(dout), F(w), I(offsets), I(perm), F(dvals), warp,
                                stream_of(dout)), "idw_blend_bwd_vals");
  return dvals;
}

TT idw_blend_bwd_coords(Tensor ref, Tensor qry, Tensor vals, Tensor idx, Tensor dout,
                        bool warp) {
  dev(ref, kF, "ref"), dev(qry, kF, "qry"), dev(vals, kF, "vals"), dev(idx, kI, "idx");
  dev(dout, kF, "dout");
  same_device(ref, qry, "qry"), same_device(ref, vals, "vals"), same_device(ref, idx, "idx");
  same_device(ref, dout, "dout");
  TORCH_CHECK(ref.dim() == 3 && ref.size(2) == 3 && qry.dim() == 3 && qry.size(2) == 3 &&
                  vals.dim() == 3 && idx.dim() == 3 && idx.size(2) == 3 &&
                  vals.size(1) == ref.size(1) && idx.size(1) == qry.size(1) &&
                  ref.size(0) == qry.size(0) && vals.size(0) == ref.size(0) &&
                  idx.size(0) == ref.size(0),
              "kdpc: idw_blend_bwd_coords expects ref (B,S,3), qry (B,N,3), vals (B,S,C), "
              "idx (B,N,3)");
  GUARD(ref);
  const int64_t b = ref.size(0), s = ref.size(1), n = qry.size(1), c = vals.size(2);
  TORCH_CHECK(dout.dim() == 3 && dout.size(0) == b && dout.size(1) == n && dout.size(2) == c,
              "kdpc: idw_blend_bwd_coords expects dout (B,N,C)");
  Tensor drow = empty_f({b, n * 3, 3}, ref);
  Tensor dq = empty_f({b, n, 3}, ref);
  check(kdpc_idw_blend_bwd_coords(b, n, s, c, F(ref), F(qry), F(vals), I(idx), F(dout),
                                  F(drow), F(dq), warp, stream_of(ref)), "idw_blend_bwd_coords");
  return {drow, dq};
}

// -------------------------------------- skinny weight gradients (dense_small.hip)
Tensor dense_tn_small(Tensor a, Tensor b) {
  dev(a, kF, "a"), dev(b, kF, "b"), same_device(a, b, "b");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(0) == b.size(0),
              "kdpc: dense_tn_small expects a (R,O), b (R,I)");
  GUARD(a);
  const int64_t r = a.size(0), o = a.size(1), i = b.size(1);
  const size_t nb = kdpc_dense_tn_small_workspace_bytes(r, o, i);
  TORCH_CHECK(nb > 0, "kdpc: dense_tn_small: unsupported shape r=", r, " o=", o, " i=", i);
  Tensor ws = workspace(nb, a);
  Tensor out = empty_f({o, i}, a);
  check(kdpc_dense_tn_small(r, o, i, F(a), F(b), F(out), ws.data_ptr(), nb, stream_of(a)),
        "dense_tn_small");
  return out;
}

Tensor dense_small(Tensor x, Tensor m, c10::optional<Tensor> bias) {
  dev(x, kF, "x"), dev(m, kF, "m"), same_device(x, m, "m");
  TORCH_CHECK(x.dim() == 2 && m.dim() == 2 && x.size(1) == m.size(0),
              "kdpc: dense_small expects x (R,K), m (K,N)");
  const int64_t r = x.size(0), k = x.size(1), n = m.size(1);
  TORCH_CHECK(std::min(k, n) <= 4 && k * n <= 4096, "kdpc: dense_small: unsupported k=", k,
              " n=", n);
  const float* bp = nullptr;
  if (bias.has_value()) {
    dev(*bias, kF, "bias");
    TORCH_CHECK(bias->numel() == n, "kdpc: dense_small: bias must have N entries");
    bp = F(*bias);
  }
  GUARD(x);
  Tensor y = empty_f({r, n}, x);
  check(kdpc_dense_small(r, k, n, F(x), F(m), bp, F(y), stream_of(x)), "dense_small");
  return y;
}

// the same into a caller tensor (a contiguous (R, N) view of an N-d output the caller owns)
void dense_small_out(Tensor x, Tensor m, c10::optional<Tensor> bias, Tensor y) {
  dev(x, kF, "x"), dev(m, kF, "m"), dev(y, kF, "y"), same_device(x, y, "y");
  TORCH_CHECK(x.dim() == 2 && m.dim() == 2 && x.size(1) == m.size(0) && y.dim() == 2 &&
                  y.size(0) == x.size(0) && y.size(1) == m.size(1) && y.is_contiguous(),
              "kdpc: dense_small_out expects x (R,K), m (K,N), y (R,N) contiguous");
  const int64_t r = x.size(0), k = x.size(1), n = m.size(1);
  TORCH_CHECK(std::min(k, n) <= 4 && k * n <= 4096, "kdpc: dense_small: unsupported k=", k,
              " n=", n);
  const float* bp = nullptr;
  if (bias.has_value()) {
    dev(*bias, kF, "bias");
    TORCH_CHECK(bias->numel() == n, "kdpc: dense_small: bias must have N entries");
    bp = F(*bias);
  }
  GUARD(x);
  check(kdpc_dense_small(r, k, n, F(x), F(m), bp, F(y), stream_of(x)), "dense_small");
}

TORCH_LIBRARY(kdpc, m) {
  // reference pointnet2_cuda surface (pointnet2_api.cpp:10-24), in-place, returns 1
  m.def("ball_query_wrapper(int b, int n, int m, float radius, int nsample, Tensor new_xyz, "
        "Tensor xyz, Tensor(a!) idx) -> int");
  m.def("group_points_wrapper(int b, int c, int n, int npoints, int nsample, Tensor points, "
        "Tensor idx, Tensor(a!) out) -> int");
  m.def("group_points_grad_wrapper(int b, int c, int n, int npoints, int nsample, "
        "Tensor grad_out, Tensor idx, Tensor(a!) grad_points) -> int");
  m.def("gather_points_wrapper(int b, int c, int n, int npoints, Tensor points, Tensor idx, "
        "Tensor(a!) out) -> int");
  m.def("gather_points_grad_wrapper(int b, int c, int n, int npoints, Tensor grad_out, "
        "Tensor idx, Tensor(a!) grad_points) -> int");
  m.def("furthest_point_sampling_wrapper(int b, int n, int m, Tensor points, Tensor(a!) temp, "
        "Tensor(b!) idx) -> int");
  m.def("three_nn_wrapper(int b, int n, int m, Tensor unknown, Tensor known, "
        "Tensor(a!) dist2, Tensor(b!) idx) -> int");
  m.def("three_interpolate_wrapper(int b, int c, int m, int n, Tensor points, Tensor idx, "
        "Tensor weight, Tensor(a!) out) -> int");
  m.def("three_interpolate_grad_wrapper(int b, int c, int n, int m, Tensor grad_out, "
        "Tensor idx, Tensor weight, Tensor(a!) grad_points) -> int");
  // functional ops used by the drop-in layers
  m.def("furthest_point_sample(Tensor xyz, int npoint) -> Tensor");
  m.def("gather_points(Tensor points, Tensor idx) -> Tensor");
  m.def("ball_query(float radius, int nsample, Tensor xyz, Tensor new_xyz) -> Tensor");
  m.def("group_points(Tensor points, Tensor idx) -> Tensor");
  m.def("three_nn(Tensor unknown, Tensor known) -> (Tensor, Tensor)");
  m.def("three_interpolate(Tensor points, Tensor idx, Tensor weight) -> Tensor");
  m.def("knn_point(int nsample, Tensor xyz, Tensor new_xyz, bool seeded=True) -> Tensor");
  m.def("knn_point_dist(int nsample, Tensor xyz, Tensor new_xyz, bool seeded=True) "
        "-> (Tensor, Tensor)");
  m.def("knn_feature(int nsample, Tensor ref, Tensor query) -> Tensor");
  m.def("knn_feature_dist(int nsample, Tensor ref, Tensor query) -> (Tensor, Tensor)");
  m.def("group_rows(Tensor points, Tensor idx) -> Tensor");
  m.def("csr_build(Tensor idx, int n) -> (Tensor, Tensor)");
  m.def("group_rows_grad(Tensor grad_out, Tensor offsets, Tensor perm, int n) -> Tensor");
  m.def("csr_rank(Tensor idx, Tensor offsets, Tensor perm, int n) -> Tensor");
  m.def("csr_sum_channels(Tensor src, Tensor offsets, Tensor perm, int b, int c, int n) "
        "-> Tensor");
  m.def("three_interpolate_grad_csr(Tensor grad_out, Tensor weight, Tensor offsets, "
        "Tensor perm, int m) -> Tensor");
  m.def("cost_volume_fwd(Tensor x1, Tensor x2, Tensor idx, Tensor p1, Tensor p2, Tensor wpos, "
        "Tensor bpos, Tensor w1, Tensor b1) -> (Tensor, Tensor)");
  m.def("cost_volume_bwd(Tensor x1, Tensor x2, Tensor idx, Tensor p1, Tensor p2, Tensor wpos, "
        "Tensor bpos, Tensor w1, Tensor out, Tensor amax, Tensor gout, Tensor? slope0=None) "
        "-> (Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("cost_volume_bwd_csr(Tensor x1, Tensor x2, Tensor idx, Tensor p1, Tensor p2, "
        "Tensor wpos, Tensor bpos, Tensor w1, Tensor out, Tensor amax, Tensor gout, "
        "Tensor offsets, Tensor rank, Tensor? slope0=None) "
        "-> (Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("cost_volume_wide_h0(Tensor x1, Tensor x2, Tensor idx, Tensor p1, Tensor p2, "
        "Tensor wpos, Tensor bpos) -> Tensor");
  m.def("cost_volume_wide_max(Tensor z1, int b, int n1, int k, int dout) -> (Tensor, Tensor)");
  m.def("cost_volume_wide_max_bwd(Tensor gout, Tensor out, Tensor amax, int k) "
        "-> (Tensor, Tensor)");
  m.def("cost_volume_wide_h0_bwd(Tensor x1, Tensor x2, Tensor idx, Tensor h0, Tensor(a!) dz) "
        "-> (Tensor, Tensor)");
  m.def("pointconv_fwd(Tensor xyz, Tensor center, Tensor feats, Tensor idx, Tensor wt, "
        "Tensor wl, Tensor bias) -> Tensor");
  m.def("pointconv_bwd(Tensor xyz, Tensor center, Tensor feats, Tensor idx, Tensor wt, "
        "Tensor wl, Tensor dy, Tensor offsets, Tensor rank, bool need_xyz) "
        "-> (Tensor?, Tensor, Tensor, Tensor, Tensor)");
  m.def("pointconv_bwd_data(Tensor xyz, Tensor center, Tensor feats, Tensor idx, Tensor wt, "
        "Tensor wl, Tensor dy, Tensor offsets, Tensor rank, bool need_xyz) "
        "-> (Tensor?, Tensor, Tensor, Tensor)");
  m.def("pointconv_bwd_weight(Tensor xyz, Tensor center, Tensor feats, Tensor idx, Tensor wt, "
        "Tensor dy, int o) -> Tensor");
  m.def("morton_order(Tensor xyz) -> Tensor");
  m.def("pointconv_bwd_weight_bias(Tensor xyz, Tensor center, Tensor feats, Tensor idx, "
        "Tensor wt, Tensor dy, int o) -> (Tensor, Tensor)");
  m.def("pointconv_fwd_tiled(Tensor xyz, Tensor center, Tensor feats, Tensor idx, Tensor wt, "
        "Tensor wl, Tensor bias, Tensor trow) -> Tensor");
  m.def("pc_tile_plan(Tensor idx, Tensor? order, int n) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("pointconv_bwd_tiled(Tensor xyz, Tensor center, Tensor feats, Tensor idx, Tensor wt, "
        "Tensor wl, Tensor dy, Tensor offsets, Tensor trow, Tensor tpair, Tensor tsoff, "
        "Tensor tdst, bool need_xyz, bool weight) -> (Tensor?, Tensor, Tensor, Tensor, Tensor?)");
  m.def("pointconv_contract_fwd(Tensor xyz, Tensor center, Tensor feats, Tensor idx, "
        "Tensor wt) -> Tensor");
  m.def("pointconv_contract_bwd(Tensor xyz, Tensor center, Tensor feats, Tensor idx, "
        "Tensor wt, Tensor dout) -> (Tensor, Tensor, Tensor)");
  m.def("weightnet_fwd(Tensor xyz, Tensor center, Tensor idx, Tensor w0, Tensor b0, Tensor w1, "
        "Tensor b1, Tensor w2, Tensor b2) -> Tensor");
  m.def("weightnet_bwd(Tensor xyz, Tensor center, Tensor idx, Tensor w0, Tensor b0, Tensor w1, "
        "Tensor b1, Tensor w2, Tensor b2, Tensor dwt, bool need_rel) -> (Tensor?, Tensor)");
  m.def("weightnet_bwd_rel(Tensor xyz, Tensor center, Tensor idx, Tensor w0, Tensor b0, "
        "Tensor w1, Tensor b1, Tensor w2, Tensor b2, Tensor dwt) -> Tensor");
  m.def("wn_wsum_fwd(Tensor dir, Tensor? idx, Tensor v, Tensor w0, Tensor b0, Tensor w1, "
        "Tensor b1, Tensor w2, Tensor b2) -> Tensor");
  m.def("wn_wsum_bwd(Tensor dir, Tensor? idx, Tensor v, Tensor w0, Tensor b0, Tensor w1, "
        "Tensor b1, Tensor w2, Tensor b2, Tensor dout) -> (Tensor, Tensor, Tensor)");
  m.def("batchnorm_lrelu_fwd(Tensor x, Tensor weight, Tensor bias, float eps, float momentum, "
        "float slope, Tensor(a!)? run_mean, Tensor(b!)? run_var) -> (Tensor, Tensor, Tensor)");
  m.def("batchnorm_lrelu_apply(Tensor x, Tensor mean, Tensor invstd, Tensor weight, "
        "Tensor bias, float slope) -> Tensor");
  m.def("batchnorm_lrelu_bwd(Tensor dy, Tensor y, Tensor x, Tensor weight, Tensor mean, "
        "Tensor invstd, float slope) -> (Tensor, Tensor, Tensor)");
  m.def("colsum(Tensor x) -> Tensor");
  m.def("idw_blend_fwd(Tensor ref, Tensor qry, Tensor vals, Tensor idx, bool warp) "
        "-> (Tensor, Tensor)");
  m.def("idw_blend_bwd_vals(Tensor dout, Tensor w, Tensor offsets, Tensor perm, int s, "
        "bool warp) -> Tensor");
  m.def("idw_blend_bwd_coords(Tensor ref, Tensor qry, Tensor vals, Tensor idx, Tensor dout, "
        "bool warp) -> (Tensor, Tensor)");
  m.def("dense_tn_small(Tensor a, Tensor b) -> Tensor");
  m.def("neg_sum_k(Tensor x) -> Tensor");
  m.def("copy_segments(Tensor(a!)[] dst, Tensor[] src) -> ()");
  m.def("adam_step(Tensor(a!) param, Tensor grad, Tensor(b!) exp_avg, Tensor(c!) exp_avg_sq, "
        "Tensor lr, Tensor step, float beta1, float beta2, float eps, float weight_decay, "
        "bool maximize, int mode) -> ()");
  m.def("dense_small(Tensor x, Tensor m, Tensor? bias) -> Tensor");
  m.def("dense_small_out(Tensor x, Tensor m, Tensor? bias, Tensor(a!) y) -> ()");
}

TORCH_LIBRARY_IMPL(kdpc, CUDA, m) {
  m.impl("ball_query_wrapper", ball_query_wrapper);
  m.impl("group_points_wrapper", group_points_wrapper);
  m.impl("group_points_grad_wrapper", group_points_grad_wrapper);
  m.impl("gather_points_wrapper", gather_points_wrapper);
  m.impl("gather_points_grad_wrapper", gather_points_grad_wrapper);
  m.impl("furthest_point_sampling_wrapper", furthest_point_sampling_wrapper);
  m.impl("three_nn_wrapper", three_nn_wrapper);
  m.impl("three_interpolate_wrapper", three_interpolate_wrapper);
  m.impl("three_interpolate_grad_wrapper", three_interpolate_grad_wrapper);
  m.impl("furthest_point_sample", furthest_point_sample);
  m.impl("gather_points", gather_points);
  m.impl("ball_query", ball_query);
  m.impl("group_points", group_points);
  m.impl("three_nn", three_nn);
  m.impl("three_interpolate", three_interpolate);
  m.impl("knn_point", knn_point);
  m.impl("knn_point_dist", knn_point_dist);
  m.impl("group_rows", group_rows);
  m.impl("csr_build", csr_build);
  m.impl("group_rows_grad", group_rows_grad);
  m.impl("csr_rank", csr_rank);
  m.impl("csr_sum_channels", csr_sum_channels);
  m.impl("three_interpolate_grad_csr", three_interpolate_grad_csr);
  m.impl("cost_volume_fwd", cost_volume_fwd);
  m.impl("cost_volume_bwd", cost_volume_bwd);
  m.impl("cost_volume_bwd_csr", cost_volume_bwd_csr);
  m.impl("cost_volume_wide_h0", cost_volume_wide_h0);
  m.impl("cost_volume_wide_max", cost_volume_wide_max);
  m.impl("cost_volume_wide_max_bwd", cost_volume_wide_max_bwd);
  m.impl("cost_volume_wide_h0_bwd", cost_volume_wide_h0_bwd);
  m.impl("pointconv_fwd", pointconv_fwd);
  m.impl("pointconv_bwd", pointconv_bwd);
  m.impl("pointconv_bwd_data", pointconv_bwd_data);
  m.impl("pointconv_bwd_weight", pointconv_bwd_weight);
  m.impl("morton_order", morton_order);
  m.impl("pointconv_bwd_weight_bias", pointconv_bwd_weight_bias);
  m.impl("pointconv_fwd_tiled", pointconv_fwd_tiled);
  m.impl("pc_tile_plan", pc_tile_plan);
  m.impl("pointconv_bwd_tiled", pointconv_bwd_tiled);
  m.impl("pointconv_contract_fwd", pointconv_contract_fwd);
  m.impl("pointconv_contract_bwd", pointconv_contract_bwd);
  m.impl("weightnet_fwd", weightnet_fwd);
  m.impl("weightnet_bwd", weightnet_bwd);
  m.impl("weightnet_bwd_rel", weightnet_bwd_rel);
  m.impl("knn_feature", knn_feature);
  m.impl("knn_feature_dist", knn_feature_dist);
  m.impl("wn_wsum_fwd", wn_wsum_fwd);
  m.impl("wn_wsum_bwd", wn_wsum_bwd);
  m.impl("batchnorm_lrelu_fwd", batchnorm_lrelu_fwd);
  m.impl("batchnorm_lrelu_apply", batchnorm_lrelu_apply);
  m.impl("batchnorm_lrelu_bwd", batchnorm_lrelu_bwd);
  m.impl("colsum", colsum);
  m.impl("idw_blend_fwd", idw_blend_fwd);
  m.impl("idw_blend_bwd_vals", idw_blend_bwd_vals);
  m.impl("idw_blend_bwd_coords", idw_blend_bwd_coords);
  m.impl("dense_tn_small", dense_tn_small);
  m.impl("neg_sum_k", neg_sum_k);
  m.impl("copy_segments", copy_segments);
  m.impl("adam_step", adam_step);
  m.impl("dense_small", dense_small);
  m.impl("dense_small_out", dense_small_out);
}
