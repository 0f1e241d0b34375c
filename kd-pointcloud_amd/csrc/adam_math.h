// Adam's per-element update, written as torch's fused Adam writes it (ATen
// native/cuda/fused_adam_utils.cuh, adam_math, ADAM_MODE::ORIGINAL, no amsgrad, no grad
// scaling): the beta / eps / weight-decay constants are doubles, so those expressions are
// evaluated in double and rounded to float on assignment; everything else is float.  The
// bits then depend on how the compiler evaluates it (contraction of the double expressions,
// correctly rounded or fast f32 division / square root): csrc/adam.hip and
// csrc/adam_fastdiv.hip compile it under both f32 division / sqrt settings, and the contract /
// no-contract forms below, and tests/test_gpu_adam.py finds the one equal to torch's kernel.
#pragma once
#include <cmath>

#include "kdpc_common.h"

namespace kdpc_adam {

struct Args {
  double beta1, beta2, eps, wd;
  int maximize;
};

// internal linkage: each including file (compiled with its own f32 division / sqrt setting)
// gets its own kernels
namespace {

__device__ __forceinline__ void elem_contract(float& param, float grad, float& exp_avg,
                                              float& exp_avg_sq, double lr, float bc1,
                                              float bc2s, const Args& a) {
  if (a.maximize) grad = -grad;
  if (a.wd != 0) grad += param * a.wd;
  exp_avg = a.beta1 * exp_avg + (1 - a.beta1) * grad;
  exp_avg_sq = a.beta2 * exp_avg_sq + (1 - a.beta2) * grad * grad;
  const float step_size = lr / bc1;
  const float denom = (std::sqrt(exp_avg_sq) / bc2s) + a.eps;
  param -= step_size * exp_avg / denom;
}

__device__ __forceinline__ void elem_plain(float& param, float grad, float& exp_avg,
                                           float& exp_avg_sq, double lr, float bc1, float bc2s,
                                           const Args& a) {
#pragma clang fp contract(off)
  if (a.maximize) grad = -grad;
  if (a.wd != 0) grad += param * a.wd;
  exp_avg = a.beta1 * exp_avg + (1 - a.beta1) * grad;
  exp_avg_sq = a.beta2 * exp_avg_sq + (1 - a.beta2) * grad * grad;
  const float step_size = lr / bc1;
  const float denom = (std::sqrt(exp_avg_sq) / bc2s) + a.eps;
  param -= step_size * exp_avg / denom;
}

template <bool CONTRACT>
__global__ __launch_bounds__(256) void adam_flat_kernel(long long n4, float4* __restrict__ param,
                                                        const float4* __restrict__ grad,
                                                        float4* __restrict__ exp_avg,
                                                        float4* __restrict__ exp_avg_sq,
                                                        const float* __restrict__ lr,
                                                        const float* __restrict__ step, Args a) {
  const double lrd = *lr;
  const float st = *step;
  // as torch: 1 - pow(beta, step) in double (pow of double base and exponent), rounded to
  // float where adam_math takes them
  const float bc1 = (float)(1 - ::pow(a.beta1, (double)st));
  const float bc2s = (float)std::sqrt(1 - ::pow(a.beta2, (double)st));
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    float4 p = param[i], m = exp_avg[i], v = exp_avg_sq[i];
    const float4 g = grad[i];
    if (CONTRACT) {
      elem_contract(p.x, g.x, m.x, v.x, lrd, bc1, bc2s, a);
      elem_contract(p.y, g.y, m.y, v.y, lrd, bc1, bc2s, a);
      elem_contract(p.z, g.z, m.z, v.z, lrd, bc1, bc2s, a);
      elem_contract(p.w, g.w, m.w, v.w, lrd, bc1, bc2s, a);
    } else {
      elem_plain(p.x, g.x, m.x, v.x, lrd, bc1, bc2s, a);
      elem_plain(p.y, g.y, m.y, v.y, lrd, bc1, bc2s, a);
      elem_plain(p.z, g.z, m.z, v.z, lrd, bc1, bc2s, a);
      elem_plain(p.w, g.w, m.w, v.w, lrd, bc1, bc2s, a);
    }
    param[i] = p;
    exp_avg[i] = m;
    exp_avg_sq[i] = v;
  }
}

inline unsigned grid_of(long long n4) {
  const long long g = kdpc::divupll(n4, 256);
  return (unsigned)(g < 4096 ? g : 4096);
}

}  // namespace

#define KDPC_ADAM_LAUNCH(NAME)                                                                  \
  hipError_t NAME(bool contract, long long n4, float* param, const float* grad, float* m,       \
                  float* v, const float* lr, const float* step, const Args& a, hipStream_t st) { \
    if (contract)                                                                               \
      hipLaunchKernelGGL(adam_flat_kernel<true>, dim3(grid_of(n4)), dim3(256), 0, st, n4,       \
                         reinterpret_cast<float4*>(param), reinterpret_cast<const float4*>(grad), \
                         reinterpret_cast<float4*>(m), reinterpret_cast<float4*>(v), lr, step, a); \
    else                                                                                        \
      hipLaunchKernelGGL(adam_flat_kernel<false>, dim3(grid_of(n4)), dim3(256), 0, st, n4,      \
                         reinterpret_cast<float4*>(param), reinterpret_cast<const float4*>(grad), \
                         reinterpret_cast<float4*>(m), reinterpret_cast<float4*>(v), lr, step, a); \
    return hipGetLastError();                                                                   \
  }

hipError_t launch_cr(bool contract, long long n4, float* param, const float* grad, float* m,
                     float* v, const float* lr, const float* step, const Args& a, hipStream_t st);
hipError_t launch_fast(bool contract, long long n4, float* param, const float* grad, float* m,
                       float* v, const float* lr, const float* step, const Args& a,
                       hipStream_t st);

}  // namespace kdpc_adam
