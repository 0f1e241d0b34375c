// f32 products on the bf16 matrix cores ("bf16x6"), shared by the PointConv and cost-volume
// kernels.  Internal linkage (header-only device code).
#pragma once

#include <hip/hip_runtime.h>

namespace kdpc_x6 {

typedef float x6f32x16 __attribute__((ext_vector_type(16)));

// ---- f32 products on the bf16 matrix cores ("bf16x6").  On gfx950 the f32-input MFMA runs at
// the f32 VECTOR rate on the vector ALUs: VALU work beside it does not overlap (measured:
// 32x32x2 f32 chains + VALU fmas, in one wave or in two, take the sum of their times), while a
// bf16 MFMA holds vector issue for 8 of its 32 cycles.  An f32 x is split into three bf16
// planes x = h + m + l + O(2^-24 x) (h = bf16(x), m = bf16(x - h), l = bf16(x - h - m), each a
// round-to-nearest of an exactly representable f32 difference), and a product a b is summed
// as the six plane products of order <= 2^-16 (al bh + am bm + ah bl + am bh + ah bm + ah bh,
// exact products, f32 accumulation): 6 bf16 MFMAs (6 x 32 cycles per 32x32x16 block) for the
// 8 f32 MFMAs (8 x 64 cycles) of the same block, at f32 accuracy (a 32x32x128 product: max
// error 2.7-4.0e-7 of max|C| vs 2.6-4.5e-7 on the f32 MFMA, tools/probe_bf16.hip).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct Planes {
  bf16x8 h, m, l;
};

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r = x - (float)h;
  m = (__bf16)r;
  l = (__bf16)(r - (float)m);
}

__device__ __forceinline__ Planes split8(const float (&x)[8]) {
  Planes p;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    __bf16 h, m, l;
    split3(x[j], h, m, l);
    p.h[j] = h;
    p.m[j] = m;
    p.l[j] = l;
  }
  return p;
}

// acc += A B over one 32x32x16 block, A / B given as planes in the bf16 MFMA operand layout
// (lane (half, i): A[i][8 half + 0..7], B[8 half + 0..7][i]); small products first
__device__ __forceinline__ x6f32x16 mfma_x6(const bf16x8& ah, const bf16x8& am, const bf16x8& al,
                                          const bf16x8& bh, const bf16x8& bm, const bf16x8& bl,
                                          x6f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
}

}  // namespace kdpc_x6
