// Strided rows -> dense rows: dst (rows, width) = src rows of `width` floats `ld` floats apart.
// The backward of a feature concatenation (pointconv_util.py: `torch.cat([feats,
// cost_volume], -1)`, the IDW blend's value input) hands each part its gradient as a slice of
// the concatenated gradient: row stride = the concatenated width.  torch's strided copy ran
// such a slice at ~50 GB/s (165 us for the level-0 (8, 8192, 32) slice in the step profile);
// here a thread moves 16-byte pieces (width % 4 == 0 and 16-byte aligned rows) or floats.
#include "kdpc_common.h"

using namespace kdpc;

namespace {

__global__ __launch_bounds__(256) void copy_rows4_kernel(long long n4, int w4, long long ld4,
                                                         const float4* __restrict__ src,
                                                         float4* __restrict__ dst) {
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n4;
       e += (long long)gridDim.x * 256) {
    const long long r = e / w4;
    dst[e] = src[r * ld4 + (e - r * w4)];
  }
}

__global__ __launch_bounds__(256) void copy_rows_kernel(long long n, int w, long long ld,
                                                        const float* __restrict__ src,
                                                        float* __restrict__ dst) {
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n;
       e += (long long)gridDim.x * 256) {
    const long long r = e / w;
    dst[e] = src[r * ld + (e - r * w)];
  }
}

}  // namespace

KDPC_API int kdpc_copy_rows(size_t rows_, int width, const float* src, size_t src_ld_,
                            float* dst, void* stream) {
  const long long rows = (long long)rows_, src_ld = (long long)src_ld_;
  KDPC_CHECK_ARG(rows >= 0 && width >= 0 && src_ld >= width);
  if (rows == 0 || width == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(src && dst);
  hipStream_t st = (hipStream_t)stream;
  const bool vec = (width % 4) == 0 && (src_ld % 4) == 0 &&
                   ((reinterpret_cast<unsigned long long>(src) |
                     reinterpret_cast<unsigned long long>(dst)) & 15ull) == 0;
  const long long n = rows * (long long)width;
  const long long units = vec ? n / 4 : n;
  long long g = divupll(units, 256);
  g = g > 8192 ? 8192 : g;  // grid-stride beyond 2M threads
  if (vec)
    hipLaunchKernelGGL(copy_rows4_kernel, dim3((unsigned)g), dim3(256), 0, st, units, width / 4,
                       src_ld / 4, reinterpret_cast<const float4*>(src),
                       reinterpret_cast<float4*>(dst));
  else
    hipLaunchKernelGGL(copy_rows_kernel, dim3((unsigned)g), dim3(256), 0, st, n, width, src_ld,
                       src, dst);
  KDPC_RETURN_LAUNCH();
}
