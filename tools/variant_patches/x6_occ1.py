# pc_bwd_weight_x6_kernel at one wave per SIMD (512 registers: no spills) instead of two
REPL = [("csrc/pointconv_fused.hip", """template <int O, int KM, bool EX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void pc_bwd_weight_x6_kernel(""", """template <int O, int KM, bool EX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
void pc_bwd_weight_x6_kernel(""")]
