REPL = [("csrc/knn.hip", "__device__ __noinline__ void compact_buffer", "__device__ __forceinline__ void compact_buffer"),
        ("csrc/knn.hip", "__device__ __noinline__ void shrink_buffer", "__device__ __forceinline__ void shrink_buffer")]
