// Adam over the graphed step's flat parameter buffer in one full-chip launch.
//
// distill.GraphedStep lays every trained parameter, its gradient and Adam's two moments out
// as views of four flat buffers (distill.py _flat_adam).  torch's fused Adam ran over them as
// 7 multi-tensor launches of 40-57 workgroups each (one 65,536-element chunk per workgroup):
// 308 us per step for ~20 M parameters, 1.9 TB/s (round-6 trace).  Here one grid-stride
// launch of 16-byte vectors with torch's per-element update (csrc/adam_math.h), so the
// graphed step stays bit-identical to the eager per-parameter optimizer
// (tests/test_gpu_adam.py, tests/test_gpu_graph.py).  The reference trains with
// torch.optim.Adam (distilTrain.py:134-135, config_train_kd_pointconv.yaml:15-24).
// This file: correctly rounded f32 division / square root (adam_fastdiv.hip: the fast ones).
#include "adam_math.h"

namespace kdpc_adam {
KDPC_ADAM_LAUNCH(launch_cr)
}  // namespace kdpc_adam

KDPC_API int kdpc_adam_step(long long n, float* param, const float* grad, float* exp_avg,
                            float* exp_avg_sq, const float* lr, const float* step, double beta1,
                            double beta2, double eps, double weight_decay, int maximize,
                            int mode, void* stream) {
  KDPC_CHECK_ARG(n >= 0 && n % 4 == 0 && mode >= 0 && mode <= 3);
  if (n == 0) return (int)hipSuccess;
  KDPC_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && lr && step);
  KDPC_CHECK_ARG(((reinterpret_cast<unsigned long long>(param) |
                   reinterpret_cast<unsigned long long>(grad) |
                   reinterpret_cast<unsigned long long>(exp_avg) |
                   reinterpret_cast<unsigned long long>(exp_avg_sq)) & 15ull) == 0);
  const kdpc_adam::Args a{beta1, beta2, eps, weight_decay, maximize ? 1 : 0};
  const bool contract = (mode & 1) != 0;
  auto launch = (mode & 2) ? kdpc_adam::launch_fast : kdpc_adam::launch_cr;
  return (int)launch(contract, n / 4, param, grad, exp_avg, exp_avg_sq, lr, step, a,
                     (hipStream_t)stream);
}
