// csrc/adam_math.h's Adam update compiled with fast (not correctly rounded) f32 division and
// square root (build_native.py EXTRA_FLAGS); kdpc_adam_step (adam.hip) mode bit 1 selects it.
#include "adam_math.h"

namespace kdpc_adam {
KDPC_ADAM_LAUNCH(launch_fast)
}  // namespace kdpc_adam
