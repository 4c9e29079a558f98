// optim_pack_kernel instantiations for optimizer op(s) 7 (see optim_pack.h: one translation unit
// per group so the build compiles the fused optimizer variants in parallel).
#define DQN_OPTIM_DEFINE_OPS
#include "optim_pack.h"

namespace dqn {
template void optim_pack_op<7>(const OptPackLaunch&);
}  // namespace dqn
