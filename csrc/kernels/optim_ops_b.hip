// optim_pack_kernel instantiations for optimizer op(s) 4, 5, 6 (see optim_pack.h: one translation unit
// per group so the build compiles the fused optimizer variants in parallel).
#define DQN_OPTIM_DEFINE_OPS
#include "optim_pack.h"

namespace dqn {
template void optim_pack_op<4>(const OptPackLaunch&);
template void optim_pack_op<5>(const OptPackLaunch&);
template void optim_pack_op<6>(const OptPackLaunch&);
}  // namespace dqn
