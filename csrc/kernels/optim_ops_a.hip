// optim_pack_kernel instantiations for optimizer op(s) -1, 0, 1, 2 (see optim_pack.h: one translation unit
// per group so the build compiles the fused optimizer variants in parallel).
#define DQN_OPTIM_DEFINE_OPS
#include "optim_pack.h"

namespace dqn {
template void optim_pack_op<-1>(const OptPackLaunch&);
template void optim_pack_op<0>(const OptPackLaunch&);
template void optim_pack_op<1>(const OptPackLaunch&);
template void optim_pack_op<2>(const OptPackLaunch&);
}  // namespace dqn
