// Bindings for the Q-network layer kernels (filled in by csrc/kernels/conv*.hip, dense*.hip).
#include "include/dqn_nets.h"

void register_net_ops(pybind11::module_& m) { (void)m; }
