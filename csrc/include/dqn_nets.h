// Registration of the Q-network kernels (conv / dense / fused layers).
#pragma once
#include <torch/extension.h>

void register_net_ops(pybind11::module_& m);
