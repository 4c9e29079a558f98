from .dist import DistContext, init_distributed, shutdown  # noqa: F401
from .dp import (GradAllReducer, broadcast_flat, broadcast_state, check_replicas_equal,  # noqa: F401
                 check_state_equal, state_tensors)
