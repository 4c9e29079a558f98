from .dist import DistContext, init_distributed, shutdown  # noqa: F401
from .dp import GradAllReducer, broadcast_flat, check_replicas_equal  # noqa: F401
