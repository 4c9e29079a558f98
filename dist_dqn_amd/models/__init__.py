from .arch import ArchSpec, ConvSpec, DenseSpec, arch_from_config, build_arch  # noqa: F401
from .params import FlatLayout, ParamStore  # noqa: F401
from .network import Network  # noqa: F401
