from .host import ReplayMemory  # noqa: F401
from .device import DeviceReplay  # noqa: F401
from .sumtree import DeviceSumTree  # noqa: F401
from .nstep import NStepAccumulator  # noqa: F401
