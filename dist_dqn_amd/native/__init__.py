"""Torch-free native host runtime (``libdqn_host.so``) loaded through ctypes."""
from .hostlib import HostLib, load  # noqa: F401
