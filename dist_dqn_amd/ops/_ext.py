"""Loader for the in-tree native extension ``dist_dqn_amd/_C*.so``.

Built by ``python setup.py build_ext --inplace`` (or ``__graft_entry__.build()``)
with hipcc for gfx950. On a GPU process every device op goes through it; if
it is missing there we raise instead of silently falling back to PyTorch.
"""
from __future__ import annotations

import importlib
import os

_ext = None
_err = None


def load(required: bool = False):
    global _ext, _err
    if _ext is None and _err is None:
        try:
            # DQN_DEBUG_EXT=1: the bounds-checked debug build (DQN_DEBUG=1 python setup.py build_ext)
            name = '_C_debug' if os.environ.get('DQN_DEBUG_EXT', '0') == '1' else '_C'
            _ext = importlib.import_module('dist_dqn_amd.' + name)
        except Exception as e:  # pragma: no cover - depends on build
            _err = e
    if _ext is None and required:
        raise RuntimeError(
            'dist_dqn_amd native extension is not built/importable (%r). Run '
            '`python setup.py build_ext --inplace` (PYTORCH_ROCM_ARCH=gfx950).' % (_err,))
    return _ext


def available() -> bool:
    return load() is not None


def path() -> str:
    ext = load()
    return getattr(ext, '__file__', '') if ext is not None else ''


def hip_required() -> bool:
    """Env override for tests: DQN_ALLOW_TORCH_FALLBACK=1 permits torch ops on GPU."""
    return os.environ.get('DQN_ALLOW_TORCH_FALLBACK', '0') != '1'
