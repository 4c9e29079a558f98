"""Loader for the in-tree native extension ``dist_dqn_amd/_C*.so``.

Built by ``python setup.py build_ext --inplace`` (or ``__graft_entry__.build()``)
with hipcc for gfx950. On a GPU process every device op goes through it; if
it is missing there we raise instead of silently falling back to PyTorch.
"""
from __future__ import annotations

import importlib
import os

_mods = {}
_errs = {}


def load(required: bool = False, variant: str = ''):
    """The native module: '' -> _C (bf16 network kernels), 'f16' -> _C_f16 (fp16 network
    kernels), 'f32' -> _C_f32 (fp32 network kernels; csrc/include/dqn_act.h). DQN_DEBUG_EXT=1
    swaps in the bounds-checked debug build (_C_debug, bf16) for the default variant."""
    name = {'f16': '_C_f16', 'f32': '_C_f32'}.get(variant, '_C')
    if name == '_C' and os.environ.get('DQN_DEBUG_EXT', '0') == '1':
        name = '_C_debug'
    if name not in _mods and name not in _errs:
        try:
            _mods[name] = importlib.import_module('dist_dqn_amd.' + name)
        except Exception as e:  # pragma: no cover - depends on build
            _errs[name] = e
    mod = _mods.get(name)
    if mod is None and required:
        raise RuntimeError(
            'dist_dqn_amd native extension %s is not built/importable (%r). Run '
            '`python setup.py build_ext --inplace` (PYTORCH_ROCM_ARCH=gfx950).' % (name, _errs.get(name)))
    return mod


def available() -> bool:
    return load() is not None


def path() -> str:
    ext = load()
    return getattr(ext, '__file__', '') if ext is not None else ''


def hip_required() -> bool:
    """Env override for tests: DQN_ALLOW_TORCH_FALLBACK=1 permits torch ops on GPU."""
    return os.environ.get('DQN_ALLOW_TORCH_FALLBACK', '0') != '1'
