"""roctx ranges around the host-side phases: learner step / graph
replay, all-reduce, actor step, Ape-X serve / drain. Enabled with DQN_TRACE=1
(rocprofv3 --marker-trace shows them; torch.cuda.nvtx is roctx on ROCm builds);
a no-op context otherwise, so the hot loop pays one attribute lookup.
"""
from __future__ import annotations

import contextlib
import os

_ENABLED = os.environ.get('DQN_TRACE', '0') not in ('', '0')
_nvtx = None
if _ENABLED:
    try:
        import torch
        _nvtx = torch.cuda.nvtx
    except Exception:      # pragma: no cover - torch without a GPU runtime
        _ENABLED = False


@contextlib.contextmanager
def _range(name: str):
    _nvtx.range_push(name)
    try:
        yield
    finally:
        _nvtx.range_pop()


_NULL = contextlib.nullcontext()


def trace(name: str):
    """``with trace('learner.step'): ...``"""
    return _range(name) if _ENABLED else _NULL


def enabled() -> bool:
    return _ENABLED
