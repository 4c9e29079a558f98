"""Fused HIP executor (placeholder until the conv/dense kernels land)."""
from __future__ import annotations


def supports(arch) -> bool:
    return False


class HipExecutor:  # pragma: no cover
    name = 'hip'

    def __init__(self, *a, **k):
        raise NotImplementedError
