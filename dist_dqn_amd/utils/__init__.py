"""Reference helper API (`/root/reference/src/utils.py:9-45`) plus shared utilities."""
from __future__ import annotations

import itertools

import numpy as np

from .image import resize_image, rgb_to_gray, resize_gray  # noqa: F401


def partition(pred, iterable):
    """Split ``iterable`` into (items where pred is false, items where pred is true).

    Same contract as `/root/reference/src/utils.py:9-17` (lazy iterators).
    """
    a, b = itertools.tee(iterable)
    return itertools.filterfalse(pred, a), filter(pred, b)


def decay(val, min_val, decay_rate):
    """Multiplicative decay with a floor (`src/utils.py:19-20`, unused upstream)."""
    return max(val * decay_rate, min_val)


def decay_per_step(init_val, min_val, steps):
    """Linear per-step decrement (`src/utils.py:22-25`)."""
    if steps <= 0:
        return 0.0
    return (init_val - min_val) / steps


def one_hot(i, n):
    """One-hot float64 vector of length n (`src/utils.py:27-37`)."""
    assert i < n, "Invalid args to one_hot"
    enc = np.zeros(n)
    enc[i] = 1
    return enc
