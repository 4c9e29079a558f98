"""Frame preprocessing dispatch (reference `utils.resize_image`, `src/utils.py:39-45`).

* host frames (actors): the C++ implementation in the extension
  (`csrc/host/preprocess.cpp`, cv2-compatible fixed point), numpy oracle if
  the extension is absent (CPU-only environments);
* device frames (batched synthetic/on-GPU envs): `preprocess_batch` HIP kernel.
Both are bit-exact to `dist_dqn_amd.utils.image` (tested).
"""
from __future__ import annotations

import numpy as np
import torch

from ..utils import image as _np_image
from . import _ext


def resize_image(image, width: int, height: int) -> np.ndarray:
    ext = _ext.load()
    img = np.ascontiguousarray(image, dtype=np.uint8)
    if ext is not None and hasattr(ext, 'preprocess_host') and img.ndim == 3 and img.shape[2] == 3:
        out = np.empty((height, width), dtype=np.uint8)
        ext.preprocess_host(torch.from_numpy(img), torch.from_numpy(out))
        return out
    return _np_image.resize_image(img, width, height)


def preprocess_batch(frames: torch.Tensor, height: int, width: int) -> torch.Tensor:
    """[N, Hs, Ws, 3] uint8 -> [N, height, width] uint8 gray+bilinear."""
    if frames.is_cuda:
        ext = _ext.load(required=True)
        out = torch.empty(frames.shape[0], height, width, dtype=torch.uint8, device=frames.device)
        ext.preprocess_batch(frames.contiguous(), out)
        return out
    return torch.from_numpy(np.stack([_np_image.resize_image(f, width, height) for f in frames.numpy()]))
