"""Frame preprocessing: RGB->gray + bilinear resize, bit-compatible with the
OpenCV calls the reference makes (`/root/reference/src/utils.py:39-45`:
``cv2.cvtColor(RGB2GRAY)`` then ``cv2.resize(gray, (W, H))``, INTER_LINEAR).

OpenCV is not installed here, so this module re-derives OpenCV's fixed-point
arithmetic:
  * gray = (4899*R + 9617*G + 1868*B + 2^13) >> 14      (coefficients * 2^14)
  * resize: half-pixel centres, per-axis 11-bit fixed-point weights
    (INTER_RESIZE_COEF_BITS = 11), horizontal pass in int, vertical pass
    rounded with >> 22.
Parity with a real cv2 build is "unpinned" (no cv2 to compare against); the C++
actor-side implementation (`csrc/host/preprocess.cpp`) and the HIP kernel
(`csrc/kernels/preprocess.hip`) are tested bit-exact against this oracle.
"""
from __future__ import annotations

import numpy as np

_COEF_BITS = 11
_COEF_SCALE = 1 << _COEF_BITS


def rgb_to_gray(image: np.ndarray) -> np.ndarray:
    img = np.asarray(image)
    if img.ndim == 2:
        return img.astype(np.uint8, copy=False)
    r = img[..., 0].astype(np.int32)
    g = img[..., 1].astype(np.int32)
    b = img[..., 2].astype(np.int32)
    return ((4899 * r + 9617 * g + 1868 * b + (1 << 13)) >> 14).astype(np.uint8)


def linear_coeffs(src: int, dst: int):
    """Source index and fixed-point weights for one axis (OpenCV INTER_LINEAR)."""
    scale = src / dst
    idx = np.empty(dst, dtype=np.int32)
    w0 = np.empty(dst, dtype=np.int32)
    for d in range(dst):
        # OpenCV: float fx = (float)((dx + 0.5) * scale - 0.5); sx = floor(fx); fx -= sx
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(np.floor(f))
        f = np.float32(f - np.float32(s))
        if s < 0:
            s, f = 0, np.float32(0.0)
        if s >= src - 1:
            s, f = src - 1, np.float32(0.0)
        # saturate_cast<short>((1.f - fx) * 2048): round half to even
        c0 = int(np.rint(np.float32(np.float32(1.0) - f) * np.float32(_COEF_SCALE)))
        idx[d] = s
        w0[d] = c0
    return idx, w0, _COEF_SCALE - w0


def resize_gray(gray: np.ndarray, width: int, height: int) -> np.ndarray:
    g = np.asarray(gray, dtype=np.uint8)
    sh, sw = g.shape
    if (sh, sw) == (height, width):
        return g.copy()
    xi, xa0, xa1 = linear_coeffs(sw, width)
    yi, yb0, yb1 = linear_coeffs(sh, height)
    gi = g.astype(np.int64)
    xi1 = np.minimum(xi + 1, sw - 1)
    horiz = gi[:, xi] * xa0[None, :] + gi[:, xi1] * xa1[None, :]     # [sh, width]
    yi1 = np.minimum(yi + 1, sh - 1)
    val = horiz[yi, :] * yb0[:, None] + horiz[yi1, :] * yb1[:, None]
    out = (val + (1 << (2 * _COEF_BITS - 1))) >> (2 * _COEF_BITS)
    return np.clip(out, 0, 255).astype(np.uint8)


def resize_image(image: np.ndarray, width: int, height: int) -> np.ndarray:
    """Reference API: grayscale + resize to (height, width)."""
    return resize_gray(rgb_to_gray(image), width, height)
