"""k-frame state stacker (API of `/root/reference/src/frame_buffer.py:13-57`).

Host-side and per-actor. The HBM replay does not store stacked states; it
stores single frames and rebuilds the stack inside the GPU gather kernel,
so this class only feeds the acting policy.
"""
from __future__ import annotations

from collections import deque

import numpy as np


class FrameBuffer:
    def __init__(self, frames_per_state, preprocessor=lambda x: x):
        if frames_per_state <= 0:
            raise RuntimeError('Frames per state should be greater than 0')
        self.frames_per_state = frames_per_state
        self.frames = deque(maxlen=frames_per_state)
        self.preprocessor = preprocessor

    def append(self, frame):
        """Preprocess and push; the first frame after ``clear`` fills every slot."""
        frame = self.preprocessor(frame)
        if not self.frames:
            self.frames.extend([frame] * self.frames_per_state)
        else:
            self.frames.append(frame)
        return frame

    def get_state(self):
        """Raw frame when k == 1, else an HWC stack ``[..., k]``; None when empty."""
        if not self.frames:
            return None
        if self.frames_per_state == 1:
            return self.frames[0]
        return np.stack(self.frames, axis=-1)

    def clear(self):
        self.frames.clear()
