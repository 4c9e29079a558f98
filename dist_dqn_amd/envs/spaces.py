from __future__ import annotations

import dataclasses
import random
from typing import Optional, Tuple

import numpy as np


class Discrete:
    def __init__(self, n: int, rng: Optional[random.Random] = None):
        self.n = int(n)
        self.shape = ()
        self._rng = rng or random.Random()

    def seed(self, seed):
        self._rng.seed(seed)

    def sample(self) -> int:
        return self._rng.randrange(self.n)

    def contains(self, x) -> bool:
        return 0 <= int(x) < self.n


class Box:
    def __init__(self, low, high, shape: Tuple[int, ...], dtype=np.float32):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype


@dataclasses.dataclass
class EnvSpec:
    id: str
    max_episode_steps: Optional[int] = None
