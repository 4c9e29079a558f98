"""Synthetic Atari-shaped environment (no ALE in this image).

Emits uint8 RGB frames of the ALE screen shape (210, 160, 3), the real game's
action count, sparse random rewards in {-1, 0, 1} and random episode ends, so
the full CNN path (preprocess -> frame stack -> replay -> learner) runs end to
end. Frames are cheap: a fixed random background plus a moving block, so the
actor cost is dominated by our own preprocessing, as with a real emulator.
"""
from __future__ import annotations

import random
from typing import Optional

import numpy as np

from .spaces import Box, Discrete, EnvSpec

ATARI_ACTIONS = {
    'Pong': 6, 'Breakout': 4, 'SpaceInvaders': 6, 'Seaquest': 18, 'BeamRider': 9,
    'Qbert': 6, 'Enduro': 9, 'MsPacman': 9, 'Asteroids': 14, 'Freeway': 3,
}


def game_name(env_id: str) -> str:
    base = env_id.split('-')[0]
    for suffix in ('NoFrameskip', 'Deterministic'):
        base = base.replace(suffix, '')
    return base


class SyntheticAtariEnv:
    SCREEN = (210, 160, 3)

    def __init__(self, env_id: str = 'Pong-v0', seed: Optional[int] = None,
                 episode_len: int = 2000, num_actions: Optional[int] = None):
        n = num_actions or ATARI_ACTIONS.get(game_name(env_id), 6)
        self.spec = EnvSpec(env_id, None)
        self.action_space = Discrete(n, random.Random(seed))
        self.observation_space = Box(0, 255, self.SCREEN, np.uint8)
        self._rng = np.random.default_rng(seed)
        self._bg = self._rng.integers(0, 256, size=self.SCREEN, dtype=np.uint8)
        self._mean_len = episode_len
        self._t = 0
        self._pos = 0

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        self.action_space.seed(seed)

    def _frame(self):
        f = self._bg.copy()
        y = (self._pos * 7) % (self.SCREEN[0] - 16)
        x = (self._pos * 3) % (self.SCREEN[1] - 16)
        f[y:y + 16, x:x + 16, :] = 255
        return f

    def reset(self):
        self._t = 0
        self._pos = int(self._rng.integers(0, 1000))
        return self._frame()

    def step(self, action):
        assert self.action_space.contains(action)
        self._t += 1
        self._pos += 1 + int(action)
        u = self._rng.random()
        reward = 1.0 if u < 0.01 else (-1.0 if u < 0.02 else 0.0)
        done = bool(self._rng.random() < 1.0 / self._mean_len)
        return self._frame(), reward, done, {}

    def close(self):
        pass


class BlockBanditEnv:
    """A LEARNABLE Atari-shaped environment (for end-to-end learning checks of the image
    learners; `SyntheticAtariEnv` rewards are pure noise). Each frame is a dark screen with
    one bright block in one of ``num_actions`` vertical bands; the reward is 1 when the action
    names the block's band of the CURRENT frame, else 0, and the next frame's band is drawn at
    random. Episodes last ``episode_len`` steps (terminal), so the best return is
    ``episode_len`` and a uniformly random policy scores ``episode_len / num_actions``.
    Solving it needs the Q-network to read the newest frame of the stack through the conv
    trunk — what the reference's Atari learner has to do (`/root/reference/src/dqn_agent.py:72-106`)."""
    SCREEN = (210, 160, 3)

    def __init__(self, env_id: str = 'SyntheticBlock-v0', seed: Optional[int] = None,
                 episode_len: int = 8, num_actions: int = 4):
        self.spec = EnvSpec(env_id, episode_len)
        self.action_space = Discrete(num_actions, random.Random(seed))
        self.observation_space = Box(0, 255, self.SCREEN, np.uint8)
        self._rng = np.random.default_rng(seed)
        self.episode_len = episode_len
        self._t = 0
        self._band = 0

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        self.action_space.seed(seed)

    def _frame(self):
        f = np.full(self.SCREEN, 16, dtype=np.uint8)
        w = self.SCREEN[1] // self.action_space.n
        x0 = self._band * w + w // 4
        f[60:150, x0:x0 + w // 2, :] = 240
        return f

    def reset(self):
        self._t = 0
        self._band = int(self._rng.integers(0, self.action_space.n))
        return self._frame()

    def step(self, action):
        assert self.action_space.contains(action)
        reward = 1.0 if int(action) == self._band else 0.0
        self._t += 1
        self._band = int(self._rng.integers(0, self.action_space.n))
        return self._frame(), reward, self._t >= self.episode_len, {}

    def close(self):
        pass
