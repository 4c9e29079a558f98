"""Classic cart-pole (Barto, Sutton & Anderson 1983) in numpy.

Same dynamics constants and termination thresholds as gym's CartPole; the
episode cap is applied here (gym applies it via its TimeLimit wrapper), and a
cap-triggered end is reported as ``done=True`` like gym does — the reference
agent therefore stores it as terminal (SURVEY.md §5.6.2 "Episode termination").
"""
from __future__ import annotations

import math
import random
from typing import Optional

import numpy as np

from .spaces import Box, Discrete, EnvSpec


class CartPoleEnv:
    gravity = 9.8
    masscart = 1.0
    masspole = 0.1
    total_mass = masscart + masspole
    length = 0.5
    polemass_length = masspole * length
    force_mag = 10.0
    tau = 0.02
    theta_threshold = 12 * 2 * math.pi / 360
    x_threshold = 2.4

    def __init__(self, env_id: str = 'CartPole-v0', max_episode_steps: Optional[int] = None,
                 seed: Optional[int] = None):
        if max_episode_steps is None:
            max_episode_steps = 500 if env_id.endswith('v1') else 200
        self.spec = EnvSpec(env_id, max_episode_steps)
        self._rng = np.random.default_rng(seed)
        self.action_space = Discrete(2, random.Random(seed))
        high = np.array([self.x_threshold * 2, np.finfo(np.float32).max,
                         self.theta_threshold * 2, np.finfo(np.float32).max], dtype=np.float32)
        self.observation_space = Box(-high, high, (4,))
        self.state = None
        self._t = 0

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        self.action_space.seed(seed)

    def reset(self):
        self.state = self._rng.uniform(-0.05, 0.05, size=4)
        self._t = 0
        return self.state.astype(np.float32)

    def step(self, action):
        assert self.action_space.contains(action), action
        x, x_dot, theta, theta_dot = self.state
        force = self.force_mag if int(action) == 1 else -self.force_mag
        ct, st = math.cos(theta), math.sin(theta)
        temp = (force + self.polemass_length * theta_dot * theta_dot * st) / self.total_mass
        thetaacc = (self.gravity * st - ct * temp) / (
            self.length * (4.0 / 3.0 - self.masspole * ct * ct / self.total_mass))
        xacc = temp - self.polemass_length * thetaacc * ct / self.total_mass
        x = x + self.tau * x_dot
        x_dot = x_dot + self.tau * xacc
        theta = theta + self.tau * theta_dot
        theta_dot = theta_dot + self.tau * thetaacc
        self.state = np.array([x, x_dot, theta, theta_dot])
        self._t += 1
        failed = (x < -self.x_threshold or x > self.x_threshold or
                  theta < -self.theta_threshold or theta > self.theta_threshold)
        capped = self.spec.max_episode_steps is not None and self._t >= self.spec.max_episode_steps
        return self.state.astype(np.float32), 1.0, bool(failed or capped), {'TimeLimit.truncated': capped and not failed}

    def close(self):
        pass
