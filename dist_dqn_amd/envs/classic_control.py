"""Acrobot-v1 and MountainCar-v0 in numpy: the reference's CONTROL preset covers gym's classic
control tasks in general (`/root/reference/scripts/dqn_params.sh:5-20`, any id through
`gym.make(args.env)` at `/root/reference/src/main.py:101`).

gym is not importable in this image, so these follow gym's published dynamics (parity
unpinned: no gym run to compare against):

* Acrobot-v1 (Sutton & Barto's "book" equations of motion, RK4 over one dt = 0.2 step, angles
  wrapped to [-pi, pi], velocities clipped to 4 pi / 9 pi, observation
  [cos t1, sin t1, cos t2, sin t2, dt1, dt2], reward -1 per step and 0 on reaching the line,
  terminal when -cos(t1) - cos(t1 + t2) > 1, TimeLimit 500);
* MountainCar-v0 (force 0.001, gravity 0.0025, position clipped to [-1.2, 0.6] with the
  velocity zeroed at the left wall, goal position >= 0.5, reward -1 per step, start position
  U(-0.6, -0.4), TimeLimit 200).

As with CartPole (cartpole.py), the registry TimeLimit is applied here and a cap-triggered
end returns ``done=True``, so the reference agent stores it as terminal.
"""
from __future__ import annotations

import math
import random
from typing import Optional

import numpy as np

from .spaces import Box, Discrete, EnvSpec


class _Capped:
    """TimeLimit bookkeeping shared by the classic-control envs."""

    def _cap(self, done: bool):
        self._t += 1
        capped = self.spec.max_episode_steps is not None and self._t >= self.spec.max_episode_steps
        return bool(done or capped), {'TimeLimit.truncated': capped and not done}

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        self.action_space.seed(seed)

    def close(self):
        pass


class AcrobotEnv(_Capped):
    dt = 0.2
    LINK_LENGTH_1 = 1.0
    LINK_MASS_1 = 1.0
    LINK_MASS_2 = 1.0
    LINK_COM_POS_1 = 0.5
    LINK_COM_POS_2 = 0.5
    LINK_MOI = 1.0
    MAX_VEL_1 = 4 * math.pi
    MAX_VEL_2 = 9 * math.pi
    AVAIL_TORQUE = (-1.0, 0.0, 1.0)

    def __init__(self, env_id: str = 'Acrobot-v1', max_episode_steps: Optional[int] = 500,
                 seed: Optional[int] = None):
        self.spec = EnvSpec(env_id, max_episode_steps)
        self._rng = np.random.default_rng(seed)
        self.action_space = Discrete(3, random.Random(seed))
        high = np.array([1.0, 1.0, 1.0, 1.0, self.MAX_VEL_1, self.MAX_VEL_2], dtype=np.float32)
        self.observation_space = Box(-high, high, (6,))
        self.state = None
        self._t = 0

    def reset(self):
        self.state = self._rng.uniform(-0.1, 0.1, size=4)
        self._t = 0
        return self._obs()

    def _obs(self):
        s = self.state
        return np.array([math.cos(s[0]), math.sin(s[0]), math.cos(s[1]), math.sin(s[1]), s[2], s[3]],
                        dtype=np.float32)

    def _dsdt(self, sa):
        m1, m2 = self.LINK_MASS_1, self.LINK_MASS_2
        l1, lc1, lc2 = self.LINK_LENGTH_1, self.LINK_COM_POS_1, self.LINK_COM_POS_2
        i1 = i2 = self.LINK_MOI
        g = 9.8
        t1, t2, dt1, dt2, a = sa
        d1 = m1 * lc1 ** 2 + m2 * (l1 ** 2 + lc2 ** 2 + 2 * l1 * lc2 * math.cos(t2)) + i1 + i2
        d2 = m2 * (lc2 ** 2 + l1 * lc2 * math.cos(t2)) + i2
        phi2 = m2 * lc2 * g * math.cos(t1 + t2 - math.pi / 2.0)
        phi1 = (-m2 * l1 * lc2 * dt2 ** 2 * math.sin(t2) - 2 * m2 * l1 * lc2 * dt2 * dt1 * math.sin(t2)
                + (m1 * lc1 + m2 * l1) * g * math.cos(t1 - math.pi / 2) + phi2)
        # "book" dynamics (gym's default)
        ddt2 = ((a + d2 / d1 * phi1 - m2 * l1 * lc2 * dt1 ** 2 * math.sin(t2) - phi2)
                / (m2 * lc2 ** 2 + i2 - d2 ** 2 / d1))
        ddt1 = -(d2 * ddt2 + phi1) / d1
        return np.array([dt1, dt2, ddt1, ddt2, 0.0])

    def step(self, action):
        assert self.action_space.contains(action), action
        y0 = np.append(self.state, self.AVAIL_TORQUE[int(action)])
        h = self.dt
        k1 = self._dsdt(y0)
        k2 = self._dsdt(y0 + h / 2 * k1)
        k3 = self._dsdt(y0 + h / 2 * k2)
        k4 = self._dsdt(y0 + h * k3)
        ns = (y0 + h / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4))[:4]
        ns[0] = _wrap(ns[0], -math.pi, math.pi)
        ns[1] = _wrap(ns[1], -math.pi, math.pi)
        ns[2] = min(max(ns[2], -self.MAX_VEL_1), self.MAX_VEL_1)
        ns[3] = min(max(ns[3], -self.MAX_VEL_2), self.MAX_VEL_2)
        self.state = ns
        terminal = bool(-math.cos(ns[0]) - math.cos(ns[1] + ns[0]) > 1.0)
        done, info = self._cap(terminal)
        return self._obs(), (0.0 if terminal else -1.0), done, info


def _wrap(x: float, lo: float, hi: float) -> float:
    d = hi - lo
    while x > hi:
        x -= d
    while x < lo:
        x += d
    return x


class MountainCarEnv(_Capped):
    min_position = -1.2
    max_position = 0.6
    max_speed = 0.07
    goal_position = 0.5
    goal_velocity = 0.0
    force = 0.001
    gravity = 0.0025

    def __init__(self, env_id: str = 'MountainCar-v0', max_episode_steps: Optional[int] = 200,
                 seed: Optional[int] = None):
        self.spec = EnvSpec(env_id, max_episode_steps)
        self._rng = np.random.default_rng(seed)
        self.action_space = Discrete(3, random.Random(seed))
        self.observation_space = Box(np.array([self.min_position, -self.max_speed], dtype=np.float32),
                                     np.array([self.max_position, self.max_speed], dtype=np.float32), (2,))
        self.state = None
        self._t = 0

    def reset(self):
        self.state = np.array([self._rng.uniform(-0.6, -0.4), 0.0])
        self._t = 0
        return self.state.astype(np.float32)

    def step(self, action):
        assert self.action_space.contains(action), action
        position, velocity = float(self.state[0]), float(self.state[1])
        velocity += (int(action) - 1) * self.force + math.cos(3 * position) * (-self.gravity)
        velocity = min(max(velocity, -self.max_speed), self.max_speed)
        position += velocity
        position = min(max(position, self.min_position), self.max_position)
        if position == self.min_position and velocity < 0:
            velocity = 0.0
        goal = bool(position >= self.goal_position and velocity >= self.goal_velocity)
        self.state = np.array([position, velocity])
        done, info = self._cap(goal)
        return self.state.astype(np.float32), -1.0, done, info
