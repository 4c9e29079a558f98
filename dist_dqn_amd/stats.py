"""Episode statistics (`/root/reference/src/stats.py:7-19`) plus throughput meters."""
from __future__ import annotations

import time
from collections import deque

import numpy as np


class Stats:
    def __init__(self):
        self.rewards = deque(maxlen=100)
        self.episodes = 0
        self.total_steps = 0

    def last_100_mean_reward(self):
        if not self.rewards:
            return float('nan')
        return float(np.mean(self.rewards))

    def log_episode(self, reward, steps):
        self.episodes += 1
        self.rewards.append(reward)
        self.total_steps += steps


class RateMeter:
    """Counts events and reports events/sec over a sliding wall-clock window."""

    def __init__(self, window_s: float = 10.0):
        self.window_s = window_s
        self.t0 = time.perf_counter()
        self.count0 = 0
        self.count = 0
        self.last_rate = 0.0

    def add(self, n: int = 1):
        self.count += n

    def rate(self) -> float:
        now = time.perf_counter()
        dt = now - self.t0
        if dt >= self.window_s or self.last_rate == 0.0 and dt > 0:
            self.last_rate = (self.count - self.count0) / dt
            if dt >= self.window_s:
                self.t0, self.count0 = now, self.count
        return self.last_rate
