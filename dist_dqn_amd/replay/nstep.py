"""n-step return accumulator (actor side).

Emits (state, action, R = sum_{i<n} gamma^i r_{t+i}, next_state = s_{t+n},
done, gamma^m) where m <= n is the number of rewards actually summed (episode
ends truncate the window). With n == 1 it reproduces the reference's
one-step transitions exactly (`/root/reference/src/dqn_agent.py:99`).
"""
from __future__ import annotations

from collections import deque
from typing import Any, List, Tuple


class NStepAccumulator:
    def __init__(self, n: int, gamma: float):
        self.n = max(1, int(n))
        self.gamma = float(gamma)
        self.buf: deque = deque()

    def push(self, state: Any, action: int, reward: float, next_state: Any, done: bool
             ) -> List[Tuple[Any, int, float, Any, bool, float]]:
        self.buf.append((state, action, reward))
        out = []
        if done:
            while self.buf:
                out.append(self._emit(next_state, True))
                self.buf.popleft()
        elif len(self.buf) >= self.n:
            out.append(self._emit(next_state, False))
            self.buf.popleft()
        return out

    def _emit(self, next_state, done):
        R, g = 0.0, 1.0
        for _, _, r in self.buf:
            R += g * r
            g *= self.gamma
        s, a, _ = self.buf[0]
        return (s, a, R, next_state, done, g)

    def reset(self):
        self.buf.clear()
