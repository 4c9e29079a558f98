"""Host replay memory with the reference API
(`/root/reference/src/replay_memory.py:18-53`).

The reference keeps ``(s, a, r, s', done)`` tuples in a ``deque(maxlen)``
and samples with ``random.sample`` (O(n) deque indexing). Here the same API
sits on a list ring (O(1) random access), and `sample_arrays` returns the
minibatch as stacked numpy arrays (non-terminal first, like the reference's
``partition`` order) for the learner.
"""
from __future__ import annotations

import random
import threading
from typing import Optional

import numpy as np

from .. import utils


class ReplayMemory:
    def __init__(self, capacity, rng: Optional[random.Random] = None):
        self._cap = int(capacity)
        self._buf = []
        self._next = 0
        self._rng = rng or random
        self._lock = threading.Lock()    # reference TODO (replay_memory.py:15-17): reader/writer safety

    def add(self, state, action, reward, observation, terminal):
        item = (state, action, reward, observation, terminal)
        with self._lock:
            if len(self._buf) < self._cap:
                self._buf.append(item)
            else:
                self._buf[self._next] = item
            self._next = (self._next + 1) % self._cap

    def size(self):
        return len(self._buf)

    def capacity(self):
        return self._cap

    def _sample(self, n):
        with self._lock:
            return [self._buf[i] for i in self._rng.sample(range(len(self._buf)), n)]

    def get_minibatch(self, minibatch_size):
        """(non_terminal_iter, terminal_iter); (None, None) if not enough samples."""
        if self.size() < minibatch_size:
            return None, None
        return utils.partition(lambda x: x[4], self._sample(minibatch_size))

    def sample_arrays(self, minibatch_size):
        """dict of stacked arrays (states, actions, rewards, next_states, dones), non-terminal first."""
        items = self._sample(minibatch_size)
        items.sort(key=lambda x: bool(x[4]))
        return {
            'states': np.stack([np.asarray(i[0]) for i in items]),
            'actions': np.array([i[1] for i in items], dtype=np.int64),
            'rewards': np.array([i[2] for i in items], dtype=np.float32),
            'next_states': np.stack([np.asarray(i[3]) for i in items]),
            'dones': np.array([float(bool(i[4])) for i in items], dtype=np.float32),
        }

    @staticmethod
    def get_states(iterable):
        return map(lambda m: m[0], iterable)

    @staticmethod
    def get_next_states(iterable):
        return map(lambda m: m[3], iterable)
