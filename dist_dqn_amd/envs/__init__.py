"""Environments with the gym-0.x API the reference agent drives
(`reset() -> obs`, `step(a) -> (obs, reward, done, info)`, `action_space.n/sample()`,
`observation_space.shape`, `spec.id`).

gym/ALE are not available, so:
  * CartPole-v0/v1, Acrobot-v1, MountainCar-v0: numpy re-implementations of the
    classic-control dynamics with the registry TimeLimit that gym applies;
  * Atari ids (``*-v0``, ``*NoFrameskip-v4`` ...): `SyntheticAtariEnv`, random
    210x160x3 frames with the real game's action count, for throughput work;
  * `VectorSyntheticAtari` (device.py): a GPU-resident batched synthetic env
    used by the Ape-X actors and the benchmark.
"""
from .spaces import Box, Discrete, EnvSpec  # noqa: F401
from .cartpole import CartPoleEnv  # noqa: F401
from .classic_control import AcrobotEnv, MountainCarEnv  # noqa: F401
from .synthetic import BlockBanditEnv, SyntheticAtariEnv, ATARI_ACTIONS  # noqa: F401
from .registry import make, is_atari  # noqa: F401
