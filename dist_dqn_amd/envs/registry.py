"""`gym.make` replacement used by the CLI (reference: `src/main.py:101`)."""
from __future__ import annotations

from typing import Optional

from .cartpole import CartPoleEnv
from .synthetic import ATARI_ACTIONS, BlockBanditEnv, SyntheticAtariEnv, game_name


def is_atari(env_id: str) -> bool:
    return game_name(env_id) in ATARI_ACTIONS or env_id.startswith('Synthetic')


def make(env_id: str, seed: Optional[int] = None):
    if env_id.startswith('CartPole'):
        return CartPoleEnv(env_id, seed=seed)
    if env_id.startswith('SyntheticBlock'):
        return BlockBanditEnv(env_id, seed=seed)
    if is_atari(env_id):
        return SyntheticAtariEnv(env_id, seed=seed)
    raise ValueError('Unknown environment %r (available: CartPole-v0/v1, Atari ids %s)'
                     % (env_id, sorted(ATARI_ACTIONS)))
