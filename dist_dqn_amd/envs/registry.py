"""`gym.make` replacement used by the CLI (reference: `src/main.py:101`).

Classic control (the reference CONTROL preset, `scripts/dqn_params.sh:5-20`): CartPole-v0/v1,
Acrobot-v1, MountainCar-v0 in numpy with gym's dynamics and TimeLimits. Atari ids map to
`SyntheticAtariEnv` (no ALE in this image): random frames of the game's screen shape and
action count, for throughput work only -- a WARNING says so, since its rewards are noise.
"""
from __future__ import annotations

import logging
from typing import Optional

from .cartpole import CartPoleEnv
from .classic_control import AcrobotEnv, MountainCarEnv
from .synthetic import ATARI_ACTIONS, BlockBanditEnv, SyntheticAtariEnv, game_name

log = logging.getLogger(__name__)

CLASSIC = {
    'CartPole-v0': (CartPoleEnv, 200), 'CartPole-v1': (CartPoleEnv, 500),
    'Acrobot-v1': (AcrobotEnv, 500), 'MountainCar-v0': (MountainCarEnv, 200),
}
_warned = set()


def is_atari(env_id: str) -> bool:
    return game_name(env_id) in ATARI_ACTIONS or env_id.startswith('Synthetic')


def make(env_id: str, seed: Optional[int] = None):
    if env_id in CLASSIC:
        cls, cap = CLASSIC[env_id]
        return cls(env_id, max_episode_steps=cap, seed=seed)
    if env_id.startswith('SyntheticBlock'):
        return BlockBanditEnv(env_id, seed=seed)
    if is_atari(env_id):
        if not env_id.startswith('Synthetic') and env_id not in _warned:
            _warned.add(env_id)
            log.warning('%s: no Atari emulator (ALE) in this build -- using SyntheticAtariEnv: random %dx%dx%d '
                        'frames with the game\'s %d actions and random rewards (throughput runs only; the agent '
                        'cannot learn the game)', env_id, *SyntheticAtariEnv.SCREEN,
                        ATARI_ACTIONS.get(game_name(env_id), 6))
        return SyntheticAtariEnv(env_id, seed=seed)
    raise ValueError('Unknown environment %r (available: %s, Atari ids %s)'
                     % (env_id, ', '.join(sorted(CLASSIC)), sorted(ATARI_ACTIONS)))
