"""Classic-control environments of the reference CONTROL preset (`/root/reference/scripts/
dqn_params.sh:5-20`, built by `gym.make(args.env)` at `/root/reference/src/main.py:101`).

gym is not importable here, so parity with gym is unpinned; these tests pin the published
dynamics' properties instead: spaces, TimeLimit caps reported as terminal, rewards, and that
the textbook control heuristics (energy pumping) solve the tasks well inside their caps while
random play does not.
"""
import logging

import numpy as np
import pytest

from dist_dqn_amd.envs import make


def _run(env, policy, max_steps=10_000):
    o = env.reset()
    total, n = 0.0, 0
    while True:
        o, r, d, info = env.step(policy(o))
        total += r
        n += 1
        if d or n >= max_steps:
            return total, n, o, info


@pytest.mark.parametrize('eid,obs,acts,cap', [('CartPole-v0', 4, 2, 200), ('CartPole-v1', 4, 2, 500),
                                              ('Acrobot-v1', 6, 3, 500), ('MountainCar-v0', 2, 3, 200)])
def test_spaces_and_time_limit(eid, obs, acts, cap):
    env = make(eid, seed=0)
    assert env.spec.id == eid and env.spec.max_episode_steps == cap
    assert env.observation_space.shape == (obs,) and env.action_space.n == acts
    o = env.reset()
    assert o.shape == (obs,) and o.dtype == np.float32


def test_acrobot_random_times_out_and_pumping_swings_up():
    env = make('Acrobot-v1', seed=1)
    total, n, _, info = _run(env, lambda o: 1)          # zero torque: hangs, never reaches the line
    assert n == 500 and total == -500.0 and info['TimeLimit.truncated']
    # torque in the direction of the second joint's velocity pumps energy in
    total, n, o, info = _run(env, lambda o: 2 if o[5] > 0 else 0)
    assert n < 200 and not info['TimeLimit.truncated']
    assert total == -(n - 1)                             # -1 per step, 0 on the terminal step
    c1, s1, c2, s2 = o[:4]
    t1, t2 = np.arctan2(s1, c1), np.arctan2(s2, c2)
    assert -np.cos(t1) - np.cos(t1 + t2) > 1.0
    assert abs(o[4]) <= 4 * np.pi + 1e-5 and abs(o[5]) <= 9 * np.pi + 1e-5


def test_mountain_car_needs_momentum():
    env = make('MountainCar-v0', seed=3)
    total, n, _, info = _run(env, lambda o: 2)           # full throttle right: too weak to climb
    assert n == 200 and total == -200.0 and info['TimeLimit.truncated']
    total, n, o, info = _run(env, lambda o: 2 if o[1] >= 0 else 0)   # push along the velocity
    assert n < 200 and o[0] >= 0.5 and not info['TimeLimit.truncated']
    # the left wall stops the car (velocity zeroed)
    env.reset()
    env.state = np.array([-1.2, -0.05])
    o, _, _, _ = env.step(0)
    assert o[0] == np.float32(-1.2) and o[1] == 0.0


def test_atari_id_maps_to_synthetic_with_warning(caplog):
    from dist_dqn_amd.envs import registry
    registry._warned.discard('Breakout-v0')
    with caplog.at_level(logging.WARNING, logger='dist_dqn_amd.envs.registry'):
        env = make('Breakout-v0', seed=0)
    assert env.action_space.n == 4 and env.reset().shape == (210, 160, 3)
    assert any('SyntheticAtariEnv' in r.getMessage() for r in caplog.records)
    with pytest.raises(ValueError):
        make('Pendulum-v0')
