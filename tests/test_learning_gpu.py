"""End-to-end learning on the HIP learners (GPU): the agent loop of the reference
(`/root/reference/src/dqn_agent.py:52-106`) driving the hand-written kernels must actually
improve returns, not only match the oracle on one step.

* image learners (`nature` bf16 MFMA trunk, reference `cnn` SAME+max-pool kernels) on
  `BlockBanditEnv` — a learnable Atari-shaped task: reward 1 for naming the band of the bright
  block in the newest frame; random play scores episode_len / A;
* the fused fp32 MLP executor on CartPole (the reference's CONTROL config on the GPU).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _episode_rewards(logdir):
    path = os.path.join(logdir, 'metrics.rank0.jsonl')
    return [r['reward'] for r in map(json.loads, open(path)) if r.get('kind') == 'episode']


@pytest.mark.parametrize('network', ['nature', 'cnn'])
def test_hip_image_learner_learns_block_bandit(tmp_path, network):
    from dist_dqn_amd.cli import run_worker
    from dist_dqn_amd.config import preset
    cfg = preset('nature' if network == 'nature' else 'atari', 'SyntheticBlock-v0',
                 '--seed=0 --device=cuda --backend=hip --dtype=bf16 --replay_memory_capacity=20000 '
                 '--replay_start_size=500 --update_freq=1 --target_update_freq=200 '
                 '--random_action_explore_steps=2000 --min_random_action_prob=0.05 --reward_discount=0.9 '
                 '--max_steps_per_episode=8 --num_episodes=100000 --max_train_steps=2500 '
                 '--checkpoint_secs=0 --logdir=%s' % tmp_path)
    agent = run_worker(cfg)
    assert agent.network.executor.name.startswith('hip'), agent.network.executor.name
    assert agent.training_steps == 2500
    r = _episode_rewards(str(tmp_path))
    chance = 8.0 / 4
    first, last = np.mean(r[:50]), np.mean(r[-100:])
    print('%s: first-50 mean %.2f, last-100 mean %.2f (chance %.2f, max 8)' % (network, first, last, chance))
    assert last > 2.0 * chance and last > first + 1.0, (first, last)


def test_hip_mlp_learner_learns_cartpole(tmp_path):
    from dist_dqn_amd.cli import run_worker
    from dist_dqn_amd.config import parse_args
    cfg = parse_args(['--env=CartPole-v0', '--network=simple', '--optimizer=adam', '--lr=0.002',
                      '--minibatch_size=64', '--num_episodes=400', '--max_steps_per_episode=200',
                      '--replay_memory_capacity=20000', '--target_update_freq=200', '--reward_discount=0.99',
                      '--init_random_action_prob=1.0', '--min_random_action_prob=0.02',
                      '--random_action_explore_steps=4000', '--logdir=%s' % tmp_path, '--seed=4',
                      '--max_train_steps=15000', '--reg_param=0', '--device=cuda', '--backend=hip',
                      '--checkpoint_secs=0'])
    agent = run_worker(cfg)
    assert agent.network.executor.name.startswith('hip'), agent.network.executor.name
    r = _episode_rewards(str(tmp_path))
    first, last = np.mean(r[:30]), np.mean(r[-30:])
    print('cartpole: first-30 mean %.1f, last-30 mean %.1f' % (first, last))
    assert last > 60 and last > 2 * first, (first, last)
