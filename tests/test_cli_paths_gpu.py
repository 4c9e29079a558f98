"""User paths through the real CLI entry on the GPU.

* ``--device_envs``: the benched fused-acting learner (GPU-resident envs acting inside the
  learner's launches) run by ``cli.run_worker`` under the supervisor: train-step budget,
  progress metrics with env frames, the final checkpoint, ``global_step``;
* the reference CONTROL preset (`/root/reference/scripts/dqn_params.sh:5-20`) on Acrobot-v1
  with the fused fp32 MLP executor: returns must improve over random play (-500 per episode).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _records(logdir, kind):
    return [r for r in map(json.loads, open(os.path.join(logdir, 'metrics.rank0.jsonl'))) if r.get('kind') == kind]


@pytest.mark.parametrize('envs', [4, 2])
def test_device_envs_cli_path(tmp_path, envs):
    from dist_dqn_amd import checkpoint as ckpt
    from dist_dqn_amd.cli import run_worker
    from dist_dqn_amd.config import preset
    cfg = preset('nature', 'Pong-v0', '--device=cuda --dtype=bf16 --device_envs=%d --max_train_steps=100 '
                 '--replay_start_size=512 --replay_memory_capacity=8192 --checkpoint_secs=600 --seed=1 '
                 '--logdir=%s' % (envs, tmp_path))
    learner = run_worker(cfg)
    assert learner.train_steps == 100
    assert int(learner.net.global_step) == 100
    # 4 envs: one fused acting step per SGD step; 2 envs: two separate acting steps per SGD step
    assert (learner.actor is not None) == (envs == 4)
    done = _records(str(tmp_path), 'done')[-1]
    assert done['training_steps'] == 100 and done['env_frames_per_sec'] > 0
    prog = _records(str(tmp_path), 'progress')
    assert prog and prog[-1]['env_frames'] >= 100 * 4
    path = ckpt.latest_checkpoint(str(tmp_path))
    assert path is not None and path.endswith('-100')       # the final save on the graceful stop


def test_hip_mlp_learner_improves_acrobot(tmp_path):
    from dist_dqn_amd.cli import run_worker
    from dist_dqn_amd.config import preset
    # (CPU torch executor, same flags: ~105 episodes, the last ones at -75 .. -130)
    cfg = preset('control', 'Acrobot-v1', '--device=cuda --backend=hip --seed=2 --minibatch_size=64 '
                 '--random_action_explore_steps=5000 --init_random_action_prob=1.0 --min_random_action_prob=0.05 '
                 '--target_update_freq=250 --reward_discount=0.99 --replay_memory_capacity=50000 '
                 '--max_steps_per_episode=500 --max_train_steps=25000 --checkpoint_secs=0 --reg_param=0 '
                 '--logdir=%s' % tmp_path)
    agent = run_worker(cfg)
    assert agent.network.executor.name.startswith('hip'), agent.network.executor.name
    r = [e['reward'] for e in _records(str(tmp_path), 'episode')]
    first, last = np.mean(r[:5]), np.mean(r[-10:])
    print('acrobot: %d episodes, first-5 mean %.1f, last-10 mean %.1f' % (len(r), first, last))
    assert last > -300 and last > first + 150, (first, last)
