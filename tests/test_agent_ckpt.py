"""Agent semantics (/root/reference/src/dqn_agent.py), checkpoint layout and
resume (Supervisor, /root/reference/src/main.py:136-167), metrics sinks and CLI."""
import json
import os

import numpy as np
import pytest
import torch

from dist_dqn_amd import checkpoint as ckpt
from dist_dqn_amd.agent import DQNAgent
from dist_dqn_amd.config import parse_args
from dist_dqn_amd.envs import CartPoleEnv, SyntheticAtariEnv, make
from dist_dqn_amd.models.network import Network
from dist_dqn_amd.replay import DeviceReplay, ReplayMemory
from dist_dqn_amd.supervisor import FaultInjected, RunSupervisor
from dist_dqn_amd.utils.metrics import EpisodeMonitor, JsonlWriter, SummaryWriter, read_tfrecords


def _cfg(tmp_path, *extra):
    return parse_args(['--device=cpu', '--seed=0', '--logdir=%s' % tmp_path] + list(extra))


def test_epsilon_schedule_decays_before_roll(tmp_path):
    cfg = _cfg(tmp_path, '--init_random_action_prob=1.0', '--min_random_action_prob=0.5',
               '--random_action_explore_steps=4', '--replay_start_size=3')
    env = CartPoleEnv(seed=0)
    net = Network.create_network(cfg, (4,), 2)
    agent = DQNAgent(env, net, None, ReplayMemory(100), cfg, enable_summary=False)
    assert agent.random_action_prob == 1.0           # prefill does not decay
    assert agent.replay_memory.size() >= 3
    seen = []
    for _ in range(4):
        agent._pick_action(env.reset())
        seen.append(agent.random_action_prob)
    np.testing.assert_allclose(seen, [0.875, 0.75, 0.625, 0.5])
    agent._pick_action(env.reset())
    assert agent.random_action_prob == pytest.approx(0.5)   # floor reached: no further decay


def test_target_update_cadence(tmp_path):
    cfg = _cfg(tmp_path, '--target_update_freq=3', '--minibatch_size=4', '--lr=0.05')
    env = CartPoleEnv(seed=0)
    net = Network.create_network(cfg, (4,), 2)
    rep = ReplayMemory(100)
    agent = DQNAgent(env, net, None, rep, cfg, enable_summary=False)
    for i in range(8):
        rep.add(np.random.rand(4), i % 2, 1.0, np.random.rand(4), False)
    synced = []
    for _ in range(7):
        agent._train_minibatch(4)
        synced.append(bool(torch.equal(net.online.flat, net.target.flat)))
    # target copied when training_steps % 3 == 0 after the increment: steps 3 and 6
    assert synced == [False, False, True, False, False, True, False]


def test_cartpole_learns(tmp_path):
    """Config 1 of BASELINE.json (plumbing): CartPole MLP on CPU learns within a bounded budget."""
    from dist_dqn_amd.cli import run_worker
    cfg = parse_args(['--env=CartPole-v0', '--network=simple', '--optimizer=adam', '--lr=0.002',
                      '--minibatch_size=64', '--num_episodes=400', '--max_steps_per_episode=200',
                      '--replay_memory_capacity=20000', '--target_update_freq=200', '--reward_discount=0.99',
                      '--init_random_action_prob=1.0', '--min_random_action_prob=0.02',
                      '--random_action_explore_steps=4000', '--logdir=%s' % tmp_path, '--seed=4',
                      '--max_train_steps=15000', '--reg_param=0', '--device=cpu', '--checkpoint_secs=0'])
    agent = run_worker(cfg)
    rewards = list(agent.stats.rewards)
    early = [r['mean100'] for r in map(json.loads, open(os.path.join(tmp_path, 'metrics.rank0.jsonl')))
             if r.get('kind') == 'episode'][20]
    # (DQN on CartPole is high-variance across seeds; runs are deterministic per seed)
    assert np.mean(rewards[-30:]) > 60 and np.mean(rewards[-30:]) > 2 * early
    assert ckpt.latest_checkpoint(str(tmp_path)) is not None      # final save on stop


def test_atari_cnn_path_on_cpu_with_device_replay(tmp_path):
    """Reference `cnn` end-to-end on the CPU executor: preprocess -> frame stack -> HBM-style replay."""
    from dist_dqn_amd.learner import Learner
    cfg = parse_args(['--env=Pong-v0', '--network=cnn', '--optimizer=rmsprop', '--lr=0.00025',
                      '--minibatch_size=8', '--frames_per_state=4', '--resize_width=84', '--resize_height=84',
                      '--update_freq=4', '--replay_start_size=40', '--replay_memory_capacity=200',
                      '--target_update_freq=5', '--device=cpu', '--seed=0', '--logdir=%s' % tmp_path])
    env = SyntheticAtariEnv('Pong-v0', seed=0, episode_len=30)
    net = Network.create_network(cfg, DQNAgent.get_input_shape(env, cfg), env.action_space.n)
    rep = DeviceReplay(200, (84, 84), 4, device='cpu', stage_size=16)
    learner = Learner(net, rep, cfg)
    agent = DQNAgent(env, net, learner, rep, cfg, enable_summary=False)
    for _ in range(50):
        agent.train_episode(60)
        if agent.training_steps >= 3:
            break
    assert agent.training_steps >= 3 and int(net.global_step) == agent.training_steps


def test_checkpoint_roundtrip_tf_names(tmp_path):
    cfg = _cfg(tmp_path, '--network=cnn', '--optimizer=adam')
    net = Network.create_network(cfg, (84, 84, 4), 6)
    net.global_step.fill_(42)
    net.optimizer.slots[0].fill_(0.25)
    path = ckpt.save(str(tmp_path), net.state_dict(), 42)
    assert os.path.basename(path) == 'model.ckpt-42'
    index = open(os.path.join(tmp_path, 'checkpoint')).read()
    assert 'model_checkpoint_path: "model.ckpt-42"' in index
    sd = ckpt.load(path)
    assert tuple(sd['conv1/w'].shape) == (8, 8, 4, 32) and tuple(sd['fcl/w'].shape) == (256, 256)
    assert 'conv1/w/Adam' in sd and 'conv1/w/Adam_1' in sd and 'beta1_power' in sd
    assert int(sd['global_step']) == 42
    net2 = Network.create_network(cfg.replace(seed=7), (84, 84, 4), 6)
    net2.load_state_dict(sd)
    assert torch.equal(net2.online.flat, net.online.flat) and int(net2.global_step) == 42
    s1, s2 = net.optimizer.state_dict(), net2.optimizer.state_dict()
    assert s1.keys() == s2.keys() and all(torch.equal(s1[k], s2[k]) for k in s1)


def test_checkpoint_manager_snapshots_inside_quiesce(tmp_path):
    """A manager with a quiesce hook (the native async-PS server's pause) takes its snapshot while
    the hook is held, and the written checkpoint holds that state."""
    cfg = _cfg(tmp_path, '--network=simple', '--optimizer=rmsprop')
    net = Network.create_network(cfg, (4,), 2)
    mgr = ckpt.CheckpointManager(str(tmp_path), net, save_secs=600, async_write=False)
    events = []
    orig = net.snapshot

    def snap():
        events.append('snapshot')
        return orig()
    net.snapshot = snap

    import contextlib

    @contextlib.contextmanager
    def quiesce():
        events.append('pause')
        net.global_step.fill_(7)          # the paused writer's last update
        yield
        events.append('resume')
        net.global_step.fill_(8)          # updates continue after the snapshot
    mgr.quiesce = quiesce
    path = mgr.maybe_save(force=True)
    assert events == ['pause', 'snapshot', 'resume']
    assert int(ckpt.load(path)['global_step']) == 7


def test_checkpoint_retention(tmp_path):
    t = {'w': torch.zeros(2)}
    for s in range(6):
        ckpt.save(str(tmp_path), t, s, max_to_keep=2)
    names = sorted(f for f in os.listdir(tmp_path) if f.startswith('model.ckpt-'))
    assert names == ['model.ckpt-4', 'model.ckpt-5']
    assert ckpt.latest_checkpoint(str(tmp_path)).endswith('model.ckpt-5')


def test_supervisor_fault_injection_and_resume(tmp_path, monkeypatch):
    cfg = _cfg(tmp_path)
    net = Network.create_network(cfg, (4,), 2)
    monkeypatch.setenv('DQN_FAULT_INJECT', 'step:3,rank:0')
    # a periodic save after every step (save_secs > 0 but tiny)
    sv = RunSupervisor(True, str(tmp_path), net, save_secs=1e-9, install_signal_handlers=False)
    sv.prepare()
    with pytest.raises(FaultInjected):
        with sv.managed():
            for step in range(1, 10):
                net.global_step.fill_(step)
                sv.on_train_step(step)
    assert sv.should_stop()
    path = ckpt.latest_checkpoint(str(tmp_path))
    # no final save after a failure: the newest checkpoint is the last periodic one (step 2; the
    # fault fires at step 3 before that step's save)
    assert path is not None and path.endswith('-2')
    # relaunch: chief restores global_step and params
    monkeypatch.delenv('DQN_FAULT_INJECT')
    net2 = Network.create_network(cfg.replace(seed=9), (4,), 2)
    sv2 = RunSupervisor(True, str(tmp_path), net2, save_secs=0, install_signal_handlers=False)
    assert sv2.prepare() == path
    assert int(net2.global_step) == 2 and torch.equal(net2.online.flat, net.online.flat)
    hb = json.load(open(os.path.join(tmp_path, 'heartbeat', 'rank0.json')))
    assert hb['rank'] == 0
    assert sv2.stale_ranks(timeout_s=3600) == []


def test_agent_state_sidecar_roundtrip(tmp_path):
    """--save_agent_state: epsilon and the local step count survive a relaunch (opt-in)."""
    from dist_dqn_amd.cli import run_worker
    args = ['--env=CartPole-v0', '--network=simple', '--device=cpu', '--seed=1', '--minibatch_size=16',
            '--replay_start_size=32', '--num_episodes=1000', '--max_steps_per_episode=50',
            '--random_action_explore_steps=1000', '--checkpoint_secs=600', '--save_agent_state',
            '--logdir=%s' % tmp_path]
    a1 = run_worker(parse_args(args + ['--max_train_steps=40']))
    eps, steps = a1.random_action_prob, a1.training_steps
    assert steps == 40 and eps < 0.9
    side = ckpt.load_sidecar(ckpt.latest_checkpoint(str(tmp_path)))
    assert side == {'random_action_prob': eps, 'training_steps': steps}
    a2 = run_worker(parse_args(args + ['--max_train_steps=45']))
    assert a2.training_steps == 45                          # continued from 40
    assert a2.random_action_prob < eps                      # epsilon kept decaying from the saved value
    assert int(a2.network.global_step) == 45


def test_tfevents_and_jsonl(tmp_path):
    w = SummaryWriter(str(tmp_path))
    w.add_scalar('loss', 1.5, 10)
    w.close()
    recs = list(read_tfrecords(w.path))
    assert len(recs) == 2 and b'brain.Event:2' in recs[0] and b'loss' in recs[1]
    j = JsonlWriter(os.path.join(tmp_path, 'm.jsonl'))
    j.write(a=1)
    m = EpisodeMonitor(str(tmp_path))
    m.episode(0, 10, 1.0)
    assert json.loads(open(os.path.join(tmp_path, 'episodes.rank0.jsonl')).readline())['length'] == 10


def test_cli_ps_job_and_env_registry():
    from dist_dqn_amd.cli import main
    assert main(['--job=ps']) == 0
    assert make('CartPole-v1').spec.max_episode_steps == 500
    assert make('BreakoutNoFrameskip-v4').action_space.n == 4
    assert make('MountainCar-v0').action_space.n == 3
    with pytest.raises(ValueError):
        make('LunarLander-v2')


def test_step_counter_writes_global_step_per_sec(tmp_path):
    """TF Supervisor's step counter (`/root/reference/src/main.py:136-143`): the chief writes
    ``global_step/sec`` into its event file every summary_secs."""
    import glob
    import time
    cfg = _cfg(tmp_path)
    net = Network.create_network(cfg, (4,), 2)
    sv = RunSupervisor(True, str(tmp_path), net, save_secs=0, install_signal_handlers=False, summary_secs=0.02)
    sv.prepare()
    with sv.managed():
        for step in range(1, 6):
            net.global_step.fill_(10 * step)
            sv.on_train_step(step)
            time.sleep(0.03)
    recs = [r for p in glob.glob(os.path.join(tmp_path, 'events.out.tfevents.*')) for r in read_tfrecords(p)]
    tagged = [r for r in recs if b'global_step/sec' in r]
    assert len(tagged) >= 3, len(tagged)
