"""Supervisor under synchronous data parallelism, through the real CLI (one process per rank,
gloo): periodic checkpoints while training, a crashed peer ends the survivor's loop, a
graceful stop request is agreed so every rank leaves after the same step, and a relaunch
restores the chief's checkpoint on EVERY rank (parameters, target, optimizer slots, beta
powers, global_step) so the replicas stay bit-identical.

Reference: `tf.train.Supervisor` (`/root/reference/src/main.py:136-143,155,167`) saves every
600 s, restores all global variables for every worker on start, and the agent checks
``should_stop()`` (`/root/reference/src/dqn_agent.py:68-70`).
"""
import glob
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _args(logdir, *extra):
    return ['--env=CartPole-v0', '--network=simple', '--device=cpu', '--seed=3', '--sync', '--optimizer=adam',
            '--minibatch_size=32', '--replay_start_size=64', '--update_freq=1', '--num_episodes=100000',
            '--max_steps_per_episode=200', '--replay_memory_capacity=5000', '--target_update_freq=25',
            '--max_to_keep=1000', '--stop_sync_steps=5', '--log_level=WARNING', '--logdir=%s' % logdir] + list(extra)


def _launch(world, logdir, args, fault=None, timeout=240):
    port = _free_port()
    procs, logs = [], []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE=str(world), LOCAL_RANK=str(r), OMP_NUM_THREADS='1')
        env.pop('DQN_FAULT_INJECT', None)
        if fault:
            env['DQN_FAULT_INJECT'] = fault
        f = open(os.path.join(logdir, 'proc%d.%d.log' % (r, len(glob.glob(os.path.join(logdir, 'proc%d.*' % r))))),
                 'w')
        logs.append(f)
        procs.append(subprocess.Popen([sys.executable, '-m', 'dist_dqn_amd'] + args, env=env, cwd=ROOT,
                                      stdout=f, stderr=subprocess.STDOUT))
    rcs = []
    try:
        for p in procs:
            rcs.append(p.wait(timeout))
    finally:
        for p in procs:                      # exact processes we started
            if p.poll() is None:
                p.kill()
                p.wait()
        for f in logs:
            f.close()
    return rcs


def _records(logdir, rank, kind):
    path = os.path.join(logdir, 'metrics.rank%d.jsonl' % rank)
    return [r for r in map(json.loads, open(path)) if r.get('kind') == kind]


def _ckpts(logdir):
    return sorted(int(p.rsplit('-', 1)[1]) for p in glob.glob(os.path.join(logdir, 'model.ckpt-*'))
                  if p.rsplit('-', 1)[1].isdigit())


def test_crash_checkpoint_and_resume_world2(tmp_path):
    logdir = str(tmp_path)
    rcs = _launch(2, logdir, _args(logdir, '--checkpoint_secs=0.05'), fault='step:150,rank:1,mode:raise')
    assert rcs[1] != 0                              # the injected crash
    # the survivor's next gradient all-reduce fails (peer gone): its loop ended, it saved
    assert rcs[0] is not None
    steps = _ckpts(logdir)
    assert len(steps) >= 2, steps                   # periodic saves during the run + the final one
    last = steps[-1]
    assert 0 < last <= 150

    # relaunch: every rank restores the chief's checkpoint and trains 3 more steps
    rcs = _launch(2, logdir, _args(logdir, '--checkpoint_secs=600', '--max_train_steps=3'))
    assert rcs == [0, 0], rcs
    starts = [_records(logdir, r, 'start')[-1] for r in range(2)]
    assert [s['global_step'] for s in starts] == [last, last]
    assert starts[0]['restored_from'] == starts[1]['restored_from'] and starts[0]['restored_from'].endswith(
        'model.ckpt-%d' % last)
    checks = [_records(logdir, r, 'replica_check')[-1] for r in range(2)]
    for c in checks:
        assert c['equal'] and all(c['tensors'].values()), c
        assert c['global_step'] == last + 3 and c['training_steps'] == 3
    assert set(checks[0]['tensors']) >= {'online', 'target', 'global_step', 'slot/Adam', 'slot/Adam_1',
                                         'beta_powers'}


def test_graceful_stop_is_agreed_world2(tmp_path):
    """A stop request on rank 1 (signal-like) ends BOTH ranks at the same agreed step, cleanly."""
    logdir = str(tmp_path)
    rcs = _launch(2, logdir, _args(logdir, '--checkpoint_secs=600'), fault='step:40,rank:1,mode:stop')
    assert rcs == [0, 0], rcs
    checks = [_records(logdir, r, 'replica_check')[-1] for r in range(2)]
    assert checks[0]['training_steps'] == checks[1]['training_steps'] == 40
    assert checks[0]['equal'] and checks[1]['equal']
    assert _ckpts(logdir)[-1] == 40                 # the chief's final save on stop
