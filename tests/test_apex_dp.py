"""Ape-X with several learner ranks (BASELINE config 4: actors + learners, sharded PER) through
the real CLI, one process per rank over gloo, 4 CPU actor processes per rank:

- every rank fills its OWN replay shard from its own actors (different contents per rank);
- the ranks take their first synchronous step together and step in lockstep (``step_many``
  bodies, each a gradient all-reduce);
- when one rank's actors all die, that rank asks to stop and BOTH ranks leave at the same
  agreed step (coordinated stop), saving cleanly;
- at the end every replica tensor is bit-identical across the ranks.

Reference: Ape-X-style actor parallelism is BASELINE config 4; the per-rank agent loop is
`/root/reference/src/main.py:100-167`, the stop check `/root/reference/src/dqn_agent.py:68-70`.
"""
import json
import os

import pytest

from test_fault_resume import _free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(world, logdir, args, fault=None, timeout=300):
    import subprocess
    import sys
    port = _free_port()
    procs, logs = [], []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE=str(world), LOCAL_RANK=str(r), OMP_NUM_THREADS='1')
        env.pop('DQN_FAULT_INJECT', None)
        if fault:
            env['DQN_FAULT_INJECT'] = fault
        f = open(os.path.join(logdir, 'proc%d.log' % r), 'w')
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


def _args(logdir, *extra):
    return ['--env=CartPole-v0', '--network=simple', '--device=cpu', '--seed=5', '--sync', '--optimizer=adam',
            '--lr=0.001', '--minibatch_size=32', '--num_actors=4', '--replay_memory_capacity=20000',
            '--replay_start_size=200', '--n_step=3', '--max_steps_per_episode=200', '--checkpoint_secs=600',
            '--stop_sync_steps=8', '--apex_graph_steps=4', '--apex_reserve_cpus=0', '--log_level=WARNING',
            '--logdir=%s' % logdir] + list(extra)


def _records(logdir, rank, kind):
    path = os.path.join(logdir, 'metrics.rank%d.jsonl' % rank)
    return [r for r in map(json.loads, open(path)) if r.get('kind') == kind]


def _log(logdir, r):
    return open(os.path.join(logdir, 'proc%d.log' % r)).read()[-3000:]


def _check_shards_and_replicas(logdir, steps=None):
    done = [_records(logdir, r, 'done')[-1] for r in range(2)]
    for d in done:
        assert d['replay_size'] >= 200 and d['env_frames'] >= 200, d
        assert d['graph_steps'] == 4
    # each rank's shard was filled by its own actors
    assert done[0]['replay_digest'] != done[1]['replay_digest'], done
    assert done[0]['training_steps'] == done[1]['training_steps'], done
    if steps is not None:
        assert done[0]['training_steps'] == steps
    checks = [_records(logdir, r, 'replica_check')[-1] for r in range(2)]
    for c in checks:
        assert c['equal'] and all(c['tensors'].values()), c
        assert c['world_size'] == 2
    assert set(checks[0]['tensors']) >= {'online', 'target', 'global_step'}
    assert any(k.startswith('slot/') for k in checks[0]['tensors']), checks[0]
    return done


@pytest.mark.timeout(400)
def test_apex_world2_shards_lockstep_replicas(tmp_path):
    logdir = str(tmp_path)
    rcs = _launch(2, logdir, _args(logdir, '--max_train_steps=96'))
    assert rcs == [0, 0], (rcs, _log(logdir, 0), _log(logdir, 1))
    done = _check_shards_and_replicas(logdir, steps=96)
    assert done[0]['global_step'] == done[1]['global_step'] == 96


@pytest.mark.timeout(400)
def test_apex_world2_actor_death_is_a_coordinated_stop(tmp_path):
    """Rank 1's actors are killed at step 40; rank 1 asks to stop and both ranks leave at the
    same agreed step (a multiple of stop_sync_steps past 40), with the chief's final save."""
    logdir = str(tmp_path)
    rcs = _launch(2, logdir, _args(logdir, '--max_train_steps=1000000'), fault='step:40,rank:1,mode:actors')
    assert rcs == [0, 0], (rcs, _log(logdir, 0), _log(logdir, 1))
    done = _check_shards_and_replicas(logdir)
    s = done[0]['training_steps']
    assert s >= 40 and s % 8 == 0, done
    assert 'actors exited' in done[1]['stop_reason'], done
    assert os.path.exists(os.path.join(logdir, 'model.ckpt-%d' % s)) or any(
        n.startswith('model.ckpt-%d' % s) for n in os.listdir(logdir)), os.listdir(logdir)


@pytest.mark.timeout(300)
def test_apex_world2_time_budget_ends_before_the_first_step(tmp_path):
    """The replay never reaches replay_start_size (larger than its capacity), so no rank ever
    takes a first step; --apex_seconds must still end BOTH ranks (the stop request rides in the
    pre-start readiness reduction) instead of spinning forever."""
    logdir = str(tmp_path)
    args = _args(logdir, '--max_train_steps=1000000', '--apex_seconds=4')
    args = [a for a in args if not a.startswith('--replay_start_size')] + ['--replay_start_size=10000000']
    rcs = _launch(2, logdir, args, timeout=200)
    assert rcs == [0, 0], (rcs, _log(logdir, 0), _log(logdir, 1))
    done = [_records(logdir, r, 'done')[-1] for r in range(2)]
    assert all(d['training_steps'] == 0 for d in done), done


def _gpu_args(logdir, *extra):
    import shlex
    from dist_dqn_amd.config import dqn_params_for_env
    return shlex.split(dqn_params_for_env('apex', 'Pong-v0')) + [
        '--num_actors=4', '--replay_memory_capacity=20000', '--replay_start_size=600', '--sync',
        '--allreduce=xgmi', '--checkpoint_secs=600', '--stop_sync_steps=8', '--apex_graph_steps=4',
        '--apex_reserve_cpus=0', '--log_level=WARNING', '--logdir=%s' % logdir] + list(extra)


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize('fault', [None, 'step:40,rank:1,mode:actors'])
def test_apex_world2_one_gpu_rehearsal(tmp_path, fault):
    """Nature-CNN Ape-X (double + dueling, PER, n-step 3) with 2 learner ranks sharing cuda:0
    over gloo + the in-graph xGMI gradient exchange: each rank's step_many replays ONE graph of
    4 step bodies, the replay shards differ, the replicas end bit-identical, and (fault) a
    rank whose actors die is a coordinated stop."""
    logdir = str(tmp_path)
    os.environ['DQN_DIST_BACKEND'] = 'gloo'
    try:
        rcs = _launch(2, logdir, _gpu_args(logdir, '--max_train_steps=%d' % (1000000 if fault else 96)),
                      fault=fault, timeout=240)
    finally:
        os.environ.pop('DQN_DIST_BACKEND', None)
    assert rcs == [0, 0], (rcs, _log(logdir, 0), _log(logdir, 1))
    done = _check_shards_and_replicas(logdir, steps=None if fault else 96)
    assert all(d['step_many'] for d in done), done           # in-graph collectives: k steps per launch
    if fault:
        assert done[0]['training_steps'] >= 40 and done[0]['training_steps'] % 8 == 0, done
        assert 'actors exited' in done[1]['stop_reason'], done


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_device_envs_world2_one_gpu_graph_probe(tmp_path):
    """--device_envs under sync DP (2 ranks on cuda:0, gloo + in-graph xGMI): the CLI runs
    bench.py's start-up G probe (identical decision on both ranks), trains to the step budget
    and ends with bit-identical replicas."""
    import shlex
    from dist_dqn_amd.config import dqn_params_for_env
    logdir = str(tmp_path)
    args = shlex.split(dqn_params_for_env('nature', 'Pong-v0')) + [
        '--dtype=bf16', '--device_envs=4', '--max_train_steps=96', '--replay_start_size=512',
        '--replay_memory_capacity=8192', '--checkpoint_secs=600', '--seed=1', '--sync', '--allreduce=xgmi',
        '--stop_sync_steps=8', '--log_level=INFO', '--logdir=%s' % logdir]
    os.environ['DQN_DIST_BACKEND'] = 'gloo'
    try:
        rcs = _launch(2, logdir, args, timeout=240)
    finally:
        os.environ.pop('DQN_DIST_BACKEND', None)
    assert rcs == [0, 0], (rcs, _log(logdir, 0), _log(logdir, 1))
    starts = [_records(logdir, r, 'start')[-1] for r in range(2)]
    assert starts[0]['steps_per_graph_launch'] == starts[1]['steps_per_graph_launch'] in (1, 8), starts
    assert 'graph-steps probe (2 ranks)' in _log(logdir, 0)
    done = [_records(logdir, r, 'done')[-1] for r in range(2)]
    assert done[0]['training_steps'] == done[1]['training_steps'] >= 96, done
    for r in range(2):
        c = _records(logdir, r, 'replica_check')[-1]
        assert c['equal'] and all(c['tensors'].values()), c
