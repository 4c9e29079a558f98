"""Command line entry (reference `src/main.py`): ``python -m dist_dqn_amd <flags>``.

Accepts every reference flag (see `config.py`). Launch modes:
  * single process: ``python -m dist_dqn_amd --env=CartPole-v0 ...``;
  * data parallel: ``torchrun --nproc-per-node N -m dist_dqn_amd ...`` (RCCL),
    or reference-style ``--worker_hosts=h:p,h:p --task_id=i`` per process;
  * ``--job=ps`` exits immediately (no parameter-server process is needed).
"""
from __future__ import annotations

import logging
import os
import random
import sys
from typing import Optional, Sequence

import numpy as np
import torch

from .config import Config, parse_args

log = logging.getLogger('dist_dqn_amd')


def run_worker(config: Config):
    """Reference `run_worker` (`src/main.py:100-167`) for one learner rank."""
    from . import envs
    from .agent import DQNAgent
    from .learner import Learner
    from .models.network import Network
    from .parallel import broadcast_state, init_distributed
    from .replay import DeviceReplay, ReplayMemory
    from .supervisor import RunSupervisor
    from .utils.metrics import EpisodeMonitor, JsonlWriter

    ctx = init_distributed(config)
    seed = config.seed if config.seed is not None else 1234
    torch.manual_seed(seed + ctx.rank)
    env = envs.make(config.env, seed=seed + 1000 * ctx.rank)
    input_shape = DQNAgent.get_input_shape(env, config)
    network = Network.create_network(config.replace(seed=seed), input_shape, env.action_space.n,
                                     num_replicas=ctx.world_size, device=ctx.device)
    log.info('rank %d/%d device=%s executor=%s params=%d', ctx.rank, ctx.world_size, ctx.device,
             network.executor.name, network.arch.num_params())

    if ctx.enabled and not (config.sync or config.async_ps):
        # reference semantics: no --sync means asynchronous PS training (network.py:186-202)
        log.warning('world size %d without --sync or --async_ps: running synchronous data parallelism '
                    '(the reference default is asynchronous parameter-server training; pass --async_ps '
                    'for that, or --sync to silence this warning)', ctx.world_size)
    coordinated = ctx.enabled and not config.async_ps
    sv = RunSupervisor(is_chief=ctx.is_chief, logdir=config.logdir, network=network, rank=ctx.rank,
                       world_size=ctx.world_size, save_secs=config.checkpoint_secs,
                       max_to_keep=config.max_to_keep, ctx=ctx, coordinated=coordinated,
                       stop_sync_steps=config.stop_sync_steps, summary_secs=config.summary_secs)
    sv.prepare(broadcast_fn=lambda: broadcast_state(ctx, network))

    if config.async_ps and ctx.enabled and ctx.rank == 0:
        return _run_parameter_server(config, ctx, network, sv)
    if config.num_actors > 1:
        return _run_apex(config, ctx, env, network, sv, seed)
    if config.device_envs > 0:
        return _run_device_envs(config, ctx, env, network, sv, seed)
    use_device_replay = ctx.device.type == 'cuda' or ctx.enabled
    if use_device_replay:
        frames = config.resize_width > 0 and config.resize_height > 0
        obs_shape = (config.resize_height, config.resize_width) if frames else tuple(env.observation_space.shape)
        replay = DeviceReplay(config.replay_memory_capacity, obs_shape, config.frames_per_state if frames else 1,
                              device=ctx.device, prioritized=config.prioritized_replay,
                              alpha=config.per_alpha, seed=seed + ctx.rank)
        ps = None
        if config.async_ps and ctx.enabled:
            from .parallel.async_ps import make_ps_client
            ps = make_ps_client(ctx, network.online.flat, config, network=network)
            # start from the PS parameters (and the PS-owned target under --disable_target_replication)
            ps.pull(network.online.flat, network.global_step,
                    target=network.target.flat if config.disable_target_replication else None)
            network.refresh_packed()
        session = Learner(network, replay, config, ctx, ps_client=ps)
        sv.attach_learner(session)
    else:
        replay = ReplayMemory(config.replay_memory_capacity, rng=random.Random(seed + 7919 * (ctx.rank + 1)))
        session = None
    monitor = EpisodeMonitor(config.monitor_path, ctx.rank) if config.monitor else None
    metrics = JsonlWriter(os.path.join(config.logdir, 'metrics.rank%d.jsonl' % ctx.rank))
    metrics.write(kind='start', rank=ctx.rank, world_size=ctx.world_size, restored_from=sv.restored_from,
                  global_step=int(network.global_step), executor=network.executor.name)
    with sv.managed():
        agent = DQNAgent(env, network, session, replay, config, enable_summary=ctx.is_chief,
                         metrics=metrics, monitor=monitor)
        if config.save_agent_state:
            sv.ckpt.agent_state_fn = agent.agent_state
            agent.load_agent_state(sv.agent_state)
        try:
            agent.train(config.num_episodes, config.max_steps_per_episode, sv)
        finally:
            if session is not None and session.ps is not None:
                session.finish_ps()
                session.ps.close()
        if coordinated and config.replica_check:
            _replica_check(ctx, network, metrics, agent.training_steps)
    return agent


def _replica_check(ctx, network, metrics, steps: int):
    """End of a sync-DP run: every replica tensor (online, target, optimizer slots, beta
    powers, global_step, noise stream) must be bit-identical to rank 0's."""
    from .parallel import check_state_equal
    eq = check_state_equal(ctx, network)
    ok = all(eq.values())
    metrics.write(kind='replica_check', equal=ok, tensors=eq, global_step=int(network.global_step),
                  training_steps=steps, world_size=ctx.world_size)
    if not ok:
        raise RuntimeError('replicas diverged on rank %d: %s' % (ctx.rank, {k: v for k, v in eq.items() if not v}))
    log.info('replica check: %d tensors bit-identical across %d ranks at global_step %d', len(eq),
             ctx.world_size, int(network.global_step))


def _run_parameter_server(config: Config, ctx, network, sv):
    """--async_ps rank 0: the parameter server (no env, no replay): applies every
    worker's gradient push in arrival order and answers with fresh parameters."""
    import time
    from .parallel.async_ps import make_ps_server
    server = make_ps_server(ctx, network, config)
    log.info('async PS on rank 0 serving %d workers (%s transport)', len(server.workers),
             getattr(server, 'transport', 'p2p'))
    t0 = time.perf_counter()
    try:
        with sv.managed():
            server.serve(supervisor=sv)
    finally:
        if hasattr(server, 'close'):
            server.close()
    el = time.perf_counter() - t0
    log.info('async PS done: %d updates (%.0f updates/s) %s', server.updates, server.updates / max(el, 1e-9),
             server.per_worker)
    return server


def _run_apex(config: Config, ctx, env, network, sv, seed: int):
    """Ape-X rank: ``--num_actors`` CPU actor processes feed this rank's HBM replay
    shard; a batched GPU inference service answers their greedy actions."""
    from .actors.apex import ApexActorPool, ApexTrainer
    from .learner import Learner
    from .replay import DeviceReplay
    from .utils.metrics import JsonlWriter
    frames = config.resize_width > 0 and config.resize_height > 0
    hw = (config.resize_height, config.resize_width) if frames else None
    obs_shape = hw if frames else tuple(env.observation_space.shape)
    obs_dim = 0 if frames else int(np.prod(obs_shape))
    replay = DeviceReplay(config.replay_memory_capacity, obs_shape, config.frames_per_state if frames else 1,
                          device=ctx.device, num_actors=config.num_actors, prioritized=config.prioritized_replay,
                          alpha=config.per_alpha, seed=seed + ctx.rank)
    learner = Learner(network, replay, config, ctx)
    sv.attach_learner(learner)
    learner.update_target_now()
    pool = ApexActorPool(config.env, config.num_actors, config.frames_per_state if frames else 1, hw, obs_dim,
                         env.action_space.n, config.max_steps_per_episode, seed=seed + 100003 * ctx.rank,
                         eps_base=config.apex_eps_base, eps_alpha=config.apex_eps_alpha,
                         ring_capacity=config.apex_ring, reward_clip=config.reward_clip,
                         n_step=config.n_step, gamma=config.reward_discount)
    metrics = JsonlWriter(os.path.join(config.logdir, 'metrics.rank%d.jsonl' % ctx.rank))
    metrics.write(kind='start', rank=ctx.rank, world_size=ctx.world_size, restored_from=sv.restored_from,
                  global_step=int(network.global_step), executor=network.executor.name,
                  num_actors=config.num_actors)
    with sv.managed():
        trainer = ApexTrainer(network, replay, learner, pool, config, metrics=metrics)
        trainer.run(max_train_steps=config.max_train_steps, max_seconds=config.apex_seconds, supervisor=sv)
    # this rank's shard: what its own actors delivered (replay contents differ across ranks)
    metrics.write(kind='done', training_steps=learner.train_steps, global_step=int(network.global_step),
                  env_frames=trainer.pool.frames, episodes=trainer.pool.episodes, replay_size=replay.size(),
                  replay_digest=replay.digest() if hasattr(replay, 'digest') else None,
                  stop_reason=sv.stop_reason, step_many=learner.can_step_many(),
                  graph_steps=trainer.graph_steps,
                  learn_seconds=(trainer.end_t - trainer.learn_t0) if trainer.learn_t0 is not None else 0.0,
                  learn_frames=trainer.pool.frames - trainer.learn_frames0)
    if ctx.enabled and not config.async_ps and config.replica_check:
        _replica_check(ctx, network, metrics, learner.train_steps)
    return trainer


def _probe_graph_steps(ctx, learner, G_max: int) -> int:
    """bench.py's start-up probe for data parallelism: G = 1 vs G = ``G_max`` SGD steps per graph
    launch (``Learner.step_many``: one graph of G step bodies whose collectives are in-graph
    kernels), timed on every rank and MAX-reduced over the control plane so every rank takes
    the same decision. The probe's steps are ordinary training steps."""
    import time
    dev = learner.device
    for _ in range(3):                       # eager warm-up + the one-step graph capture
        if learner._graphs is not None:
            break
        learner.step()
    if not learner.can_step_many():
        return 1
    failed = 0
    try:
        learner.step_many(G_max)             # capture the G-step graph outside the timing
    except RuntimeError as e:
        log.warning('rank %d: %d-step graph unavailable (%s)', ctx.rank, G_max, e)
        torch.cuda.synchronize(dev)
        failed = 1
    # agreed fallback: under DP every step is a collective, so all ranks drop to G = 1 together,
    # and a rank whose capture failed makes up the G steps its peers just ran
    if ctx.ctrl_allreduce_max(failed):
        for _ in range(G_max if failed else 0):
            learner.step()
        log.warning('one graph per step (a %d-step capture failed on some rank)', G_max)
        return 1

    def timed(fn):
        ctx.ctrl_allreduce_max(0)            # line the ranks up
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        return ctx.ctrl_allreduce_max(int(1e6 * (time.perf_counter() - t0)))

    n = 4 * G_max
    t1 = timed(lambda: [learner.step() for _ in range(n)])
    tg = timed(lambda: [learner.step_many(G_max) for _ in range(n // G_max)])
    G = G_max if tg < t1 else 1
    log.info('graph-steps probe (%d ranks): G=1 %.1f us/step, G=%d %.1f us/step -> G=%d', ctx.world_size,
             t1 / n, G_max, tg / n, G)
    return G


def _run_device_envs(config: Config, ctx, env, network, sv, seed: int):
    """--device_envs=E: E GPU-resident synthetic Atari envs (DeviceActor) whose eps-greedy / env /
    replay-append step rides inside the learner's launches (fused acting: one more trunk / fc
    instance and one head workgroup per env) -- the path bench.py times -- under the Supervisor
    (checkpoints, stop agreement, fault injection), with the reference metrics. The replay is
    prefilled with ``replay_start_size`` random transitions (the synthetic env's frames are random
    anyway: reference prefill, `dqn_agent.py:191-213`); ``update_freq`` env frames are stepped per
    SGD step (``update_freq / E`` fused acting steps; fused only at one step per SGD step)."""
    import time
    from .actors.device_actor import DeviceActor
    from .envs import is_atari
    from .learner import Learner
    from .replay import DeviceReplay
    from .utils.metrics import JsonlWriter, SummaryWriter
    frames = config.resize_width > 0 and config.resize_height > 0
    if not (ctx.device.type == 'cuda' and frames and is_atari(config.env)):
        raise ValueError('--device_envs needs a GPU and a (synthetic) Atari id with frame preprocessing, '
                         'got env=%s device=%s' % (config.env, ctx.device))
    E = int(config.device_envs)
    A = env.action_space.n
    replay = DeviceReplay(config.replay_memory_capacity, (config.resize_height, config.resize_width),
                          config.frames_per_state, device=ctx.device, prioritized=config.prioritized_replay,
                          alpha=config.per_alpha, seed=seed + ctx.rank)
    replay.fill_synthetic(max(config.replay_start_size, config.minibatch_size), A, seed=seed + ctx.rank)
    actor = DeviceActor(network, replay, config, num_envs=E, steps_per_call=max(1, config.update_freq // E),
                        seed=seed + 1000 * (ctx.rank + 1))
    fused = actor.can_fuse(config.minibatch_size)
    learner = Learner(network, replay, config, ctx, actor=actor if fused else None)
    sv.attach_learner(learner)
    learner.update_target_now()
    G = max(1, int(config.device_graph_steps)) if fused and learner.use_graph else 1
    if G > 1 and ctx.enabled:
        G = _probe_graph_steps(ctx, learner, G)
    metrics = JsonlWriter(os.path.join(config.logdir, 'metrics.rank%d.jsonl' % ctx.rank))
    writer = SummaryWriter(config.logdir) if ctx.is_chief else None
    metrics.write(kind='start', rank=ctx.rank, world_size=ctx.world_size, restored_from=sv.restored_from,
                  global_step=int(network.global_step), executor=network.executor.name, device_envs=E,
                  fused_acting=fused, steps_per_graph_launch=G)
    log.info('device envs: %d GPU envs, acting %s, %d SGD steps per graph launch', E,
             'fused into the learner launches' if fused else 'separate launches', G)
    budget = int(config.max_train_steps)
    t0 = t_log = time.time()
    f0 = f_log = actor.env_frames
    s_log = 0
    with sv.managed():
        while not sv.should_stop():
            if budget and learner.train_steps >= budget:
                break
            if G > 1 and (not budget or budget - learner.train_steps >= G) and learner._graphs is not None:
                learner.step_many(G)
            else:
                if not fused:
                    actor.step()
                learner.step()
            sv.on_train_step(learner.train_steps)
            now = time.time()
            if now - t_log >= 10.0 or (budget and learner.train_steps >= budget):
                fr = actor.env_frames
                loss = float(learner.loss)
                rate = (learner.train_steps - s_log) / max(now - t_log, 1e-9)
                fps = (fr - f_log) / max(now - t_log, 1e-9)
                metrics.write(kind='progress', training_steps=learner.train_steps,
                              global_step=int(network.global_step), loss=loss, epsilon=actor.epsilon,
                              sgd_steps_per_sec=rate, env_frames_per_sec=fps, env_frames=fr,
                              replay_size=replay.size())
                if writer is not None:
                    writer.add_scalar('loss', loss, learner.train_steps)
                log.info('training steps = %d, %.0f SGD steps/s, %.0f env frames/s, epsilon = %.3f, loss = %.4f',
                         learner.train_steps, rate, fps, actor.epsilon, loss)
                t_log, f_log, s_log = now, fr, learner.train_steps
    el = max(time.time() - t0, 1e-9)
    metrics.write(kind='done', training_steps=learner.train_steps, sgd_steps_per_sec=learner.train_steps / el,
                  env_frames_per_sec=(actor.env_frames - f0) / el, global_step=int(network.global_step))
    if ctx.enabled and not config.async_ps and config.replica_check:
        _replica_check(ctx, network, metrics, learner.train_steps)
    return learner


def main(argv: Optional[Sequence[str]] = None) -> int:
    config = parse_args(argv)
    logging.basicConfig(level=getattr(logging, config.log_level.upper(), logging.INFO),
                        format='%(asctime)s %(levelname)s %(name)s: %(message)s')
    if config.job == 'ps':
        log.warning('--job=ps: no parameter server is needed (synchronous RCCL data parallelism); exiting.')
        return 0
    from .parallel.dist import shutdown
    try:
        run_worker(config)
    finally:
        shutdown()      # tear the process group down before interpreter exit (gloo's threads)
    return 0


if __name__ == '__main__':
    sys.exit(main())
