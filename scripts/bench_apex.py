"""Ape-X throughput (BASELINE.json config 4, single rank): N CPU actor processes
(synthetic Atari, C++ preprocessing) -> SPSC rings -> HBM PER replay shard,
batched GPU inference service, Double+Dueling n-step learner on the HIP executor.

    python scripts/bench_apex.py --actors 16 --seconds 60
    python scripts/bench_apex.py --world 8 --actors 32 --seconds 60     # 256 actors + 8 learners

Prints one JSON line: env frames/s (all actors), SGD steps/s, served batch stats.

``--world N`` (BASELINE config 4 on one node): the script starts itself under
``torch.distributed.run`` with N ranks (one GPU each, RCCL / in-graph xGMI gradient exchange);
every rank runs the CLI's Ape-X path (``cli.run_worker``: ``--actors`` actor processes into its
own HBM PER shard, synchronous data-parallel learner, coordinated time-budget stop, end-of-run
replica check) and rank 0 prints the aggregate: env frames/s summed over ranks, learner SGD
steps/s (lockstep: every rank takes the same steps).
"""
import argparse
import json
import logging
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--actors', type=int, default=min(16, os.cpu_count() or 4))
    ap.add_argument('--seconds', type=float, default=60.0)
    ap.add_argument('--capacity', type=int, default=200000)
    ap.add_argument('--extra', default='')
    ap.add_argument('--world', type=int, default=1, help='learner ranks (one GPU each)')
    args = ap.parse_args()
    if args.world > 1:
        return main_world(args)
    logging.basicConfig(level=logging.INFO, format='%(asctime)s %(name)s: %(message)s')
    import torch
    from dist_dqn_amd.actors.apex import ApexActorPool, ApexTrainer
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    from dist_dqn_amd.utils.cpus import cfs_quota_cpus
    dev = torch.device('cuda', 0) if torch.cuda.is_available() else torch.device('cpu')
    cfg = preset('apex', 'Pong-v0', '--num_actors=%d --replay_memory_capacity=%d --replay_start_size=2000 '
                 '--logdir=%s %s' % (args.actors, args.capacity, tempfile.mkdtemp(), args.extra))
    net = Network.create_network(cfg, (84, 84, 4), 6, device=dev)
    rep = DeviceReplay(cfg.replay_memory_capacity, (84, 84), 4, device=dev, num_actors=cfg.num_actors,
                       prioritized=cfg.prioritized_replay, alpha=cfg.per_alpha, seed=1)
    ln = Learner(net, rep, cfg)
    pool = ApexActorPool(cfg.env, cfg.num_actors, 4, (84, 84), 0, 6, cfg.max_steps_per_episode, seed=1,
                         eps_base=cfg.apex_eps_base, eps_alpha=cfg.apex_eps_alpha, ring_capacity=cfg.apex_ring,
                         n_step=cfg.n_step, gamma=cfg.reward_discount)
    tr = ApexTrainer(net, rep, ln, pool, cfg)
    t0 = time.time()
    tr.run(max_seconds=args.seconds, log_every=10.0)
    t1 = time.time()
    wall = t1 - t0
    lw = t1 - tr.learn_t0 if tr.learn_t0 is not None else 0.0      # steady state: learner running
    print(json.dumps({
        'metric': 'Ape-X env frames/sec + learner SGD steps/sec (1 rank)', 'actors': cfg.num_actors,
        'seconds': round(wall, 1), 'env_frames': pool.frames, 'env_frames_per_sec': round(pool.frames / wall, 1),
        'sgd_steps': ln.train_steps, 'sgd_steps_per_sec': round(ln.train_steps / wall, 1),
        'learning_seconds': round(lw, 1),
        'learner_sgd_steps_per_sec': round(ln.train_steps / lw, 1) if lw > 0 else None,
        'learner_env_frames_per_sec': round((pool.frames - tr.learn_frames0) / lw, 1) if lw > 0 else None,
        'greedy_actions_served': pool.served, 'serve_calls': tr.serve_calls,
        'mean_serve_batch': round(pool.served / max(1, tr.serve_calls), 2), 'executor': net.executor.name,
        'cpus_visible': len(os.sched_getaffinity(0)), 'cfs_quota_cpus': cfs_quota_cpus(),
        'main_loop_s': {k: round(v, 2) for k, v in tr.loop_time.items()},
        'config': 'apex preset: double+dueling, PER, n_step=3, nature-cnn', 'dtype': net.executor.compute_dtype,
        'device': str(dev)}))


def main_world(args):
    """N learner ranks; relaunches itself under torch.distributed.run (as a child process,
    before anything touches the GPU) when not started by a launcher."""
    if 'RANK' not in os.environ:
        import socket
        import subprocess
        s = socket.socket()
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=%d' % args.world,
               '--master-addr=127.0.0.1', '--master-port=%d' % port, os.path.abspath(__file__)] + sys.argv[1:]
        return subprocess.call(cmd)
    logging.basicConfig(level=logging.WARNING, format='%(asctime)s %(name)s: %(message)s')
    import torch.distributed as dist
    from dist_dqn_amd.cli import run_worker
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.utils.cpus import cfs_quota_cpus
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    assert world == args.world, (world, args.world)
    logdir = os.path.join(tempfile.gettempdir(), 'bench_apex_w%d_%d' % (world, int(os.environ.get('MASTER_PORT', 0))))
    cfg = preset('apex', 'Pong-v0', '--num_actors=%d --replay_memory_capacity=%d --replay_start_size=2000 '
                 '--sync --apex_seconds=%g --checkpoint_secs=0 --logdir=%s %s'
                 % (args.actors, args.capacity, args.seconds, logdir, args.extra))
    tr = run_worker(cfg)
    ln = tr.learner
    lw = tr.end_t - tr.learn_t0 if tr.learn_t0 is not None else 0.0
    mine = dict(rank=rank, frames=tr.pool.frames, learn_frames=tr.pool.frames - tr.learn_frames0, learn_s=lw,
                steps=ln.train_steps, served=tr.pool.served, calls=tr.serve_calls,
                replay=tr.replay.size(), step_many=ln.can_step_many(), reducer=getattr(ln.reducer, 'mode', None),
                cpus=len(os.sched_getaffinity(0)))
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    if rank == 0:
        lw_max = max(r['learn_s'] for r in allr) or 1e-9
        steps = allr[0]['steps']
        print(json.dumps({
            'metric': 'Ape-X env frames/sec + learner SGD steps/sec (%d ranks)' % world, 'world': world,
            'actors_per_rank': args.actors, 'actors': args.actors * world, 'seconds': args.seconds,
            'learner_env_frames_per_sec': round(sum(r['learn_frames'] for r in allr) / lw_max, 1),
            'learner_sgd_steps_per_sec': round(steps / lw_max, 1),
            'samples_per_sec': round(steps * cfg.minibatch_size * world / lw_max, 1),
            'sgd_steps': steps, 'steps_equal': len({r['steps'] for r in allr}) == 1,
            'per_rank': allr, 'reducer': allr[0]['reducer'], 'cfs_quota_cpus': cfs_quota_cpus(),
            'config': 'apex preset: double+dueling, PER (sharded per rank), n_step=3, nature-cnn, sync DP',
            'dtype': tr.net.executor.compute_dtype}))
    return 0


if __name__ == '__main__':
    sys.exit(main())
