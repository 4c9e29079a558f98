#!/usr/bin/env python3
"""Headline benchmark: learner SGD steps/sec (+ env frames/sec) for the Atari
Nature-CNN DQN on 1..8 MI355X (BASELINE.json "metric").

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Per GPU (weak scaling): minibatch 32 from an HBM replay of synthetic 84x84x4
uint8 frames, random-init Nature-CNN (VALID convs 32/64/64, FC512, A=6),
RMSProp (TF semantics), MSE TD loss, target copy every 10k steps — one full
SGD step per timed step (sample, gather, online+target forward, loss,
backward, gradient all-reduce when N > 1 (peer-to-peer xGMI kernel inside the step's
HIP graph, or RCCL, whichever the start-up probe measured faster), optimizer, target
predicate). The device actor runs inside each timed step and writes its
frames into the same replay: ``--actor_envs`` envs x ``update_freq // envs``
batched eps-greedy steps = update_freq (4) env frames per SGD step, the
reference's 1:4 acting/learning ratio (`scripts/dqn_params.sh:38`).
Prints ONE JSON line on rank 0; ``value`` = total SGD steps/s over all ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# (ref: the reference's own Q-network and preset -- `cnn` (SAME convs + max-pools, FC256), the atari
#  preset of scripts/dqn_params.sh:24-42 (RMSProp 2.5e-4, B = 32, no input scaling) -- in the reference's
#  fp32 by default)
VARIANT_DTYPE = {'rainbow': 'fp16', 'ref': 'fp32'}
METRIC = "learner SGD steps/sec + env frames/sec, Atari Nature-CNN DQN at 1/2/4/8 MI355X"
VARIANTS = {
    'dqn': '',
    'dd': '--dueling --double_dqn --loss=huber',
    'rainbow': '--dueling --double_dqn --distributional --noisy --prioritized_replay --optimizer=adam --lr=0.0000625',
    'ref': '',
}


def relaunch(n: int) -> int:
    """Run this benchmark as ``n`` ranks (one per GPU) under torch.distributed.run and return the
    worst rank's exit code; rank 0's JSON line reaches stdout unchanged. Refuses loudly when the
    node has fewer than ``n`` GPUs, unless DQN_DIST_BACKEND=gloo asks for a one-GPU rehearsal
    (ranks sharing a device, process group over gloo, data over the in-graph xgmi kernels)."""
    import socket
    import subprocess
    shared_ok = os.environ.get('DQN_DIST_BACKEND') == 'gloo'
    ndev = torch.cuda.device_count()
    if ndev < n and not shared_ok:
        print('bench: --gpus %d needs %d GPUs, this node has %d (one rank per GPU; DQN_DIST_BACKEND=gloo '
              'rehearses several ranks on one GPU)' % (n, n, ndev), file=sys.stderr, flush=True)
        return 2
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=%d' % n,
           '--master-addr=127.0.0.1', '--master-port=%d' % port, os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def timed_split(steps: int, g_max: int):
    """(G, graph launches, single steps) for the timed region: G = the largest step count per graph
    launch in [4, g_max] that divides ``steps`` (no single-step graphs mixed into the timing), else
    g_max with the remainder as single steps (reported)."""
    if g_max <= 1:
        return 1, 0, steps
    for g in range(g_max, 3, -1):
        if steps % g == 0:
            return g, steps // g, 0
    return g_max, steps // g_max, steps % g_max


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=500)
    ap.add_argument('--warmup', type=int, default=50)
    ap.add_argument('--network', default='nature')
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--dtype', default=None, choices=['bf16', 'fp16', 'fp32'],
                    help='compute dtype (default: the variant\'s BASELINE config -- bf16, Rainbow fp16)')
    ap.add_argument('--backend', default='auto', choices=['auto', 'hip', 'torch'])
    ap.add_argument('--replay', type=int, default=1000000, help='replay capacity (the Atari preset: 1M transitions)')
    ap.add_argument('--actions', type=int, default=6)
    ap.add_argument('--actor_envs', type=int, default=4)
    ap.add_argument('--update_freq', type=int, default=4)
    ap.add_argument('--graph', type=int, default=1)
    ap.add_argument('--extra', default='', help='extra config flags, e.g. "--dueling --double_dqn"')
    ap.add_argument('--variant', default='dqn', choices=sorted(VARIANTS),
                    help='algorithm variant (BASELINE.json configs): dqn = Nature DQN, dd = Double+Dueling+Huber, '
                         'rainbow = C51 + noisy nets + dueling + double + PER + Adam, ref = the reference\'s own '
                         '`cnn` Q-network on its atari preset (fp32 by default)')
    ap.add_argument('--fuse_acting', type=int, default=1,
                    help='run the device actors\' step inside the learner step\'s launches when possible')
    ap.add_argument('--graph_steps', type=int, default=16,
                    help='SGD steps per HIP-graph launch (Learner.step_many: the same per-step work, one host '
                         'launch per G steps -- the inter-graph gap is amortised); 1 = one graph per step '
                         '(profiles/r4_graph_steps.txt: 16 / 32 measured 0.5-1%% above 8)')
    ap.add_argument('--dp_path', type=int, default=0,
                    help='1 (one GPU only): run the data-parallel step at W = 1 -- a one-rank RCCL group with every '
                         'DP code path on (in-graph xgmi gather + in-launch gradient exchange): the per-rank cost of '
                         'the multi-GPU step without peers')
    args = ap.parse_args()
    if args.dp_path and args.gpus != 1:
        ap.error('--dp_path is the one-rank probe of the DP step (--gpus 1)')
    if args.variant == 'ref':
        args.network = 'cnn'
    if args.dtype is None:             # BASELINE.json config 5: "Rainbow ... fp16 conv MFMA path"
        args.dtype = VARIANT_DTYPE.get(args.variant, 'bf16')
    if args.gpus < 1:
        ap.error('--gpus must be >= 1')
    # --gpus N > 1 started without a launcher: relaunch N ranks under torch.distributed.run as a
    # CHILD process, before anything touches the GPU (device_count() does not initialise it here)
    if 'RANK' not in os.environ and args.gpus > 1:
        return relaunch(args.gpus)
    world_env = int(os.environ.get('WORLD_SIZE', '1'))
    if world_env != args.gpus:
        print('bench: --gpus %d but the launcher started %d rank(s); pass --gpus equal to --nproc-per-node'
              % (args.gpus, world_env), file=sys.stderr, flush=True)
        return 2

    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.parallel import broadcast_state, check_state_equal, init_distributed
    from dist_dqn_amd.parallel.dist import device_id
    from dist_dqn_amd.replay import DeviceReplay

    cfg = preset('nature' if args.network == 'nature' else 'atari', 'Pong-v0',
                 '--minibatch_size=%d --dtype=%s --backend=%s --hip_graph=%d --replay_memory_capacity=%d '
                 '--update_freq=%d --seed=0 %s' % (args.batch, args.dtype, args.backend, args.graph, args.replay,
                                                    args.update_freq, VARIANTS[args.variant] + ' ' + args.extra))
    if args.network not in ('nature', 'cnn'):
        cfg = cfg.replace(network=args.network)
    ctx = init_distributed(cfg, device='cuda', force_dp=bool(args.dp_path))
    dev = ctx.device
    assert dev.type == 'cuda', 'bench.py needs a GPU'
    if ctx.enabled and ctx.ranks_share_gpu() and ctx.backend != 'gloo':
        print('bench: ranks share a GPU (%s); one rank per GPU is required (DQN_DIST_BACKEND=gloo for a '
              'one-GPU rehearsal)' % ctx.device_ids(), file=sys.stderr, flush=True)
        return 2
    net = Network.create_network(cfg, (84, 84, 4), args.actions, num_replicas=ctx.world_size, device=dev)
    net.target.copy_from(net.online)
    net.refresh_packed()
    broadcast_state(ctx, net)          # every replica tensor from rank 0 (params, target, slots, noise)
    replay = DeviceReplay(cfg.replay_memory_capacity, (84, 84), 4, device=dev,
                          prioritized=cfg.prioritized_replay, seed=ctx.rank)
    replay.fill_synthetic(cfg.replay_memory_capacity, args.actions, seed=ctx.rank)
    actor = None
    if args.actor_envs > 0:
        from dist_dqn_amd.actors.device_actor import DeviceActor
        actor = DeviceActor(net, replay, cfg, num_envs=args.actor_envs,
                            steps_per_call=max(1, args.update_freq // args.actor_envs),
                            seed=1000 + ctx.rank)
    fused = bool(args.fuse_acting) and actor is not None and actor.can_fuse(args.batch)
    learner = Learner(net, replay, cfg, ctx, actor=actor if fused else None)

    def step():
        if actor is not None and not fused:
            actor.step()
        learner.step()

    # G steps per graph launch (Learner.step_many) when the whole step is one in-graph body (fused or
    # no acting; one process, or DP with in-graph xgmi collectives). Whether G > 1 pays is decided
    # by a start-up probe (below), identically on every rank.
    # G_max divides --steps when it can (timed_split), so the timed region is G-step launches only
    G_max = timed_split(args.steps, max(1, args.graph_steps))[0] if (actor is None or fused) and args.graph else 1

    def run(n, G):
        if G > 1:
            for _ in range(n // G):
                learner.step_many(G)
            n %= G
        for _ in range(n):
            step()

    def timed(fn):
        ctx.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if ctx.enabled:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el)

    # warm-up: eager steps and the one-step graph capture, then (G_max > 1) the G-step graph's
    # capture and first replay -- W steps in all when W >= G + 3, else W single steps + one G-step launch
    w1 = args.warmup - G_max if G_max > 1 and args.warmup >= G_max + 3 else args.warmup
    for _ in range(w1):
        step()
    for _ in range(3):                          # (tiny W: the one-step graph must exist first)
        if learner._graphs is not None or not args.graph:
            break
        step()
    if G_max > 1 and not learner.can_step_many():
        G_max = 1
    if G_max > 1:
        failed = 0
        try:
            learner.step_many(G_max)            # captures the G-step graph outside the timed region
        except RuntimeError as e:               # (capture refused): one graph per step instead
            print('bench: rank %d: %d-step graph unavailable (%s)' % (ctx.rank, G_max, e), file=sys.stderr,
                  flush=True)
            torch.cuda.synchronize(dev)
            failed = 1
        # every rank falls back together (DP: each step is a collective, so the ranks' step
        # sequences must stay identical); a rank whose capture succeeded ran G steps, the others
        # catch up with single steps
        if ctx.ctrl_allreduce_max(failed):
            for _ in range(G_max if failed else 0):
                step()
            G_max = 1
            print('bench: one graph per step (a G-step capture failed on some rank)', file=sys.stderr, flush=True)
    # probe (untimed, identical decision on every rank: MAX-reduced times): G = 1 vs G = G_max
    probe_steps = 4 * G_max if G_max > 1 else 16
    t_g1 = timed(lambda: run(probe_steps, 1))
    G = 1
    if G_max > 1:
        t_gm = timed(lambda: run(probe_steps, G_max))
        G = G_max if t_gm < t_g1 else 1
    ms_g1 = 1000.0 * t_g1 / probe_steps
    G, n_launch, n_single = timed_split(args.steps, G)
    ctx.barrier()
    torch.cuda.synchronize(dev)
    frames0 = actor.env_frames if actor is not None else 0
    t0 = time.perf_counter()
    run(args.steps, G)
    torch.cuda.synchronize(dev)
    ctx.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if ctx.enabled:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t)
    # env frames the device actors actually stepped in the timed region (device counter), summed
    frames = torch.tensor([(actor.env_frames - frames0) if actor is not None else 0], dtype=torch.float64,
                          device=dev)
    if ctx.enabled:
        dist.all_reduce(frames)
    frames = float(frames)
    loss = float(learner.loss)
    xgmi_ok = learner.reducer.xgmi.check() if learner.reducer.xgmi is not None else True
    # (outside the timed region) every replica tensor must still be bit-identical to rank 0's
    eq = check_state_equal(ctx, net)
    replicas_equal = all(eq.values())
    dev_ids = ctx.device_ids() if ctx.enabled else [device_id(dev)]
    if ctx.rank == 0:
        sps = args.steps * ctx.world_size / el
        out = {
            'metric': METRIC, 'value': round(sps, 2), 'unit': 'SGD steps/s (all GPUs)',
            'n_gpus': ctx.world_size, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': round(1000.0 * el / args.steps, 4), 'ms_per_step_g1': round(ms_g1, 4),
            'graph_steps': G, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': getattr(net.executor, 'compute_dtype', 'fp32'), 'data': 'synthetic (random uint8 84x84 frames, random init)',
            'env_frames_per_sec': round(frames / el, 1),
            'samples_per_sec': round(sps * args.batch, 1),
            'config': {'model': 'nature-cnn' if args.network == 'nature' else args.network,
                       'global_batch': args.batch * ctx.world_size, 'seq_len': None,
                       'parallelism': 'dp%d' % ctx.world_size + (' (DP step forced at one rank)' if ctx.force_dp else ''),
                       'per_gpu_batch': args.batch,
                       'frames_per_state': 4, 'optimizer': cfg.optimizer + '(tf)', 'executor': net.executor.name,
                       'hip_graph': bool(args.graph), 'steps_per_graph_launch': G,
                       'timed_launches': {'graph_launches_of_G': n_launch, 'single_step_graphs': n_single},
                       'graph_steps_probe': {'candidates': sorted({1, G_max}), 'probe_steps': probe_steps,
                                             'ms_per_step_g1': round(ms_g1, 4)},
                       'actor_envs': args.actor_envs,
                       'acting': 'fused into the learner launches' if fused else 'separate launches',
                       'update_freq': args.update_freq, 'replay_capacity': cfg.replay_memory_capacity,
                       'num_actions': args.actions, 'variant': args.variant, 'extra': args.extra,
                       'final_loss': loss,
                       'allreduce': learner.reducer.mode if ctx.enabled else None,
                       'allreduce_probe_us': learner.reducer.timings or None,
                       'xgmi_vs_rccl_max_rel': (learner.reducer.timings or {}).get('xgmi_vs_rccl_max_rel'),
                       'rank_devices': dev_ids, 'ranks_share_gpu': len(set(dev_ids)) < len(dev_ids),
                       'lowrank_dense': learner._lowrank is not None,
                       'dp_fused_update': bool(getattr(learner, '_dp_fused', False)),
                       'allreduce_ranges': learner._ar_ranges or None,
                       'allreduce_peer_timeouts': not xgmi_ok,
                       'world_size': ctx.world_size, 'dist_backend': ctx.backend,
                       'replicas_equal': replicas_equal,
                       'replicas_diverged': sorted(k for k, v in eq.items() if not v),
                       'sampling': learner._sample_mode()},
        }
        print(json.dumps(out), flush=True)
        if os.environ.get('DQN_OPT_PROF'):            # optimizer phase stamps of the last launch
            t = net.executor.ext.optim_prof()
            print('optim_pack stamps (cycles from block start): block0 %s | block1 %s'
                  % ([t[i] - t[0] for i in range(1, 5)], [t[8 + i] - t[8] if t[8 + i] else 0 for i in range(1, 8)]),
                  file=sys.stderr, flush=True)
    if ctx.enabled:
        dist.destroy_process_group()
    if not replicas_equal or not xgmi_ok:
        print('bench: replicas diverged (%s) or an xgmi peer wait timed out (%s)'
              % (sorted(k for k, v in eq.items() if not v), not xgmi_ok), file=sys.stderr, flush=True)
        return 3
    return 0


if __name__ == '__main__':
    sys.exit(main())
