"""Data parallelism without a cluster: gloo process groups on the CPU (world 2-3).

Replaces the reference's localhost PS/worker emulation (scripts/dqn_multi_gpu.sh)
with torch.distributed ranks; checks the sync-DP invariants the RCCL path relies on:
averaged gradients equal the big-batch gradient, replicas stay bit-identical,
the chief's parameters reach every rank, and the reference cluster flags map to ranks.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(seed, B=6):
    g = torch.Generator().manual_seed(seed)
    return {'states': torch.randn(B, 4, generator=g), 'next_states': torch.randn(B, 4, generator=g),
            'actions': torch.randint(0, 2, (B,), generator=g), 'rewards': torch.randn(B, generator=g),
            'dones': (torch.rand(B, generator=g) < 0.3).float(), 'gammas': torch.full((B,), 0.9)}


def _worker_grads(rank, world, port, tmpdir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from dist_dqn_amd.config import parse_args
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.parallel import GradAllReducer, broadcast_flat, check_replicas_equal, init_distributed
    cfg = parse_args(['--device=cpu', '--seed=%d' % (100 + rank), '--optimizer=rmsprop', '--lr=0.01'])
    ctx = init_distributed(cfg, device='cpu')
    assert ctx.world_size == world and ctx.rank == rank and ctx.backend == 'gloo'
    net = Network.create_network(cfg, (4,), 2)
    broadcast_flat(ctx, net.online.flat)          # chief init reaches every rank (reference M8)
    net.target.copy_from(net.online)
    assert check_replicas_equal(ctx, net.online.flat)
    red = GradAllReducer(ctx, net.grad, bucket_mb=0.0005)   # force several buckets
    assert len(red.buckets) > 1
    for step in range(3):
        net.compute_grads(_batch(1000 * step + rank))
        red.allreduce()
        g_avg = net.grad * red.scale
        # reference: one process computing the gradient over the union of the batches
        if rank == 0:
            ref = Network.create_network(cfg, (4,), 2)
            ref.online.flat.copy_(net.online.flat)
            ref.target.flat.copy_(net.target.flat)
            big = {k: torch.cat([_batch(1000 * step + r)[k] for r in range(world)]) for k in _batch(0)}
            ref.compute_grads(big)
            torch.testing.assert_close(g_avg, ref.grad, rtol=1e-5, atol=1e-7)
        net.apply_grads(red.scale)
        assert check_replicas_equal(ctx, net.online.flat)
    assert int(net.global_step) == 3
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_dp_grads_equal_big_batch_and_replicas_stay_equal(tmp_path, world):
    mp.spawn(_worker_grads, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)


def _worker_learner(rank, world, port, tmpdir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import numpy as np
    from dist_dqn_amd.config import parse_args
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.parallel import broadcast_flat, check_replicas_equal, init_distributed
    from dist_dqn_amd.replay import DeviceReplay
    cfg = parse_args(['--device=cpu', '--seed=5', '--network=cnn', '--optimizer=rmsprop', '--minibatch_size=4',
                      '--target_update_freq=2', '--replay_memory_capacity=64'])
    ctx = init_distributed(cfg, device='cpu')
    net = Network.create_network(cfg, (84, 84, 4), 6)
    broadcast_flat(ctx, net.online.flat)
    net.target.copy_from(net.online)
    rep = DeviceReplay(64, (84, 84), 4, device='cpu', seed=rank)
    rep.fill_synthetic(64, 6, seed=rank, episode_len=16)    # different data per rank
    ln = Learner(net, rep, cfg, ctx)
    for _ in range(4):
        ln.step()
    assert check_replicas_equal(ctx, net.online.flat)
    assert check_replicas_equal(ctx, net.target.flat)
    assert int(net.global_step) == 4 and ln.train_steps == 4
    dist.barrier()
    dist.destroy_process_group()


def test_dp_learner_cnn_world2(tmp_path):
    mp.spawn(_worker_learner, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)


def test_reference_cluster_flags_map_to_ranks(monkeypatch):
    from dist_dqn_amd.config import parse_args
    from dist_dqn_amd.parallel.dist import _from_cluster_flags
    cfg = parse_args(['--worker_hosts=localhost:8090,localhost:8091,localhost:8092', '--task_id=2',
                      '--gpu_id=3'])
    m = _from_cluster_flags(cfg)
    assert m == dict(rank=2, world=3, addr='127.0.0.1', port='8090', local_rank=3)
    assert _from_cluster_flags(parse_args([])) is None


def _worker_async(rank, world, port, tmpdir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from dist_dqn_amd.config import parse_args
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.parallel import broadcast_flat, init_distributed
    from dist_dqn_amd.parallel.async_ps import AsyncPSClient, AsyncPSServer
    cfg = parse_args(['--device=cpu', '--seed=7', '--optimizer=sgd', '--lr=1.0', '--reg_param=0'])
    ctx = init_distributed(cfg, device='cpu')
    net = Network.create_network(cfg, (4,), 2)
    broadcast_flat(ctx, net.online.flat)
    init = net.online.flat.clone()
    steps = 5
    if rank == 0:
        srv = AsyncPSServer(ctx, net)
        assert srv.serve() == steps * (world - 1)
        # SGD lr=1: every push of worker w subtracted w * ones, in whatever order they arrived
        total = sum(w * steps for w in range(1, world))
        torch.testing.assert_close(net.online.flat, init - total)
        assert int(net.global_step) == steps * (world - 1)
        assert srv.per_worker == {w: steps for w in range(1, world)}
    else:
        cli = AsyncPSClient(ctx, net.online.flat)
        cli.pull(net.online.flat, net.global_step)
        torch.testing.assert_close(net.online.flat, init)
        seen = []
        for _ in range(steps):
            cli.exchange(torch.full_like(net.online.flat, float(rank)), net.online.flat, net.global_step)
            seen.append(int(net.global_step))
        assert seen == sorted(seen) and len(set(seen)) == steps    # PS step only moves forward
        cli.close()
    dist.barrier()
    dist.destroy_process_group()


def test_async_parameter_server_arrival_order(tmp_path):
    mp.spawn(_worker_async, args=(3, _free_port(), str(tmp_path)), nprocs=3, join=True)


def _worker_async_cli(rank, world, port, tmpdir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from dist_dqn_amd.cli import run_worker
    from dist_dqn_amd.config import parse_args
    cfg = parse_args(['--env=CartPole-v0', '--network=simple', '--device=cpu', '--seed=3', '--async_ps',
                      '--optimizer=adam', '--minibatch_size=16', '--num_episodes=6', '--max_steps_per_episode=60',
                      '--replay_memory_capacity=2000', '--target_update_freq=7', '--checkpoint_secs=0',
                      '--logdir=%s/r%d' % (tmpdir, rank)])
    out = run_worker(cfg)
    if rank == 0:
        assert out.updates > 0 and sum(out.per_worker.values()) == out.updates
    else:
        assert out.session.ps.pushes == out.training_steps > 0, (out.session.ps.pushes, out.training_steps)
    dist.barrier()
    dist.destroy_process_group()


def test_async_ps_training_cli_world3(tmp_path):
    """--async_ps end to end: rank 0 serves, ranks 1-2 run the agent against it."""
    mp.spawn(_worker_async_cli, args=(3, _free_port(), str(tmp_path)), nprocs=3, join=True)


def _worker_bf16_wire(rank, world, port, tmpdir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from dist_dqn_amd.config import parse_args
    from dist_dqn_amd.parallel import GradAllReducer, init_distributed
    ctx = init_distributed(parse_args(['--device=cpu']), device='cpu')
    g = torch.Generator().manual_seed(rank)
    flat = torch.randn(1000, generator=g)
    ref = flat.clone()
    dist.all_reduce(ref)
    red = GradAllReducer(ctx, flat, wire_dtype='bf16')
    assert len(red.buckets) == 1                      # default: ONE collective per step
    red.allreduce()
    torch.testing.assert_close(flat, ref, rtol=2e-2, atol=2e-2)
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_bf16_wire(tmp_path):
    mp.spawn(_worker_bf16_wire, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)


def _worker_broadcast_state(rank, world, port, tmpdir):
    """Chief-only restore, then broadcast_state: every replica tensor equal on every rank."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from dist_dqn_amd.config import parse_args
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.parallel import broadcast_state, check_state_equal, init_distributed
    cfg = parse_args(['--device=cpu', '--seed=%d' % (10 + rank), '--optimizer=adam', '--network=cnn'])
    ctx = init_distributed(cfg, device='cpu')
    net = Network.create_network(cfg, (84, 84, 4), 6)
    if rank == 0:                      # the chief "restored" a trained state
        net.global_step.fill_(123456789)
        net.optimizer.slots[1].fill_(0.5)
        net.optimizer.beta_powers.fill_(0.25)
        net.target.flat.mul_(2.0)
    assert not all(check_state_equal(ctx, net).values())
    broadcast_state(ctx, net)
    eq = check_state_equal(ctx, net)
    assert all(eq.values()), eq
    assert int(net.global_step) == 123456789 and float(net.optimizer.beta_powers[0]) == 0.25
    dist.barrier()
    dist.destroy_process_group()


def test_broadcast_state_world2(tmp_path):
    mp.spawn(_worker_broadcast_state, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)


def _worker_async_owned_target(rank, world, port, tmpdir):
    """--disable_target_replication under --async_ps: the PS owns the target, a worker's sync
    request copies PS online -> PS target, and the new target reaches the workers; the int64
    header carries a global_step beyond fp32's exact range."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from dist_dqn_amd.config import parse_args
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.parallel import broadcast_flat, init_distributed
    from dist_dqn_amd.parallel.async_ps import AsyncPSClient, AsyncPSServer
    cfg = parse_args(['--device=cpu', '--seed=7', '--optimizer=sgd', '--lr=1.0', '--reg_param=0',
                      '--disable_target_replication'])
    ctx = init_distributed(cfg, device='cpu')
    net = Network.create_network(cfg, (4,), 2)
    broadcast_flat(ctx, net.online.flat)
    big = (1 << 24) + 1                 # not representable in fp32
    if rank == 0:
        net.global_step.fill_(big)
        net.target.flat.fill_(3.0)
        srv = AsyncPSServer(ctx, net)
        assert srv.own_target
        srv.serve()
        assert srv.target_syncs == 1
        torch.testing.assert_close(net.target.flat, net.online.flat + 1.0)   # synced before push 2
    else:
        cli = AsyncPSClient(ctx, net.online.flat)
        cli.pull(net.online.flat, net.global_step, target=net.target.flat)
        assert int(net.global_step) == big and cli.target_updated
        assert bool((net.target.flat == 3.0).all())                     # the PS-owned target arrived
        ones = torch.ones_like(net.online.flat)
        cli.exchange(ones, net.online.flat, net.global_step, sync_target=True, target=net.target.flat)
        assert cli.target_updated and torch.equal(net.target.flat, net.online.flat)
        assert int(net.global_step) == big + 1
        cli.exchange(ones, net.online.flat, net.global_step, target=net.target.flat)
        assert not cli.target_updated and int(net.global_step) == big + 2
        cli.close()
    dist.barrier()
    dist.destroy_process_group()


def test_async_ps_owned_target_and_int64_step(tmp_path):
    mp.spawn(_worker_async_owned_target, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)


def _worker_sync_owned_target(rank, world, port, tmpdir):
    """Sync DP + --disable_target_replication: rank 0's target is broadcast after each sync."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from dist_dqn_amd.config import parse_args
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.parallel import broadcast_state, check_state_equal, init_distributed
    from dist_dqn_amd.replay import DeviceReplay
    cfg = parse_args(['--device=cpu', '--seed=5', '--network=cnn', '--optimizer=rmsprop', '--minibatch_size=4',
                      '--target_update_freq=2', '--replay_memory_capacity=64', '--disable_target_replication'])
    ctx = init_distributed(cfg, device='cpu')
    net = Network.create_network(cfg, (84, 84, 4), 6)
    broadcast_state(ctx, net)
    rep = DeviceReplay(64, (84, 84), 4, device='cpu', seed=rank)
    rep.fill_synthetic(64, 6, seed=rank, episode_len=16)
    ln = Learner(net, rep, cfg, ctx)
    assert ln._own_target
    for _ in range(4):
        ln.step()
        if rank == 1:                   # a stray local target write is overwritten by rank 0's copy
            net.target.flat.add_(1.0)
    eq = check_state_equal(ctx, net)
    assert eq['online'] and eq['global_step'] and not eq['target']     # step 4 was a sync, then rank 1 wrote
    ln.step()
    ln.step()                           # step 6 syncs + broadcasts again
    assert all(check_state_equal(ctx, net).values())
    dist.barrier()
    dist.destroy_process_group()


def test_sync_dp_owned_target_broadcast(tmp_path):
    mp.spawn(_worker_sync_owned_target, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)


@pytest.mark.parametrize('extra', ['', '--dueling --double_dqn', '--dueling --double_dqn --distributional --noisy'])
def test_lowrank_reduce_ranges_cover_every_summed_tensor(extra):
    """Low-rank DP: the all-reduce pieces cover every tensor whose gradient is still per-rank,
    never touch the fc weights (already the global sum), skip the noisy sigma tensors (derived in
    the optimizer), stay 64-element multiples and fit one multi-range launch."""
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import _reduce_ranges
    from dist_dqn_amd.models.network import Network
    cfg = preset('nature', 'Pong-v0', '--seed=0 --backend=torch ' + extra)
    lay = Network.create_network(cfg, (84, 84, 4), 6).layout
    names = ['value/fcl/w', 'advantage/fcl/w'] if '--dueling' in extra else ['fcl/w']
    fc = [(lay.offsets[n], lay.offsets[n] + lay.numel(n)) for n in names]
    skip = [(lay.offsets[n], lay.offsets[n] + lay.numel(n)) for n in lay.names if n.endswith('_sigma')]
    r = _reduce_ranges(lay, lay.total, fc + skip, forbidden=fc)
    assert r and len(r) <= 8
    assert all(lo % 64 == 0 and (hi - lo) % 64 == 0 for lo, hi in r)
    assert all(hi <= a or lo >= b for lo, hi in r for a, b in fc)
    for n in lay.names:
        lo, hi = lay.offsets[n], lay.offsets[n] + lay.numel(n)
        if (lo, hi) in fc or (lo, hi) in skip:
            continue
        assert any(a <= lo and hi <= b for a, b in r), n
    # forced merging never crosses an fc range
    r2 = _reduce_ranges(lay, lay.total, fc + skip, forbidden=fc, max_ranges=2)
    assert r2 is None or all(hi <= a or lo >= b for lo, hi in r2 for a, b in fc)
