"""Multi-rank learner on ONE MI355X: 2, 4 or 8 ranks share cuda:0 over a gloo process group
(DQN_DIST_BACKEND=gloo; RCCL refuses two ranks per device). This runs the exact
world > 1 code path of the learner that RCCL runs on an 8-GPU node — split HIP
graphs, dense-range all-reduce started before the conv-backward graph, second
collective, optimizer graph; with --allreduce=xgmi the peer-to-peer kernels at their
world-size instantiations (WC = 2 / 4 / 8), the 8-peer gather and the low-rank fc exchange
feeding the fused optimizer with W*B rows — with real GPU tensors, and checks it against the
non-overlapped single-collective path and across replicas.
"""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(target, args, world=2, timeout=100):
    ctx = mp.get_context('spawn')
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + tuple(args) + (errq,)) for r in range(world)]
    # (a hung rank dumps its Python stacks shortly before the deadline: _setup)
    os.environ['DQN_TEST_STACK_DUMP_S'] = str(max(5, timeout - 10))
    for p in procs:
        p.start()
    deadline = time.monotonic() + timeout          # one deadline for all ranks, not one per join
    for p in procs:
        p.join(timeout=max(0.0, deadline - time.monotonic()))
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not alive, 'rank(s) hung'
    assert not errs, '\n'.join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def _setup(rank, world, port):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0', DQN_DIST_BACKEND='gloo')
    if world > 4:
        # 8 ranks (+ this test process) on ONE GPU: 2 hardware queues each keeps every rank's
        # queues mapped at once (their spinning peer waits need all ranks running together)
        os.environ['GPU_MAX_HW_QUEUES'] = '2'
    import faulthandler
    import sys
    faulthandler.dump_traceback_later(float(os.environ.get('DQN_TEST_STACK_DUMP_S', '90')), exit=False)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _worker_xgmi(rank, world, port, wire, concurrent, errq):
    try:
        _setup(rank, world, port)
        from dist_dqn_amd.parallel import init_distributed
        from dist_dqn_amd.parallel.xgmi import XgmiAllReduce
        ctx = init_distributed(None, device='cuda')
        cap = 1 << 20
        x = XgmiAllReduce(ctx, cap, wire)
        assert x.self_test(cap), x.self_test_log
        g = torch.Generator(device='cuda').manual_seed(1234)
        for n in (8 * world, 4096 + 8 * world, cap):
            for call in range(3):                          # both staging parities, then again
                parts = [torch.randn(n, generator=g, device='cuda') for _ in range(world)]
                t = parts[rank].clone()
                x.allreduce(t, channel=call % 2)
                torch.cuda.synchronize()
                if wire == 'bf16':
                    ref = sum(p.bfloat16().float() for p in parts).bfloat16().float()
                else:
                    ref = parts[0].clone()
                    for p in parts[1:]:
                        ref += p                            # same rank order as the kernel
                assert torch.equal(t, ref), (n, call, (t - ref).abs().max())
        assert x.check(), x.error_info()
        # both channels back to back on one stream (the learner's one linear graph) or, concurrent,
        # on two streams at once
        a = torch.full((cap,), float(rank + 1), device='cuda')
        b = torch.full((4096,), float(10 * (rank + 1)), device='cuda')
        side = torch.cuda.Stream() if concurrent else torch.cuda.current_stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            x.allreduce(a, channel=0)
        x.allreduce(b, channel=1)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        s = world * (world + 1) / 2
        assert x.check(), x.error_info()
        assert bool((a == s).all()) and bool((b == 10 * s).all())
        # every rank done with x (a peer's phase C may still read my staging after my kernel
        # returned) before any rank frees its buffers and maps new ones
        torch.cuda.synchronize()
        dist.barrier()
        x.close()
        dist.barrier()
        # the gather channel (low-rank DP exchange): two segments, every rank's bytes in rank order,
        # both staging parities, concurrently with an all-reduce on another stream
        y = XgmiAllReduce(ctx, cap, wire, gather_bytes=96 * 1024)
        assert y.self_test(4096) and y.self_test_gather()
        for call in range(3):
            n0, n1 = 64 * 1024, 32 * 1024 - 16 * call
            n1 -= n1 % 16
            segs = [torch.randint(0, 256, (world, n), dtype=torch.uint8, generator=torch.Generator().manual_seed(
                call * 10 + n), device='cpu').cuda() for n in (n0, n1)]
            src = [segs[0][rank].clone(), segs[1][rank].clone()]
            out = [torch.zeros(world * n0, dtype=torch.uint8, device='cuda'),
                   torch.zeros(world * n1, dtype=torch.uint8, device='cuda')]
            t = torch.full((4096,), float(rank + 1), device='cuda')
            side = torch.cuda.Stream() if concurrent else torch.cuda.current_stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                y.allreduce(t, channel=0)
            y.allgather2([src[0].data_ptr(), src[1].data_ptr()], [out[0].data_ptr(), out[1].data_ptr()], [n0, n1])
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            assert y.check(), y.error_info()
            assert torch.equal(out[0], segs[0].reshape(-1)) and torch.equal(out[1], segs[1].reshape(-1)), call
            assert bool((t == world * (world + 1) / 2).all())
        # several disjoint pieces of one buffer summed as ONE vector (the low-rank step's remainder)
        flat = torch.full((8192,), float(rank + 1), device='cuda')
        pieces = [(64, 192), (1024, 1088), (4096, 8192)]
        y.allreduce_ranges(flat, pieces, channel=1)
        torch.cuda.synchronize()
        mask = torch.zeros(8192, dtype=torch.bool, device='cuda')
        for lo, hi in pieces:
            mask[lo:hi] = True
        s = world * (world + 1) / 2
        assert y.check(), y.error_info()
        assert bool((flat[mask] == s).all()) and bool((flat[~mask] == rank + 1).all())
        y.close()
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001 - report to the parent
        import traceback
        errq.put('rank %d: %s\n%s' % (rank, e, traceback.format_exc()))
        raise


# The production schedule is one stream per rank (the DP step is ONE linear HIP graph): strict at
# every world size. The two-stream sub-case (both channels / the gather beside an all-reduce at
# the same time) stops at W = 4 here: with every rank on ONE GPU, 8 processes x 2 streams of
# spinning peer-wait kernels ask for more user-mode hardware queues than the scheduler keeps
# mapped at once, so a kernel can wait on a peer whose queue is not resident (round-3 runs: 5
# timed-out W = 8 runs in 6). On the 8-GPU node each rank owns its GPU's queues.
@pytest.mark.parametrize('world,wire,concurrent', [(2, 'fp32', True), (2, 'bf16', True), (4, 'fp32', True),
                                                   (8, 'fp32', False), (8, 'bf16', False)])
def test_xgmi_allreduce_ranks_one_gpu(world, wire, concurrent):
    """The peer-to-peer kernel (IPC-mapped fine-grained buffers) against exact sums, at the
    world sizes the node runs (the WC = 2 / 4 / 8 instantiations, the 8-peer gather)."""
    _gpu_free_parent(world)
    _run_ranks(_worker_xgmi, (wire, concurrent), world=world, timeout=100 + 20 * world)


RAINBOW_DP = '--distributional --noisy --dueling --double_dqn --optimizer=adam --lr=0.0000625'


def _worker(rank, world, port, network, extra, errq):
    try:
        _setup(rank, world, port)
        from dist_dqn_amd.config import preset
        from dist_dqn_amd.learner import Learner
        from dist_dqn_amd.models.network import Network
        from dist_dqn_amd.parallel import broadcast_state, check_state_equal, init_distributed
        from dist_dqn_amd.replay import DeviceReplay
        outs = {}
        ctx = None
        for overlap in (1, 0):
            # a different init seed per rank: broadcast_state must carry EVERYTHING (params, target,
            # slots, noise stream) and every rank must rebuild its packed / premixed fragments
            cfg = preset(network, 'Pong-v0', '--dtype=bf16 --seed=%d --backend=hip --replay_memory_capacity=2048 '
                         '--overlap_allreduce=%d %s' % (3 + rank, overlap, extra))
            if ctx is None:
                ctx = init_distributed(cfg, device='cuda')
                assert ctx.world_size == world and ctx.backend == 'gloo' and ctx.device.index == 0
            net = Network.create_network(cfg, (84, 84, 4), 6, num_replicas=world, device=ctx.device)
            broadcast_state(ctx, net)
            init = net.online.flat.clone()
            rep = DeviceReplay(2048, (84, 84), 4, device=ctx.device, seed=rank)
            rep.fill_synthetic(2048, 6, seed=rank)          # different data per rank
            ln = Learner(net, rep, cfg, ctx)
            assert ln.use_graph
            for _ in range(6):                              # 2 eager warm-up steps, then graphs
                ln.step()
            torch.cuda.synchronize()
            assert torch.isfinite(ln.loss).all()
            if ln.reducer.xgmi is not None:
                ln.reducer.check()                          # a timed-out peer wait raises here
            eq = check_state_equal(ctx, net)
            assert all(eq.values()), 'replicas diverged (overlap=%d): %s' % (overlap, eq)
            assert int(net.global_step) == 6
            xgmi = '--allreduce=xgmi' in extra
            assert ln.reducer.mode == ('xgmi' if xgmi else 'rccl')
            if xgmi:
                assert len(ln._graphs) == 1, 'xgmi DP step should be one graph'
                ln.reducer.check()
                # the fc weight gradient travels as all-gathered factors (overlap=1, Nature,
                # no noisy layers, fp32 wire); overlap=0 is the full all-reduce it is compared with
                lowrank = bool(overlap) and network == 'nature' and 'bf16' not in extra
                assert (ln._lowrank is not None) == lowrank, (overlap, extra)
                # ... and then feeds the fused optimizer (fc dW from the W*B gathered rows), whose launch
                # also runs the conv / output-layer weight gradients and sums them over the ranks
                # itself (in-launch exchange: no all-reduce launch)
                assert ln._defer_fc == lowrank, (overlap, extra)
                assert ln._dp_fused == lowrank and ln._defer_wgrad == lowrank, (overlap, extra)
            elif overlap and network == 'nature':
                assert ln._graphs is not None and ln._graphs[2] is not None, 'no split graph captured'
            outs[overlap] = net.online.flat.clone()
        # same data, same init: the overlapped schedule reduces the same sums. The conv weight
        # gradients accumulate M-chunk partials with fp32 atomics, so their last bits depend on
        # arrival order. SGD / RMSProp keep such differences at rounding level; Adam turns a
        # near-zero gradient into a ~lr * sign(g) step, and the flipped elements then perturb
        # every later gradient, so there the two runs' parameter updates must agree in direction
        # and size per tensor instead of elementwise.
        if cfg.optimizer == 'adam':
            lay = net.layout
            for name in lay.names:
                o, n = lay.offsets[name], lay.numel(name)
                d1, d0 = outs[1][o:o + n] - init[o:o + n], outs[0][o:o + n] - init[o:o + n]
                cos = float(torch.nn.functional.cosine_similarity(d1, d0, dim=0))
                ratio = float(d1.norm() / (d0.norm() + 1e-30))
                assert cos > 0.99 and abs(ratio - 1) < 0.02, (name, cos, ratio)
        else:
            torch.testing.assert_close(outs[1], outs[0], rtol=1e-4, atol=1e-6)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001 - report to the parent
        import traceback
        errq.put('rank %d: %s\n%s' % (rank, e, traceback.format_exc()))
        raise


@pytest.mark.parametrize('world,network,extra', [
    (2, 'nature', '--allreduce=rccl'),
    (2, 'nature', '--allreduce=rccl --dueling --double_dqn --loss=huber'),
    (2, 'atari', '--allreduce=rccl'),
    (2, 'nature', '--allreduce=rccl --allreduce_dtype=bf16'),
    (2, 'nature', '--allreduce=xgmi'),
    (2, 'nature', '--allreduce=xgmi --dueling --double_dqn --loss=huber'),
    (2, 'atari', '--allreduce=xgmi'),
    (2, 'nature', '--allreduce=xgmi --allreduce_dtype=bf16'),
    # Rainbow minus PER: noisy sigma gradients are derived in the optimizer from the all-reduced
    # mu gradients under the rank-shared noise stream, so replicas stay bit-identical
    (2, 'nature', '--allreduce=rccl ' + RAINBOW_DP),
    (2, 'nature', '--allreduce=xgmi ' + RAINBOW_DP),
    # the node's world sizes: W*B = 128 / 256 all-gathered rows into the fused optimizer, the
    # WC = 4 / 8 all-reduce of the remaining ranges
    (4, 'nature', '--allreduce=xgmi'),
    (4, 'nature', '--allreduce=rccl'),
    (4, 'nature', '--allreduce=xgmi --dueling --double_dqn --loss=huber'),
    (8, 'nature', '--allreduce=xgmi'),
    (8, 'nature', '--allreduce=xgmi ' + RAINBOW_DP)])
def test_dp_learner_ranks_one_gpu(world, network, extra):
    """(--allreduce=rccl means the process group's collective: gloo in this rehearsal.)"""
    _gpu_free_parent(world)
    _run_ranks(_worker, (network, extra), world=world, timeout=100 + 25 * world)


@pytest.mark.parametrize('world', [2, 4])
def test_bench_ranks_replicas_equal(tmp_path, world):
    """bench.py under torchrun (2 / 4 ranks on one GPU over gloo): the JSON line reports the
    end-of-run replica check, the world size, the transport and the graph-steps probe."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DQN_DIST_BACKEND='gloo', OMP_NUM_THREADS='4')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=%d' % world,
           '--master-addr=127.0.0.1', '--master-port=%d' % _free_port(), os.path.join(root, 'bench.py'),
           '--gpus', str(world), '--steps', '20', '--warmup', '5', '--replay', '20000']
    out = subprocess.run(cmd, env=env, cwd=root, capture_output=True, text=True, timeout=200)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith('{')][-1]
    d = json.loads(line)
    assert d['n_gpus'] == world and d['config']['world_size'] == world
    assert d['graph_steps'] in (1, 10) and d['ms_per_step_g1'] > 0        # 10: the largest G <= 16 dividing 20
    assert d['config']['replicas_equal'] is True and d['config']['replicas_diverged'] == []
    assert d['config']['dist_backend'] == 'gloo'


def test_bench_gpus_flag_launches_ranks_itself(tmp_path):
    """`python bench.py --gpus 2` with NO launcher: bench.py relaunches itself under
    torch.distributed.run as 2 ranks (here sharing cuda:0 over gloo), rank 0's line reports
    n_gpus == 2, both ranks' device ids, bit-equal replicas and a timed region of G-step
    launches only."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK')}
    env.update(DQN_DIST_BACKEND='gloo', OMP_NUM_THREADS='4')
    cmd = [sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--steps', '20', '--warmup', '5',
           '--replay', '20000']
    out = subprocess.run(cmd, env=env, cwd=root, capture_output=True, text=True, timeout=200)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out.stdout                  # rank 0 only
    d = json.loads(lines[0])
    assert d['n_gpus'] == 2 and d['config']['world_size'] == 2
    assert d['config']['replicas_equal'] is True
    assert len(d['config']['rank_devices']) == 2 and d['config']['ranks_share_gpu'] is True
    tl = d['config']['timed_launches']
    assert tl['graph_launches_of_G'] * d['graph_steps'] + tl['single_step_graphs'] == 20


def _worker_rccl_one_rank(rank, world, port, errq):
    """A real RCCL (backend 'nccl') process group of ONE rank: RCCL refuses two ranks on one GPU, so
    this is the only RCCL run a one-GPU box allows. The context is forced 'enabled' so the data
    parallel code takes its RCCL branches: first contact, the bucketed fp32 and bf16-wire all-reduce,
    the async range all-reduce of the overlapped backward, the state broadcast, and learner steps
    whose gradient all-reduce is RCCL's."""
    try:
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK='0', WORLD_SIZE='1', LOCAL_RANK='0')
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from dist_dqn_amd.config import preset
        from dist_dqn_amd.learner import Learner
        from dist_dqn_amd.models.network import Network
        from dist_dqn_amd.parallel.dist import DistContext, first_contact
        from dist_dqn_amd.parallel.dp import GradAllReducer, broadcast_state
        from dist_dqn_amd.replay import DeviceReplay
        dev = torch.device('cuda', 0)
        torch.cuda.set_device(dev)
        dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
        assert dist.get_backend() == 'nccl'
        ctrl = dist.new_group(backend='gloo')

        class _Ctx(DistContext):
            enabled = property(lambda self: True)
        ctx = _Ctx(0, 1, 0, dev, 'nccl', ctrl)
        first_contact(ctx)                                  # checked 4-element RCCL all-reduce
        g = torch.Generator(device=dev).manual_seed(1)
        flat = torch.randn(3 * 1024 * 1024 + 12, device=dev, generator=g)
        ref = flat.clone()
        red = GradAllReducer(ctx, flat, bucket_mb=2.0, mode='rccl')
        assert red.xgmi is None and len(red.buckets) > 1, red.buckets
        red.allreduce()                                     # one rank: the sum is the value itself
        assert torch.equal(flat, ref)
        h = [red.allreduce_range_async(0, 1000), red.allreduce_range_async(1000, flat.numel())]
        red.wait_all(h)
        assert torch.equal(flat, ref)
        red16 = GradAllReducer(ctx, flat, bucket_mb=2.0, mode='rccl', wire_dtype='bf16')
        red16.allreduce()                                   # bf16 wire: rounded once
        assert torch.equal(flat, ref.to(torch.bfloat16).float())
        cfg = preset('nature', 'Pong-v0', '--dtype=bf16 --seed=3 --backend=hip --replay_memory_capacity=4096 '
                     '--allreduce=rccl')
        net = Network.create_network(cfg, (84, 84, 4), 6, device=dev)
        broadcast_state(ctx, net)
        rep = DeviceReplay(4096, (84, 84), 4, device=dev, seed=3)
        rep.fill_synthetic(4096, 6, seed=3)
        ln = Learner(net, rep, cfg, ctx)
        assert ln.reducer.xgmi is None and ln.reducer.ctx is ctx
        p0 = net.online.flat.clone()
        for _ in range(4):
            ln.step()
        torch.cuda.synchronize()
        assert int(net.global_step) == 4 and torch.isfinite(net.online.flat).all()
        assert not torch.equal(p0, net.online.flat)
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001
        import traceback
        errq.put('rank %d: %s\n%s' % (rank, e, traceback.format_exc()))
        raise


def test_rccl_one_rank_data_parallel_paths():
    _run_ranks(_worker_rccl_one_rank, (), world=1, timeout=150)


def _worker_dp_fused_one_rank(rank, world, port, extra, errq):
    """The fused DP step at W = 1 (``init_distributed(force_dp=True)``: a one-rank RCCL group, every DP
    code path on): the fc gather side duty, the weight-gradient tiles inside the update launch and
    its in-launch exchange, all in ONE graph per G steps. Against a one-process learner from the
    same init on the same minibatches: the same parameters (to the conv wgrad's fp32-atomic order)."""
    try:
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        for k in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'DQN_DIST_BACKEND'):
            os.environ.pop(k, None)
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from dist_dqn_amd.config import preset
        from dist_dqn_amd.learner import Learner
        from dist_dqn_amd.models.network import Network
        from dist_dqn_amd.parallel import init_distributed
        from dist_dqn_amd.replay import DeviceReplay
        cfg = preset('nature', 'Pong-v0', '--dtype=bf16 --seed=3 --backend=hip --replay_memory_capacity=4096 '
                     '--allreduce=xgmi ' + extra)
        ctx = init_distributed(cfg, device='cuda', force_dp=True)
        assert ctx.enabled and ctx.world_size == 1 and ctx.backend == 'nccl'
        outs, losses = [], []
        for dp in (True, False):
            net = Network.create_network(cfg, (84, 84, 4), 6, device=ctx.device)
            rep = DeviceReplay(4096, (84, 84), 4, device=ctx.device, seed=3,
                               prioritized=cfg.prioritized_replay)
            rep.fill_synthetic(4096, 6, seed=3)
            ln = Learner(net, rep, cfg, ctx if dp else None)
            if dp:
                assert ln._dp_fused and ln._defer_wgrad and ln.reducer.mode == 'xgmi', \
                    (ln._dp_fused, ln._defer_wgrad, ln.reducer.mode)
                assert ln.reducer.xgmi.dpx is not None
            else:
                assert not ln.ctx.enabled and ln._defer_wgrad
            for _ in range(3):                          # eager warm-up, then the one-step graph
                ln.step()
            assert ln.can_step_many()
            ln.step_many(4)                             # a 4-step graph (the bench's shape)
            torch.cuda.synchronize()
            assert int(net.global_step) == 7
            if dp:
                ln.reducer.check()
                ln._device_checks()
            losses.append(float(ln.loss))
            outs.append(net.online.flat.clone())
        assert all(torch.isfinite(o).all() for o in outs)
        if cfg.optimizer == 'adam':
            assert float(torch.nn.functional.cosine_similarity(outs[0], outs[1], dim=0)) > 0.9999
        else:
            torch.testing.assert_close(outs[0], outs[1], rtol=1e-4, atol=1e-6)
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001
        import traceback
        errq.put('rank %d: %s\n%s' % (rank, e, traceback.format_exc()))
        raise


@pytest.mark.parametrize('extra', ['', '--dueling --double_dqn --loss=huber', RAINBOW_DP])
def test_dp_fused_step_one_rank_matches_one_process(extra):
    _run_ranks(_worker_dp_fused_one_rank, (extra,), world=1, timeout=200)


def test_bench_gpus_more_than_the_node_has_fails_loudly():
    """`--gpus 8` on a one-GPU box (no gloo rehearsal asked for) must refuse with a message and a
    non-zero exit, never run one rank and print n_gpus 1."""
    import subprocess
    import sys
    if torch.cuda.device_count() >= 8:
        pytest.skip('node has 8 GPUs')
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'DQN_DIST_BACKEND')}
    out = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', '8', '--steps', '4'],
                         env=env, cwd=root, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    assert 'needs 8 GPUs' in out.stderr


def _worker_async_ps(rank, world, port, transport, errq, pipeline=0):
    """--async_ps on the GPU: rank 0 is the parameter server (HIP fused optimizer on its HBM
    copy), ranks 1..world-1 run the HIP Nature-CNN learner against it (push gradient, pull
    parameters + int64 global_step). Three ranks share cuda:0 over gloo (p2p: the messages;
    xgmi: setup only -- the data moves by one-sided peer access, the control words through a
    host-shared page)."""
    try:
        _setup(rank, world, port)
        from dist_dqn_amd.config import preset
        from dist_dqn_amd.learner import Learner
        from dist_dqn_amd.models.network import Network
        from dist_dqn_amd.parallel import broadcast_state, init_distributed
        from dist_dqn_amd.parallel.async_ps import make_ps_client, make_ps_server
        from dist_dqn_amd.replay import DeviceReplay
        cfg = preset('nature', 'Pong-v0', '--dtype=bf16 --seed=5 --backend=hip --replay_memory_capacity=2048 '
                     '--async_ps --target_update_freq=3 --ps_transport=%s --ps_pipeline=%d' % (transport, pipeline))
        ctx = init_distributed(cfg, device='cuda')
        net = Network.create_network(cfg, (84, 84, 4), 6, num_replicas=world, device=ctx.device)
        assert net.executor.name.startswith('hip'), net.executor.name
        broadcast_state(ctx, net)
        init = net.online.flat.clone()
        steps = 5
        if rank == 0:
            srv = make_ps_server(ctx, net, cfg)
            assert getattr(srv, 'transport', 'p2p') == transport, srv
            n = srv.serve()
            torch.cuda.synchronize()
            assert n == steps * (world - 1) and srv.per_worker == {w: steps for w in range(1, world)}
            assert int(net.global_step) == n
            assert torch.isfinite(net.online.flat).all()
            assert not torch.equal(net.online.flat, init), 'the PS applied no update'
            ps_params = net.online.flat.clone()
            if hasattr(srv, 'close'):
                dist.barrier()                            # (workers verified their last pull)
                srv.close()
        else:
            rep = DeviceReplay(2048, (84, 84), 4, device=ctx.device, seed=rank)
            rep.fill_synthetic(2048, 6, seed=rank)
            ps = make_ps_client(ctx, net.online.flat, cfg, network=net)
            assert getattr(ps, 'transport', 'p2p') == transport, ps
            ps.pull(net.online.flat, net.global_step)
            net.refresh_packed()
            ln = Learner(net, rep, cfg, ctx, ps_client=ps)
            seen = []
            for _ in range(steps):
                ln.step()
                seen.append(int(net.global_step))
            torch.cuda.synchronize()
            assert torch.isfinite(ln.loss).all()
            assert ps.pushes == steps
            if pipeline:
                # each step takes the answer to the PREVIOUS push: the first one is the initial
                # parameters (step 0), and the PS step still only moves forward
                assert seen == sorted(seen) and seen[0] == 0, seen
                assert all(0 <= s < steps * (world - 1) for s in seen), seen
            else:
                assert seen == sorted(seen) and len(set(seen)) == steps, seen    # the PS step only moves forward
                assert all(1 <= s <= steps * (world - 1) for s in seen), seen
            if transport == 'xgmi':
                assert ps.check()
                ps.close()
                dist.barrier()
            else:
                ps.close()
        if transport != 'xgmi':
            dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001 - report to the parent
        import traceback
        errq.put('rank %d: %s\n%s' % (rank, e, traceback.format_exc()))
        raise


@pytest.mark.parametrize('transport', ['p2p', 'xgmi'])
def test_async_ps_hip_learners_one_gpu(transport):
    _run_ranks(_worker_async_ps, (transport,), world=3, timeout=150)


def _worker_async_ps_pipelined(rank, world, port, errq):
    _worker_async_ps(rank, world, port, 'xgmi', errq, pipeline=1)


def test_async_ps_pipelined_hip_learners_one_gpu():
    """--ps_pipeline=1 (xgmi): every push is still applied exactly once in arrival order, the server's
    step counts them all, and the workers' parameters lag one answer behind."""
    _run_ranks(_worker_async_ps_pipelined, (), world=3, timeout=150)


class _QuiesceProbeSupervisor:
    """Stands in for the RunSupervisor on the PS rank: every new update count triggers a
    'checkpoint' that reads the PS state inside the checkpoint manager's quiesce hook and checks
    that nothing moves while it is held (parameters, every optimizer slot, global_step)."""

    def __init__(self, net):
        import types
        self.net = net
        self.reads = []
        self.ckpt = types.SimpleNamespace(quiesce=None)

    def on_train_step(self, u):
        import time
        q = self.ckpt.quiesce
        assert q is not None, 'native serve did not install the quiesce hook'
        if len(self.reads) >= 6:
            return
        with q():
            net = self.net
            g0 = int(net.global_step)
            p0 = net.online.flat.clone()
            s0 = [s.clone() for s in net.optimizer.slots]
            torch.cuda.synchronize()
            time.sleep(0.005)                        # workers keep pushing meanwhile
            torch.cuda.synchronize()
            moved = (int(net.global_step) != g0 or not torch.equal(p0, net.online.flat)
                     or any(not torch.equal(a, b) for a, b in zip(s0, net.optimizer.slots)))
            self.reads.append((g0, moved))

    def should_stop(self):
        return False


def _worker_async_ps_quiesce(rank, world, port, errq):
    """Native xgmi PS serve with periodic 'checkpoints': the server thread pauses (drains its stream)
    around each snapshot, so a save reads ONE update's parameters, slots and global_step."""
    try:
        _setup(rank, world, port)
        from dist_dqn_amd.config import preset
        from dist_dqn_amd.learner import Learner
        from dist_dqn_amd.models.network import Network
        from dist_dqn_amd.parallel import broadcast_state, init_distributed
        from dist_dqn_amd.parallel.async_ps import make_ps_client, make_ps_server
        from dist_dqn_amd.replay import DeviceReplay
        cfg = preset('nature', 'Pong-v0', '--dtype=bf16 --seed=5 --backend=hip --replay_memory_capacity=2048 '
                     '--async_ps --ps_transport=xgmi')
        ctx = init_distributed(cfg, device='cuda')
        net = Network.create_network(cfg, (84, 84, 4), 6, num_replicas=world, device=ctx.device)
        broadcast_state(ctx, net)
        steps = 40
        if rank == 0:
            srv = make_ps_server(ctx, net, cfg)
            sup = _QuiesceProbeSupervisor(net)
            n = srv.serve(supervisor=sup)
            assert n == steps * (world - 1)
            assert sup.reads and not any(m for _, m in sup.reads), sup.reads
            assert srv.pauses >= len(sup.reads), (srv.pauses, len(sup.reads))
            assert sup.ckpt.quiesce is None                     # removed when serving ends
            dist.barrier()
            srv.close()
        else:
            rep = DeviceReplay(2048, (84, 84), 4, device=ctx.device, seed=rank)
            rep.fill_synthetic(2048, 6, seed=rank)
            ps = make_ps_client(ctx, net.online.flat, cfg, network=net)
            ps.pull(net.online.flat, net.global_step)
            net.refresh_packed()
            ln = Learner(net, rep, cfg, ctx, ps_client=ps)
            for _ in range(steps):
                ln.step()
            torch.cuda.synchronize()
            assert ps.check()
            ps.close()
            dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001 - report to the parent
        import traceback
        errq.put('rank %d: %s\n%s' % (rank, e, traceback.format_exc()))
        raise


def test_async_ps_native_serve_quiesces_for_checkpoints():
    _run_ranks(_worker_async_ps_quiesce, (), world=3, timeout=150)


def _worker_ps_stall(rank, world, port, errq):
    """The server answers 2 pushes, then stops answering (a stalled / dead PS): the worker's pull
    times out on the device (2 s) and the learner's next device check raises instead of training
    on un-pulled parameters."""
    try:
        _setup(rank, world, port)
        from dist_dqn_amd.config import preset
        from dist_dqn_amd.learner import Learner
        from dist_dqn_amd.models.network import Network
        from dist_dqn_amd.parallel import broadcast_state, init_distributed
        from dist_dqn_amd.parallel.async_ps import make_ps_client, make_ps_server
        from dist_dqn_amd.replay import DeviceReplay
        cfg = preset('nature', 'Pong-v0', '--dtype=bf16 --seed=5 --backend=hip --replay_memory_capacity=2048 '
                     '--async_ps --ps_transport=xgmi --ps_timeout_s=2 --allreduce_check_steps=1 --hip_graph=0')
        ctx = init_distributed(cfg, device='cuda')
        net = Network.create_network(cfg, (84, 84, 4), 6, num_replicas=world, device=ctx.device)
        broadcast_state(ctx, net)
        if rank == 0:
            srv = make_ps_server(ctx, net, cfg)
            assert srv.serve(max_updates=2) == 2
            dist.barrier()                                  # (the worker saw its error)
            srv.close()
        else:
            rep = DeviceReplay(2048, (84, 84), 4, device=ctx.device, seed=rank)
            rep.fill_synthetic(2048, 6, seed=rank)
            ps = make_ps_client(ctx, net.online.flat, cfg, network=net)
            ps.pull(net.online.flat, net.global_step)
            net.refresh_packed()
            ln = Learner(net, rep, cfg, ctx, ps_client=ps)
            raised = None
            for _ in range(5):
                try:
                    ln.step()
                except RuntimeError as e:
                    raised = str(e)
                    break
            assert raised is not None and 'parameter server' in raised, raised
            assert ln.train_steps <= 4, ln.train_steps
            torch.cuda.synchronize()
            ps.close()
            dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001 - report to the parent
        import traceback
        errq.put('rank %d: %s\n%s' % (rank, e, traceback.format_exc()))
        raise


def test_async_ps_worker_raises_when_the_server_stalls():
    _run_ranks(_worker_ps_stall, (), world=2, timeout=150)


# ------------------------------------------------------- DP == the big-batch step
# The reference's synchronous mode aggregates the replicas' gradients into ONE update
# (SyncReplicasOptimizer, /root/reference/src/network.py:186-202): W ranks with B samples each
# must take the step one process takes on the W*B samples. Every rank (and the one process) holds
# the same replay and the same init; rank r's minibatch is transitions [OFF + rB, OFF + (r+1)B),
# the one process's [OFF, OFF + WB). The one-process step at W*B > 32 runs other kernels than the
# ranks' (per-layer weight gradients instead of the grouped / FcFuse ones), so a shared error in
# the DP arithmetic (1/W scale, the W*B-row fc factors) cannot cancel out.
BIG_OFF = 100


def _fixed_batch(rep, idx):
    """A slot minibatch of the given transitions (what the sampler kernel writes for them)."""
    i = idx.long()
    st = rep.state_idx.index_select(0, i).to(torch.int32)
    nx = torch.cat([st[:, 1:], rep.next_idx.index_select(0, i).view(-1, 1).to(torch.int32)], 1).contiguous()
    return {'idx': idx.to(torch.int32), 'actions': rep.actions.index_select(0, i).to(torch.int32).contiguous(),
            'rewards': rep.rewards.index_select(0, i).contiguous(), 'dones': rep.dones.index_select(0, i).contiguous(),
            'gammas': rep.gammas.index_select(0, i).contiguous(), 'state_slots': st.contiguous(), 'next_slots': nx,
            'frames': rep.frames}


def _big_batch_net(cfg_str, B, W, rank, device):
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    cfg = preset('nature', 'Pong-v0', cfg_str % B)
    net = Network.create_network(cfg, (84, 84, 4), 6, num_replicas=W, device=device)
    g = torch.Generator(device=device).manual_seed(11)
    net.online.flat.normal_(0.0, 0.03, generator=g)      # larger-than-init weights: signal in every layer
    net.target.flat.copy_(net.online.flat)
    net.refresh_packed()
    rep = DeviceReplay(4096, (84, 84), 4, device=device, seed=0)
    rep.fill_synthetic(4096, 6, seed=0)                 # identical on every rank
    idx = torch.arange(BIG_OFF + rank * B, BIG_OFF + (rank + 1) * B, device=device, dtype=torch.int32)
    batch = _fixed_batch(rep, idx)
    rep.sample_slots = lambda *a, **k: dict(batch)      # every step trains on these transitions
    return cfg, net, rep


BIG_CFG = ('--dtype=bf16 --seed=0 --backend=hip --minibatch_size=%d --replay_memory_capacity=4096 '
           '--optimizer=sgd --lr=0.05 --reg_param=0 --fuse_sampling=0 --hip_graph=0 ')


def _worker_bigbatch(rank, world, port, extra, out, errq):
    try:
        _setup(rank, world, port)
        from dist_dqn_amd.learner import Learner
        from dist_dqn_amd.parallel import check_state_equal, init_distributed
        ctx = init_distributed(None, device='cuda')
        cfg, net, rep = _big_batch_net(BIG_CFG + extra, 32, world, rank, ctx.device)
        ln = Learner(net, rep, cfg, ctx)
        w0 = net.online.flat.clone()
        ln.step()
        torch.cuda.synchronize()
        if ln.reducer.xgmi is not None:
            ln.reducer.check()
        eq = check_state_equal(ctx, net)
        assert all(eq.values()), eq
        lowrank = '--lowrank_dense=0' not in extra and '--allreduce=xgmi' in extra
        assert (ln._lowrank is not None) == lowrank, (extra, ln._lowrank)
        if rank == 0:
            torch.save({'w0': w0.cpu(), 'w1': net.online.flat.cpu(), 'step': int(net.global_step)}, out)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001 - report to the parent
        import traceback
        errq.put('rank %d: %s\n%s' % (rank, e, traceback.format_exc()))
        raise


def _worker_bigbatch_ref(rank, world, port, extra, W, out, errq):
    """The single-process W*B reference step, in a child too: the test process itself never
    opens a GPU context here (see _gpu_free_parent)."""
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from dist_dqn_amd.learner import Learner
        dev = torch.device('cuda', 0)
        cfg, net, rep = _big_batch_net(BIG_CFG + extra, 32 * W, 1, 0, dev)
        w0 = net.online.flat.clone()
        ln = Learner(net, rep, cfg)
        ln.step()
        torch.cuda.synchronize()
        torch.save({'w0': w0.cpu(), 'w1': net.online.flat.cpu(), 'step': int(net.global_step),
                    'names': list(net.layout.names),
                    'spans': [(net.layout.offsets[n], net.layout.numel(n)) for n in net.layout.names]}, out)
    except BaseException as e:  # noqa: BLE001 - report to the parent
        import traceback
        errq.put('reference: %s\n%s' % (e, traceback.format_exc()))
        raise


def _gpu_free_parent(world):
    """8 ranks on ONE GPU need the test process itself to hold no GPU context: with it they are
    9 GPU processes, and round 4's diagnostics showed the resulting starvation -- the W=8 self-test
    of the second big-batch case (after the first case's reference had opened a context here)
    timed out with every wait pointing at one never-run block (ranks 1, 2: reduce-scatter, peer 0
    block 6, flag 2 of 3; the others all-gather on peer 1), while the same case passed first in a
    fresh process. The full GPU suite opens a context in earlier modules: skip there, run the
    module on its own (scripts/gpu_dp.sh) for the 8-rank evidence."""
    if world >= 8 and torch.cuda.is_initialized():
        pytest.skip('8 ranks + a GPU-holding test process on one device: run this module in a fresh '
                    'process (scripts/gpu_dp.sh)')


@pytest.mark.parametrize('world,extra', [
    (2, '--allreduce=xgmi'),                           # low-rank fc exchange into the fused optimizer
    (2, '--allreduce=xgmi --lowrank_dense=0'),         # full all-reduce of the flat gradient
    (2, '--allreduce=rccl'),                           # the process-group collective (gloo here)
    (2, '--allreduce=xgmi --dueling'),
    (2, '--allreduce=xgmi --lowrank_dense=0 --dueling'),
    (4, '--allreduce=xgmi'),
    (4, '--allreduce=xgmi --lowrank_dense=0 --dueling'),
    (8, '--allreduce=xgmi'),
    (8, '--allreduce=xgmi --dueling')])
def test_dp_step_equals_big_batch_step(tmp_path, world, extra):
    _gpu_free_parent(world)
    out = str(tmp_path / 'dp.pt')
    _run_ranks(_worker_bigbatch, (extra, out), world=world, timeout=100 + 25 * world)
    dp = torch.load(out, weights_only=True)
    ex = ' '.join(a for a in extra.split() if not a.startswith('--allreduce') and not a.startswith('--lowrank'))
    ref = str(tmp_path / 'big.pt')
    _run_ranks(_worker_bigbatch_ref, (ex, world, ref), world=1, timeout=200)
    bb = torch.load(ref, weights_only=True)
    assert torch.equal(bb['w0'], dp['w0']), 'different initial parameters'
    assert bb['step'] == dp['step'] == 1
    big = bb['w1'] - dp['w0']
    small = dp['w1'] - dp['w0']

    class _Lay:
        names = bb['names']
        offsets = {n: o for n, (o, _) in zip(bb['names'], bb['spans'])}

        def numel(self, n):
            return dict(zip(bb['names'], bb['spans']))[n][1]
    lay = _Lay()
    for name in lay.names:
        o, n = lay.offsets[name], lay.numel(name)
        a, b = small[o:o + n].double(), big[o:o + n].double()
        if float(b.norm()) == 0.0:
            assert float(a.norm()) == 0.0, name
            continue
        cos = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
        ratio = float(a.norm() / b.norm())
        assert cos > 0.999 and abs(ratio - 1.0) < 0.01, (name, cos, ratio)
