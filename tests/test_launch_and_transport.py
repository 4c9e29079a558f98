"""CPU checks of the multi-GPU launch contract and the all-reduce transport decision.

* ``bench.py --gpus N`` launches N ranks itself and refuses loudly when the node cannot host
  them (the reference's multi-GPU launcher starts one worker per GPU,
  `/root/reference/scripts/dqn_multi_gpu.sh:31-36,84-105`);
* the first data-backend collective runs right after the process group forms
  (`parallel/dist.py:first_contact`; the reference's cluster bootstrap is
  `/root/reference/src/main.py:174-186`);
* `GradAllReducer._setup_xgmi` picks xgmi or RCCL for every failure / timing outcome, with a
  mocked transport (no GPU).
"""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _clean_env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT', 'DQN_DIST_BACKEND')}
    env.update(kw)
    return env


def test_timed_split_prefers_a_dividing_graph_size():
    import bench
    assert bench.timed_split(20, 16) == (10, 2, 0)
    assert bench.timed_split(2000, 16) == (16, 125, 0)
    assert bench.timed_split(500, 16) == (10, 50, 0)
    assert bench.timed_split(17, 16) == (16, 1, 1)         # prime: reported mix
    assert bench.timed_split(3, 16) == (16, 0, 3)
    assert bench.timed_split(64, 1) == (1, 0, 64)


def test_bench_gpus_beyond_the_node_refuses_without_running():
    """No GPU here: --gpus 8 must exit non-zero with a message and print no JSON line."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '8', '--steps', '4'],
                         env=_clean_env(), cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert out.returncode == 2, out.stderr
    assert 'needs 8 GPUs' in out.stderr
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith('{')]


def test_bench_world_size_must_match_gpus_flag():
    """Under a launcher, WORLD_SIZE != --gpus is an error (not a silently different run)."""
    env = _clean_env(RANK='0', WORLD_SIZE='2', LOCAL_RANK='0')
    out = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '3', '--steps', '4'],
                         env=env, cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert out.returncode == 2
    assert 'launcher started 2 rank' in out.stderr


def _worker_first_contact(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        from dist_dqn_amd.parallel import init_distributed
        ctx = init_distributed(None, device='cpu')      # runs first_contact inside
        assert ctx.world_size == world and ctx.backend == 'gloo'
        assert ctx.device_ids() == ['cpu'] * world
        assert ctx.ranks_share_gpu() is False           # CPU ranks: no GPU to share
        got = ctx.ctrl_all_gather_object(rank * 10)
        assert got == [r * 10 for r in range(world)]
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put('rank %d: %r' % (rank, e))


def test_first_contact_and_device_ids_world3():
    ctx = mp.get_context('spawn')
    q = ctx.SimpleQueue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_first_contact, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    errs = []
    while not q.empty():
        errs.append(q.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in ps)


# ------------------------------------------------------------------ transport decision (mocked)
class _FakeCtx:
    rank, world_size, enabled, is_chief = 0, 2, True, True


class _FakeXgmi:
    """Stands in for parallel/xgmi.XgmiAllReduce: behaviour set per test through class attributes."""
    raise_in_ctor = False
    self_test_ok = True
    gather_ok = True
    closed = 0

    def __init__(self, ctx, n, wire, gather_bytes=0, exchange_slots=0):
        if _FakeXgmi.raise_in_ctor:
            raise RuntimeError('ipc mapping refused')

    def self_test(self, n):
        return _FakeXgmi.self_test_ok

    def self_test_gather(self):
        return _FakeXgmi.gather_ok

    def allreduce(self, t, ch):
        pass

    def close(self):
        _FakeXgmi.closed += 1


def _reducer(monkeypatch, agree=True, t_x=10.0, t_r=20.0, gather_bytes=0):
    from dist_dqn_amd.parallel import dp, xgmi
    monkeypatch.setattr(xgmi, 'XgmiAllReduce', _FakeXgmi)
    single = type('C', (), {'enabled': False, 'world_size': 1, 'rank': 0})()
    r = dp.GradAllReducer(single, torch.zeros(1024), mode='rccl')
    r.ctx = _FakeCtx()
    r.gather_bytes = gather_bytes
    times = iter([t_x, t_r])
    monkeypatch.setattr(r, '_cross_check', lambda x: agree)
    monkeypatch.setattr(r, '_time', lambda fn: next(times))
    return r


@pytest.fixture(autouse=False)
def fake_reset():
    _FakeXgmi.raise_in_ctor, _FakeXgmi.self_test_ok, _FakeXgmi.gather_ok, _FakeXgmi.closed = False, True, True, 0
    yield


def test_auto_keeps_faster_xgmi(monkeypatch, fake_reset):
    r = _reducer(monkeypatch, t_x=10.0, t_r=20.0)
    assert isinstance(r._setup_xgmi('auto'), _FakeXgmi)
    assert r.timings == {'xgmi_us': 10.0, 'rccl_us': 20.0}


def test_auto_picks_rccl_when_xgmi_is_slower_without_gather(monkeypatch, fake_reset):
    r = _reducer(monkeypatch, t_x=30.0, t_r=20.0)
    assert r._setup_xgmi('auto') is None and _FakeXgmi.closed == 1


def test_auto_keeps_slower_xgmi_with_a_working_gather(monkeypatch, fake_reset):
    r = _reducer(monkeypatch, t_x=30.0, t_r=20.0, gather_bytes=4096)
    assert isinstance(r._setup_xgmi('auto'), _FakeXgmi) and r.can_gather


def test_auto_falls_back_to_rccl_on_setup_error(monkeypatch, fake_reset):
    _FakeXgmi.raise_in_ctor = True
    r = _reducer(monkeypatch)
    assert r._setup_xgmi('auto') is None
    with pytest.raises(RuntimeError, match='ipc mapping refused'):
        r._setup_xgmi('xgmi')


def test_auto_falls_back_to_rccl_on_self_test_failure(monkeypatch, fake_reset):
    _FakeXgmi.self_test_ok = False
    r = _reducer(monkeypatch)
    assert r._setup_xgmi('auto') is None and _FakeXgmi.closed == 1
    with pytest.raises(RuntimeError, match='self-test'):
        r._setup_xgmi('xgmi')


def test_auto_falls_back_to_rccl_on_disagreement(monkeypatch, fake_reset):
    r = _reducer(monkeypatch, agree=False)
    assert r._setup_xgmi('auto') is None and _FakeXgmi.closed == 1
    r2 = _reducer(monkeypatch, agree=False)
    with pytest.raises(RuntimeError, match='disagrees'):
        r2._setup_xgmi('xgmi')


def test_failed_gather_self_test_keeps_allreduce_but_no_gather(monkeypatch, fake_reset):
    _FakeXgmi.gather_ok = False
    r = _reducer(monkeypatch, t_x=10.0, t_r=20.0, gather_bytes=4096)
    assert isinstance(r._setup_xgmi('auto'), _FakeXgmi) and not r.can_gather


# ------------------------------------------------------------------ async PS low-rank push plan
class _StubEx:
    FLAT, HH, noisy, dist = 3136, 512, False, False

    def __init__(self, HH=512):
        self.HH = HH

    def can_defer_fc(self, B, sigma_grads=False):
        return B <= 32

    def update_and_pack(self, *a, **k):
        pass


@pytest.mark.parametrize('dueling', [False, True])
def test_ps_lowrank_plan_pushes_everything_but_the_fc_weights(dueling):
    """--ps_lowrank: the pushed pieces cover the flat buffer outside the fc weight tensors exactly,
    and the fc factor rows (X [B][3136], dL/dh [B][HH], 16-bit) fit where the first fc weight
    gradient would be."""
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.parallel.async_ps import ps_lowrank_plan
    cfg = preset('nature', 'Pong-v0', '--device=cpu --backend=torch --async_ps' + (' --dueling' if dueling else ''))
    net = Network.create_network(cfg, (84, 84, 4), 6)
    net.executor = _StubEx(1024 if dueling else 512)
    plan = ps_lowrank_plan(net, cfg)
    lay = net.layout
    fcw = [(lay.offsets[n], lay.offsets[n] + lay.numel(n)) for n in lay.names if n.endswith('fcl/w')]
    covered = sorted(plan['keep'] + fcw)
    assert covered[0][0] == 0 and covered[-1][1] == lay.total
    assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))          # no gap, no overlap
    B = cfg.minibatch_size
    assert plan['x_off'] == 4 * fcw[0][0] and plan['xbytes'] == B * 3136 * 2
    assert plan['dh_off'] == plan['x_off'] + plan['xbytes'] and plan['dbytes'] == B * (1024 if dueling else 512) * 2
    assert plan['dh_off'] + plan['dbytes'] <= 4 * fcw[0][1]
    pushed = sum(4 * (b - a) for a, b in plan['keep']) + plan['xbytes'] + plan['dbytes']
    assert pushed < 4 * lay.total / 8                       # > 8x fewer bytes than the full gradient
    # not applicable: flag off, noisy heads, minibatch beyond the fused path
    assert ps_lowrank_plan(net, cfg.replace(ps_lowrank=0)) is None
    net.executor.noisy = True
    assert ps_lowrank_plan(net, cfg) is None
    net.executor.noisy = False
    assert ps_lowrank_plan(net, cfg.replace(minibatch_size=64)) is None


def _worker_agree_plan(rank, world, port, differ, q):
    try:
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        from dist_dqn_amd.parallel import init_distributed
        from dist_dqn_amd.parallel.async_ps import _agree_lowrank
        ctx = init_distributed(None, device='cpu')
        plan = {'B': 32, 'keep': [(0, 64), (128, 256)], 'x_off': 256, 'dh_off': 512, 'xbytes': 64, 'dbytes': 32}
        if differ and rank == 1:
            plan = None                              # e.g. a worker built without the network
        try:
            _agree_lowrank(ctx, plan)
            raised = False
        except ValueError:
            raised = True
        assert raised == bool(differ), (rank, raised)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put('rank %d: %r' % (rank, e))


@pytest.mark.parametrize('differ', [False, True])
def test_async_ps_lowrank_plan_agreement(differ):
    """The xgmi PS server and its workers must agree on the low-rank push plan: identical plans pass,
    a worker without one fails on EVERY rank (ValueError, no fallback) instead of corrupting the
    parameters (the server would read 16-bit factor rows as an fp32 gradient)."""
    ctx = mp.get_context('spawn')
    q = ctx.SimpleQueue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_agree_plan, args=(r, 2, port, differ, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    errs = []
    while not q.empty():
        errs.append(q.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in ps)


def test_kernel_tuning_parse():
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.ops.tuning import KernelTuning
    assert KernelTuning.parse('') == KernelTuning()
    t = KernelTuning.parse('wg_conv_chunks=2, dep_at=300,tfact=1')
    assert (t.wg_conv_chunks, t.dep_at, t.fold_two_per_cu, t.tfact) == (2, 300, 1, 1)
    auto = KernelTuning()                           # -1: the measured best per net / build
    assert (auto.conv_chunks('nature', 'bf16'), auto.conv_chunks('nature', 'fp32'), auto.conv_chunks('cnn', 'bf16'),
            auto.conv_chunks('cnn', 'fp32')) == (3, 4, 2, 4)
    assert t.conv_chunks('cnn', 'fp32') == 2
    assert (auto.cnn_parts('fp32'), auto.cnn_parts('bf16'), KernelTuning.parse('cnn_bwd_parts=1').cnn_parts('fp32')) \
        == (4, 4, 1)
    with pytest.raises(ValueError):
        KernelTuning.parse('cnn_bwd_parts=3')  # (1, 2 or 4)
    with pytest.raises(ValueError):
        KernelTuning.parse('wg_mix=1')              # removed knob: refused, not ignored
    cfg = preset('nature', 'Pong-v0', '--kernel_tuning=dep_at=0')
    assert KernelTuning.parse(cfg.kernel_tuning).dep_at == 0
