"""Ape-X on the GPU: the native ingest thread (csrc/ingest_server.cpp) against the Python
staging path, and the actor pool end to end with it.

* The same actor records pushed through SPSC rings land in an HBM replay either through the
  native thread (ingest + pinned staging + H2D copies on its own stream, events against the
  learner stream, PER insert at max priority) or through DeviceReplay.begin_episode /
  add_step(_nstep) + flush: the device replay columns, frame ring, size and sum-tree must match
  exactly.
* A short Ape-X run (image actors, PER, n-step) with the native ingest and the CPU reservation:
  the learner steps, frames and episodes are counted and the replay's host cursors are handed
  back consistent with the device.

Reference: the worker's own actor loop feeding a Python deque (`/root/reference/src/
dqn_agent.py:72-106`, `src/replay_memory.py:22-23`).
"""
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)


def _records(n, H, W, seed):
    from dist_dqn_amd.actors.apex import HEADER
    rng = np.random.default_rng(seed)
    rb = HEADER.itemsize + H * W
    recs = np.zeros((n, rb), dtype=np.uint8)
    hdr = recs[:, :HEADER.itemsize].view(HEADER).reshape(-1)
    recs[:, HEADER.itemsize:] = rng.integers(0, 256, (n, H * W), dtype=np.uint8)
    ep_left = 0
    for i in range(n):
        if ep_left == 0:
            hdr[i] = (0, 0, 0, 0, 0.0, 0.0)
            ep_left = int(rng.integers(3, 15))
            continue
        ep_left -= 1
        done = int(ep_left == 0 and rng.random() < 0.7)
        ep_left = 0 if done else ep_left
        hdr[i] = (1, done, 0, int(rng.integers(0, 6)), float(rng.normal()), 5.0 if done else np.nan)
    return recs, hdr


@pytest.mark.parametrize('nstep,per', [(1, False), (3, True)])
def test_native_ingest_thread_matches_python_path(nstep, per):
    from dist_dqn_amd.actors.apex import HEADER
    from dist_dqn_amd.native import load
    from dist_dqn_amd.ops import _ext
    from dist_dqn_amd.replay import DeviceReplay
    from dist_dqn_amd.replay.nstep import NStepAccumulator
    ext = _ext.load(required=True)
    L = load()
    H = W = 84
    k, gamma, actors, n = 4, 0.9, 3, 700
    rb = HEADER.itemsize + H * W
    cap = 1024
    data = [_records(n, H, W, seed=a) for a in range(actors)]
    # Python path: actor by actor, record by record (same order as one ingest pass per actor)
    ref = DeviceReplay(4096, (H, W), k, device=DEV, prioritized=per, stage_size=256)
    for a in range(actors):
        recs, hdr = data[a]
        acc = NStepAccumulator(nstep, gamma)
        for i in range(n):
            h, obs = hdr[i], recs[i, HEADER.itemsize:].reshape(H, W)
            if h['kind'] == 0:
                ref.begin_episode(obs.copy())
                acc.reset()
            elif nstep > 1:
                ref.add_step_nstep(acc, int(h['action']), float(h['reward']), obs.copy(), bool(h['done']))
            else:
                ref.add_step(int(h['action']), float(h['reward']), obs.copy(), bool(h['done']), gamma_n=gamma)
        ref.flush()
    torch.cuda.synchronize()
    # native thread: all records pushed before start, so each actor's ring drains in one pass
    rings = [np.zeros(L.ring_bytes(cap, rb), dtype=np.uint8) for _ in range(actors)]
    for a in range(actors):
        L.ring_init(rings[a], cap, rb)
        assert L.ring_push(rings[a], data[a][0], n) == n
    nat = DeviceReplay(4096, (H, W), k, device=DEV, prioritized=per, stage_size=256)
    words = nat.ingest_state_size(k, nstep)
    states = np.zeros((actors, words), dtype=np.int32)
    addrs = np.array([r.ctypes.data for r in rings], dtype=np.int64)
    dev = [nat.frames.data_ptr(), nat.state_idx.data_ptr(), nat.next_idx.data_ptr(), nat.actions.data_ptr(),
           nat.rewards.data_ptr(), nat.dones.data_ptr(), nat.gammas.data_ptr(), nat.size_dev.data_ptr()]
    pr = [nat.tree.sum.data_ptr(), nat.tree.min.data_ptr(), nat.tree.max_p.data_ptr(), nat.tree.P] if per else [0] * 4
    # stage sets of 8192 transitions: one flush per pass, like the reference's per-actor flushes
    cfg = [k, nstep, H * W, nat.capacity, nat.num_frames, 8192, 3, 1 << 30, 1 << 40, 0, -1]
    srv = ext.IngestServer(int(addrs.ctypes.data), actors, int(states.ctypes.data), words, gamma, dev, pr,
                           [0, 0, 0], cfg, int(torch.cuda.current_stream().cuda_stream))
    srv.start()
    t0 = time.time()
    while srv.stats()[0] < actors * n and time.time() - t0 < 30:
        time.sleep(0.01)
    srv.stop()
    consumed, frames, eps, flushes, size, err = srv.stats()
    assert not err, err
    f, t, sz = srv.cursors()
    torch.cuda.synchronize()
    assert consumed == actors * n and size == sz == ref.size() > 0
    assert frames == sum(int((d[1]['kind'] == 1).sum()) for d in data)
    assert eps == sum(int(d[1]['done'].sum()) for d in data)
    rets = srv.pop_returns()
    assert len(rets) == eps and all(r == 5.0 for r in rets)
    assert int(nat.size_dev[0]) == sz and f == ref._f_next and t == ref._t_next
    m = ref.size()
    for name in ('state_idx', 'next_idx', 'actions', 'rewards', 'dones', 'gammas'):
        assert torch.equal(getattr(nat, name)[:m], getattr(ref, name)[:m]), name
    assert torch.equal(nat.frames[:f], ref.frames[:f])
    if per:
        assert torch.equal(nat.tree.sum, ref.tree.sum) and torch.equal(nat.tree.min, ref.tree.min)


def test_apex_native_ingest_end_to_end(tmp_path):
    from dist_dqn_amd.cli import run_worker
    from dist_dqn_amd.config import preset
    cfg = preset('apex', 'Pong-v0', '--device=cuda --dtype=bf16 --num_actors=6 --replay_memory_capacity=20000 '
                 '--replay_start_size=400 --max_train_steps=300 --checkpoint_secs=0 --seed=3 '
                 '--apex_reserve_cpus=3 --logdir=%s' % tmp_path)
    tr = run_worker(cfg)
    assert tr.learner.train_steps >= 300
    assert tr.pool.frames >= 400 and tr.pool.served > 0
    r = tr.replay
    assert r._size == int(r.size_dev[0]) >= 400          # host cursors handed back from the thread
    assert tr._ingest is None


def test_apex_trainer_native_paths():
    """Tiny Ape-X run (BASELINE config 4 shape): CPU actor processes, the native ingest thread into
    the HBM PER replay, the native inference server thread replaying captured inference graphs, and
    the multi-step learner graphs; with the Python drain path (--apex_native_ingest=0) too."""
    import tempfile
    from dist_dqn_amd.actors.apex import ApexActorPool, ApexTrainer
    from dist_dqn_amd.config import preset
    from dist_dqn_amd.learner import Learner
    from dist_dqn_amd.models.network import Network
    from dist_dqn_amd.replay import DeviceReplay
    dev = torch.device('cuda', 0)
    for native in (1, 0):
        cfg = preset('apex', 'Pong-v0', '--num_actors=3 --replay_memory_capacity=20000 --replay_start_size=500 '
                     '--apex_ring=256 --apex_native_ingest=%d --logdir=%s' % (native, tempfile.mkdtemp()))
        net = Network.create_network(cfg, (84, 84, 4), 6, device=dev)
        rep = DeviceReplay(cfg.replay_memory_capacity, (84, 84), 4, device=dev, num_actors=cfg.num_actors,
                           prioritized=True, alpha=cfg.per_alpha, seed=1)
        ln = Learner(net, rep, cfg)
        pool = ApexActorPool(cfg.env, cfg.num_actors, 4, (84, 84), 0, 6, 200, seed=1, ring_capacity=cfg.apex_ring,
                             n_step=cfg.n_step, gamma=cfg.reward_discount)
        tr = ApexTrainer(net, rep, ln, pool, cfg)
        tr.run(max_seconds=12.0, log_every=100.0)
        assert getattr(tr, '_server', 'gone') is None, 'native server not stopped'
        assert tr._ingest is None, 'native ingest not stopped'
        assert pool.served > 0 and tr.serve_calls > 0, 'no greedy action served'
        assert pool.frames > 500 and rep.size() > 500
        assert rep.size() == int(rep.size_dev[0])
        assert ln.train_steps > 100 and ln.train_steps % cfg.apex_graph_steps == 0
        assert torch.isfinite(net.online.flat).all() and torch.isfinite(ln.loss).all()
