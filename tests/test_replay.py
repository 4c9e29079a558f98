"""Replay memories: reference API (/root/reference/src/replay_memory.py:18-53),
the HBM replay's frame-dedup layout, n-step returns and the PER sum-tree (CPU paths)."""
import random

import numpy as np
import pytest
import torch

from dist_dqn_amd.frame_buffer import FrameBuffer
from dist_dqn_amd.ops import kernels
from dist_dqn_amd.replay import DeviceReplay, DeviceSumTree, NStepAccumulator, ReplayMemory


def test_host_replay_reference_api():
    r = ReplayMemory(5, rng=random.Random(0))
    assert r.size() == 0 and r.capacity() == 5
    assert r.get_minibatch(1) == (None, None)
    for i in range(8):
        r.add(np.full(2, i), i % 2, float(i), np.full(2, i + 1), i % 3 == 0)
    assert r.size() == 5                                   # deque(maxlen) semantics
    nt, t = r.get_minibatch(4)
    nt, t = list(nt), list(t)
    assert len(nt) + len(t) == 4 and all(not x[4] for x in nt) and all(x[4] for x in t)
    assert len({int(x[0][0]) for x in nt + t}) == 4        # without replacement
    assert all(int(x[0][0]) >= 3 for x in nt + t)          # oldest evicted
    assert [s for s in ReplayMemory.get_states([(1, 0, 0, 2, False)])] == [1]
    assert [s for s in ReplayMemory.get_next_states([(1, 0, 0, 2, False)])] == [2]
    b = r.sample_arrays(3)
    assert b['states'].shape == (3, 2) and b['dones'].dtype == np.float32
    assert list(b['dones']) == sorted(b['dones'])          # non-terminal first


def test_device_replay_frame_dedup_matches_frame_buffer():
    """The HBM replay rebuilds exactly the reference FrameBuffer stacks (first frame duplicated)."""
    rng = np.random.default_rng(0)
    rep = DeviceReplay(50, (6, 8), 4, device='cpu', stage_size=7)
    fb = FrameBuffer(4)
    expected = []
    for ep in range(3):
        fb.clear()
        f0 = rng.integers(0, 256, (6, 8), dtype=np.uint8)
        fb.append(f0)
        rep.begin_episode(f0)
        s = fb.get_state()
        for t in range(5):
            f = rng.integers(0, 256, (6, 8), dtype=np.uint8)
            fb.append(f)
            ns = fb.get_state()
            done = t == 4
            rep.add_step(t % 3, float(t), f, done, gamma_n=0.9)
            expected.append((s, t % 3, float(t), ns, done))
            s = ns
    rep.flush()
    assert rep.size() == 15
    idx = torch.arange(15, dtype=torch.int32)
    batch = rep.gather(idx)
    for i, (s, a, r, ns, d) in enumerate(expected):
        np.testing.assert_array_equal(batch['states'][i].numpy(), s)
        np.testing.assert_array_equal(batch['next_states'][i].numpy(), ns)
        assert int(batch['actions'][i]) == a and float(batch['rewards'][i]) == r and float(batch['dones'][i]) == d
    assert rep.nbytes() > 0


def test_device_replay_vector_mode_and_sampling():
    rep = DeviceReplay(10, (3,), 1, device='cpu', stage_size=4)
    rep.begin_episode(np.zeros(3))
    for i in range(12):
        rep.add_step(i % 2, 1.0, np.full(3, i + 1.0), False)
    rep.flush()
    assert rep.size() == 10
    out = rep.sample_indices(8)
    assert len(set(out.tolist())) == 8 and int(out.max()) < 10
    b = rep.gather(out)
    assert b['states'].shape == (8, 3)
    assert torch.allclose(b['next_states'] - b['states'], torch.ones(8, 3))


def test_fill_synthetic_consistency():
    rep = DeviceReplay(200, (84, 84), 4, device='cpu')
    rep.fill_synthetic(200, 6, episode_len=50)
    si, ni = rep.state_idx[:200], rep.next_idx[:200]
    # within an episode the next state's newest frame is the following state's newest frame
    assert torch.equal(si[1:50, 3], ni[0:49])
    assert len(set(si[0].tolist())) == 1                  # episode start: duplicated reset frame
    assert float(rep.dones[49]) == 1.0


def test_nstep_accumulator():
    acc = NStepAccumulator(3, 0.5)
    out = []
    for t in range(5):
        out += acc.push('s%d' % t, t, 1.0, 's%d' % (t + 1), t == 4)
    assert [o[0] for o in out] == ['s0', 's1', 's2', 's3', 's4']
    s, a, R, ns, d, g = out[0]
    assert R == pytest.approx(1 + 0.5 + 0.25) and ns == 's3' and not d and g == pytest.approx(0.125)
    assert out[-1][3] == 's5' and out[-1][4] and out[-1][2] == pytest.approx(1.0)


def test_sumtree_cpu_proportional_and_weights():
    C = 64
    t = DeviceSumTree(C, 'cpu')
    t.set_max_priority(torch.arange(C, dtype=torch.int32))
    assert t.total() == pytest.approx(C)
    pr = torch.zeros(C)
    pr[5] = 9.0
    t.update(torch.arange(C, dtype=torch.int32), pr, alpha=1.0, eps=1e-4)
    assert t.total() == pytest.approx(9.0, rel=1e-3) and float(t.max_p) == pytest.approx(9.0, rel=1e-3)
    rng = torch.tensor([1, 0], dtype=torch.int64)
    idx = torch.zeros(16, dtype=torch.int32)
    w = torch.zeros(16)
    t.sample(rng, torch.tensor([C], dtype=torch.int32), torch.tensor([0.5]), idx, w)
    assert (idx == 5).all()
    # max-normalised IS weight of the dominant leaf: (p_min / p)^beta
    assert torch.allclose(w, torch.full((16,), (1e-4 / 9.0001) ** 0.5), rtol=1e-3)
    # duplicate indices in one update: last writer wins on the leaf, parents stay consistent
    t.update(torch.tensor([1, 1], dtype=torch.int32), torch.tensor([2.0, 4.0]), 1.0, 0.0)
    assert float(t.sum[1]) == pytest.approx(float(t.sum[t.P:t.P + C].sum()))


def test_prioritized_device_replay_cpu():
    rep = DeviceReplay(32, (4,), 1, device='cpu', prioritized=True, stage_size=8)
    rep.begin_episode(np.zeros(4))
    for i in range(32):
        rep.add_step(0, 0.0, np.full(4, i), False)
    rep.flush()
    idx, w = rep.sample_prioritized(8, torch.tensor([0.4]))
    assert idx.shape == (8,) and float(w.max()) <= 1.0 + 1e-6
    rep.update_priorities(idx, torch.rand(8))
    assert rep.tree.total() > 0
