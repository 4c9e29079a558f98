"""Ape-X acting path: the torch-free host runtime
(SPSC rings + inference mailboxes, also under ThreadSanitizer), the actor pool's
processes / shared memory lifecycle, and end-to-end Ape-X training on the CPU."""
import glob
import os
import shutil
import subprocess

import numpy as np
import pytest

from dist_dqn_amd.actors.apex import HEADER, ApexActorPool, apex_epsilons
from dist_dqn_amd.config import parse_args
from dist_dqn_amd.native import load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_ring_roundtrip_and_backpressure():
    L = load()
    rec = 24
    buf = np.zeros(L.ring_bytes(8, rec), dtype=np.uint8)
    L.ring_init(buf, 8, rec)
    recs = np.arange(10 * rec, dtype=np.uint8).reshape(10, rec)
    assert L.ring_push(buf, recs, 10) == 8            # full after capacity
    assert L.ring_size(buf) == 8
    out = np.zeros((10, rec), dtype=np.uint8)
    assert L.ring_pop(buf, out, 5) == 5
    np.testing.assert_array_equal(out[:5], recs[:5])
    assert L.ring_push(buf, recs[8:], 2) == 2          # wraps around
    assert L.ring_pop(buf, out, 10) == 5
    np.testing.assert_array_equal(out[:3], recs[5:8])
    np.testing.assert_array_equal(out[3:5], recs[8:10])


def test_mailbox_protocol_single_process():
    L = load()
    n, sb = 3, 8
    region = np.zeros(L.mbox_region_bytes(n, sb), dtype=np.uint8)
    L.mbox_init(region, n, sb)
    st = np.full(sb, 5, dtype=np.uint8)
    assert L.mbox_request(region, 1, st, timeout_us=1000) == -1      # nobody serves: timeout
    states = np.zeros((n, sb), dtype=np.uint8)
    ids, seq = np.zeros(n, np.int32), np.zeros(n, np.uint64)
    m = L.mbox_collect(region, n, sb, states, ids, seq, n)
    assert m == 1 and ids[0] == 1 and states[0, 0] == 5                # the posted request is pending
    L.mbox_respond(region, sb, ids, seq, np.array([4], np.int32), 1)
    assert L.mbox_collect(region, n, sb, states, ids, seq, n) == 0
    L.mbox_set_stop(region, 1)
    assert L.mbox_stopped(region) and L.mbox_request(region, 0, st) == -2


@pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++')
def test_host_runtime_under_thread_sanitizer(tmp_path):
    exe = str(tmp_path / 'host_stress')
    src = [os.path.join(ROOT, 'csrc', 'host', f) for f in ('tests/host_stress.cpp', 'spsc_ring.cpp', 'mailbox.cpp')]
    r = subprocess.run(['g++', '-std=c++17', '-O1', '-g', '-fsanitize=thread', '-o', exe] + src + ['-lpthread'],
                       capture_output=True, text=True)
    if r.returncode != 0 and 'tsan' in (r.stderr + r.stdout).lower():
        pytest.skip('ThreadSanitizer runtime unavailable')
    assert r.returncode == 0, r.stderr
    run = subprocess.run([exe], capture_output=True, text=True, timeout=600,
                         env=dict(os.environ, TSAN_OPTIONS='halt_on_error=1'))
    assert run.returncode == 0, run.stdout + run.stderr
    assert 'ThreadSanitizer' not in run.stderr, run.stderr
    assert 'ring errors 0, mailbox errors 0' in run.stdout


@pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++')
def test_ingest_service_under_thread_sanitizer(tmp_path):
    """The native ingest service's core (csrc/host/ingest_core.h, the code the GPU binding runs)
    with a fake device whose stream is a worker thread: actor threads -> rings -> rotating
    staging sets -> late "H2D" copies, stats polled during the run, stop + cursor hand-back."""
    exe = str(tmp_path / 'ingest_stress')
    src = [os.path.join(ROOT, 'csrc', 'host', f) for f in ('tests/ingest_stress.cpp', 'apex_ingest.cpp',
                                                           'spsc_ring.cpp')]
    r = subprocess.run(['g++', '-std=c++17', '-O1', '-g', '-fsanitize=thread', '-I' + os.path.join(ROOT, 'csrc'),
                        '-o', exe] + src + ['-lpthread'], capture_output=True, text=True)
    if r.returncode != 0 and 'tsan' in (r.stderr + r.stdout).lower():
        pytest.skip('ThreadSanitizer runtime unavailable')
    assert r.returncode == 0, r.stderr
    run = subprocess.run([exe], capture_output=True, text=True, timeout=600,
                         env=dict(os.environ, TSAN_OPTIONS='halt_on_error=1'))
    assert run.returncode == 0, run.stdout + run.stderr
    assert 'ThreadSanitizer' not in run.stderr, run.stderr
    assert 'errors 0' in run.stdout, run.stdout


@pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++')
def test_inference_service_under_thread_sanitizer(tmp_path):
    """The native inference service's core (csrc/host/infer_core.h, the code the GPU binding
    runs) on a fake device: actor threads' mailbox requests answered through late "H2D / graph /
    D2H" ops on a stream thread, stats polled during the run, stop."""
    exe = str(tmp_path / 'infer_stress')
    src = [os.path.join(ROOT, 'csrc', 'host', f) for f in ('tests/infer_stress.cpp', 'mailbox.cpp')]
    r = subprocess.run(['g++', '-std=c++17', '-O1', '-g', '-fsanitize=thread', '-I' + os.path.join(ROOT, 'csrc'),
                        '-o', exe] + src + ['-lpthread'], capture_output=True, text=True)
    if r.returncode != 0 and 'tsan' in (r.stderr + r.stdout).lower():
        pytest.skip('ThreadSanitizer runtime unavailable')
    assert r.returncode == 0, r.stderr
    run = subprocess.run([exe], capture_output=True, text=True, timeout=600,
                         env=dict(os.environ, TSAN_OPTIONS='halt_on_error=1'))
    assert run.returncode == 0, run.stdout + run.stderr
    assert 'ThreadSanitizer' not in run.stderr, run.stderr
    assert 'errors 0' in run.stdout, run.stdout


def test_apex_epsilons():
    e = apex_epsilons(8)
    assert e[0] == pytest.approx(0.4) and e[-1] == pytest.approx(0.4 ** 8)
    assert all(a > b for a, b in zip(e, e[1:]))


def test_pool_serves_and_drains_image_actors():
    """Synthetic Atari actors: C++ preprocessing, frame records, batched serving."""
    from dist_dqn_amd.replay import DeviceReplay
    pool = ApexActorPool('Pong-v0', 2, 4, (84, 84), 0, 6, max_steps_per_episode=50, seed=1,
                         ring_capacity=64, max_frames_per_actor=120)
    rep = DeviceReplay(1000, (84, 84), 4, device='cpu', num_actors=2)
    seen = []

    def q_fn(batch):
        assert batch.shape[1:] == (84, 84, 4) and batch.dtype == np.uint8
        seen.append(len(batch))
        return np.zeros(len(batch), dtype=np.int64)

    import time
    with pool:
        t0 = time.time()
        while pool.frames < 240 and time.time() - t0 < 60:
            pool.serve(q_fn)
            pool.drain(rep)
        paths = (pool.ring_path, pool.mbox_path)
    assert pool.frames == 240 and rep.size() == 240          # every env step became a transition
    assert pool.episodes >= 4 and pool.served > 0 and max(seen) >= 1
    assert not any(os.path.exists(p) for p in paths)         # shared memory removed
    # stacks are rebuilt from frame slots per actor: the s' of every transition that was
    # followed by another step of its episode is the s of that later transition
    st, nx = rep.state_idx.numpy()[:240], rep.next_idx.numpy()[:240]
    states = {tuple(r) for r in st}
    follow = [tuple(st[i, 1:]) + (nx[i],) in states for i in range(240)]
    assert sum(follow) >= 240 - 2 * 4        # all but the last step of each (cut) episode


@pytest.mark.parametrize('nstep,many', [(1, False), (3, False), (3, True)])
def test_native_ingest_matches_python_path(nstep, many):
    """csrc/host/apex_ingest.cpp (one call per actor ring, staging flushes included) stages
    exactly the transitions of DeviceReplay.begin_episode / add_step(_nstep) per record."""
    from dist_dqn_amd.replay import DeviceReplay
    from dist_dqn_amd.replay.nstep import NStepAccumulator
    L = load()
    H = W = 84
    k, gamma = 4, 0.9
    rb = HEADER.itemsize + H * W
    cap = 512
    ring = np.zeros(L.ring_bytes(cap, rb), dtype=np.uint8)
    L.ring_init(ring, cap, rb)
    rng = np.random.default_rng(0)
    recs = np.zeros((300, rb), dtype=np.uint8)
    hdr = recs[:, :HEADER.itemsize].view(HEADER).reshape(-1)
    recs[:, HEADER.itemsize:] = rng.integers(0, 256, (300, H * W), dtype=np.uint8)
    ep_left = 0
    for i in range(300):
        if ep_left == 0:
            hdr[i] = (0, 0, 0, 0, 0.0, 0.0)                 # reset record
            ep_left = int(rng.integers(3, 15))
            continue
        ep_left -= 1
        done = int(ep_left == 0 and rng.random() < 0.7)
        ep_left = 0 if done else ep_left
        hdr[i] = (1, done, 0, int(rng.integers(0, 6)), float(rng.normal()), 5.0 if done else np.nan)
    # the Python path
    ref = DeviceReplay(2000, (H, W), k, device='cpu', stage_size=64)
    acc = NStepAccumulator(nstep, gamma)
    for i in range(300):
        h, obs = hdr[i], recs[i, HEADER.itemsize:].reshape(H, W)
        if h['kind'] == 0:
            ref.begin_episode(obs.copy())
            acc.reset()
        elif nstep > 1:
            ref.add_step_nstep(acc, int(h['action']), float(h['reward']), obs.copy(), bool(h['done']))
        else:
            ref.add_step(int(h['action']), float(h['reward']), obs.copy(), bool(h['done']), gamma_n=gamma)
    ref.flush()
    # the native path, in two ring fills (state carried across calls), small staging sets
    nat = DeviceReplay(2000, (H, W), k, device='cpu', stage_size=64)
    state = np.zeros(nat.ingest_state_size(k, nstep), dtype=np.int32)
    got = [0, 0, 0]
    for lo, hi in ((0, 170), (170, 300)):
        assert L.ring_push(ring, recs[lo:hi], hi - lo) == hi - lo
        if many:                                            # the all-actors call (one ring here)
            m, frames, eps, rets = nat.ingest_rings(L, np.array([ring.ctypes.data], dtype=np.int64), state[None],
                                                    nstep, gamma)
        else:
            m, frames, eps, rets = nat.ingest_ring(L, ring, state, nstep, gamma)
        got = [got[0] + m, got[1] + frames, got[2] + eps]
        assert all(r == 5.0 for r in rets)
    nat.flush()
    assert got[0] == 300 and got[1] == int((hdr['kind'] == 1).sum()) and got[2] == int(hdr['done'].sum())
    assert nat.size() == ref.size() > 0
    n = ref.size()
    for name in ('state_idx', 'next_idx', 'actions', 'rewards', 'dones', 'gammas'):
        np.testing.assert_array_equal(getattr(nat, name).numpy()[:n], getattr(ref, name).numpy()[:n], err_msg=name)
    nf = ref._f_next
    assert nat._f_next == nf
    np.testing.assert_array_equal(nat.frames.numpy()[:nf], ref.frames.numpy()[:nf])


def test_apex_cartpole_end_to_end(tmp_path):
    from dist_dqn_amd.cli import run_worker
    cfg = parse_args(['--env=CartPole-v0', '--network=simple', '--optimizer=adam', '--lr=0.001',
                      '--minibatch_size=32', '--num_actors=3', '--replay_memory_capacity=5000',
                      '--max_train_steps=200', '--device=cpu', '--logdir=%s' % tmp_path, '--checkpoint_secs=0',
                      '--replay_start_size=200', '--n_step=3', '--actor_param_sync_freq=50'])
    tr = run_worker(cfg)
    assert tr.learner.train_steps == 200 and tr.pool.frames >= 200
    assert tr.pool.episodes > 0 and tr.pool.served > 0 and tr.pool.alive() == 0
    assert not glob.glob(tr.pool.ring_path + '*')
