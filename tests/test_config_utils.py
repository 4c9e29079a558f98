"""Config parity with /root/reference/src/main.py:12-98 and helper semantics
(/root/reference/src/utils.py, frame_buffer.py, stats.py)."""
import numpy as np
import pytest

from dist_dqn_amd import utils
from dist_dqn_amd.config import build_parser, defaults, dqn_params_for_env, preset
from dist_dqn_amd.frame_buffer import FrameBuffer
from dist_dqn_amd.stats import Stats

REFERENCE_DEFAULTS = {
    'log_level': 'INFO', 'env': 'CartPole-v0', 'monitor': False, 'monitor_path': '/tmp/gym',
    'disable_video': False, 'network': 'simple', 'lr': 0.001, 'reg_param': 0.001, 'optimizer': 'sgd',
    'momentum': 0.9, 'rmsprop_decay': 0.95, 'num_episodes': 10000, 'max_steps_per_episode': 1000,
    'minibatch_size': 30, 'frames_per_state': 1, 'resize_width': 0, 'resize_height': 0,
    'reward_discount': 0.9, 'replay_memory_capacity': 10000, 'replay_start_size': 0,
    'init_random_action_prob': 0.9, 'min_random_action_prob': 0.1, 'random_action_explore_steps': 10000,
    'update_freq': 1, 'target_update_freq': 10000, 'ps_hosts': '', 'worker_hosts': 'localhost:0',
    'job': 'worker', 'task_id': 0, 'gpu_id': 0, 'sync': False, 'disable_cpu_param_pinning': False,
    'disable_target_replication': False, 'logdir': '/tmp/train_logs', 'summary_freq': 100,
}


def test_reference_flag_defaults():
    c = defaults()
    for k, v in REFERENCE_DEFAULTS.items():
        assert getattr(c, k) == v, k


def test_reference_choices():
    p = build_parser()
    acts = {a.dest: a for a in p._actions}
    assert set(acts['optimizer'].choices) >= {'adadelta', 'adagrad', 'adam', 'ftrl', 'sgd', 'momentum', 'rmsprop'}
    assert {'simple', 'cnn'} <= set(acts['network'].choices)
    assert set(acts['job'].choices) == {'ps', 'worker'}


def test_presets_match_reference_scripts():
    a = preset('atari', 'Pong-v0')
    assert (a.env, a.network, a.optimizer, a.lr, a.minibatch_size) == ('Pong-v0', 'cnn', 'rmsprop', 0.00025, 32)
    assert (a.frames_per_state, a.update_freq, a.replay_start_size, a.resize_width, a.resize_height) == (4, 4, 10000, 84, 84)
    assert (a.replay_memory_capacity, a.target_update_freq, a.reward_discount) == (1000000, 10000, 0.99)
    c = preset('control', 'CartPole-v0')
    assert (c.network, c.optimizer, c.minibatch_size, c.max_steps_per_episode, c.target_update_freq) == \
        ('simple', 'adam', 100, 200, 3000)
    assert dqn_params_for_env('control', 'X').startswith('--env=X ')
    with pytest.raises(ValueError):
        dqn_params_for_env('bogus', 'X')


def test_partition_order_and_laziness():
    nt, t = utils.partition(lambda x: x[4], [(0, 0, 0, 0, False), (1, 0, 0, 0, True), (2, 0, 0, 0, False)])
    assert [x[0] for x in nt] == [0, 2]
    assert [x[0] for x in t] == [1]


def test_decay_and_one_hot():
    assert utils.decay_per_step(1.0, 0.1, 0) == 0.0
    assert utils.decay_per_step(1.0, 0.1, 9) == pytest.approx(0.1)
    assert utils.decay(1.0, 0.5, 0.1) == 0.5
    np.testing.assert_array_equal(utils.one_hot(2, 4), [0, 0, 1, 0])
    with pytest.raises(AssertionError):
        utils.one_hot(4, 4)


def test_frame_buffer_semantics():
    fb = FrameBuffer(3)
    assert fb.get_state() is None
    fb.append(np.full((2, 2), 1))
    s = fb.get_state()
    assert s.shape == (2, 2, 3) and (s == 1).all()       # first frame duplicated k times
    fb.append(np.full((2, 2), 2))
    assert list(fb.get_state()[0, 0]) == [1, 1, 2]         # HWC stack, newest last
    fb1 = FrameBuffer(1, preprocessor=lambda x: x * 10)
    fb1.append(np.ones(3))
    assert (fb1.get_state() == 10).all() and fb1.get_state().shape == (3,)
    with pytest.raises(RuntimeError):
        FrameBuffer(0)


def test_stats():
    s = Stats()
    for r in range(150):
        s.log_episode(r, 1)
    assert s.last_100_mean_reward() == pytest.approx(np.mean(range(50, 150)))
    assert s.episodes == 150 and s.total_steps == 150


def test_resize_image_properties():
    img = np.zeros((210, 160, 3), np.uint8)
    img[..., 0] = 255
    out = utils.resize_image(img, 84, 84)
    assert out.shape == (84, 84) and out.dtype == np.uint8
    assert (out == ((4899 * 255 + (1 << 13)) >> 14)).all()   # constant image stays constant
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (210, 160, 3), dtype=np.uint8)
    out = utils.resize_image(img, 84, 84)
    gray = utils.rgb_to_gray(img).astype(float)
    assert abs(out.astype(float).mean() - gray.mean()) < 3.0


def test_resize_native_matches_oracle():
    from dist_dqn_amd.ops import _ext, preprocess
    if not _ext.available():
        pytest.skip('extension not built')
    rng = np.random.default_rng(1)
    for shape, (w, h) in [((210, 160, 3), (84, 84)), ((100, 90, 3), (84, 60)), ((50, 50, 3), (84, 84))]:
        img = rng.integers(0, 256, shape, dtype=np.uint8)
        np.testing.assert_array_equal(preprocess.resize_image(img, w, h), utils.resize_image(img, w, h))
