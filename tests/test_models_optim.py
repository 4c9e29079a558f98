"""Model specs (/root/reference/src/network.py:258-424), TF-exact optimizers
 and TD losses (/root/reference/src/network.py:141-157)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from dist_dqn_amd.config import parse_args
from dist_dqn_amd.models import build_arch, ParamStore
from dist_dqn_amd.models import losses, torch_net
from dist_dqn_amd.optim import FlatOptimizer


def test_reference_cnn_param_count_and_shapes():
    arch = build_arch('cnn', (84, 84, 4), 6)
    assert arch.num_params() == 145318
    assert [c.conv_hw for c in arch.convs] == [(21, 21), (6, 6), (3, 3)]
    assert [c.out_hw for c in arch.convs] == [(11, 11), (3, 3), (2, 2)]
    assert arch.convs[0].pads() == (2, 2, 2, 2)
    names = [n for n, _, _ in arch.param_specs()]
    assert names == ['conv1/w', 'conv1/b', 'conv2/w', 'conv2/b', 'conv3/w', 'conv3/b', 'fcl/w', 'fcl/b',
                     'output/w', 'output/b']
    assert arch.reg_names() == ['fcl/w', 'output/w']
    with pytest.raises(RuntimeError):
        build_arch('cnn', (64, 64, 4), 6)                   # reference would silently mis-reshape


def test_simple_and_nature_shapes():
    s = build_arch('simple', (4,), 2)
    assert s.num_params() == 4 * 20 + 20 + 20 * 20 + 20 + 20 * 2 + 2
    assert s.reg_names() == ['hidden1/w', 'hidden2/w', 'output/w']
    n = build_arch('nature', (84, 84, 4), 6)
    assert [c.conv_hw for c in n.convs] == [(20, 20), (9, 9), (7, 7)]
    assert n.flat_features == 3136 and n.num_params() == 1687206
    d = build_arch('nature', (84, 84, 4), 6, dueling=True, distributional=True, num_atoms=51, noisy=True)
    assert d.dueling and d.distributional and d.head[-1].fout == 6 * 51 and d.value[-1].fout == 51


def test_flat_layout_alignment_and_reg_prefix():
    arch = build_arch('cnn', (84, 84, 4), 6)
    ps = ParamStore(arch).init_(0)
    lay = ps.layout
    assert all(o % 64 == 0 for o in lay.offsets.values())
    assert lay.offsets['fcl/w'] < lay.reg_end and lay.offsets['output/w'] < lay.reg_end
    assert lay.offsets['conv1/w'] >= lay.reg_end
    w = ps.tensors['conv1/w']
    assert w.abs().max() <= 0.02 + 1e-7 and float(w.std()) == pytest.approx(0.0088, rel=0.15)  # trunc-normal(0.01)
    assert (ps.tensors['conv1/b'] == 0).all()


def _tf_conv_same_ref(x, w, b, stride):
    """Independent SAME conv: explicit TF padding formula, NHWC/HWIO via unfold."""
    N, H, W, C = x.shape
    k = w.shape[0]
    oh, ow = -(-H // stride), -(-W // stride)
    ph = max((oh - 1) * stride + k - H, 0)
    pw = max((ow - 1) * stride + k - W, 0)
    xp = np.pad(x, ((0, 0), (ph // 2, ph - ph // 2), (pw // 2, pw - pw // 2), (0, 0)))
    out = np.zeros((N, oh, ow, w.shape[3]))
    for i in range(oh):
        for j in range(ow):
            patch = xp[:, i * stride:i * stride + k, j * stride:j * stride + k, :]
            out[:, i, j, :] = np.tensordot(patch, w, axes=([1, 2, 3], [0, 1, 2]))
    return out + b


def test_cnn_forward_matches_tf_semantics():
    arch = build_arch('cnn', (84, 84, 4), 6)
    ps = ParamStore(arch).init_(1)
    ps.flat.mul_(30.0)
    x = torch.randint(0, 256, (2, 84, 84, 4), dtype=torch.uint8)
    q = torch_net.forward(arch, ps.flat, ps.layout, x, 1.0 / 255)
    p = {k: v.double().numpy() for k, v in ps.tensors.items()}
    h = x.double().numpy() / 255
    for c in arch.convs:
        h = np.maximum(_tf_conv_same_ref(h, p[c.name + '/w'], p[c.name + '/b'], c.stride), 0)
        # 2x2/2 SAME max pool (pad bottom/right with -inf)
        N, H, W, C = h.shape
        oh, ow = -(-H // 2), -(-W // 2)
        hp = np.full((N, oh * 2, ow * 2, C), -np.inf)
        hp[:, :H, :W] = h
        h = hp.reshape(N, oh, 2, ow, 2, C).max(axis=(2, 4))
    h = h.reshape(2, -1)
    h = np.maximum(h @ p['fcl/w'] + p['fcl/b'], 0)
    ref = h @ p['output/w'] + p['output/b']
    # fp32 forward vs float64: errors scale with the output magnitude (~1e3), not per element
    np.testing.assert_allclose(q.double().numpy(), ref, rtol=1e-4, atol=1e-6 * np.abs(ref).max())


def test_grad_through_unflatten_is_flat():
    arch = build_arch('simple', (4,), 2)
    ps = ParamStore(arch).init_(0)
    flat = ps.flat.clone().requires_grad_(True)
    q = torch_net.forward(arch, flat, ps.layout, torch.randn(5, 4))
    q.sum().backward()
    assert flat.grad.shape == flat.shape and flat.grad.abs().sum() > 0


# ------------------------------------------------------------------ optimizers
def _np_tf_update(name, w, g, steps, lr=0.01, reg=0.0, reg_mask=None):
    w = w.astype(np.float64).copy()
    s0 = {'rmsprop': np.ones_like(w), 'adagrad': np.full_like(w, 0.1), 'ftrl': np.full_like(w, 0.1)}.get(name, np.zeros_like(w))
    s1 = np.zeros_like(w)
    b1p, b2p = 0.9, 0.999
    for t in range(steps):
        gg = g[t].astype(np.float64) + (reg * w * reg_mask if reg else 0)
        if name == 'sgd':
            w -= lr * gg
        elif name == 'momentum':
            s0 = 0.9 * s0 + gg
            w -= lr * s0
        elif name == 'rmsprop':
            s0 = 0.95 * s0 + 0.05 * gg * gg
            s1 = 0.0 * s1 + lr * gg / np.sqrt(s0 + 1e-10)
            w -= s1
        elif name == 'adam':
            lr_t = lr * math.sqrt(1 - b2p) / (1 - b1p)
            s0 = 0.9 * s0 + 0.1 * gg
            s1 = 0.999 * s1 + 0.001 * gg * gg
            w -= lr_t * s0 / (np.sqrt(s1) + 1e-8)
            b1p *= 0.9
            b2p *= 0.999
        elif name == 'adagrad':
            s0 += gg * gg
            w -= lr * gg / np.sqrt(s0)
        elif name == 'adadelta':
            s0 = 0.95 * s0 + 0.05 * gg * gg
            upd = np.sqrt(s1 + 1e-8) / np.sqrt(s0 + 1e-8) * gg
            s1 = 0.95 * s1 + 0.05 * upd * upd
            w -= lr * upd
        elif name == 'ftrl':
            na = s0 + gg * gg
            s1 = s1 + gg - (np.sqrt(na) - np.sqrt(s0)) / lr * w
            w = np.where(np.abs(s1) > 0, -s1 / (np.sqrt(na) / lr), 0.0)
            s0 = na
    return w


@pytest.mark.parametrize('name', ['sgd', 'momentum', 'rmsprop', 'adam', 'adagrad', 'adadelta', 'ftrl'])
def test_tf_exact_optimizers(name):
    arch = build_arch('simple', (4,), 2)
    ps = ParamStore(arch).init_(0)
    lay = ps.layout
    opt = FlatOptimizer(name, lay, 'cpu', lr=0.01, reg_param=0.01)
    rng = np.random.default_rng(0)
    g = rng.normal(size=(5, lay.total)).astype(np.float32)
    mask = np.zeros(lay.total)
    mask[:lay.reg_end] = 1
    w0 = ps.flat.numpy().copy()
    step = torch.zeros(1, dtype=torch.int64)
    for t in range(5):
        opt.step(ps.flat, torch.from_numpy(g[t]), 1.0, step)
    ref = _np_tf_update(name, w0, g, 5, lr=0.01, reg=0.01, reg_mask=mask)
    np.testing.assert_allclose(ps.flat.numpy(), ref, rtol=2e-4, atol=2e-6)
    assert int(step) == 5
    sd = opt.state_dict()
    assert all(k.split('/')[-1] in ('RMSProp', 'RMSProp_1', 'Adam', 'Adam_1', 'Momentum', 'Adagrad', 'Adadelta',
                                    'Adadelta_1', 'Ftrl', 'Ftrl_1') or k.endswith('_power') for k in sd)


# ---------------------------------------------------------------------- losses
def test_reference_td_target_and_mse():
    q = torch.tensor([[1.0, 2.0], [0.5, -1.0], [3.0, 0.0]], requires_grad=True)
    qn = torch.tensor([[0.2, 0.7], [1.0, 5.0], [9.0, 9.0]])
    a = torch.tensor([1, 0, 0])
    r = torch.tensor([1.0, 0.0, 2.0])
    d = torch.tensor([0.0, 0.0, 1.0])
    loss, td = losses.scalar_td_loss(q, a, r, d, qn, None, 0.9, 'mse')
    y = np.array([1 + 0.9 * 0.7, 0 + 0.9 * 5.0, 2.0])      # terminal -> y = r
    qa = np.array([2.0, 0.5, 3.0])
    assert float(loss) == pytest.approx(np.mean((qa - y) ** 2), rel=1e-6)
    np.testing.assert_allclose(td.numpy(), np.abs(qa - y), rtol=1e-6)
    loss.backward()
    g = q.grad.numpy()
    assert g[0, 1] == pytest.approx(2 * (qa[0] - y[0]) / 3, rel=1e-5) and g[0, 0] == 0


def test_double_dqn_and_huber():
    q = torch.zeros(1, 3)
    qn_t = torch.tensor([[1.0, 5.0, 2.0]])
    qn_o = torch.tensor([[9.0, 0.0, 1.0]])
    loss, td = losses.scalar_td_loss(q, torch.tensor([0]), torch.tensor([0.0]), torch.tensor([0.0]), qn_t, qn_o,
                                     1.0, 'huber', 1.0)
    assert float(td) == pytest.approx(1.0)          # online argmax = 0 -> target Q = 1
    assert float(loss) == pytest.approx(0.5)
    l2, _ = losses.scalar_td_loss(q, torch.tensor([0]), torch.tensor([4.0]), torch.tensor([1.0]), qn_t, None, 1.0,
                                  'huber', 1.0)
    assert float(l2) == pytest.approx(3.5)


def test_c51_projection_mass_and_loss():
    B, A, N = 4, 3, 11
    p = torch.softmax(torch.randn(B, N), -1)
    m = losses.categorical_projection(p, torch.tensor([0.0, 1.0, -20.0, 20.0]), torch.tensor([0.0, 0.0, 1.0, 1.0]),
                                      0.99, -10.0, 10.0)
    np.testing.assert_allclose(m.sum(-1).numpy(), 1.0, rtol=1e-5)
    assert float(m[2, 0]) == pytest.approx(1.0) and float(m[3, -1]) == pytest.approx(1.0)
    lg = torch.randn(B, A, N, requires_grad=True)
    loss, ce = losses.c51_loss(lg, torch.tensor([0, 1, 2, 0]), torch.zeros(B), torch.zeros(B), torch.randn(B, A, N),
                               None, 0.99, -10.0, 10.0)
    loss.backward()
    assert ce.shape == (B,) and torch.isfinite(lg.grad).all()
